#!/bin/bash
# Round 4: per-step batch size sweep of the config-3 step (65,536 vs 131,072 molecules per GPU).
set -o pipefail
TAG=${1:-r4o}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
for mps in 131072 65536; do
  timeout -k 10 400 python3 -u bench.py --steps 10 --warmup 3 --mols-per-step $mps --no-inference --no-cpu-baseline --view-only-steps 0 > $OUT/bench_$mps.json 2> $OUT/bench_$mps.err || { tail -30 $OUT/bench_$mps.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$mps.json')); print($mps, {k: d.get(k) for k in ('value','ms_per_step','untimed_ms_per_step')}, d['roofline_gemm']['frac'], d['allocator'])"
done
