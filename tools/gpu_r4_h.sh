#!/bin/bash
# Round 4: head-mean backward by source atom on config 3 (microbench + whole step, A/B).
# Usage: tools/gpu_r4_h.sh TAG
set -o pipefail
TAG=${1:-r4h}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
for ms in 0 1; do
  MVML_MEAN_SRC=$ms timeout -k 10 200 python3 -u tools/agg_bench.py --config 3 --mols 65536 --layers 1 --no-fwd > $OUT/agg_c3_ms$ms.log 2>&1 || { tail -30 $OUT/agg_c3_ms$ms.log; exit 1; }
  echo "mean_src $ms: $(grep agg_bwd $OUT/agg_c3_ms$ms.log)"
done
for ms in 1 0; do
  MVML_MEAN_SRC=$ms timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-inference --no-cpu-baseline --view-only-steps 0 > $OUT/bench_ms$ms.json 2> $OUT/bench_ms$ms.err || { tail -30 $OUT/bench_ms$ms.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_ms$ms.json')); print('mean_src $ms', {k: d.get(k) for k in ('value','ms_per_step')}, d['roofline_agg_bwd']['frac'], d['kernel_ms_per_step']['mvml_gat_agg_bwd'])"
done
