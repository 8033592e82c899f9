#!/bin/bash
# Round-3: BASELINE config 4 (the whole MVP step) with fp32-accurate and bf16 projections, plus
# the config-3 bench with the per-kernel breakdown.  Usage: tools/gpu_r3_mvp.sh TAG
set -o pipefail
TAG=${1:-mvp}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --workload mvp --steps 6 --warmup 2 --no-cpu-baseline \
  --view-only-steps 0 --no-inference > $OUT/mvp.json 2> $OUT/mvp.err || { tail -30 $OUT/mvp.err; exit 1; }
cat $OUT/mvp.json; grep -E "mvml_" $OUT/mvp.err | head -16
timeout -k 10 400 python -u bench.py --workload mvp --proj-bf16 --steps 6 --warmup 2 --no-cpu-baseline \
  --view-only-steps 0 --no-inference > $OUT/mvp_bf16.json 2> $OUT/mvp_bf16.err || { tail -30 $OUT/mvp_bf16.err; exit 1; }
cat $OUT/mvp_bf16.json
timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline --view-only-steps 0 \
  --no-inference > $OUT/c3.json 2> $OUT/c3.err || { tail -30 $OUT/c3.err; exit 1; }
cat $OUT/c3.json | head -c 600; echo; grep -E "mvml_" $OUT/c3.err | head -30
