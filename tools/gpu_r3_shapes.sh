#!/bin/bash
# Short config-3 bench with the per-kernel and per-GEMM-shape breakdowns.  Usage: tools/gpu_r3_shapes.sh TAG [bench args]
set -o pipefail
TAG=${1:-shapes}; shift; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
MVML_GEMM_SHAPES=1 timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline --view-only-steps 0 \
  --no-inference "$@" > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
head -c 400 $OUT/bench.json; echo; grep -E "mvml_|gemm" $OUT/bench.err | head -60
