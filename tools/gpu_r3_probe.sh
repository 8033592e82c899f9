#!/bin/bash
# Round-3 probe: GEMM time per shape in the bench step, then current counters of the split-fp16
# GEMM (L2 fwd / dX / dW / LSTM gates shapes).  Usage: tools/gpu_r3_probe.sh TAG
set -o pipefail
TAG=${1:-probe}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
MVML_GEMM_SHAPES=1 timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline \
  --view-only-steps 0 --no-inference > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
grep -E "gemm|mvml_" $OUT/bench.err | head -60
bash tools/pmc_gemm.sh $TAG/pmc f16x2 0,1,2,4
