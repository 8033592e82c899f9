#!/bin/bash
# Round-3 call E: fused attention + Conv2d backward without flat weight loads / spills — fusion
# tests, the attn-conv microbench, then the hipBLASLt yardstick for the split-fp16 GEMM.
set -o pipefail
TAG=${1:-e}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_fusion.py tests/test_gpu_mvp.py > $OUT/pytest_fusion.log 2>&1 || { tail -40 $OUT/pytest_fusion.log; exit 1; }
tail -3 $OUT/pytest_fusion.log
timeout -k 10 200 python -u tools/attn_conv_bench.py > $OUT/attn_conv.txt 2>&1 || { tail -20 $OUT/attn_conv.txt; exit 1; }
cat $OUT/attn_conv.txt
timeout -k 10 300 python -u tools/ceiling_bench.py > $OUT/ceiling.txt 2>&1 || { tail -20 $OUT/ceiling.txt; exit 1; }
cat $OUT/ceiling.txt
