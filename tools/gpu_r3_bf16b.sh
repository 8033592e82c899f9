#!/bin/bash
# Round-3: bf16 projection on the el / er GEMM-column path — bf16 / MVP tests, then the benches.
set -o pipefail
TAG=${1:-bf16b}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bf16.py tests/test_gpu_mvp.py \
  > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
bash tools/gpu_r3_bf16.sh $TAG
