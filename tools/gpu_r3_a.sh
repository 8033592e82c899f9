#!/bin/bash
# Round-3 call A: new parity tests (bench-size, ReLU branch capture, bf16 MVP, GEMM dynamic
# range), then the GEMM probe.  Usage: tools/gpu_r3_a.sh TAG
set -o pipefail
TAG=${1:-a}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
export MVML_MARGINS_DIR=$OUT/margins
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k "dynamic_range" tests/test_gpu_fusion.py tests/test_gpu_mvp.py \
  > $OUT/pytest_small.log 2>&1; rc=$?; tail -15 $OUT/pytest_small.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 900 --timeout-method thread \
  tests/test_gpu_parity_bench.py > $OUT/pytest_bench.log 2>&1; rc=$?; tail -15 $OUT/pytest_bench.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
bash tools/gpu_r3_probe.sh $TAG/probe
