#!/bin/bash
# Round-3 call B: fused attention + Conv2d kernels (fusion tests), the bench-size parity test,
# then a short bench with the per-kernel breakdown.  Usage: tools/gpu_r3_b.sh TAG
set -o pipefail
TAG=${1:-b}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
export MVML_MARGINS_DIR=$OUT/margins
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_fusion.py tests/test_gpu_mvp.py > $OUT/pytest_fusion.log 2>&1 || { tail -40 $OUT/pytest_fusion.log; exit 1; }
tail -3 $OUT/pytest_fusion.log
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 900 --timeout-method thread \
  tests/test_gpu_parity_bench.py -k config3 > $OUT/pytest_bench.log 2>&1 || { tail -40 $OUT/pytest_bench.log; exit 1; }
tail -3 $OUT/pytest_bench.log
timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline --view-only-steps 0 \
  --no-inference > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json; grep -E "mvml_" $OUT/bench.err | head -40
