#!/bin/bash
# Round-3 call D: counters of the two split-fp16 GEMM kernels (ring on / off) on the L2 forward /
# dX shapes, the bench-size parity test, then a short bench.  Usage: tools/gpu_r3_d.sh TAG
set -o pipefail
TAG=${1:-d}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
MVML_GEMM_RING=1 bash tools/pmc_gemm.sh $TAG/pmc_ring1 f16x2 0,1 > $OUT/pmc_ring1.txt 2>&1 || { tail -20 $OUT/pmc_ring1.txt; exit 1; }
MVML_GEMM_RING=0 bash tools/pmc_gemm.sh $TAG/pmc_ring0 f16x2 0,1 > $OUT/pmc_ring0.txt 2>&1 || { tail -20 $OUT/pmc_ring0.txt; exit 1; }
export MVML_MARGINS_DIR=$OUT/margins
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 900 --timeout-method thread \
  tests/test_gpu_parity_bench.py -k config3 > $OUT/pytest_bench.log 2>&1 || { tail -40 $OUT/pytest_bench.log; exit 1; }
tail -3 $OUT/pytest_bench.log
timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline --view-only-steps 0 \
  --no-inference > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json; grep -E "mvml_" $OUT/bench.err | head -40
