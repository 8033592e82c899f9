#!/bin/bash
# Round 4: the bench-size parity tests (float64 oracle on the GPU; margins to $OUT/margins).
# Usage: tools/gpu_r4_parity.sh TAG [pytest -k expr]
set -o pipefail
TAG=${1:-parity}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
export MVML_MARGINS_DIR=$OUT/margins
timeout -k 10 1100 python3 -u -m pytest tests/test_gpu_parity_bench.py -m gpu -v --durations=10 --timeout 1050 --timeout-method thread \
  ${2:+-k "$2"} > $OUT/parity.log 2>&1 || { tail -80 $OUT/parity.log; exit 1; }
tail -14 $OUT/parity.log
