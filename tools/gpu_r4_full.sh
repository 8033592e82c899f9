#!/bin/bash
# Round 4: the whole GPU suite (the bench-size parity file separately: tools/gpu_r4_parity.sh) and smoke().
# Usage: tools/gpu_r4_full.sh TAG
set -o pipefail
TAG=${1:-full}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
export MVML_MARGINS_DIR=$OUT/margins
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -v --durations=15 --timeout 300 --timeout-method thread \
  --deselect tests/test_gpu_parity_bench.py > $OUT/gputest.log 2>&1 || { tail -80 $OUT/gputest.log; exit 1; }
tail -4 $OUT/gputest.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -30 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
