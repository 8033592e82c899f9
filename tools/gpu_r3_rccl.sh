#!/bin/bash
# Round-3: RCCL collectives on the box (one rank) next to the HIP library.
set -o pipefail
TAG=${1:-rccl}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_gpu_rccl.py > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
