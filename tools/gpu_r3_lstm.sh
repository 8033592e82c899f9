#!/bin/bash
# Round-3: wide BiLSTM recurrence — SMILES / MVP GPU tests, then the MVP bench (fp32 projection).
set -o pipefail
TAG=${1:-lstm}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_smiles.py tests/test_gpu_mvp.py > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 400 python -u bench.py --workload mvp --steps 6 --warmup 2 --no-cpu-baseline \
  --view-only-steps 0 --no-inference > $OUT/mvp.json 2> $OUT/mvp.err || { tail -30 $OUT/mvp.err; exit 1; }
head -c 300 $OUT/mvp.json; echo; grep -E "mvml_" $OUT/mvp.err | head -14
