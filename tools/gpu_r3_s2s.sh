#!/bin/bash
# Round-3: Set2Set gates + cell on the 128x128 kernel (MVML_LSTM_TILE=128) vs the 256x256 plan.
set -o pipefail
TAG=${1:-s2s}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "set2set" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
for t in 0 128 0 128; do
  MVML_LSTM_TILE=$t timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline --view-only-steps 0 --no-inference > $OUT/c3_$t.json 2> $OUT/c3_$t.err || { tail -30 $OUT/c3_$t.err; exit 1; }
  echo "tile $t: $(head -c 200 $OUT/c3_$t.json)"; grep -E "lstm_gates_cell_fwd" $OUT/c3_$t.err
done
