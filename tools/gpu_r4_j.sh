#!/bin/bash
# Round 4: per-atom dst / src backward pair (two rows in flight) vs windows on configs 3 / 5;
# forward big window vs gather kernel on config 5.  Usage: tools/gpu_r4_j.sh TAG
set -o pipefail
TAG=${1:-r4j}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity_configs.py -k "atomwise or fallback or config5" \
  -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -E "^FAILED|^ERROR|Error|assert" $OUT/pytest.log | head -40; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for cfg in 5 3; do
  mols=$([ $cfg = 3 ] && echo 65536 || echo 8192)
  for aw in 0 1; do
    MVML_BWD_ATOMWISE=$aw timeout -k 10 200 python3 -u tools/agg_bench.py --config $cfg --mols $mols --layers 01 > $OUT/agg_c${cfg}_aw$aw.log 2>&1 || { tail -30 $OUT/agg_c${cfg}_aw$aw.log; exit 1; }
    echo "== config $cfg atomwise $aw"; grep "agg_" $OUT/agg_c${cfg}_aw$aw.log
  done
done
MVML_BIG_WINDOW=0 timeout -k 10 200 python3 -u tools/agg_bench.py --config 5 --mols 8192 --layers 01 --no-bwd > $OUT/agg_c5_bw0.log 2>&1 || { tail -30 $OUT/agg_c5_bw0.log; exit 1; }
echo "== config 5 big_window 0 (forward gather kernel)"; grep "agg_" $OUT/agg_c5_bw0.log
