#!/bin/bash
# Round 4: flatten-layer backward by source atom: parity, microbench (configs 5 / 3), config-5 bench.
# Usage: tools/gpu_r4_p.sh TAG
set -o pipefail
TAG=${1:-r4p}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity_configs.py -k "flat_src or flat or hubs or fallback or overflow or gy_max" \
  -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -E "^FAILED|^ERROR|Error|assert" $OUT/pytest.log | head -40; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for cfg in 5 3; do
  mols=$([ $cfg = 3 ] && echo 65536 || echo 8192)
  for fs in 0 1; do
    MVML_FLAT_SRC=$fs timeout -k 10 200 python3 -u tools/agg_bench.py --config $cfg --mols $mols --layers 0 --no-fwd > $OUT/agg_c${cfg}_fs$fs.log 2>&1 || { tail -30 $OUT/agg_c${cfg}_fs$fs.log; exit 1; }
    echo "== config $cfg flat_src $fs: $(grep agg_bwd $OUT/agg_c${cfg}_fs$fs.log)"
  done
done
timeout -k 10 300 python3 -u bench.py --workload config5 --steps 6 --warmup 2 --no-cpu-baseline --no-inference > $OUT/bench5.json 2> $OUT/bench5.err || { tail -30 $OUT/bench5.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench5.json')); print({k: d.get(k) for k in ('value','ms_per_step')}); print(d['roofline']['frac'], d['roofline_agg_bwd'])"
