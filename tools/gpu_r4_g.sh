#!/bin/bash
# Round 4: config-5 head-mean backward (source atom) parity + microbench + kernel stats, PMC
# traffic of the config-5 bench batch, config-5 bench line, config-2 per-layer refresh.
# Usage: tools/gpu_r4_g.sh TAG
set -o pipefail
TAG=${1:-r4g}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity_configs.py -k "mean_src or row_maxima or layer1_config5" \
  -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -E "^FAILED|^ERROR|Error|assert" $OUT/pytest.log | head -40; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
MVML_MEAN_SRC=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt5 -o run -- python3 tools/agg_bench.py --config 5 --mols 8192 --layers 1 --no-fwd > $OUT/agg_c5.log 2>&1 || { tail -30 $OUT/agg_c5.log; exit 1; }
grep "agg_" $OUT/agg_c5.log
python3 - "$OUT" <<'PY'
import csv, glob, sys
p = glob.glob(sys.argv[1] + "/kt5/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(p)))[:6]:
    print(f"{r['Name'][:100]:100s} n={r['Calls']:>4s} avg={float(r['AverageNs'])/1e3:9.1f} us")
PY
for c in FETCH_SIZE WRITE_SIZE; do
  MVML_MEAN_SRC=1 timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $OUT/p5_$c -o run -- python3 tools/agg_bench.py --config 5 --mols 8192 --layers 1 --no-fwd > $OUT/p5_$c.log 2>&1 || { tail -20 $OUT/p5_$c.log; exit 1; }
  python3 tools/pmc_summary.py $OUT/p5_$c '(gat_\w+)(<[^>]*>)?'
done
WORKLOAD=config5 bash tools/pmc_bench.sh $TAG/pmc5 > $OUT/pmc5.log 2>&1 || { tail -30 $OUT/pmc5.log; exit 1; }
cp $OUT/pmc5/pmc_traffic.json profiles/pmc_traffic.json
python3 -c "import json; d=json.load(open('profiles/pmc_traffic.json'))['config5/mols_per_step=8192']; print({k: (v['hbm_bytes_per_launch'], v['calls']) for k, v in d.items()})"
timeout -k 10 300 python3 -u bench.py --workload config5 --steps 6 --warmup 2 --no-cpu-baseline --no-inference > $OUT/bench5.json 2> $OUT/bench5.err || { tail -30 $OUT/bench5.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench5.json')); print({k: d.get(k) for k in ('value','ms_per_step')}); print(d['roofline']); print(d['roofline_agg_bwd'])"
timeout -k 10 200 python3 -u tools/agg_bench.py --config 2 --mols 65536 --layers 01 > $OUT/agg_c2.log 2>&1 || { tail -30 $OUT/agg_c2.log; exit 1; }
grep "agg_" $OUT/agg_c2.log
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $OUT/p2_$c -o run -- python3 tools/agg_bench.py --config 2 --mols 65536 --layers 01 > $OUT/p2_$c.log 2>&1 || { tail -20 $OUT/p2_$c.log; exit 1; }
  python3 tools/pmc_summary.py $OUT/p2_$c '(gat_\w+)(<[^>]*>)?'
done
