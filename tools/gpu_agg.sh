#!/bin/bash
# Aggregation microbench + kernel trace + HBM PMC passes on the GPU box.  Usage: tools/gpu_agg.sh TAG [extra agg_bench args]
set -o pipefail
TAG=${1:-agg}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 240 python -u tools/agg_bench.py "$@" > $OUT/agg.log 2>&1 || { tail -30 $OUT/agg.log; exit 1; }
cat $OUT/agg.log
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 tools/agg_bench.py "$@" > $OUT/kt.log 2>&1 || { tail -30 $OUT/kt.log; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, sys
p = glob.glob(sys.argv[1] + "/kt/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(p)):
    print(f"{r['Name'][:110]:110s} n={r['Calls']:>4s} avg={float(r['AverageNs'])/1e3:9.1f} us")
PY
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pf -o run -- python3 tools/agg_bench.py "$@" > $OUT/pf.log 2>&1 || { tail -30 $OUT/pf.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pw -o run -- python3 tools/agg_bench.py "$@" > $OUT/pw.log 2>&1 || { tail -30 $OUT/pw.log; exit 1; }
python3 tools/pmc_summary.py $OUT/pf '(gat_\w+|seg_\w+)(<[^>]*>)?'
python3 tools/pmc_summary.py $OUT/pw '(gat_\w+|seg_\w+)(<[^>]*>)?'
