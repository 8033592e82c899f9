#!/bin/bash
# Round-3: config-5 aggregation microbench + the config-5 bench line on the current build.
set -o pipefail
TAG=${1:-c5}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/agg_bench.py --config 5 --mols 8192 > $OUT/agg_c5.txt 2>&1 || { tail -20 $OUT/agg_c5.txt; exit 1; }
cat $OUT/agg_c5.txt
timeout -k 10 400 python -u bench.py --workload config5 --steps 6 --warmup 2 --no-cpu-baseline --view-only-steps 0 \
  --no-inference > $OUT/c5.json 2> $OUT/c5.err || { tail -30 $OUT/c5.err; exit 1; }
head -c 400 $OUT/c5.json; echo; grep -E "mvml_" $OUT/c5.err | head -24
