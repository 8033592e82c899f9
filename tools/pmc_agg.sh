#!/bin/bash
# HBM traffic + L2 hit + SQ wait counters for the aggregation microbench.  Usage: tools/pmc_agg.sh TAG
set -o pipefail
TAG=${1:-pa}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
run() { timeout -s KILL 120 rocprofv3 --pmc $2 --output-format csv -d $OUT/$1 -o run -- python3 tools/agg_bench.py > $OUT/$1.log 2>&1 || { tail -20 $OUT/$1.log; exit 1; }; }
run pf "FETCH_SIZE"
run pw "WRITE_SIZE"
run ph "TCC_HIT_sum TCC_MISS_sum"
run sq "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU GRBM_GUI_ACTIVE"
for d in pf pw ph sq; do python3 tools/pmc_summary.py $OUT/$d '(gat_\w+)(<[^>]*>)?'; done
