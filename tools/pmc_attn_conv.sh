#!/bin/bash
# Fused attention + Conv2d kernels vs the separate ones (tools/attn_conv_bench.py, 65,536 molecules):
# timings, then HBM traffic of the fused pair (FETCH_SIZE / WRITE_SIZE, separate passes) and the
# kernel trace.  Usage: tools/pmc_attn_conv.sh TAG
set -o pipefail
TAG=${1:-pac}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 180 python3 tools/attn_conv_bench.py > $OUT/t.txt 2>&1 || { tail -20 $OUT/t.txt; exit 1; }
cat $OUT/t.txt
A="tools/attn_conv_bench.py --only fused --reps 2"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pf -o run -- python3 $A > $OUT/pf.log 2>&1 || { tail -20 $OUT/pf.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pw -o run -- python3 $A > $OUT/pw.log 2>&1 || { tail -20 $OUT/pw.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $OUT/p1 -o run -- python3 $A > $OUT/p1.log 2>&1 || { tail -20 $OUT/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run -- python3 tools/attn_conv_bench.py > $OUT/kt.log 2>&1 || { tail -20 $OUT/kt.log; exit 1; }
python3 tools/pmc_summary.py $OUT/pf 'attn_conv_\w+_kernel'
python3 tools/pmc_summary.py $OUT/pw 'attn_conv_\w+_kernel'
python3 tools/pmc_summary.py $OUT/p1 'attn_conv_\w+_kernel'
find $OUT/kt -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/kernel_stats.csv
