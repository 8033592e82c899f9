#!/bin/bash
# SQ counters of the conv3 kernels (tools/conv_bench.py), two --pmc passes.  Usage: tools/pmc_conv.sh TAG
set -o pipefail
TAG=${1:-pconv}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 120 python3 tools/conv_bench.py > $OUT/t.txt 2>&1 || { tail -20 $OUT/t.txt; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $OUT/p1 -o run -- python3 tools/conv_bench.py --reps 2 > $OUT/p1.log 2>&1 || { tail -20 $OUT/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA SQ_INSTS_SMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/p2 -o run -- python3 tools/conv_bench.py --reps 2 > $OUT/p2.log 2>&1 || { tail -20 $OUT/p2.log; exit 1; }
cat $OUT/t.txt
python3 tools/pmc_summary.py $OUT/p1 'conv3_\w+_kernel'
python3 tools/pmc_summary.py $OUT/p2 'conv3_\w+_kernel'
