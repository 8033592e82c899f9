#!/bin/bash
# SQ issue/wait counters of the config-5 aggregation microbench (big-window kernels), two --pmc
# passes.  Usage: tools/pmc_sq5.sh TAG
set -o pipefail
TAG=${1:-sq5}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
ARGS="--config 5 --mols 4096"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $OUT/p1 -o run -- python3 tools/agg_bench.py $ARGS > $OUT/p1.log 2>&1 || { tail -20 $OUT/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_LDS_IDX_ACTIVE --output-format csv -d $OUT/p2 -o run -- python3 tools/agg_bench.py $ARGS > $OUT/p2.log 2>&1 || { tail -20 $OUT/p2.log; exit 1; }
python3 tools/pmc_summary.py $OUT/p1 'gat_agg_\w+_kernel<[^>]*true>'
python3 tools/pmc_summary.py $OUT/p2 'gat_agg_\w+_kernel<[^>]*true>'
