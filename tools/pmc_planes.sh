#!/bin/bash
# Counters of the LDS-DMA split-fp16 tile and the register-staged tile on one product shape
# (tools/planes_bench.py shape IDX), three --pmc passes + a kernel trace, each its own run.
#   tools/pmc_planes.sh TAG IDX   -> gpurun_out/TAG/{p1,p2,p3,kt}; report:
#   python tools/pmc_gemm_report.py gpurun_out/TAG/p1 gpurun_out/TAG/p2 gpurun_out/TAG/p3 \
#       --stats gpurun_out/TAG/kt/run_kernel_stats.csv
set -o pipefail
TAG=${1:-pp}; SH=${2:-0}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
run() { timeout -s KILL 240 rocprofv3 --pmc $2 --output-format csv -d $OUT/$1 -o run -- python3 tools/planes_bench.py $SH --iters 3 > $OUT/$1.log 2>&1 || { tail -20 $OUT/$1.log; exit 1; }; }
run p1 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
run p2 "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM"
run p3 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_ACTIVE_INST_VMEM"
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 tools/planes_bench.py $SH --iters 3 > $OUT/kt.log 2>&1 || { tail -20 $OUT/kt.log; exit 1; }
