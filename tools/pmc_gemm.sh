#!/bin/bash
# MFMA / VALU / LDS / wait counters of the GEMM microbench.  Usage: tools/pmc_gemm.sh TAG ALGOS SHAPES
set -o pipefail
TAG=${1:-pg}; ALG=${2:-x3-256}; SH=${3:-0}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
run() { timeout -s KILL 180 rocprofv3 --pmc $2 --output-format csv -d $OUT/$1 -o run -- python3 tools/gemm_bench.py $ALG $SH > $OUT/$1.log 2>&1 || { tail -20 $OUT/$1.log; exit 1; }; }
run p1 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
run p2 "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM"
run p3 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_ACTIVE_INST_VMEM"
for d in p1 p2 p3; do python3 tools/pmc_summary.py $OUT/$d 'gemm_\w+_kernel<[^>]*>'; done
