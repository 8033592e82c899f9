#!/bin/bash
# MFMA / VALU / wait counters of the GEMM microbench.  Usage: tools/pmc_gemm.sh TAG
set -o pipefail
TAG=${1:-pg}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
run() { timeout -s KILL 180 rocprofv3 --pmc $2 --output-format csv -d $OUT/$1 -o run -- python3 tools/gemm_bench.py > $OUT/$1.log 2>&1 || { tail -20 $OUT/$1.log; exit 1; }; }
run p1 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
run p2 "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM"
for d in p1 p2; do python3 tools/pmc_summary.py $OUT/$d 'gemm_f32_kernel<[^>]*>'; done
