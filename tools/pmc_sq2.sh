#!/bin/bash
# SQ counters of the aggregation backward (agg_bench --no-fwd), three --pmc passes.  Usage: tools/pmc_sq2.sh TAG [agg_bench args]
set -o pipefail
TAG=${1:-sq}; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
run() {
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$N -o run -- python3 tools/agg_bench.py --no-fwd $ARGS > $OUT/$N.log 2>&1 || { tail -20 $OUT/$N.log; exit 1; }
  python3 tools/pmc_summary.py $OUT/$N 'gat_agg_\w+_kernel<[^>]*>'
}
ARGS="$*"
N=p1 run SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE
N=p2 run SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH
N=p3 run SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_WAIT_INST_ANY SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA
