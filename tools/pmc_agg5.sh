#!/bin/bash
# Counters of the config-5 aggregation backward fallback kernels (agg_bench --no-fwd, L2 mean).
set -o pipefail
TAG=${1:-a5}; shift; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
ARGS="--config 5 --mols 8192 --layers ${LAYERS:-1} --no-fwd"
run() {
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$N -o run -- python3 tools/agg_bench.py $ARGS > $OUT/$N.log 2>&1 || { tail -20 $OUT/$N.log; exit 1; }
  python3 tools/pmc_summary.py $OUT/$N 'gat_agg_\w+_kernel<[^>]*>'
}
N=p1 run SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE
N=p2 run TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum
N=p3 run FETCH_SIZE
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 tools/agg_bench.py $ARGS > $OUT/kt.log 2>&1 || exit 1
cat $OUT/kt.log | grep -v amdgpu.ids
