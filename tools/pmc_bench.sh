#!/bin/bash
# HBM traffic of the bench's aggregation / readout kernels (two --pmc passes, default workload)
# -> gpurun_out/$TAG/pmc_traffic.json under the bench's workload key (copy into profiles/).
set -o pipefail
TAG=${1:-pmcb}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
# WORKLOAD=config5 profiles the config-5 bench batch (8,192 molecules per step) instead
WORKLOAD=${WORKLOAD:-config3}
if [ "$WORKLOAD" = config5 ]; then
  ARGS="--workload config5 --steps 1 --warmup 1 --no-cpu-baseline --no-kernel-timer --view-only-steps 0 --no-inference"
  KEY="config5/mols_per_step=8192"
else
  ARGS="--total-mols 131072 --steps 1 --warmup 1 --no-cpu-baseline --no-kernel-timer --view-only-steps 0 --no-inference"
  KEY="config3/mols_per_step=65536"
fi
cp profiles/pmc_traffic.json $OUT/pmc_traffic.json
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pf -o run -- python3 bench.py $ARGS > $OUT/pf.log 2>&1 || { tail -20 $OUT/pf.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pw -o run -- python3 bench.py $ARGS > $OUT/pw.log 2>&1 || { tail -20 $OUT/pw.log; exit 1; }
python3 tools/pmc_traffic.py $OUT/pf $OUT/pw --workload "$KEY" --out $OUT/pmc_traffic.json
