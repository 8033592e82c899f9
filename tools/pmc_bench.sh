#!/bin/bash
# HBM traffic of the bench's aggregation / readout kernels (two --pmc passes) -> profiles/pmc_traffic.json
set -o pipefail
TAG=${1:-pmcb}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
ARGS="--steps 1 --warmup 1 --no-cpu-baseline --no-kernel-timer"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pf -o run -- python3 bench.py $ARGS > $OUT/pf.log 2>&1 || { tail -20 $OUT/pf.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pw -o run -- python3 bench.py $ARGS > $OUT/pw.log 2>&1 || { tail -20 $OUT/pw.log; exit 1; }
python3 tools/pmc_traffic.py $OUT/pf $OUT/pw --out $OUT/pmc_traffic.json
