#!/bin/bash
# PMC traffic (FETCH_SIZE / WRITE_SIZE passes) of the config-3 and config-5 bench batches
set -o pipefail
cd "$(dirname "$0")/.."
WORKLOAD=config3 bash tools/pmc_bench.sh pmc3 > gpurun_out/pmc3.txt 2>&1 || { tail -30 gpurun_out/pmc3.txt; exit 1; }
cp gpurun_out/pmc3/pmc_traffic.json profiles/pmc_traffic.json
WORKLOAD=config5 bash tools/pmc_bench.sh pmc5 > gpurun_out/pmc5.txt 2>&1 || { tail -30 gpurun_out/pmc5.txt; exit 1; }
cp gpurun_out/pmc5/pmc_traffic.json gpurun_out/pmc_traffic_new.json
