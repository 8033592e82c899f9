#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 300 python -u tools/smallk_bench.py --kinds 1,3,4,1,3,4,0 > gpurun_out/smallk_chunk.txt 2>&1; rc=$?; cat gpurun_out/smallk_chunk.txt; exit $rc
