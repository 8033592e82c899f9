#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
tools/gpu_r5.sh tests sk tests/test_gpu_smallk.py tests/test_gpu_rows.py tests/test_gpu_parity.py -k "smallk or il4 or shard or gnn or gat" || exit 1
timeout -k 10 300 python -u tools/smallk_bench.py > gpurun_out/smallk_bench.txt 2>&1; rc=$?; cat gpurun_out/smallk_bench.txt; [ $rc = 0 ] || exit $rc
tools/gpu_r5.sh bench c3g --steps 16 --warmup 2 --no-cpu-baseline --no-inference
