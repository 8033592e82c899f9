#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
tools/gpu_r5.sh tests sk tests/test_gpu_smallk.py || exit 1
timeout -k 10 300 python -u tools/smallk_bench.py > gpurun_out/smallk_bench.txt 2>&1; rc=$?; cat gpurun_out/smallk_bench.txt; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u tools/smallk_bench.py --random --kinds 1,7,0 > gpurun_out/smallk_bench_rand.txt 2>&1; rc=$?; cat gpurun_out/smallk_bench_rand.txt; exit $rc
