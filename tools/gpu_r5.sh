#!/bin/bash
# Round-5 GPU runner: one named step per call, every GPU step under its own time limit.
#   tools/gpu_r5.sh <step> [args...]
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
step=$1; shift
case "$step" in
  tests)   # pytest selection: tools/gpu_r5.sh tests <tag> <pytest args...>
    tag=$1; shift
    timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread "$@" \
      > gpurun_out/tests_$tag.log 2>&1; rc=$?; tail -5 gpurun_out/tests_$tag.log; exit $rc ;;
  agg)     # aggregation A/B: tools/gpu_r5.sh agg <tag> <agg_bench args...>
    tag=$1; shift
    timeout -k 10 600 python -u tools/agg_bench.py "$@" > gpurun_out/agg_$tag.txt 2>&1; rc=$?
    cat gpurun_out/agg_$tag.txt; exit $rc ;;
  bench)   # bench.py: tools/gpu_r5.sh bench <tag> <bench args...>
    tag=$1; shift
    timeout -k 10 900 python -u bench.py "$@" > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err; rc=$?
    tail -3 gpurun_out/bench_$tag.err; cat gpurun_out/bench_$tag.json; exit $rc ;;
  prof)    # rocprofv3 kernel stats of a command: tools/gpu_r5.sh prof <tag> <python args...>
    tag=$1; shift
    export TMPDIR=/tmp
    timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- python3 "$@" \
      > gpurun_out/prof_$tag.log 2>&1; rc=$?; tail -3 gpurun_out/prof_$tag.log; exit $rc ;;
  pmc)     # one PMC pass: tools/gpu_r5.sh pmc <tag> "<counters>" <python args...>
    tag=$1; ctr=$2; shift 2
    export TMPDIR=/tmp
    timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/pmc_$tag -o run -- python3 "$@" \
      > gpurun_out/pmc_$tag.log 2>&1; rc=$?; tail -3 gpurun_out/pmc_$tag.log; exit $rc ;;
  *) echo "unknown step $step"; exit 2 ;;
esac
