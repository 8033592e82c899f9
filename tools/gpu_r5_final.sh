#!/bin/bash
# Round-5 final passes (one per gpurun call): tests | bench | extra
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
case "$1" in
  tests)
    timeout -k 10 900 python -u -m pytest tests -m gpu -q --durations=15 --timeout 300 --timeout-method thread \
      > gpurun_out/r05_gputest_final.log 2>&1; rc=$?; tail -4 gpurun_out/r05_gputest_final.log; [ $rc = 0 ] || exit $rc
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05_smoke.log 2>&1; rc=$?
    tail -3 gpurun_out/r05_smoke.log; exit $rc ;;
  bench)
    timeout -k 10 600 python -u bench.py > gpurun_out/r05_bench_final.json 2> gpurun_out/r05_bench_final.err; rc=$?
    cat gpurun_out/r05_bench_final.json; [ $rc = 0 ] || exit $rc
    export TMPDIR=/tmp
    timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05_prof_final -o run -- \
      python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-inference > gpurun_out/r05_prof_final.log 2>&1; rc=$?
    tail -2 gpurun_out/r05_prof_final.log; exit $rc ;;
  extra)
    timeout -k 10 400 python -u bench.py --workload config5 --steps 10 --warmup 3 --no-cpu-baseline --no-inference \
      > gpurun_out/r05_bench_config5_final.json 2> gpurun_out/r05_bench_config5_final.err || exit 1
    timeout -k 10 300 python -u bench.py --workload mvp --steps 10 --warmup 3 --no-cpu-baseline --no-inference \
      > gpurun_out/r05_bench_mvp_final.json 2> gpurun_out/r05_bench_mvp_final.err || exit 1
    timeout -k 10 300 python -u bench.py --workload mvp --proj-bf16 --steps 10 --warmup 3 --no-cpu-baseline --no-inference \
      > gpurun_out/r05_bench_mvp_bf16_final.json 2> gpurun_out/r05_bench_mvp_bf16_final.err
    exit $? ;;
esac
