#!/bin/bash
# One parameterised runner for the GPU passes (one gpurun call may chain several):
#   tools/gpu_run.sh TAG PASS [PASS ...]
# Passes:
#   tests[:EXPR]   pytest -m gpu (optionally -k EXPR)       -> gpurun_out/TAG_gputest.log
#   smoke          __graft_entry__.smoke()                   -> gpurun_out/TAG_smoke.log
#   bench          python bench.py (the driver's command)    -> gpurun_out/TAG_bench.json
#   prof           rocprofv3 kernel trace + stats of a short bench -> gpurun_out/TAG_prof/
#   config5 | mvp | mvpbf16   the other bench workloads      -> gpurun_out/TAG_<pass>.json
#   ab[:V,V..]     bench.py (20 steps) of each tree back to back on one box: variants/<V> (the
#                  round-4 / round-5 trees with their own libraries) or . (this tree); default r04,r05,.
#   dp2            bench.py --gpus 2, both ranks on cuda:0 over gloo -> gpurun_out/TAG_dp2.json
#   planes[:IDX]   tools/planes_bench.py (IDX: shape indices) -> gpurun_out/TAG_planes.txt
#   pmc[:WL]       tools/pmc_bench.sh: PMC HBM traffic of the bench workload WL (config3 | config5)
# Every GPU step runs under its own time limit; the first failing step ends the call.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=$1
shift
O=gpurun_out/$TAG
for P in "$@"; do
  NAME=${P%%:*}
  ARG=${P#*:}
  [ "$ARG" = "$P" ] && ARG=""
  echo "== $TAG $P"
  case "$NAME" in
    tests)
      K=()
      [ -n "$ARG" ] && K=(-k "$ARG")
      timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --durations=10 --timeout 300 --timeout-method thread \
        "${K[@]}" > ${O}_gputest.log 2>&1; rc=$?; tail -4 ${O}_gputest.log; [ $rc = 0 ] || exit $rc ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > ${O}_smoke.log 2>&1
      rc=$?; tail -3 ${O}_smoke.log; [ $rc = 0 ] || exit $rc ;;
    bench)
      timeout -k 10 600 python -u bench.py > ${O}_bench.json 2> ${O}_bench.err; rc=$?
      cat ${O}_bench.json; [ $rc = 0 ] || exit $rc ;;
    config5|mvp|mvpbf16)
      EXTRA=(--workload $NAME)
      [ $NAME = mvpbf16 ] && EXTRA=(--workload mvp --proj-bf16)
      timeout -k 10 500 python -u bench.py "${EXTRA[@]}" --steps 10 --warmup 3 --no-cpu-baseline --no-inference \
        > ${O}_$NAME.json 2> ${O}_$NAME.err; rc=$?; cat ${O}_$NAME.json; [ $rc = 0 ] || exit $rc ;;
    prof)
      export TMPDIR=/tmp
      timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d ${O}_prof -o run -- \
        python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-inference > ${O}_prof.log 2>&1; rc=$?
      tail -2 ${O}_prof.log; [ $rc = 0 ] || exit $rc ;;
    ab)
      VL=${ARG:-r04,r05,.}
      for V in ${VL//,/ }; do
        VN=$V; [ "$V" = . ] && VN=head
        [ "$V" != . ] && V=variants/$V
        (cd $V && timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline \
          --no-inference) > ${O}_ab_$VN.json 2> ${O}_ab_$VN.err; rc=$?
        cat ${O}_ab_$VN.json; [ $rc = 0 ] || exit $rc
      done ;;
    dp2)  # the 2-rank DP path rehearsed on the one GPU (gloo; RCCL refuses two ranks per device)
      MVML_BENCH_ONE_DEVICE=1 MVML_BENCH_BACKEND=gloo timeout -k 10 600 python -u bench.py --gpus 2 --steps 6 \
        --warmup 2 --no-cpu-baseline --no-inference > ${O}_dp2.json 2> ${O}_dp2.err; rc=$?
      cat ${O}_dp2.json; [ $rc = 0 ] || exit $rc ;;
    planes)
      timeout -k 10 600 python -u tools/planes_bench.py $ARG > ${O}_planes.txt 2>&1; rc=$?
      cat ${O}_planes.txt; [ $rc = 0 ] || exit $rc ;;
    pmc)  # HBM traffic (FETCH_SIZE / WRITE_SIZE passes) of the bench workload ARG (config3 | config5)
      WORKLOAD=${ARG:-config3} timeout -k 10 700 bash tools/pmc_bench.sh ${TAG}_pmc_${ARG:-config3} \
        > ${O}_pmc_${ARG:-config3}.log 2>&1; rc=$?
      tail -3 ${O}_pmc_${ARG:-config3}.log; [ $rc = 0 ] || exit $rc ;;
    *) echo "unknown pass $P"; exit 2 ;;
  esac
done
