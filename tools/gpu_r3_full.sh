#!/bin/bash
# Round-3 full pass: the whole -m gpu suite (margins on file), smoke, the default bench line, and
# the rocprofv3 kernel stats of the same bench.  Usage: tools/gpu_r3_full.sh TAG
set -o pipefail
TAG=${1:-full}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
export MVML_MARGINS_DIR=$OUT/margins
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --durations=40 --timeout 600 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -30 $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json; grep -E "mvml_" $OUT/bench.err | head -40
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --view-only-steps 0 --no-inference --no-kernel-timer > $OUT/prof.log 2>&1 || { tail -30 $OUT/prof.log; exit 1; }
find $OUT/prof -name '*kernel_stats.csv' | head -n 1 | xargs -I{} cp {} $OUT/kernel_stats.csv
head -n 14 $OUT/kernel_stats.csv | cut -c1-200
timeout -k 10 400 python -u bench.py --workload mvp --steps 6 --warmup 2 --no-cpu-baseline \
  --view-only-steps 0 --no-inference > $OUT/mvp.json 2> $OUT/mvp.err || { tail -30 $OUT/mvp.err; exit 1; }
head -c 300 $OUT/mvp.json; echo; grep -E "mvml_" $OUT/mvp.err | head -12
timeout -k 10 400 python -u bench.py --workload mvp --proj-bf16 --steps 6 --warmup 2 --no-cpu-baseline \
  --view-only-steps 0 --no-inference > $OUT/mvp_bf16.json 2> $OUT/mvp_bf16.err || { tail -30 $OUT/mvp_bf16.err; exit 1; }
head -c 300 $OUT/mvp_bf16.json; echo
