#!/bin/bash
# Round 4: the driver's exact bench command, then the same command under rocprofv3 --kernel-trace
# (idle time between kernels per timed step, tools/trace_gaps.py).  Usage: tools/gpu_r4_gap.sh TAG [bench args]
set -o pipefail
TAG=${1:-gap}; shift; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 "$@" > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python3 -c "import json,sys; d=json.load(open('$OUT/bench.json')); print({k: d.get(k) for k in ('value','ms_per_step','untimed_ms_per_step','allocator')}); print(d.get('step_ms'))"
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python3 bench.py --steps 20 --warmup 5 \
  --no-cpu-baseline --view-only-steps 0 --no-inference "$@" > $OUT/trace.json 2> $OUT/trace.err || { tail -30 $OUT/trace.err; exit 1; }
python3 tools/trace_gaps.py $OUT/trace --steps 20 > $OUT/gaps.txt && cat $OUT/gaps.txt
