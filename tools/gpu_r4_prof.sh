#!/bin/bash
# Round 4: the driver's bench command, then the same bench under rocprofv3 --kernel-trace --stats
# (kernel stats for profiles/, idle gaps per step, GEMM time per dispatch shape).
# Usage: tools/gpu_r4_prof.sh TAG [bench args]
set -o pipefail
TAG=${1:-prof}; shift; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 "$@" > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print({k: d.get(k) for k in ('value','ms_per_step','untimed_ms_per_step')}); print(d['roofline']['frac'], d['roofline_agg_bwd']['frac'], d['roofline_gemm']['frac'], d['roofline_gemm']['achieved'])"
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --steps 20 --warmup 5 \
  --no-cpu-baseline --view-only-steps 0 --no-inference "$@" > $OUT/trace.json 2> $OUT/trace.err || { tail -30 $OUT/trace.err; exit 1; }
python3 tools/trace_gaps.py $OUT/trace --steps 20 --marker layernorm_fwd > $OUT/gaps.txt && head -24 $OUT/gaps.txt | tail -3
python3 tools/trace_shapes.py $OUT/trace --steps 25 --match gemm > $OUT/shapes.txt && cat $OUT/shapes.txt
