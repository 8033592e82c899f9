#!/bin/bash
# Round 4 final pass: whole GPU suite (bench-size parity included), smoke, the driver's bench
# command, rocprofv3 kernel stats of it.  Usage: tools/gpu_r4_final.sh TAG
set -o pipefail
TAG=${1:-r4final}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
export MVML_MARGINS_DIR=$OUT/margins
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --durations=10 --timeout 600 --timeout-method thread > $OUT/gputest.log 2>&1 || { grep -E "^FAILED|^ERROR" $OUT/gputest.log | head; tail -40 $OUT/gputest.log; exit 1; }
tail -1 $OUT/gputest.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -30 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print({k: d.get(k) for k in ('value','ms_per_step','untimed_ms_per_step')}); print(d['roofline']['frac'], d['roofline']['traffic_over_algorithmic'], d['roofline_agg_bwd']['frac'], d['roofline_gemm']['frac'], d['cpu_baseline']['value'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-inference --view-only-steps 0 > $OUT/kt.log 2>&1 || { tail -30 $OUT/kt.log; exit 1; }
cp $OUT/kt/run_kernel_stats.csv $OUT/kernel_stats.csv
