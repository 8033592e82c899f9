#!/bin/bash
# Round 4: whole GPU suite, config-5 bench-size parity, smoke, the driver's bench command.
# Usage: tools/gpu_r4_f.sh TAG
set -o pipefail
TAG=${1:-r4f}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
export MVML_MARGINS_DIR=$OUT/margins
timeout -k 10 700 python3 -u -m pytest tests -m gpu -v --durations=10 --timeout 300 --timeout-method thread \
  --deselect tests/test_gpu_parity_bench.py > $OUT/gputest.log 2>&1 || { grep -E "^FAILED|^ERROR" $OUT/gputest.log | head; tail -40 $OUT/gputest.log; exit 1; }
tail -2 $OUT/gputest.log
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity_bench.py -k config5 -v --timeout 380 --timeout-method thread > $OUT/parity5.log 2>&1 || { tail -30 $OUT/parity5.log; exit 1; }
tail -2 $OUT/parity5.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -30 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print({k: d.get(k) for k in ('value','ms_per_step','untimed_ms_per_step')}); print(d['roofline']['frac'], d['roofline_agg_bwd']['frac'], d['roofline_gemm']['frac'], d['cpu_baseline']['value'])"
