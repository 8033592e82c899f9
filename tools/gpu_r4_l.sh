#!/bin/bash
# Round 4: bench-size parity (all cases) on the source-atom default; MVP (config 4) lines, fp32 and
# bf16 projection.  Usage: tools/gpu_r4_l.sh TAG
set -o pipefail
TAG=${1:-r4l}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
export MVML_MARGINS_DIR=$OUT/margins
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_parity_bench.py -v --timeout 600 --timeout-method thread > $OUT/parity.log 2>&1 || { grep -E "^FAILED|^ERROR" $OUT/parity.log; tail -30 $OUT/parity.log; exit 1; }
tail -1 $OUT/parity.log
timeout -k 10 300 python3 -u bench.py --workload mvp --steps 10 --warmup 3 --no-cpu-baseline --no-inference > $OUT/mvp.json 2> $OUT/mvp.err || { tail -30 $OUT/mvp.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/mvp.json')); print('mvp', {k: d.get(k) for k in ('value','ms_per_step')})"
timeout -k 10 300 python3 -u bench.py --workload mvp --proj-bf16 --steps 10 --warmup 3 --no-cpu-baseline --no-inference > $OUT/mvp_bf16.json 2> $OUT/mvp_bf16.err || { tail -30 $OUT/mvp_bf16.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/mvp_bf16.json')); print('mvp bf16 proj', {k: d.get(k) for k in ('value','ms_per_step')})"
