#!/bin/bash
# Round 4: the re-associated first layer — its tests, the module / bench-size parity files, DP2,
# then the driver's bench line.  Usage: tools/gpu_r4_c.sh TAG
set -o pipefail
TAG=${1:-r4c}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
export MVML_MARGINS_DIR=$OUT/margins
timeout -k 10 900 python3 -u -m pytest ${TESTS:-tests/test_gpu_reassoc.py tests/test_gpu_parity_configs.py tests/test_gpu_dp2.py tests/test_gpu_parity_bench.py} \
  -v --timeout 600 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -E "^FAILED|^ERROR|Error|assert" $OUT/pytest.log | head -40; tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print({k: d.get(k) for k in ('value','ms_per_step','untimed_ms_per_step')}); print(d['roofline']['frac'], d['roofline_agg_bwd']['frac'], d['roofline_gemm']['frac'], d['roofline_gemm']['achieved'])"
grep -E "mvml_" $OUT/bench.err | head -34
