#!/bin/bash
# Round 4: re-associated layer + mean-src iteration: parity, microbench (config 3 / 5), kernel
# stats of the config-5 microbench, bench GEMM shapes.  Usage: tools/gpu_r4_e.sh TAG
set -o pipefail
TAG=${1:-r4e}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_reassoc.py tests/test_gpu_parity_configs.py -k "mean_src or row_maxima or reassociated or elu_link or reassoc" \
  -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -E "^FAILED|^ERROR|Error|assert" $OUT/pytest.log | head -40; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
MVML_MEAN_SRC=1 timeout -k 10 200 python3 -u tools/agg_bench.py --config 3 --mols 65536 --layers x1 > $OUT/agg_c3.log 2>&1 || { tail -30 $OUT/agg_c3.log; exit 1; }
grep -v amdgpu.ids $OUT/agg_c3.log
MVML_MEAN_SRC=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt5 -o run -- python3 tools/agg_bench.py --config 5 --mols 8192 --layers x1 > $OUT/agg_c5.log 2>&1 || { tail -30 $OUT/agg_c5.log; exit 1; }
grep -v amdgpu.ids $OUT/agg_c5.log | grep -v "^\[\|^W2\|rocprof"
python3 - "$OUT" <<'PY'
import csv, glob, sys
p = glob.glob(sys.argv[1] + "/kt5/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(p)))[:24]:
    print(f"{r['Name'][:100]:100s} n={r['Calls']:>4s} avg={float(r['AverageNs'])/1e3:9.1f} us")
PY
MVML_GEMM_SHAPES=1 timeout -k 10 300 python3 -u bench.py --steps 6 --warmup 2 --no-inference --no-cpu-baseline --view-only-steps 0 > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print({k: d.get(k) for k in ('value','ms_per_step','untimed_ms_per_step')})"
grep -E "gemm \(" $OUT/bench.err | grep -E " 76|152|1928, 0, 1" | head -30
grep -E "mvml_" $OUT/bench.err | head -20
