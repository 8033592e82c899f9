#!/bin/bash
# Round 4: the new / changed GPU tests, then the default bench line.  Usage: tools/gpu_r4_b.sh TAG
set -o pipefail
TAG=${1:-r4b}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
export MVML_MARGINS_DIR=$OUT/margins
# timeout -k 10 300 python3 -u tools/gemm_bench.py f16x2,f16x2r,f16x2i,f16x2ri 0,1,2,4,5,6 > $OUT/gemm.txt 2>&1 || { tail -20 $OUT/gemm.txt; exit 1; }
# cat $OUT/gemm.txt
timeout -k 10 900 python3 -u -m pytest ${TESTS:-tests/test_gpu_rows.py tests/test_gpu_dp2.py tests/test_gpu_fusion.py tests/test_gpu_smiles.py} -v --timeout 600 --timeout-method thread > $OUT/pytest_new.log 2>&1 || { tail -60 $OUT/pytest_new.log; exit 1; }
tail -5 $OUT/pytest_new.log
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print({k: d.get(k) for k in ('value','ms_per_step','untimed_ms_per_step','allocator')}); print(d['roofline']['frac'], d['roofline_agg_bwd']['frac'], d['roofline_gemm'])"
grep -E "mvml_" $OUT/bench.err | head -30
