#!/bin/bash
# Round 4: persistent tile loop (MVML_X3W_PERSIST = 256 workgroups) across the GEMM shapes and the
# whole config-3 step.  Usage: tools/gpu_r4_u.sh TAG
set -o pipefail
TAG=${1:-r4u}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
for p in 0 256; do
  MVML_X3W_PERSIST=$p timeout -k 10 300 python3 -u tools/gemm_bench.py f16x2ri,f16x2 0,1,2,4,5,6 > $OUT/g_$p.log 2>&1 || { tail -30 $OUT/g_$p.log; exit 1; }
  echo "== persist $p"; grep -v amdgpu $OUT/g_$p.log
done
for p in 256 0; do
  MVML_X3W_PERSIST=$p timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-inference --no-cpu-baseline --view-only-steps 0 > $OUT/bench_$p.json 2> $OUT/bench_$p.err || { tail -30 $OUT/bench_$p.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$p.json')); print('persist $p', {k: d.get(k) for k in ('value','ms_per_step')}, d['roofline_gemm']['frac'])"
done
