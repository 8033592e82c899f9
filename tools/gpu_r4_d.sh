#!/bin/bash
# Round 4: mean-src backward parity + aggregation microbench (configs 3 / 5, both paths), then
# bench GEMM shapes with / without the re-associated first layer.  Usage: tools/gpu_r4_d.sh TAG
set -o pipefail
TAG=${1:-r4d}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_reassoc.py tests/test_gpu_parity_configs.py -k "mean_src or row_maxima or reassociated or elu_link" \
  -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -E "^FAILED|^ERROR|Error|assert" $OUT/pytest.log | head -40; tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
for cfg in 3 5; do
  mols=$([ $cfg = 3 ] && echo 65536 || echo 8192)
  for ms in 0 1; do
    MVML_MEAN_SRC=$ms timeout -k 10 200 python3 -u tools/agg_bench.py --config $cfg --mols $mols --layers x1 > $OUT/agg_c${cfg}_ms${ms}.log 2>&1 || { tail -30 $OUT/agg_c${cfg}_ms${ms}.log; exit 1; }
    echo "== config $cfg mean_src $ms"; grep -v amdgpu.ids $OUT/agg_c${cfg}_ms${ms}.log
  done
done
for ra in 1 0; do
  MVML_GEMM_SHAPES=1 MVML_GAT_REASSOC=$ra timeout -k 10 300 python3 -u bench.py --steps 6 --warmup 2 --no-inference --no-cpu-baseline --view-only-steps 0 > $OUT/bench_ra$ra.json 2> $OUT/bench_ra$ra.err || { tail -30 $OUT/bench_ra$ra.err; exit 1; }
  echo "== reassoc $ra"; python3 -c "import json; d=json.load(open('$OUT/bench_ra$ra.json')); print({k: d.get(k) for k in ('value','ms_per_step','untimed_ms_per_step')})"
  grep -E "gemm \(" $OUT/bench_ra$ra.err | head -30
done
