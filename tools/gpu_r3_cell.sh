#!/bin/bash
# Round-3: float4 LSTM-cell GEMM epilogue and split-fp16 skinny GEMMs — GEMM / cell / Set2Set /
# BiLSTM / MVP parity, then the config-3 bench with GEMM shapes and the MVP bench.
# Usage: tools/gpu_r3_cell.sh TAG
set -o pipefail
TAG=${1:-cell}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k "set2set or cell or lstm or gemm" tests/test_gpu_smiles.py tests/test_gpu_mvp.py \
  > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
MVML_GEMM_SHAPES=1 timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline --view-only-steps 0 \
  --no-inference > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
head -c 300 $OUT/bench.json; echo; grep -E "cell|mvml_|76|384" $OUT/bench.err | head -60
timeout -k 10 400 python -u bench.py --workload mvp --steps 6 --warmup 2 --no-cpu-baseline \
  --view-only-steps 0 --no-inference > $OUT/mvp.json 2> $OUT/mvp.err || { tail -30 $OUT/mvp.err; exit 1; }
head -c 300 $OUT/mvp.json; echo; grep -E "mvml_" $OUT/mvp.err | head -12
