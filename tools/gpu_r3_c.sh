#!/bin/bash
# Round-3 call C: the LDS-DMA ring split-fp16 GEMM — bitwise vs the register-staged kernel,
# GEMM parity, then the microbench (ring on / off) on the step's big shapes.  Usage: tools/gpu_r3_c.sh TAG
set -o pipefail
TAG=${1:-c}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k "ring_bitwise or gemm_layouts or f16x2 or set2set" > $OUT/pytest_gemm.log 2>&1 || { tail -40 $OUT/pytest_gemm.log; exit 1; }
tail -3 $OUT/pytest_gemm.log
MVML_GEMM_RING=1 timeout -k 10 300 python -u tools/gemm_bench.py f16x2 0,1,2,4,5,6 > $OUT/gemm_ring1.txt 2>&1 || { tail -20 $OUT/gemm_ring1.txt; exit 1; }
MVML_GEMM_RING=0 timeout -k 10 300 python -u tools/gemm_bench.py f16x2 0,1,2,4,5,6 > $OUT/gemm_ring0.txt 2>&1 || { tail -20 $OUT/gemm_ring0.txt; exit 1; }
grep TF $OUT/gemm_ring1.txt; grep TF $OUT/gemm_ring0.txt
