#!/bin/bash
# Round 4: tile plans for the layer-1 (K = 76 / N = 76) products.  Usage: tools/gpu_r4_k.sh TAG
set -o pipefail
TAG=${1:-r4k}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/gemm_bench.py f16x2ri,f16x2ri-128,f16x2ri-256 11 > $OUT/g1.log 2>&1 || { tail -30 $OUT/g1.log; exit 1; }
cat $OUT/g1.log | grep -v amdgpu
timeout -k 10 300 python3 -u tools/gemm_bench.py f16x2,f16x2-128,f16x2-256 10 > $OUT/g2.log 2>&1 || { tail -30 $OUT/g2.log; exit 1; }
cat $OUT/g2.log | grep -v amdgpu
