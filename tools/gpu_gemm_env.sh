#!/bin/bash
# GEMM timings under several environment settings.  Usage: tools/gpu_gemm_env.sh TAG "VAR=a VAR=b" [shapes]
TAG=${1:-ge}; SETS=${2:-}; SH=${3:-}; OUT=gpurun_out/$TAG; mkdir -p $OUT
for e in $SETS; do
  env $e timeout -k 10 240 python3 tools/gemm_bench.py x3 $SH > $OUT/$e.txt 2>&1 || exit $?
  echo "== $e"; grep -v amdgpu.ids $OUT/$e.txt
done
