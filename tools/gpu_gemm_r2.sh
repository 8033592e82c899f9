#!/bin/bash
# GEMM timings of the default library and variants, then MFMA-busy / wait / LDS counters of the
# default x3w kernel on the L2-forward shape.  Usage: tools/gpu_gemm_r2.sh TAG "variant1 variant2"
TAG=${1:-g2}; VARS=${2:-}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 240 python3 tools/gemm_bench.py x3 > $OUT/default.txt 2>&1 || exit $?
for v in $VARS; do
  MVML_GAT_LIB=variants/$v.so timeout -k 10 240 python3 tools/gemm_bench.py x3 > $OUT/$v.txt 2>&1 || exit $?
done
for f in $OUT/*.txt; do echo "== $f"; grep -v amdgpu.ids $f; done
