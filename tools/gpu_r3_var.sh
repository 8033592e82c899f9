#!/bin/bash
# GEMM microbench of the default library and variants/*.so (tools/build_variant.sh) on the big
# split-fp16 shapes.  Usage: tools/gpu_r3_var.sh TAG "v1 v2 ..." [shapes]
set -o pipefail
TAG=${1:-var}; VARS=${2:-}; SH=${3:-0,1,2,4,5}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 240 python3 -u tools/gemm_bench.py f16x2 $SH > $OUT/default.txt 2>&1 || { tail -20 $OUT/default.txt; exit 1; }
echo "== default"; grep TF $OUT/default.txt
for v in $VARS; do
  MVML_GAT_LIB=variants/$v.so timeout -k 10 240 python3 -u tools/gemm_bench.py f16x2 $SH > $OUT/$v.txt 2>&1 || { tail -20 $OUT/$v.txt; exit 1; }
  echo "== $v"; grep TF $OUT/$v.txt
done
timeout -k 10 240 python3 -u tools/gemm_bench.py f16x2 $SH > $OUT/default2.txt 2>&1 || { tail -20 $OUT/default2.txt; exit 1; }
echo "== default again"; grep TF $OUT/default2.txt
