#!/bin/bash
# conv3 kernel timings of the default library and variants.  Usage: tools/gpu_conv_var.sh TAG "v1 v2"
TAG=${1:-cv}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 120 python3 tools/conv_bench.py > $OUT/default.txt 2>&1 || exit $?
for v in $2; do
  MVML_GAT_LIB=variants/$v.so timeout -k 10 120 python3 tools/conv_bench.py > $OUT/$v.txt 2>&1 || exit $?
done
for f in $OUT/*.txt; do echo "== $f"; grep -v amdgpu.ids $f; done
