#!/bin/bash
# Round 4: staggered split for the pre-split-B GEMMs.  Usage: tools/gpu_r4_s.sh TAG
set -o pipefail
TAG=${1:-r4s}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
for v in default stagger; do
  LIB=mvml-mpi_amd/mvml_gat/libmvml_gat.so; [ $v != default ] && LIB=variants/$v.so
  MVML_GAT_LIB=$LIB timeout -k 10 300 python3 -u tools/gemm_bench.py f16x2ri,f16x2 0,1,2,4 > $OUT/g_$v.log 2>&1 || { tail -30 $OUT/g_$v.log; exit 1; }
  echo "== $v"; grep -v amdgpu $OUT/g_$v.log
done
