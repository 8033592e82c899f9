#!/bin/bash
# Round 4: forward chunk width 32 (new default) vs 16; backward chunk width 32 vs 64.
# Usage: tools/gpu_r4_n.sh TAG
set -o pipefail
TAG=${1:-r4n}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
for v in default cw16 bwdcw32; do
  LIB=""; [ $v != default ] && LIB=variants/$v.so
  for cfg in 3 2; do
    MVML_GAT_LIB=${LIB:-mvml-mpi_amd/mvml_gat/libmvml_gat.so} timeout -k 10 200 python3 -u tools/agg_bench.py --config $cfg --mols 65536 --layers 01 > $OUT/agg_${v}_c$cfg.log 2>&1 || { tail -30 $OUT/agg_${v}_c$cfg.log; exit 1; }
    echo "== $v config $cfg"; grep "agg_" $OUT/agg_${v}_c$cfg.log
  done
done
