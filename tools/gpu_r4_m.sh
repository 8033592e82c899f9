#!/bin/bash
# Round 4: forward aggregation variants (64- vs 32-column chunks, ring depth) on configs 3 / 2.
# Usage: tools/gpu_r4_m.sh TAG
set -o pipefail
TAG=${1:-r4m}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
for v in default cw32 ring3; do
  LIB=""; [ $v != default ] && LIB=variants/$v.so
  for cfg in 3 2; do
    MVML_GAT_LIB=${LIB:-mvml-mpi_amd/mvml_gat/libmvml_gat.so} timeout -k 10 200 python3 -u tools/agg_bench.py --config $cfg --mols 65536 --layers 01 --no-bwd > $OUT/agg_${v}_c$cfg.log 2>&1 || { tail -30 $OUT/agg_${v}_c$cfg.log; exit 1; }
    echo "== $v config $cfg"; grep "agg_fwd" $OUT/agg_${v}_c$cfg.log
  done
done
