#!/bin/bash
# Build an experimental variant of libmvml_gat.so with extra -D flags into variants/<name>.so
#   tools/build_variant.sh NAME -DFOO=1 ...      (run agg_bench with MVML_GAT_LIB=variants/NAME.so)
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
OUT=$ROOT/variants/$NAME; mkdir -p "$OUT"
for f in "$ROOT"/mvml-mpi_amd/csrc/*.hip "$ROOT"/mvml-mpi_amd/csrc/*.cpp; do
  /opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 "$@" -c "$f" -o "$OUT/$(basename "$f").o" &
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 "$OUT"/*.o -o "$ROOT/variants/$NAME.so"
rm -rf "$OUT"
echo "$ROOT/variants/$NAME.so"
