#!/bin/bash
# Build an experimental variant of libmvml_gat.so with extra -D flags into variants/<name>.so
#   tools/build_variant.sh NAME [-s SRC.hip] -DFOO=1 ...
# With -s only that source is recompiled with the flags; the other objects come from the
# default in-tree build (mvml-mpi_amd/build/).  Run with MVML_GAT_LIB=variants/NAME.so.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
ONLY=""
if [ "$1" = "-s" ]; then ONLY=$2; shift 2; fi
OUT=$ROOT/variants/$NAME; mkdir -p "$OUT"
for f in "$ROOT"/mvml-mpi_amd/csrc/*.hip "$ROOT"/mvml-mpi_amd/csrc/*.cpp; do
  b=$(basename "$f")
  if [ -n "$ONLY" ] && [ "$b" != "$ONLY" ]; then cp "$ROOT/mvml-mpi_amd/build/$b.o" "$OUT/$b.o"; continue; fi
  /opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 "$@" -c "$f" -o "$OUT/$b.o" &
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 "$OUT"/*.o -o "$ROOT/variants/$NAME.so"
rm -rf "$OUT"
echo "$ROOT/variants/$NAME.so"
