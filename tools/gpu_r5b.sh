#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
tools/gpu_r5.sh agg c5lr --config 5 --mols 8192 --layers 1 --no-bwd --ab "dst_fwd=1;dst_fwd=1,dst_unr=5;dst_fwd=2;dst_fwd=2,dst_unr=5" || exit 1
tools/gpu_r5.sh agg c3lr --config 3 --mols 65536 --layers 1 --no-bwd --ab "dst_fwd=2;dst_fwd=2,dst_unr=5;dst_fwd=1;dst_fwd=1,dst_unr=5"
