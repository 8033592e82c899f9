#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
tools/gpu_r5.sh agg c5o6 --config 5 --mols 8192 --layers 1 --no-bwd --ab "dst_fwd=1;dst_fwd=1,dst_unr=7;dst_fwd=1;dst_fwd=1,dst_unr=7" || exit 1
tools/gpu_r5.sh agg c3o6 --config 3 --mols 65536 --layers 1 --no-bwd --ab "dst_fwd=2;dst_fwd=2,dst_unr=7;dst_fwd=2;dst_fwd=2,dst_unr=7"
