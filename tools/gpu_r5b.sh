#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
tools/gpu_r5.sh agg c5rs --config 5 --mols 8192 --layers 1 --no-bwd --ab "dst_fwd=1;dst_fwd=1,dst_unr=8;dst_fwd=1;dst_fwd=1,dst_unr=8"
