#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
tools/gpu_r5.sh tests p6 tests/test_gpu_smallk.py tests/test_gpu_parity_configs.py tests/test_gpu_bf16.py tests/test_gpu_mvp.py tests/test_gpu_rows.py -k "not bench" || exit 1
tools/gpu_r5.sh agg c5p --config 5 --mols 8192 --layers 01 --no-bwd --ab "dst_fwd=1,dst_parts=1;dst_fwd=1,dst_parts=2;dst_fwd=1,dst_parts=3;dst_fwd=2,dst_parts=2;dst_fwd=2,dst_parts=3" || exit 1
tools/gpu_r5.sh bench c3f --steps 10 --warmup 3 --no-cpu-baseline --no-inference
