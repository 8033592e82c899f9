#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
tools/gpu_r5.sh tests am tests/test_gpu_rows.py tests/test_gpu_parity.py tests/test_gpu_mvp.py -k "absmax or gnn or mvp or gemm" || exit 1
tools/gpu_r5.sh bench am --steps 16 --warmup 2 --no-cpu-baseline --no-inference
