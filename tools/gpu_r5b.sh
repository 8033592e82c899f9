#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
MVML_BENCH_ADAM=foreach tools/gpu_r5.sh bench adf --steps 16 --warmup 2 --no-cpu-baseline --no-inference || exit 1
tools/gpu_r5.sh bench adu --steps 16 --warmup 2 --no-cpu-baseline --no-inference
