#!/bin/bash
# Round-3: BASELINE config 4 as written (MVP step with the bf16 projection) and the config-3 bf16
# projection line.  Usage: tools/gpu_r3_bf16.sh TAG
set -o pipefail
TAG=${1:-bf16}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --workload mvp --proj-bf16 --steps 6 --warmup 2 --no-cpu-baseline \
  --view-only-steps 0 --no-inference > $OUT/mvp_bf16.json 2> $OUT/mvp_bf16.err || { tail -30 $OUT/mvp_bf16.err; exit 1; }
head -c 600 $OUT/mvp_bf16.json; echo; grep -E "mvml_" $OUT/mvp_bf16.err | head -14
timeout -k 10 400 python -u bench.py --proj-bf16 --steps 6 --warmup 2 --no-cpu-baseline \
  --view-only-steps 0 --no-inference > $OUT/c3_bf16.json 2> $OUT/c3_bf16.err || { tail -30 $OUT/c3_bf16.err; exit 1; }
head -c 600 $OUT/c3_bf16.json; echo; grep -E "mvml_" $OUT/c3_bf16.err | head -8
