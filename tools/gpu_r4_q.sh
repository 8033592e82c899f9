#!/bin/bash
# Round 4: rehearsal of bench.py's N-rank path on the one-GPU box (2 ranks on cuda:0 over gloo,
# self-launched), a small global set.  Usage: tools/gpu_r4_q.sh TAG
set -o pipefail
TAG=${1:-r4q}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
export MVML_BENCH_ONE_DEVICE=1 MVML_BENCH_BACKEND=gloo
timeout -k 10 600 python3 -u bench.py --gpus 2 --steps 4 --warmup 1 --total-mols 262144 --no-cpu-baseline > $OUT/bench2.json 2> $OUT/bench2.err || { tail -40 $OUT/bench2.err; exit 1; }
cat $OUT/bench2.json | head -c 1500; echo
grep -v amdgpu.ids $OUT/bench2.err | head -20
