#!/bin/bash
set -o pipefail
TAG=${1:-r4t}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
cd tools && timeout -k 10 300 python3 -u persist_bench.py > ../$OUT/persist.log 2>&1 || { tail -30 ../$OUT/persist.log; exit 1; }
grep -v amdgpu ../$OUT/persist.log
