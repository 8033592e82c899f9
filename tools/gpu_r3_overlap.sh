#!/bin/bash
# Round-3: MVP step with the SMILES view on a side stream vs one stream (fp32 projection).
set -o pipefail
TAG=${1:-ovl}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
for m in ovl seq; do
  X=""; [ $m = seq ] && X="--no-view-overlap"
  timeout -k 10 400 python -u bench.py --workload mvp --steps 6 --warmup 2 --no-cpu-baseline \
    --view-only-steps 0 --no-inference $X > $OUT/mvp_$m.json 2> $OUT/mvp_$m.err || { tail -30 $OUT/mvp_$m.err; exit 1; }
  head -c 300 $OUT/mvp_$m.json; echo
done
grep -E "mvml_" $OUT/mvp_ovl.err | head -14
