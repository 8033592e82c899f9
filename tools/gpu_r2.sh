#!/bin/bash
# Round-2 GPU check: GPU test suite, then the default bench line (+ stderr kernel breakdown).
# Usage: tools/gpu_r2.sh TAG [pytest-args...]   (bench skipped if pytest crashed or hung)
TAG=${1:-r2}; shift; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "$@" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 500 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
rc2=$?; echo "bench rc=$rc2"; cat $OUT/bench.json; tail -40 $OUT/bench.err
exit $rc2
