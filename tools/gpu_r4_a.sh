#!/bin/bash
# Round 4, first pass: GEMM A/B (round-3 library vs this build, per-row scales), the driver's exact
# bench command with its kernel trace (untimed gaps), then the new GPU tests.
# Usage: tools/gpu_r4_a.sh TAG
set -o pipefail
TAG=${1:-r4a}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
export MVML_MARGINS_DIR=$OUT/margins
timeout -k 10 300 python3 -u tools/gemm_bench.py f16x2,f16x2r 0,1,2,4,5,6 > $OUT/gemm_new.txt 2>&1 || { tail -20 $OUT/gemm_new.txt; exit 1; }
cat $OUT/gemm_new.txt
MVML_GAT_LIB=$PWD/mvml-mpi_amd/mvml_gat/libmvml_gat_base.so timeout -k 10 300 python3 -u tools/gemm_bench.py f16x2 0,1,2,4,5,6 > $OUT/gemm_base.txt 2>&1 || { tail -20 $OUT/gemm_base.txt; exit 1; }
cat $OUT/gemm_base.txt
tools/gpu_r4_gap.sh $TAG/gap || exit 1
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_rows.py tests/test_gpu_dp2.py tests/test_gpu_smiles.py -x -v --timeout 400 --timeout-method thread > $OUT/pytest_new.log 2>&1 || { tail -60 $OUT/pytest_new.log; exit 1; }
tail -5 $OUT/pytest_new.log
