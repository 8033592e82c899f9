#!/bin/bash
# Round 4: GPU suite on the source-atom default, config-3 PMC traffic refresh, the driver's bench
# command, kernel stats of it.  Usage: tools/gpu_r4_i.sh TAG
set -o pipefail
TAG=${1:-r4i}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
export MVML_MARGINS_DIR=$OUT/margins
timeout -k 10 700 python3 -u -m pytest tests -m gpu -v --durations=10 --timeout 300 --timeout-method thread \
  --deselect tests/test_gpu_parity_bench.py > $OUT/gputest.log 2>&1 || { grep -E "^FAILED|^ERROR" $OUT/gputest.log | head; tail -40 $OUT/gputest.log; exit 1; }
tail -1 $OUT/gputest.log
bash tools/pmc_bench.sh $TAG/pmc3 > $OUT/pmc3.log 2>&1 || { tail -30 $OUT/pmc3.log; exit 1; }
cp $OUT/pmc3/pmc_traffic.json profiles/pmc_traffic.json
WORKLOAD=config5 bash tools/pmc_bench.sh $TAG/pmc5 > $OUT/pmc5.log 2>&1 || { tail -30 $OUT/pmc5.log; exit 1; }
cp $OUT/pmc5/pmc_traffic.json profiles/pmc_traffic.json
cp profiles/pmc_traffic.json $OUT/pmc_traffic.json
python3 -c "import json; d=json.load(open('profiles/pmc_traffic.json')); print({w: {k: (v['hbm_bytes_per_launch'], v['calls']) for k, v in d[w].items()} for w in ('config3/mols_per_step=65536', 'config5/mols_per_step=8192')})"
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print({k: d.get(k) for k in ('value','ms_per_step','untimed_ms_per_step')}); print(d['roofline']['frac'], d['roofline']['traffic_over_algorithmic'], d['roofline_agg_bwd']['frac'], d['roofline_agg_bwd'].get('traffic_over_algorithmic'), d['roofline_gemm']['frac'], d['cpu_baseline']['value'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-inference --view-only-steps 0 > $OUT/kt.log 2>&1 || { tail -30 $OUT/kt.log; exit 1; }
cp $OUT/kt/run_kernel_stats.csv $OUT/kernel_stats.csv
timeout -k 10 300 python3 -u bench.py --workload config5 --steps 6 --warmup 2 --no-cpu-baseline --no-inference > $OUT/bench5.json 2> $OUT/bench5.err || { tail -30 $OUT/bench5.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench5.json')); print({k: d.get(k) for k in ('value','ms_per_step')}); print(d['roofline']); print(d['roofline_agg_bwd'])"
