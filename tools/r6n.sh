set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for o in 0 1 0 1; do
  MVML_DST_ORDER=$o timeout -k 10 400 python -u bench.py --workload config5 --steps 10 --warmup 3 --no-cpu-baseline --no-inference > gpurun_out/r6n_c5_$o.json 2> gpurun_out/r6n_c5_$o.err || exit 1
  python3 -c "
import json;d=json.load(open('gpurun_out/r6n_c5_$o.json'))
print('order=$o', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['kernel_ms_per_step']['mvml_gat_agg_fwd'])"
done
