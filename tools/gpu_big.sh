set -eo pipefail
mkdir -p gpurun_out
for c in C4 C5; do
  timeout -k 10 400 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err
  python -c "import json;d=json.load(open('gpurun_out/bench_$c.json'));print('$c', round(d['value'],1), d['config']['ms_per_lm_iteration'], d['roofline']['kernel'], {k: v['us_per_launch'] for k,v in d['kernels'].items()})"
done
timeout -k 10 400 python bench.py --config C4 --mode shard --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_C4s.json 2> gpurun_out/bench_C4s.err
python -c "import json;d=json.load(open('gpurun_out/bench_C4s.json'));print('C4 shard(1 rank rccl)', round(d['value'],1), {k: v['us_per_launch'] for k,v in d['kernels'].items()})"
