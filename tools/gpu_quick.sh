set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_q.log 2>&1 || { tail -40 gpurun_out/gpu_tests_q.log; exit 1; }
tail -2 gpurun_out/gpu_tests_q.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_q.json
python -c "import json;d=json.load(open('gpurun_out/bench_q.json'));print(d['value'],d['config']['ms_per_lm_iteration']);[print(k,v['us_per_launch']) for k,v in d['kernels'].items()]"
