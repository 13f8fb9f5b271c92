# A/B: tests (quick subset) + bench in the default mode and with an env override.
# Usage: tools/gpu_ab.sh "ENV=1" [pytest -k expr]
set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${2:+-k "$2"} > gpurun_out/gpu_tests_ab.log 2>&1 || { tail -40 gpurun_out/gpu_tests_ab.log; exit 1; }
tail -1 gpurun_out/gpu_tests_ab.log
for v in "" "$1"; do
  env $v timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_ab.json
  python -c "import json;d=json.load(open('gpurun_out/bench_ab.json'));print('[$v]', round(d['value'],1), {k: v['us_per_launch'] for k,v in d['kernels'].items()})"
done
