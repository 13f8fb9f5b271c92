# Timing experiments (wrong results): bench per-kernel times under several PLBA_DIAG masks.
# Usage: tools/diag_ab.sh "0 1 2 4"
set -eo pipefail
mkdir -p gpurun_out
for v in $1; do
  PLBA_DIAG=$v timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_diag.json 2> gpurun_out/bench_diag.err || true
  python -c "import json;d=json.load(open('gpurun_out/bench_diag.json'));print('[diag $v]', round(d['value'],1), {k: v['us_per_launch'] for k,v in d['kernels'].items()})" || tail -3 gpurun_out/bench_diag.err
done
