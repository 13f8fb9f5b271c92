# A/B of the Schur assembly: staged (default) vs PLBA_CHUNK_DIRECT=1, C3 and C5, after the -m gpu suite.
# Usage (GPU box, repo root): tools/chunk_ab.sh [pytest -k expr]
set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${1:+-k "$1"} > gpurun_out/gpu_tests_chunk.log 2>&1 || { tail -40 gpurun_out/gpu_tests_chunk.log; exit 1; }
tail -1 gpurun_out/gpu_tests_chunk.log
for cfg in C3 C5; do
  for v in "PLBA_CHUNK_DIRECT=1" "PLBA_X=0"; do
    env $v timeout -k 10 300 python bench.py --config $cfg --steps 10 --no-cpu-baseline > gpurun_out/bench_chunk_${cfg}_${v%%=*}.json
    python -c "import json;d=json.load(open('gpurun_out/bench_chunk_${cfg}_${v%%=*}.json'));print('$cfg [$v]', round(d['value'],1), {k: v['us_per_launch'] for k,v in d['kernels'].items()}, repr(d.get('final_chi2_gpu')))"
  done
done
