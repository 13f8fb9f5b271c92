#!/bin/bash
# GPU-box round check: parity tests, smoke, default bench, rocprofv3 stats + PMC passes.
# Usage (from the repo root, on the GPU box): tools/gpu_round.sh <tag> [pytest -k expr]
set -eo pipefail
TAG=${1:-r01}
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "[gpu_round] tests" >&2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    ${2:+-k "$2"} > gpurun_out/gpu_tests_${TAG}.log 2>&1
tail -3 gpurun_out/gpu_tests_${TAG}.log >&2
echo "[gpu_round] smoke" >&2
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1
echo "[gpu_round] bench" >&2
timeout -k 10 400 python bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err
cat gpurun_out/bench_${TAG}.json >&2
echo "[gpu_round] profile" >&2
bash tools/profile_bench.sh ${TAG} C3
echo "[gpu_round] done" >&2
