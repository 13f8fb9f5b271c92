#!/bin/bash
# GPU-box: the -m gpu suite (optionally -k filtered), one process, bounded.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-t}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${2:+-k "$2"} \
    > gpurun_out/gpu_tests_${TAG}.log 2>&1
rc=$?
tail -25 gpurun_out/gpu_tests_${TAG}.log
exit $rc
