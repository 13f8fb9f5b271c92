#!/bin/bash
# r06 GPU step: full GPU suite, then C3 A/B (chunked vs row-by-row back substitution)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06/$1_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r06/$1_tests.log
[ $rc -ne 0 ] && exit $rc
bash tools/ab_env.sh $1 C3 - PLBA_BWD_SERIAL=1
