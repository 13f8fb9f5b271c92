#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "bcr or C4 or C5 or large or spec or shard or hlm or gba" > gpurun_out/r06/$1_tests.log 2>&1 || { tail -40 gpurun_out/r06/$1_tests.log; exit 1; }
tail -2 gpurun_out/r06/$1_tests.log
bash tools/ab_env.sh $1 C5 - PLBA_BCR_SPLIT=1
