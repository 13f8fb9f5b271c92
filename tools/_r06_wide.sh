#!/bin/bash
# GPU box: wide-band parity tests, then the current build against libplba_ab.so (A/B) at C3R / C2R
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "revisit or widest or wide_band or wide_bands or spec or band" > gpurun_out/r06/$1_tests.log 2>&1 || { tail -40 gpurun_out/r06/$1_tests.log; exit 1; }
tail -2 gpurun_out/r06/$1_tests.log
bash tools/ab_env.sh $1_C3R C3R - PLBA_LIB=pl-slam-plucker_amd/libplba_ab.so && \
bash tools/ab_env.sh $1_C2R C2R - PLBA_LIB=pl-slam-plucker_amd/libplba_ab.so
