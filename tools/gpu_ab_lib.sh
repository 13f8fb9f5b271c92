#!/bin/bash
# GPU box: parity subset + timing of library builds (make variant V=...).
# usage: tools/gpu_ab_lib.sh <tag> <cfgs> <lib> [<lib> ...]   (cfgs comma-separated, e.g. C3,C5)
set -o pipefail
TAG=$1; CFGS=$2; shift 2
mkdir -p gpurun_out
for L in "$@"; do
  PLBA_LIB=$PWD/pl-slam-plucker_amd/$L timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_spec.py \
      tests/test_gpu_edge_cases.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/abt_${TAG}_${L}.log 2>&1 \
      || { tail -30 gpurun_out/abt_${TAG}_${L}.log; exit 1; }
  tail -1 gpurun_out/abt_${TAG}_${L}.log
done
for C in ${CFGS//,/ }; do
  timeout -k 10 300 python -u tools/variant_time.py $C "$@" | tee gpurun_out/var_${TAG}_${C}.log || exit 1
done
