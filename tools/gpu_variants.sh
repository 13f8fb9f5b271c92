#!/bin/bash
# GPU box: A/B of libplba builds (make variant V=...) with tools/variant_time.py.
# usage: tools/gpu_variants.sh <tag> <cfg> <lib> [<lib> ...]
set -eo pipefail
TAG=$1; CFG=$2; shift 2
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/variant_time.py $CFG "$@" > gpurun_out/var_${TAG}_${CFG}.log 2>&1
