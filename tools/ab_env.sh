#!/bin/bash
# GPU box, repo root: bench.py at one config under several environment settings, one line each.
# usage: tools/ab_env.sh <tag> <config> "<ENV=val ...>" ["<ENV=val ...>" ...]   ("-" = no extra env)
set -o pipefail
TAG=$1; CFG=$2; shift 2
mkdir -p gpurun_out
for rep in 1 2; do
for e in "$@"; do
  [ "$e" = "-" ] && e=""
  env $e timeout -k 10 120 python3 bench.py --config $CFG --steps 20 --warmup 3 --no-cpu-baseline --no-host-mirror --windows 0 \
      > gpurun_out/ab_${TAG}.json 2> gpurun_out/ab_${TAG}.err || { tail -5 gpurun_out/ab_${TAG}.err; exit 1; }
  python3 -c "
import json,sys
d=json.load(open('gpurun_out/ab_${TAG}.json'))
k=d['kernels']
print('%-28s %8.1f it/s steps %s fac %s  ' % ('$e' or 'default', d['value'], d['config']['speculative_trials'].get('device_steps_per_lba'), d['config']['factorisation']) + ' '.join('%s=%.1f' % (n[2:], v['us_per_launch']) for n, v in k.items()))
" | tee -a gpurun_out/ab_${TAG}.txt
done
done
