#!/bin/bash
# A/B of the factorisation modes (PLBA_FACTOR=bcr|cl) at C3, C4, C5 (bench, no CPU baseline).
set -eo pipefail
mkdir -p gpurun_out
for c in ${CONFIGS:-C3 C4 C5}; do
  for f in ${MODES:-bcr cl}; do
    PLBA_FACTOR=$f timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline \
        > gpurun_out/ab_${c}_${f}.json 2> gpurun_out/ab_${c}_${f}.err
    python -c "import json;d=json.load(open('gpurun_out/ab_${c}_${f}.json'));print('$c $f', round(d['value'],1), 'it/s', d['config']['ms_per_lm_iteration'], 'ms/it', {k: v['us_per_launch'] for k,v in d['kernels'].items()})"
  done
done
