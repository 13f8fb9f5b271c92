#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
T=$1; shift
for c in C3 C5 C3 C5; do
  timeout -k 10 300 python -u tools/variant_time.py $c "$@" >> gpurun_out/r06/${T}_var.log 2>&1 || { tail -20 gpurun_out/r06/${T}_var.log; exit 1; }
done
python3 - <<PY
import json
for l in open('gpurun_out/r06/${T}_var.log'):
    l=l.strip()
    if not l.startswith('{'): print(l[:200]); continue
    d=json.loads(l); k=d['kernels_us']
    print(d['lib'], 'lba %.3f ms' % d['lba_ms_median'], 'lm_solve', [v for n,v in k.items() if 'lm_solve' in n], 'chi2', d['chi2'][:1])
PY
