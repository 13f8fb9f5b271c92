#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
T=$1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_spec.py tests/test_gpu_edge_cases.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06/${T}_tests.log 2>&1 || { tail -40 gpurun_out/r06/${T}_tests.log; exit 1; }
tail -2 gpurun_out/r06/${T}_tests.log
for c in C3 C2 C3 C2; do
  timeout -k 10 300 python -u tools/variant_time.py $c libplba_base.so libplba.so >> gpurun_out/r06/${T}_var.log 2>&1 || { tail -20 gpurun_out/r06/${T}_var.log; exit 1; }
done
python3 - <<PY
import json
for l in open('gpurun_out/r06/${T}_var.log'):
    l=l.strip()
    if not l.startswith('{'): print(l[:200]); continue
    d=json.loads(l); k=d['kernels_us']
    print(d['lib'], 'lba %.3f ms' % d['lba_ms_median'], 'factor', [v for n,v in k.items() if 'factor' in n], 'chi2', d['chi2'])
PY
