#!/bin/bash
# GPU box: full GPU suite, smoke and the default + C5 bench lines at HEAD (outputs under gpurun_out/r06/).
set -eo pipefail
export TMPDIR=/tmp
T=${1:-check}
O=gpurun_out/r06
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/${T}_gpu_tests.log 2>&1 || { tail -30 $O/${T}_gpu_tests.log; exit 1; }
tail -2 $O/${T}_gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/${T}_smoke.log 2>&1
echo smoke ok
timeout -k 10 400 python bench.py > $O/${T}_bench_default.json 2> $O/${T}_bench_default.err
timeout -k 10 300 python bench.py --config C5 --no-cpu-baseline > $O/${T}_bench_C5.json 2> $O/${T}_bench_C5.err
python3 -c "
import json
for f in ['$O/${T}_bench_default.json', '$O/${T}_bench_C5.json']:
    d = json.load(open(f)); r = d['roofline']
    print(f.split('/')[-1], d['value'], d['unit'], 'ms/step', round(d['ms_per_step'], 3), 'factor us', round(r['avg_launch_us'], 2), 'cpu', (d.get('cpu_baseline') or {}).get('value'))
"
