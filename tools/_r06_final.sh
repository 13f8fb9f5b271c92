#!/bin/bash
# GPU box, round-6 evidence: full GPU suite, smoke, benches (C3 default, C5, C3R), rocprofv3 kernel
# stats + HBM PMC passes at C3 and C5, SQ pass at C3. Outputs under gpurun_out/r06/.
set -eo pipefail
export TMPDIR=/tmp
T=${1:-final}
O=gpurun_out/r06
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/${T}_gpu_tests.log 2>&1 || { tail -30 $O/${T}_gpu_tests.log; exit 1; }
tail -2 $O/${T}_gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/${T}_smoke.log 2>&1
echo smoke ok
timeout -k 10 400 python bench.py > $O/${T}_bench_default.json 2> $O/${T}_bench_default.err
timeout -k 10 300 python bench.py --config C5 --no-cpu-baseline > $O/${T}_bench_C5.json 2> $O/${T}_bench_C5.err
timeout -k 10 300 python bench.py --config C3R --no-cpu-baseline --no-host-mirror > $O/${T}_bench_C3R.json 2> $O/${T}_bench_C3R.err
echo benches ok
bash tools/profile_bench.sh ${T}_C3 C3
bash tools/profile_bench.sh ${T}_C5 C5
bash tools/pmc_sq.sh ${T}_C3
echo all done
