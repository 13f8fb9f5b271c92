#!/bin/bash
# GPU box, repo root: round-3 evidence, part $1 (a: benches + GBA/PGO timings, b: rocprofv3 C3, c: rocprofv3 C5)
set -eo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03
mkdir -p $O
case "${1:-a}" in
a)
    timeout -k 10 300 python -u bench.py > $O/bench_C3.json 2> $O/bench_C3.err
    timeout -k 10 400 python -u bench.py --config C5 --steps 10 --cpu-runs 1 --windows 0 > $O/bench_C5.json 2> $O/bench_C5.err
    timeout -k 10 300 python -u tools/pgo_bench.py 40 150 400 1000 > $O/pgo_timing.jsonl 2>&1
    timeout -k 10 500 python -u tools/gba_timing.py C4 C5:2 > $O/gba_timing.jsonl 2>&1
    ;;
b) bash tools/profile_round.sh r03 C3 10 ;;
c) bash tools/profile_round.sh r03 C5 5 ;;
esac
echo "evidence part ${1:-a} done"
