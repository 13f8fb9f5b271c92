#!/bin/bash
# Run on the GPU box from the repo root: rocprofv3 kernel stats + HBM PMC passes of bench.py.
# Usage: tools/profile_bench.sh <tag> [config]
set -eo pipefail
TAG=${1:-r01}; CFG=${2:-C3}
export TMPDIR=/tmp
OUT=gpurun_out/prof_${TAG}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o bench --output-format csv -- \
    python3 bench.py --config $CFG --steps 10 --warmup 2 --no-cpu-baseline --no-host-mirror --windows 0 > $OUT/bench_trace.json
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o bench --output-format csv -- \
    python3 bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline --no-host-mirror --windows 0 > $OUT/bench_fetch.json
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o bench --output-format csv -- \
    python3 bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline --no-host-mirror --windows 0 > $OUT/bench_write.json
echo done
