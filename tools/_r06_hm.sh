#!/bin/bash
# r06: host-mirror GPU tests, default bench (incremental gather, pinned window), bench without pinned window
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "host or shard or hlm" > gpurun_out/r06/$1_tests.log 2>&1 || { tail -30 gpurun_out/r06/$1_tests.log; exit 1; }
tail -2 gpurun_out/r06/$1_tests.log
timeout -k 10 400 python bench.py > gpurun_out/r06/$1_bench.json 2> gpurun_out/r06/$1_bench.err || { tail -20 gpurun_out/r06/$1_bench.err; exit 1; }
PLSLAM_NO_PINNED=1 timeout -k 10 400 python bench.py --no-cpu-baseline --windows 0 > gpurun_out/r06/$1_bench_nopin.json 2> gpurun_out/r06/$1_bench_nopin.err || { tail -20 gpurun_out/r06/$1_bench_nopin.err; exit 1; }
python3 - <<PY
import json
for f in ("gpurun_out/r06/$1_bench.json", "gpurun_out/r06/$1_bench_nopin.json"):
    d = json.load(open(f))
    print(f, d["value"], json.dumps(d.get("host_mirror")), json.dumps(d.get("host_mirror_c5_map")))
PY
