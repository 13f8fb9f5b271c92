#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "build or host or edge" > gpurun_out/r06/$1_tests.log 2>&1 || { tail -30 gpurun_out/r06/$1_tests.log; exit 1; }
tail -2 gpurun_out/r06/$1_tests.log
for t in 1 8; do
  PLSLAM_THREADS=$t timeout -k 10 300 python tools/host_map_timing.py 5 > gpurun_out/r06/$1_hmt_$t.json 2> gpurun_out/r06/$1_hmt_$t.err || { tail gpurun_out/r06/$1_hmt_$t.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r06/$1_hmt_$t.json')); s=d['scan']
print('threads $t', 'inc gather %.3f upload %.3f sum %.3f wb %.3f | scan gather %.3f upload %.3f wb %.3f' % (d['gather_ms'], d['upload_ms'], d['gather_ms']+d['upload_ms'], d['outlier_and_writeback_ms'], s['gather_ms'], s['upload_ms'], s['outlier_and_writeback_ms']))"
done
