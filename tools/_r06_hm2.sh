#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
for t in 1 2 4 8; do
  PLSLAM_THREADS=$t timeout -k 10 300 python tools/host_map_timing.py 5 > gpurun_out/r06/hmt_$t.json 2> gpurun_out/r06/hmt_$t.err || { tail gpurun_out/r06/hmt_$t.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r06/hmt_$t.json')); s=d['scan']
print('threads $t', 'inc gather %.3f upload %.3f wb %.3f | scan gather %.3f upload %.3f wb %.3f' % (d['gather_ms'], d['upload_ms'], d['outlier_and_writeback_ms'], s['gather_ms'], s['upload_ms'], s['outlier_and_writeback_ms']))"
done
PLBA_TIMING=1 timeout -k 10 300 python tools/host_map_timing.py 3 > gpurun_out/r06/hmt_timing.json 2> gpurun_out/r06/hmt_timing.err
grep "plba upload" gpurun_out/r06/hmt_timing.err | tail -14
