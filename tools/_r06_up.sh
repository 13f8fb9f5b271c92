#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
PLBA_TIMING=1 timeout -k 10 300 python tools/host_map_timing.py 4 > gpurun_out/r06/$1_hmt.json 2> gpurun_out/r06/$1_hmt.err || { tail gpurun_out/r06/$1_hmt.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r06/$1_hmt.json'))
print('inc gather %.3f upload %.3f sum %.3f' % (d['gather_ms'], d['upload_ms'], d['gather_ms']+d['upload_ms']))"
grep -E "stage1|plba upload" gpurun_out/r06/$1_hmt.err | tail -60
