#!/bin/bash
# GPU box: the revisit window C3R through RCM + band, the dense MFMA path and the scalar dense
# kernel (bench lines), plus a rocprofv3 kernel trace of the dense MFMA path.
set -o pipefail
mkdir -p gpurun_out/dense_ab
export TMPDIR=/tmp
B="python3 bench.py --config C3R --steps 5 --warmup 2 --no-cpu-baseline"
timeout -k 10 200 $B > gpurun_out/dense_ab/rcm.json || exit 1
PLBA_NO_RCM=1 timeout -k 10 200 $B > gpurun_out/dense_ab/mfma.json || exit 1
PLBA_NO_RCM=1 PLBA_DENSE_SCALAR=1 timeout -k 10 300 $B > gpurun_out/dense_ab/scalar.json || exit 1
PLBA_NO_RCM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/dense_ab/trace -o mfma --output-format csv -- $B > /dev/null || exit 1
for f in rcm mfma scalar; do python3 -c "import json;d=json.load(open('gpurun_out/dense_ab/$f.json'));print('$f', round(d['value'],1), d['config']['factorisation'], d['roofline']['kernel'], round(d['roofline']['avg_launch_us'],1), d['roofline']['launches_per_lba'])"; done
