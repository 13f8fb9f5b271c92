#!/bin/bash
# SQ counter pass over a short C3 bench (diagnostic): per-kernel VALU/LDS/VMEM instruction and wait counts.
# Usage (GPU box, repo root): tools/pmc_sq.sh <tag>
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc_sq_${1:-x}
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT \
    -d $OUT -o pmc --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-mirror --windows 0 > $OUT/bench.json
echo done
