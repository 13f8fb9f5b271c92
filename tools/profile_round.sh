#!/bin/bash
# GPU box, repo root: rocprofv3 evidence for one config of bench.py — kernel trace stats, then
# separate PMC passes (HBM FETCH_SIZE, WRITE_SIZE; SQ occupancy / instruction mix; GRBM busy).
# Usage: tools/profile_round.sh <tag> <config> [steps]
set -eo pipefail
TAG=${1:-r02}; CFG=${2:-C3}; ST=${3:-10}
export TMPDIR=/tmp
OUT=gpurun_out/prof_${TAG}_${CFG}
mkdir -p $OUT
B="python3 bench.py --config $CFG --steps $ST --warmup 2 --no-cpu-baseline --windows 0 --no-host-mirror"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o bench --output-format csv -- $B > $OUT/bench_trace.json
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o bench --output-format csv -- $B > $OUT/bench_fetch.json
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o bench --output-format csv -- $B > $OUT/bench_write.json
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY \
    -d $OUT/sq -o bench --output-format csv -- $B > $OUT/bench_sq.json
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d $OUT/grbm -o bench --output-format csv -- $B > $OUT/bench_grbm.json
echo "profile $TAG $CFG done"
