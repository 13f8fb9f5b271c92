set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench_r02f.json 2> gpurun_out/bench_r02f.err
cat gpurun_out/bench_r02f.json
timeout -k 10 300 python bench.py --config C5 --steps 10 > gpurun_out/bench_r02f_C5.json 2> gpurun_out/bench_r02f_C5.err
bash tools/profile_round.sh r02f C3
bash tools/profile_round.sh r02f C5 5
