#!/bin/bash
# GPU check: dense panel rewrite — tests, phase stamps, PGO timing
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_pgo.py tests/test_gpu_dense.py -m gpu > gpurun_out/dp_t.log 2>&1 &&
timeout -k 10 120 python -u tools/dense_stamps.py C3R > gpurun_out/dp_stamps.log 2>&1 &&
timeout -k 10 300 python -u tools/pgo_bench.py 150 400 1000 > gpurun_out/pgo_dp.log 2>&1
