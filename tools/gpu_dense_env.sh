#!/bin/bash
# GPU check: envelope-aware dense factorisation (LBA dense path + pose graph): tests, then timing
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_pgo.py tests/test_gpu_dense.py -m gpu > gpurun_out/de_t.log 2>&1 &&
timeout -k 10 300 python -u tools/pgo_bench.py 150 400 1000 > gpurun_out/pgo_env.log 2>&1
