#!/bin/bash
# GPU check: output download path tests, upload/e2e phase timing, step-graph depth A/B
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_build.py tests/test_g2o_facade.py tests/test_gpu_parity.py -m gpu > gpurun_out/dl_t.log 2>&1 &&
timeout -k 10 120 python -u tools/upload_timing.py C3 C5 > gpurun_out/ut2.log 2>&1 &&
for L in 4 2 1; do PLBA_GRAPH_LEVELS=$L timeout -k 10 120 python -u bench.py --steps 40 --warmup 3 --no-cpu-baseline > gpurun_out/bL$L.json 2>&1 || exit 1; done
