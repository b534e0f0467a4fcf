#!/bin/bash
set -e
mkdir -p gpurun_out/rt2
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "fista or coef" > gpurun_out/rt2/tests.log 2>&1 || { tail -30 gpurun_out/rt2/tests.log; exit 1; }
tail -2 gpurun_out/rt2/tests.log
SC_FISTA_RT1=1 timeout -k 10 300 python scripts/bench_configs.py fistaloss --steps 10 --warmup 2 --iters 50 > gpurun_out/rt2/fl_rt1.json
timeout -k 10 300 python scripts/bench_configs.py fistaloss --steps 10 --warmup 2 --iters 50 > gpurun_out/rt2/fl_rt2.json
grep -o '"ms_per_step": [0-9.]*' gpurun_out/rt2/*.json
