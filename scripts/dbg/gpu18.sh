#!/bin/bash
# pipelined Gram-form FISTA: numerics, then config 5 with 32-row (default) and 16-row workgroups
set -e
mkdir -p gpurun_out/fi
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "fista" > gpurun_out/fi/tests.log 2>&1
timeout -k 10 300 python scripts/bench_configs.py fista --steps 6 --warmup 2 > gpurun_out/fi/rt2.json
timeout -k 10 300 python scripts/bench_configs.py fista --steps 6 --warmup 2 --ratio 2 > gpurun_out/fi/direct_r2.json
cat gpurun_out/fi/*.json
