#!/bin/bash
# top-k decode A/B (gather vs dense GEMM) + numerics + per-kernel profile of both
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/tk
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "topk" > gpurun_out/tk/tests.log 2>&1
timeout -k 10 200 python scripts/bench_configs.py topk --steps 40 --warmup 5 --decode gather > gpurun_out/tk/gather.json
timeout -k 10 200 python scripts/bench_configs.py topk --steps 40 --warmup 5 --decode gemm > gpurun_out/tk/gemm.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/tk/prof_gemm -o run -- python3 scripts/bench_configs.py topk --steps 20 --warmup 3 --decode gemm > gpurun_out/tk/prof_gemm.log 2>&1
cat gpurun_out/tk/*.json
