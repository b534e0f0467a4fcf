#!/bin/bash
# top-k weight-gradient split-K A/B (1 / 2 / 3) on config 4 + numerics with split 2
set -e
mkdir -p gpurun_out/ws
SC_TOPK_WSPLIT=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "fused_topk" > gpurun_out/ws/tests.log 2>&1 || { tail -30 gpurun_out/ws/tests.log; exit 1; }
for r in 1 2; do
  for s in 1 2 3; do
    SC_TOPK_WSPLIT=$s timeout -k 10 120 python scripts/bench_configs.py topk --steps 40 --warmup 5 >> gpurun_out/ws/s$s.jsonl
  done
done
grep -o '"ms_per_step": [0-9.]*' gpurun_out/ws/*.jsonl
