#!/bin/bash
set -e
mkdir -p gpurun_out/ru2
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "topk" > gpurun_out/ru2/tests.log 2>&1 || { tail -30 gpurun_out/ru2/tests.log; exit 1; }
for r in 1 2; do
  for ru in 0 16 4; do
    SC_TOPK_RU=$ru timeout -k 10 120 python scripts/bench_configs.py topk --steps 40 --warmup 5 >> gpurun_out/ru2/ru$ru.jsonl
  done
done
grep -o '"ms_per_step": [0-9.]*' gpurun_out/ru2/*.jsonl
