#!/bin/bash
# decode gather depth A/B (rows per iteration 2 / 4 / 8) on config 4
set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "coef or fista or topk" > gpurun_out/ru_tests.log 2>&1 || { tail -30 gpurun_out/ru_tests.log; exit 1; }
mkdir -p gpurun_out/ru
for r in 1 2; do
  for ru in 4 8 2; do
    SC_TOPK_RU=$ru timeout -k 10 120 python scripts/bench_configs.py topk --steps 40 --warmup 5 >> gpurun_out/ru/ru$ru.jsonl
  done
done
grep -o '"ms_per_step": [0-9.]*' gpurun_out/ru/*.jsonl
