#!/bin/bash
# alternating A/B of the bracketed select on config 4 (3 rounds each)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "topk" > gpurun_out/tk4_tests.log 2>&1
set -e
mkdir -p gpurun_out/tk4
for r in 1 2 3; do
  SC_TOPK_NOXCD=1 timeout -k 10 120 python scripts/bench_configs.py topk --steps 60 --warmup 10 >> gpurun_out/tk4/noxcd.jsonl
  timeout -k 10 120 python scripts/bench_configs.py topk --steps 60 --warmup 10 >> gpurun_out/tk4/xcd.jsonl
done
grep -o '"ms_per_step": [0-9.]*' gpurun_out/tk4/noxcd.jsonl gpurun_out/tk4/xcd.jsonl
