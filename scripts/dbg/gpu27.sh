#!/bin/bash
set -e
mkdir -p gpurun_out/galt
for r in 1 2; do
  for a in 0 1 2; do
    SC_FISTA_GRAM_ALT=$a timeout -k 10 300 python scripts/bench_configs.py fista --steps 6 --warmup 2 >> gpurun_out/galt/a$a.jsonl
  done
done
grep -o '"solve_ms_all_models": [0-9.]*' gpurun_out/galt/*.jsonl
