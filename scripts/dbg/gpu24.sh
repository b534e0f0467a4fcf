#!/bin/bash
# non-temporal Adam state stores A/B on the headline bench (alternating, 3 runs each)
set -e
mkdir -p gpurun_out/nt
for r in 1 2 3; do
  SC_ADAM_NT=0 timeout -k 10 200 python bench.py --steps 100 --warmup 20 --no-eval >> gpurun_out/nt/nt0.jsonl
  SC_ADAM_NT=1 timeout -k 10 200 python bench.py --steps 100 --warmup 20 --no-eval >> gpurun_out/nt/nt1.jsonl
done
grep -o '"ms_per_step": [0-9.]*' gpurun_out/nt/*.jsonl
