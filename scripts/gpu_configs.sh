#!/bin/bash
# BASELINE configs 4 and 5 on one MI355X (config 2 = bench.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m sparse_coding__amd.ops.build > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 1; }
timeout -k 10 300 python scripts/bench_configs.py topk --steps 50 --warmup 5 > gpurun_out/config4_topk.json 2> gpurun_out/config4.err || { tail -20 gpurun_out/config4.err; exit 1; }
cat gpurun_out/config4_topk.json
timeout -k 10 400 python scripts/bench_configs.py fista --steps 10 --warmup 2 --models 4 --batch 1024 > gpurun_out/config5_fista.json 2> gpurun_out/config5.err || { tail -20 gpurun_out/config5.err; exit 1; }
cat gpurun_out/config5_fista.json
