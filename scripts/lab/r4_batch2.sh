#!/bin/bash
# Round-4 GPU batch 2: step-GEMM block-shape lab on the current tree, then the other BASELINE
# configs on the current tree (top-k, masked, FISTA 300-iteration solve at a small ring).
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4b2; mkdir -p $O
timeout -k 10 300 python3 -u scripts/gemm_lab.py --which step_enc,step_dec,step_dc,step_wgrad --cfgs 1,2,3,6,10 --rounds 5 --out $O/gemm_cfgs.jsonl > $O/gemm_cfgs.log 2>&1
grep -o '"case": "[a-z_0-9]*", "median_us": [0-9.]*' $O/gemm_cfgs.jsonl
timeout -k 10 300 python3 scripts/bench_configs.py topk --steps 40 --warmup 10 > $O/topk.json 2> $O/topk.err; cat $O/topk.json
timeout -k 10 300 python3 scripts/bench_configs.py masked --steps 40 --warmup 10 > $O/masked.json 2> $O/masked.err; cat $O/masked.json
timeout -k 10 400 python3 scripts/bench_configs.py fista --steps 6 --warmup 2 --ratio 1.0 > $O/fista.json 2> $O/fista.err; cat $O/fista.json
