#!/bin/bash
# Top-k config 4: slot-list / dense weight-gradient split point (sparse_k) sweep.
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O="$GRAFT_REPO_ROOT/gpurun_out/r4topksk"; mkdir -p "$O"
for r in 1 2; do
  for sk in auto 16 32 48 0; do
    timeout -k 10 300 python3 scripts/bench_configs.py topk --sparse-k $sk --steps 40 --warmup 10 > "$O/topk_sk${sk}_$r.json" 2> "$O/topk_sk${sk}_$r.err"
    echo "sparse_k=$sk run $r $(grep -o '"ms_per_step": [0-9.]*' "$O/topk_sk${sk}_$r.json" | head -1) $(grep -o '"sparse_wgrad_models": [0-9]*' "$O/topk_sk${sk}_$r.json")"
  done
done
