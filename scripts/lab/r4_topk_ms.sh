#!/bin/bash
# Top-k config 4: multi-step graphs with the in-graph batch gather vs host sampling + one replay per step.
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O="$GRAFT_REPO_ROOT/gpurun_out/r4topkms"; mkdir -p "$O"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_graphs_gpu.py -k "topk" > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
tail -2 "$O/tests.log"
for r in 1 2; do
  for gs in 1 8; do
    timeout -k 10 300 python3 scripts/bench_configs.py topk --graph-steps $gs --steps 40 --warmup 8 > "$O/topk_gs${gs}_$r.json" 2> "$O/topk_gs${gs}_$r.err"
    echo "graph_steps=$gs run $r $(grep -o '"ms_per_step": [0-9.]*' "$O/topk_gs${gs}_$r.json" | head -1)"
  done
done
