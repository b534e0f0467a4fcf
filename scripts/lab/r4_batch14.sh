#!/bin/bash
# Round-4 GPU batch 14: masked ensembles with the compacted tail grid: tests, masked config (both
# variants), masked kernel stats.
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O="$GRAFT_REPO_ROOT/gpurun_out/r4b14"; mkdir -p "$O"
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_masked_gpu.py tests/test_graphs_gpu.py > "$O/t.log" 2>&1 || { tail -40 "$O/t.log"; exit 1; }
tail -1 "$O/t.log"
for r in 1 2; do
  timeout -k 10 300 python3 scripts/bench_configs.py masked --steps 96 --warmup 16 > "$O/masked_$r.json" 2> "$O/masked_$r.err"; cat "$O/masked_$r.json"
done
# per-rank ensemble-sharded layouts (N = 4, 8) under weight-gradient split-K factors
for ws in auto 4 2 1; do
  timeout -k 10 300 python3 scripts/es_projection.py --ns 4,8 --wsplit $ws > "$O/esp_ws$ws.jsonl" 2> "$O/esp_ws$ws.err"
  echo "wsplit=$ws $(grep -o '"N": [0-9]*\|"ms_per_step": [0-9.]*' "$O/esp_ws$ws.jsonl" | tr '\n' ' ')"
done
