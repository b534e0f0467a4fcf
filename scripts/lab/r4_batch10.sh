#!/bin/bash
# Round-4 GPU batch 10: the full GPU suite + smoke on the current tree; an in-step A/B of the
# encoder / code-gradient pipeline config (cfg 13 = 128x128, BK32 x 3 stages) against the
# defaults; the driver command next to 200/20.
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O="$GRAFT_REPO_ROOT/gpurun_out/r4b10"; mkdir -p "$O"
bash scripts/gpu.sh tests smoke > "$O/suite.log" 2>&1 || { tail -40 "$O/suite.log"; exit 1; }
grep -E "passed|failed" "$O/suite.log" | tail -2
for r in 1 2; do
  for v in "" "0:13,6:13,7:13"; do
    SC_GEMM_CFG="$v" timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --no-eval > "$O/cfg_${v:-def}_$r.json" 2> "$O/cfg_$r.err"
    echo "cfg=${v:-default} run $r $(grep -o '"ms_per_step": [0-9.]*' "$O/cfg_${v:-def}_$r.json")"
  done
done
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$O/driver_$r.json" 2> "$O/driver_$r.err"
  echo "driver $r $(grep -o '"ms_per_step": [0-9.]*' "$O/driver_$r.json")"
done
