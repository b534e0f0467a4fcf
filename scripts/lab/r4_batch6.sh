#!/bin/bash
# Round-4 GPU batch 6: masked ensembles through the fused tail (tests + config), the settle-load
# experiment for the driver's 20/5 command, then the one-rank RCCL multi-GPU paths (graphed DP /
# ZeRO-1 after the unique-id fix, ensemble sharding) at 200/20.
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O="$GRAFT_REPO_ROOT/gpurun_out/r4b6"; mkdir -p "$O"
PT="python3 -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 300 $PT tests/test_masked_gpu.py tests/test_graphs_gpu.py > "$O/t_masked.log" 2>&1 || { tail -30 "$O/t_masked.log"; exit 1; }
tail -2 "$O/t_masked.log"
timeout -k 10 300 python3 scripts/bench_configs.py masked --steps 96 --warmup 16 > "$O/masked.json" 2> "$O/masked.err"; cat "$O/masked.json"
bash scripts/lab/r4_settle.sh
for m in "dp 1" "zero1 1" "es 0" "dp 0"; do
  set -- $m
  timeout -k 10 200 python3 bench.py --force-dist --parallelism $1 --dp-graph $2 --steps 200 --warmup 20 --no-eval > "$O/dist_$1_$2.json" 2> "$O/dist_$1_$2.err"
  echo "dist $1 graph=$2 $(grep -o '"ms_per_step": [0-9.]*' "$O/dist_$1_$2.json" | head -1)"
done
timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --no-eval > "$O/single.json" 2> "$O/single.err"
echo "single $(grep -o '"ms_per_step": [0-9.]*' "$O/single.json")"
