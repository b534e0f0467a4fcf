#!/bin/bash
# Driver command (twice) next to 200/20 and the one-rank RCCL modes, on another box.
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O="$GRAFT_REPO_ROOT/gpurun_out/r4final2"; mkdir -p "$O"
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$O/driver_$r.json" 2> "$O/driver_$r.err"
  echo "driver $r $(grep -o '"ms_per_step": [0-9.]*' "$O/driver_$r.json") lines=$(wc -l < "$O/driver_$r.json")"
done
timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --no-eval > "$O/long.json" 2> "$O/long.err"
echo "200/20 $(grep -o '"ms_per_step": [0-9.]*' "$O/long.json")"
for m in es dp zero1; do
  timeout -k 10 200 python3 bench.py --force-dist --parallelism $m --compare-parallelism 0 --steps 200 --warmup 20 --no-eval > "$O/dist_$m.json" 2> "$O/dist_$m.err"
  echo "dist $m $(grep -o '"ms_per_step": [0-9.]*' "$O/dist_$m.json" | head -1)"
done
