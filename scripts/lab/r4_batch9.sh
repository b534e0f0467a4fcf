#!/bin/bash
# Round-4 GPU batch 9: graphed ES / DP / ZeRO-1 with the batch fed into the engine input by the
# previous step's fused tail; tests, one-rank benches (x2) next to the single-GPU step.
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O="$GRAFT_REPO_ROOT/gpurun_out/r4b9"; mkdir -p "$O"
PT="python3 -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 400 $PT tests/test_graphs_gpu.py tests/test_train_gpu.py > "$O/t.log" 2>&1 || { tail -40 "$O/t.log"; exit 1; }
tail -2 "$O/t.log"
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --no-eval > "$O/single_$r.json" 2> "$O/single_$r.err"
  echo "single $r $(grep -o '"ms_per_step": [0-9.]*' "$O/single_$r.json")"
  for m in es dp zero1; do
    timeout -k 10 200 python3 bench.py --force-dist --parallelism $m --compare-parallelism 0 --steps 200 --warmup 20 --no-eval > "$O/dist_${m}_$r.json" 2> "$O/dist_${m}_$r.err"
    echo "dist $m $r $(grep -o '"ms_per_step": [0-9.]*' "$O/dist_${m}_$r.json" | head -1)"
  done
done
