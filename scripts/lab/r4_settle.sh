#!/bin/bash
# Driver command (20/5) under the settle loads -- GEMM-only (default), the step's own kernel mix on
# a scratch ensemble, none -- next to 200/20 on the same box; then kernel traces (per-step
# timelines) of the gemm and step settles.
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O="$GRAFT_REPO_ROOT/gpurun_out/r4settle"; mkdir -p "$O"
for r in 1 2; do
  for m in "gemm 150" "step 150" "gemm 0" "step 400"; do
    set -- $m
    timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-eval --settle-mode $1 --settle-ms $2 > "$O/d_$1_$2_$r.json" 2> "$O/d_$1_$2_$r.err"
    echo "20/5 settle=$1 $2 run $r $(grep -o '"ms_per_step": [0-9.]*' "$O/d_$1_$2_$r.json")"
  done
  timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --no-eval > "$O/l_$r.json" 2> "$O/l_$r.err"
  echo "200/20 run $r $(grep -o '"ms_per_step": [0-9.]*' "$O/l_$r.json")"
done
for m in gemm step; do
  (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace -d "$O/tr_$m" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 --no-eval --settle-mode $m > "$O/tr_$m.json" 2> "$O/tr_$m.err")
  python3 scripts/lab/step_timeline.py "$O/tr_$m" 25 > "$O/tr_$m.steps.jsonl"
  rm -rf "$O/tr_$m"
  echo "trace settle=$m $(grep -o '"ms_per_step": [0-9.]*' "$O/tr_$m.json") $(tail -1 "$O/tr_$m.steps.jsonl")"
done
