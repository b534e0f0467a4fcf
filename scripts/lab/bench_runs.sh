#!/bin/bash
# Fresh-process bench runs: bash scripts/lab/bench_runs.sh OUTDIR "label|args" ...   (one JSON per run)
set -e
O="$GRAFT_REPO_ROOT/gpurun_out/$1"; shift; mkdir -p "$O"
for spec in "$@"; do
  label="${spec%%|*}"; args="${spec#*|}"
  timeout -k 10 300 python3 bench.py $args > "$O/$label.json" 2> "$O/$label.err"
  echo "$label $(grep -o '"ms_per_step": [0-9.]*' "$O/$label.json" | head -1) $(grep -o '"settle": {[^}]*}' "$O/$label.json" | head -1 | cut -c1-60)"
done
