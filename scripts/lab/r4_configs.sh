#!/bin/bash
# Round-4 refresh of the other BASELINE configs on the final tree: config 5 FISTA (small ring),
# FISTA in the loss, Pythia-70m MLP configs.
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O="$GRAFT_REPO_ROOT/gpurun_out/r4cfgs"; mkdir -p "$O"
timeout -k 10 400 python3 scripts/bench_configs.py fista --steps 6 --warmup 2 --ratio 1.0 > "$O/fista.json" 2> "$O/fista.err"; cat "$O/fista.json"
timeout -k 10 300 python3 scripts/bench_configs.py fistaloss --steps 20 --warmup 5 > "$O/fistaloss.json" 2> "$O/fistaloss.err"; cat "$O/fistaloss.json"
timeout -k 10 300 python3 scripts/bench_configs.py mlp --steps 50 --warmup 10 > "$O/mlp.json" 2> "$O/mlp.err"; cat "$O/mlp.json"
