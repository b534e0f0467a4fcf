#!/bin/bash
# In-step A/B of GEMM block configurations (SC_GEMM_CFG = "epi:cfg,...", cfg = shape | pipeline << 2):
# epi 0 encoder, 6 encoder + counts, 7 code gradient, 1 decoder, 3 weight gradients.
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O="$GRAFT_REPO_ROOT/gpurun_out/${CFG_OUT:-r4cfg}"; mkdir -p "$O"
V=(${CFG_VARIANTS:-"new:" "old:0:1,6:1,7:1" "dec13:1:13" "dec9:1:9" "encdc9:0:9,6:9,7:9" "encdc15:0:15,6:15,7:15" "wg11:3:11" "wg9:3:9"})
for r in 1 2; do
  for spec in "${V[@]}"; do
    name=${spec%%:*}; cfg=${spec#*:}
    SC_GEMM_CFG="$cfg" timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --no-eval > "$O/${name}_$r.json" 2> "$O/${name}_$r.err"
    echo "$name run $r $(grep -o '"ms_per_step": [0-9.]*' "$O/${name}_$r.json")"
  done
done
