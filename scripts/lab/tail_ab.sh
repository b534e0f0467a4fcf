#!/bin/bash
# Same-box A/B of the fused step tail (SC_FUSED_TAIL=1, default) vs the separate Adam / loss / bias
# kernels (SC_FUSED_TAIL=0), alternating fresh processes, then the driver command.
set -e
O="$GRAFT_REPO_ROOT/gpurun_out/tail_ab3"; mkdir -p "$O"
for r in 1 2; do
  for v in 1 0; do
    SC_FUSED_TAIL=$v timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --no-eval > "$O/t${v}_$r.json" 2> "$O/t${v}_$r.err"
    echo "tail=$v run $r $(grep -o '"ms_per_step": [0-9.]*' "$O/t${v}_$r.json")"
  done
done
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 > "$O/driver.json" 2> "$O/driver.err"
echo "driver $(grep -o '"ms_per_step": [0-9.]*' "$O/driver.json")"
