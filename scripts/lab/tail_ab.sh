#!/bin/bash
# Same-box A/B, alternating fresh processes: the fused step tail (SC_FUSED_TAIL=1, default) vs the
# separate Adam / loss / bias kernels (0), and bf16 weight-gradient storage; then the driver command.
set -e
O="$GRAFT_REPO_ROOT/gpurun_out/tail_ab3"; mkdir -p "$O"
for r in 1 2; do
  for v in "t1|1|fp32" "t0|0|fp32" "t1bf|1|bf16"; do
    IFS='|' read -r lab tail gdt <<< "$v"
    SC_FUSED_TAIL=$tail timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --no-eval --wgrad-dtype $gdt > "$O/${lab}_$r.json" 2> "$O/${lab}_$r.err"
    echo "$lab run $r $(grep -o '"ms_per_step": [0-9.]*' "$O/${lab}_$r.json")"
  done
done
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 > "$O/driver.json" 2> "$O/driver.err"
echo "driver $(grep -o '"ms_per_step": [0-9.]*' "$O/driver.json")"
