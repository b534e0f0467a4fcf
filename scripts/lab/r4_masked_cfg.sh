#!/bin/bash
# Masked config (masked variant alone) under encoder / code-gradient block configurations.
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O="$GRAFT_REPO_ROOT/gpurun_out/r4mcfg"; mkdir -p "$O"
for r in 1 2; do
  for spec in "c13:" "c9:0:9,6:9,7:9" "c1:0:1,6:1,7:1" "c11:0:11,6:11,7:11" "c9dec9:0:9,6:9,7:9,1:9"; do
    name=${spec%%:*}; cfg=${spec#*:}
    rc=0; SC_GEMM_CFG="$cfg" timeout -k 10 300 python3 scripts/bench_configs.py masked --variant masked --steps 96 --warmup 16 > "$O/m_${name}_$r.json" 2> "$O/m_${name}_$r.err" || rc=$?
    [ $rc -gt 1 ] && { echo "$name rc=$rc"; exit 1; }
    echo "masked $name $r rc=$rc $(grep -o '"masked_ms_per_step": [0-9.]*' "$O/m_${name}_$r.json")"
  done
done
