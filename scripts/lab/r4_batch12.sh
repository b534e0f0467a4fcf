#!/bin/bash
# Round-4 GPU batch 12: masked ensembles under both encoder / code-gradient configurations (the
# compacted launches have fewer tiles than the unmasked step); then the full GPU suite + smoke.
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O="$GRAFT_REPO_ROOT/gpurun_out/r4b12"; mkdir -p "$O"
for r in 1 2; do
  for spec in "new:" "old:0:1,6:1,7:1"; do
    name=${spec%%:*}; cfg=${spec#*:}
    SC_GEMM_CFG="$cfg" timeout -k 10 300 python3 scripts/bench_configs.py masked --variant masked --steps 96 --warmup 16 > "$O/masked_${name}_$r.json" 2> "$O/masked_${name}_$r.err"
    echo "masked $name $r $(grep -o '"masked_ms_per_step": [0-9.]*' "$O/masked_${name}_$r.json")"
  done
done
bash scripts/gpu.sh tests smoke > "$O/suite.log" 2>&1 || { tail -40 "$O/suite.log"; exit 1; }
grep -E "passed|failed|smoke" "$O/suite.log" | tail -3
