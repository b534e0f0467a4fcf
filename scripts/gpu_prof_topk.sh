#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m sparse_coding__amd.ops.build > gpurun_out/build.log 2>&1 || exit 1
rm -rf gpurun_out/prof_topk
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_topk" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/scripts/bench_configs.py" topk --steps 20 --warmup 3 > "$GRAFT_REPO_ROOT/gpurun_out/prof_topk.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof_topk.log"; exit 1; }
cd "$GRAFT_REPO_ROOT" && python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/prof_topk/run_kernel_stats.csv")))
for r in rows[:14]:
    print(f"{r['Name'][:80]:80s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:10.2f}us {float(r['Percentage']):6.2f}%")
PY
