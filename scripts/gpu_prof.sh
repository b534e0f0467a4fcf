#!/bin/bash
# Kernel-level profile of the bench step: rocprofv3 kernel trace + stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m sparse_coding__amd.ops.build > gpurun_out/build.log 2>&1 || exit 1
rm -rf gpurun_out/prof
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 30 --warmup 5 --no-eval ${BENCH_ARGS} > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof.log"; exit 1; }
cd "$GRAFT_REPO_ROOT" && python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/prof/run_kernel_stats.csv")))
for r in rows[:16]:
    print(f"{r['Name'][:70]:70s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:9.2f}us {float(r['Percentage']):6.2f}%")
PY
