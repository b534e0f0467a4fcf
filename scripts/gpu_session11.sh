#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD FAIL; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 400 python scripts/bench_configs.py mlp --steps 50 --warmup 5 > gpurun_out/config3_mlp.json 2> gpurun_out/config3.err || { tail -20 gpurun_out/config3.err; exit 1; }
cat gpurun_out/config3_mlp.json
rm -rf gpurun_out/prof
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 50 --warmup 5 --no-eval > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof.log"; exit 1; }
cd "$GRAFT_REPO_ROOT" && python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/prof/run_kernel_stats.csv")))
for r in rows[:16]:
    print(f"{r['Name'][:70]:70s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:9.2f}us {float(r['Percentage']):6.2f}%")
PY
bash scripts/gpu_pmc2.sh > gpurun_out/pmc_run.log 2>&1 || { tail -20 gpurun_out/pmc_run.log; exit 1; }
tail -12 gpurun_out/pmc_run.log | cut -c1-200
