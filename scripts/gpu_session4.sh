#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD FAIL; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "fista or topk" > gpurun_out/gputests_fista.log 2>&1; rc=$?
tail -12 gpurun_out/gputests_fista.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/bench_configs.py fista --steps 10 --warmup 2 --ring-gb 150 > gpurun_out/config5_fista.json 2> gpurun_out/config5.err || { tail -20 gpurun_out/config5.err; exit 1; }
cat gpurun_out/config5_fista.json
timeout -k 10 300 python scripts/bench_configs.py topk --steps 50 --warmup 5 > gpurun_out/config4_topk.json 2> gpurun_out/config4.err || { tail -20 gpurun_out/config4.err; exit 1; }
cat gpurun_out/config4_topk.json
rm -rf gpurun_out/prof_topk
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_topk" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/scripts/bench_configs.py" topk --steps 20 --warmup 3 > "$GRAFT_REPO_ROOT/gpurun_out/prof_topk.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof_topk.log"; exit 1; }
cd "$GRAFT_REPO_ROOT" && python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/prof_topk/run_kernel_stats.csv")))
for r in rows[:14]:
    print(f"{r['Name'][:80]:80s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:10.2f}us {float(r['Percentage']):6.2f}%")
PY
