#!/bin/bash
# One consolidated GPU validation call: build, GPU tests, smoke, bench (config 2),
# configs 4/5, and a rocprofv3 kernel-stats profile of the bench step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD FAIL; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1; rc=$?
tail -8 gpurun_out/gputests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 300 python bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
if [ -n "$WITH_CONFIGS" ]; then
timeout -k 10 300 python scripts/bench_configs.py topk --steps 50 --warmup 5 > gpurun_out/config4_topk.json 2> gpurun_out/config4.err || { tail -20 gpurun_out/config4.err; exit 1; }
cat gpurun_out/config4_topk.json
timeout -k 10 400 python scripts/bench_configs.py fista --steps 10 --warmup 2 --models 4 --batch 1024 > gpurun_out/config5_fista.json 2> gpurun_out/config5.err || { tail -20 gpurun_out/config5.err; exit 1; }
cat gpurun_out/config5_fista.json
fi
rm -rf gpurun_out/prof
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 30 --warmup 5 --no-eval > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof.log"; exit 1; }
cd "$GRAFT_REPO_ROOT" && python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/prof/run_kernel_stats.csv")))
for r in rows[:16]:
    print(f"{r['Name'][:70]:70s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:9.2f}us {float(r['Percentage']):6.2f}%")
PY
