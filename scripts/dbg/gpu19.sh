#!/bin/bash
# FISTA in the loss on the kernels: numerics + training run; FISTA solver tests after the save-slab change
set -e
mkdir -p gpurun_out/fl
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "fista" > gpurun_out/fl/tests.log 2>&1
timeout -k 10 300 python scripts/bench_configs.py fistaloss --steps 10 --warmup 2 --iters 50 --batch 2048 > gpurun_out/fl/run.json
cat gpurun_out/fl/run.json
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/fl/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/bench_configs.py fistaloss --steps 4 --warmup 1 --iters 50 --batch 2048 > $GRAFT_REPO_ROOT/gpurun_out/fl/prof.log 2>&1)
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/fl/prof/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:12]:
    print(f"{r['Name'][:90]:90s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:9.2f}us {float(r['Percentage']):6.2f}%")
PY
