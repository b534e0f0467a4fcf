#!/bin/bash
# bracketed top-k select: numerics + config-4 A/B (bracket vs full bisection)
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/tk2
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "topk" > gpurun_out/tk2/tests.log 2>&1
SC_TOPK_NOBRACKET=1 timeout -k 10 200 python scripts/bench_configs.py topk --steps 40 --warmup 5 > gpurun_out/tk2/nobracket.json
timeout -k 10 200 python scripts/bench_configs.py topk --steps 40 --warmup 5 > gpurun_out/tk2/bracket.json
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/tk2/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/bench_configs.py topk --steps 20 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/tk2/prof.log 2>&1)
cat gpurun_out/tk2/*.json
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/tk2/prof/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:12]:
    print(f"{r['Name'][:90]:90s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:9.2f}us {float(r['Percentage']):6.2f}%")
PY
