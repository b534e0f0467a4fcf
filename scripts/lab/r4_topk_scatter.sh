#!/bin/bash
# Top-k config 4: decode scatters into the dense buffers for every model vs only the dense-wgrad ones.
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O="$GRAFT_REPO_ROOT/gpurun_out/r4topksc"; mkdir -p "$O"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_graphs_gpu.py -k "topk" > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
tail -2 "$O/tests.log"
for r in 1 2 3; do
  for a in 1 0; do
    SC_TOPK_SCATTER_ALL=$a timeout -k 10 300 python3 scripts/bench_configs.py topk --steps 48 --warmup 8 > "$O/topk_all${a}_$r.json" 2> "$O/topk_all${a}_$r.err"
    echo "scatter_all=$a run $r $(grep -o '"ms_per_step": [0-9.]*' "$O/topk_all${a}_$r.json" | head -1)"
  done
done
