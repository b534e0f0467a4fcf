#!/bin/bash
# Top-k config 4: select kernel occupancy hint (launch bounds) A/B.
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O="$GRAFT_REPO_ROOT/gpurun_out/r4topkocc"; mkdir -p "$O"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "topk" > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
tail -2 "$O/tests.log"
for r in 1 2; do
  for x in 0 2 4; do
    SC_TOPK_SELECT_OCC=$x timeout -k 10 300 python3 scripts/bench_configs.py topk --steps 40 --warmup 10 > "$O/topk_x${x}_$r.json" 2> "$O/topk_x${x}_$r.err"
    echo "occ=$x run $r $(grep -o '"ms_per_step": [0-9.]*' "$O/topk_x${x}_$r.json" | head -1)"
  done
done
cd /tmp
for x in 0 2 4; do
  SC_TOPK_SELECT_OCC=$x timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_x$x" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/scripts/bench_configs.py" topk --steps 20 --warmup 5 > "$O/prof_x$x.log" 2>&1
  f=$(find "$O/prof_x$x" -name "*kernel_stats.csv" | head -1); cp "$f" "$O/stats_x$x.csv"
  grep -E "topk_block_kernel" "$O/stats_x$x.csv" | cut -c1-200
done
