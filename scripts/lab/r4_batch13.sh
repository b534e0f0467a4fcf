#!/bin/bash
# Round-4 GPU batch 13: graphed ES after the update-only wait (tests + bench), top-k GEMM block shapes
# in-step (scores GEMM EPI_F32 = epi 3, dense bf16 weight gradient EPI_BF16 = epi 4; BK64 x 2 rings).
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O="$GRAFT_REPO_ROOT/gpurun_out/r4b13"; mkdir -p "$O"
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_graphs_gpu.py > "$O/t.log" 2>&1 || { tail -40 "$O/t.log"; exit 1; }
tail -1 "$O/t.log"
timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --no-eval > "$O/single.json" 2> "$O/single.err"
echo "single $(grep -o '"ms_per_step": [0-9.]*' "$O/single.json")"
timeout -k 10 200 python3 bench.py --force-dist --parallelism es --compare-parallelism 0 --steps 200 --warmup 20 --no-eval > "$O/es.json" 2> "$O/es.err"
echo "es $(grep -o '"ms_per_step": [0-9.]*' "$O/es.json" | head -1)"
for spec in "def:" "f1:3:1" "f2:3:2" "b1:4:1" "b2:4:2" "b3:4:3"; do
  name=${spec%%:*}; cfg=${spec#*:}
  rc=0; SC_GEMM_CFG="$cfg" timeout -k 10 300 python3 scripts/bench_configs.py topk --steps 40 --warmup 10 > "$O/topk_$name.json" 2> "$O/topk_$name.err" || rc=$?
  [ $rc -gt 1 ] && { echo "topk $name rc=$rc"; exit 1; }
  echo "topk $name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$O/topk_$name.json")"
done
