#!/bin/bash
# Round-4 GPU batch 5: fused code/encoder gradient with L2 warm-up touches (test, A/B, stats, PMC);
# then the graphed data-parallel paths after the RCCL unique-id fix (rehearsal + force-dist benches).
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O="$GRAFT_REPO_ROOT/gpurun_out/r4b5"; mkdir -p "$O"
PT="python3 -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 200 $PT tests/test_kernels_gpu.py -k code_grad_wgrad > "$O/t_dcw.log" 2>&1 || { tail -30 "$O/t_dcw.log"; exit 1; }
tail -2 "$O/t_dcw.log"
for v in 1 0; do
  SC_FUSED_DCW=$v timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --no-eval > "$O/dcw$v.json" 2> "$O/dcw$v.err"
  echo "dcw=$v $(grep -o '"ms_per_step": [0-9.]*' "$O/dcw$v.json")"
done
(cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$O/p1" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 64 --warmup 16 --no-eval > "$O/p1.log" 2>&1)
python3 - "$O/p1" > "$O/stats_dcw1.txt" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:14]:
    print(f"{r['Name'][:90]:90s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:9.2f}us")
PY
rm -rf "$O/p1"; cat "$O/stats_dcw1.txt"
bash scripts/gpu.sh pmc > "$O/pmc.log" 2>&1 || { tail -20 "$O/pmc.log"; exit 1; }
grep "dcw\|Shape<2, 4, 8, 4>, false\|, 7, 64" gpurun_out/pmc_summary.md || true
for m in dp zero1; do
  timeout -k 10 200 python3 -u scripts/lab/dp_graph_repro.py $m engines-first on > "$O/repro_$m.log" 2>&1 || { tail -30 "$O/repro_$m.log"; exit 1; }
  tail -2 "$O/repro_$m.log"
done
for m in "dp 1" "zero1 1" "dp 0" "es 0"; do
  set -- $m
  timeout -k 10 200 python3 bench.py --force-dist --parallelism $1 --dp-graph $2 --steps 200 --warmup 20 --no-eval > "$O/dist_$1_$2.json" 2> "$O/dist_$1_$2.err"
  echo "dist $1 graph=$2 $(grep -o '"ms_per_step": [0-9.]*' "$O/dist_$1_$2.json" | head -1)"
done
