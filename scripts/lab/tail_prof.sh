#!/bin/bash
# Fused step tail vs separate kernels: alternating 200-step benches, then a kernel-stats profile of each.
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O="$GRAFT_REPO_ROOT/gpurun_out/tail_prof"; mkdir -p "$O"
for r in 1 2; do
  for v in 1 0; do
    SC_FUSED_TAIL=$v timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --no-eval > "$O/t${v}_$r.json" 2> "$O/t${v}_$r.err"
    echo "tail=$v run $r $(grep -o '"ms_per_step": [0-9.]*' "$O/t${v}_$r.json")"
  done
done
for v in 1 0; do
  (cd /tmp && SC_FUSED_TAIL=$v timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$O/p$v" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 64 --warmup 16 --no-eval > "$O/p$v.log" 2>&1)
  python3 - "$O/p$v" > "$O/stats_t$v.txt" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:14]:
    print(f"{r['Name'][:80]:80s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:9.2f}us")
PY
  rm -rf "$O/p$v"; echo "== tail=$v"; cat "$O/stats_t$v.txt"
done
