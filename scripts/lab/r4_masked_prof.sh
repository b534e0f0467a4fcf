#!/bin/bash
# Per-kernel stats of the masked and the unmasked variant of the masked config, each alone.
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O="$GRAFT_REPO_ROOT/gpurun_out/r4mprof"; mkdir -p "$O"
for v in masked unmasked; do
  (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$O/p_$v" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/scripts/bench_configs.py" masked --variant $v --steps 64 --warmup 16 > "$O/p_$v.log" 2>&1)
  python3 - "$O/p_$v" > "$O/stats_$v.txt" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:16]:
    if "scamd" in r["Name"]:
        print(f"{r['Name'][:100]:100s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:9.2f}us")
PY
  rm -rf "$O/p_$v"; echo "== $v"; cat "$O/stats_$v.txt"
done
