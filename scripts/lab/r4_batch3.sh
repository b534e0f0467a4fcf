#!/bin/bash
# Round-4 GPU batch 3: the driver's command (two fresh processes) next to a 200/20 run on the
# same box; the other BASELINE configs (top-k, masked + its kernel profile, FISTA); then the
# one-rank RCCL multi-GPU paths (es, host-issued dp, graphed dp / zero1) at 200/20.
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O="$GRAFT_REPO_ROOT/gpurun_out/r4b3"; mkdir -p "$O"
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$O/driver_$r.json" 2> "$O/driver_$r.err"
  echo "driver $r $(grep -o '"ms_per_step": [0-9.]*' "$O/driver_$r.json")"
done
timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --no-eval > "$O/long.json" 2> "$O/long.err"
echo "200/20 $(grep -o '"ms_per_step": [0-9.]*' "$O/long.json")"
timeout -k 10 300 python3 scripts/bench_configs.py topk --steps 40 --warmup 10 > "$O/topk.json" 2> "$O/topk.err"; cat "$O/topk.json"
timeout -k 10 300 python3 scripts/bench_configs.py masked --steps 40 --warmup 10 > "$O/masked.json" 2> "$O/masked.err"; cat "$O/masked.json"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/pm" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/scripts/bench_configs.py" masked --steps 20 --warmup 5 > "$O/pm.log" 2>&1)
python3 - "$O/pm" > "$O/masked_kernels.txt" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:24]:
    print(f"{r['Name'][:100]:100s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:9.2f}us")
PY
rm -rf "$O/pm"; cat "$O/masked_kernels.txt"
for m in "es 0" "dp 0" "dp 1" "zero1 1"; do
  set -- $m
  timeout -k 10 200 python3 -X faulthandler bench.py --force-dist --parallelism $1 --dp-graph $2 --steps 200 --warmup 20 --no-eval > "$O/dist_$1_$2.json" 2> "$O/dist_$1_$2.err"
  echo "dist $1 graph=$2 $(grep -o '"ms_per_step": [0-9.]*' "$O/dist_$1_$2.json")"
done
