#!/bin/bash
# Round-4 GPU batch 8: ZeRO-1 graphed update through the fused tail (row shard); tests; one-rank
# benches; kernel stats + timelines of the graphed es / zero1 runs (what the N=1 rehearsal adds).
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O="$GRAFT_REPO_ROOT/gpurun_out/r4b8"; mkdir -p "$O"
PT="python3 -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 400 $PT tests/test_graphs_gpu.py tests/test_train_gpu.py > "$O/t.log" 2>&1 || { tail -40 "$O/t.log"; exit 1; }
tail -2 "$O/t.log"
timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --no-eval > "$O/single.json" 2> "$O/single.err"
echo "single $(grep -o '"ms_per_step": [0-9.]*' "$O/single.json")"
for m in es dp zero1; do
  timeout -k 10 200 python3 bench.py --force-dist --parallelism $m --compare-parallelism 0 --steps 200 --warmup 20 --no-eval > "$O/dist_$m.json" 2> "$O/dist_$m.err"
  echo "dist $m $(grep -o '"ms_per_step": [0-9.]*' "$O/dist_$m.json" | head -1)"
done
for m in es zero1; do
  (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$O/tr_$m" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --force-dist --parallelism $m --compare-parallelism 0 --settle-ms 0 --steps 64 --warmup 16 --no-eval > "$O/tr_$m.json" 2> "$O/tr_$m.err")
  python3 scripts/lab/step_timeline.py "$O/tr_$m" 4 > "$O/tr_$m.steps.jsonl"
  python3 - "$O/tr_$m" > "$O/stats_$m.txt" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:24]:
    print(f"{r['Name'][:90]:90s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:9.2f}us")
PY
  rm -rf "$O/tr_$m"; echo "== $m"; cat "$O/stats_$m.txt"; cat "$O/tr_$m.steps.jsonl"
done
