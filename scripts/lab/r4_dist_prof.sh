#!/bin/bash
# Kernel stats + per-step timelines of the one-rank RCCL multi-GPU paths next to the single-GPU step.
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O="$GRAFT_REPO_ROOT/gpurun_out/r4dist"; mkdir -p "$O"
for spec in "single" "es --force-dist --parallelism es" "dpg --force-dist --parallelism dp --dp-graph 1" "z1g --force-dist --parallelism zero1 --dp-graph 1"; do
  set -- $spec; n=$1; shift
  (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$O/tr_$n" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 64 --warmup 16 --no-eval "$@" > "$O/tr_$n.json" 2> "$O/tr_$n.err")
  python3 scripts/lab/step_timeline.py "$O/tr_$n" 6 > "$O/tr_$n.steps.jsonl"
  python3 - "$O/tr_$n" > "$O/stats_$n.txt" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:22]:
    print(f"{r['Name'][:90]:90s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:9.2f}us")
PY
  rm -rf "$O/tr_$n"
  echo "== $n $(grep -o '"ms_per_step": [0-9.]*' "$O/tr_$n.json" | head -1) $(tail -1 "$O/tr_$n.steps.jsonl")"
done
timeout -k 10 400 python3 -u scripts/gemm_lab.py --which step_enc,step_dec,step_dc,step_wgrad,step_torch --cfgs 1,5,9,13,2,6,10,14,3,7,11,15 --rounds 5 --out "$O/gemm_cfgs.jsonl" > "$O/gemm_cfgs.log" 2>&1
grep -o '"case": "[a-z_0-9]*", "median_us": [0-9.]*' "$O/gemm_cfgs.jsonl"
