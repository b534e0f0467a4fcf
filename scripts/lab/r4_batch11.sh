#!/bin/bash
# Round-4 GPU batch 11 (new GEMM defaults): driver command and 200/20 on the same box, kernel stats
# of the headline step, the masked and top-k configs, the one-rank RCCL modes.
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O="$GRAFT_REPO_ROOT/gpurun_out/r4b11"; mkdir -p "$O"
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$O/driver_$r.json" 2> "$O/driver_$r.err"
  echo "driver $r $(grep -o '"ms_per_step": [0-9.]*' "$O/driver_$r.json")"
  timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --no-eval > "$O/long_$r.json" 2> "$O/long_$r.err"
  echo "200/20 $r $(grep -o '"ms_per_step": [0-9.]*' "$O/long_$r.json")"
done
(cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$O/p" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 64 --warmup 16 --no-eval --settle-ms 0 > "$O/p.log" 2>&1)
python3 - "$O/p" > "$O/stats.txt" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:14]:
    print(f"{r['Name'][:90]:90s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:9.2f}us")
PY
rm -rf "$O/p"; cat "$O/stats.txt"
timeout -k 10 300 python3 scripts/bench_configs.py masked --steps 96 --warmup 16 > "$O/masked.json" 2> "$O/masked.err"; cat "$O/masked.json"
timeout -k 10 300 python3 scripts/bench_configs.py topk --steps 40 --warmup 10 > "$O/topk.json" 2> "$O/topk.err"; cat "$O/topk.json"
for m in es dp zero1; do
  timeout -k 10 200 python3 bench.py --force-dist --parallelism $m --compare-parallelism 0 --steps 200 --warmup 20 --no-eval > "$O/dist_$m.json" 2> "$O/dist_$m.err"
  echo "dist $m $(grep -o '"ms_per_step": [0-9.]*' "$O/dist_$m.json" | head -1)"
done
# top-k config 4: scores GEMM (EPI_F32, epi 3) and dense bf16 weight gradient (EPI_BF16, epi 4) configs
for spec in "def:" "f13:3:13" "f9:3:9" "b13:4:13" "b9:4:9"; do
  name=${spec%%:*}; cfg=${spec#*:}
  rc=0; SC_GEMM_CFG="$cfg" timeout -k 10 300 python3 scripts/bench_configs.py topk --steps 40 --warmup 10 > "$O/topk_$name.json" 2> "$O/topk_$name.err" || rc=$?
  # (rc 1 = a configuration the library does not instantiate: a host-side error, nothing ran)
  [ $rc -gt 1 ] && { echo "topk $name rc=$rc"; exit 1; }
  echo "topk $name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$O/topk_$name.json")"
done
