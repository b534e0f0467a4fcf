#!/bin/bash
# Round-4 GPU batch 4: the fused code-gradient / encoder-weight-gradient kernel (csrc/sae_dcw.hip):
# its numerics test, then the engine tests that run it (headline gradient, graph replays), a
# same-box A/B of the step with and without it (200/20) and kernel stats of both; kernel traces
# of the driver's 20/5 command and a 200/20 run (per-step timelines); last the graphed-DP
# rehearsal (segfaulted in bench.py before).
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O="$GRAFT_REPO_ROOT/gpurun_out/r4b4"; mkdir -p "$O"
PT="python3 -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 200 $PT tests/test_kernels_gpu.py -k code_grad_wgrad > "$O/t_dcw.log" 2>&1 || { tail -30 "$O/t_dcw.log"; exit 1; }
tail -3 "$O/t_dcw.log"
timeout -k 10 400 $PT tests/test_headline_grad_gpu.py tests/test_graphs_gpu.py tests/test_train_gpu.py > "$O/t_eng.log" 2>&1 || { tail -30 "$O/t_eng.log"; exit 1; }
tail -3 "$O/t_eng.log"
for r in 1 2; do
  for v in 1 0; do
    SC_FUSED_DCW=$v timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --no-eval > "$O/dcw${v}_$r.json" 2> "$O/dcw${v}_$r.err"
    echo "dcw=$v run $r $(grep -o '"ms_per_step": [0-9.]*' "$O/dcw${v}_$r.json")"
  done
done
for v in 1 0; do
  (cd /tmp && SC_FUSED_DCW=$v timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$O/p$v" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 64 --warmup 16 --no-eval > "$O/p$v.log" 2>&1)
  python3 - "$O/p$v" > "$O/stats_dcw$v.txt" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:16]:
    print(f"{r['Name'][:90]:90s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:9.2f}us")
PY
  rm -rf "$O/p$v"; echo "== dcw=$v"; cat "$O/stats_dcw$v.txt"
done
for spec in "d20 --steps 20 --warmup 5" "l200 --steps 200 --warmup 20"; do
  set -- $spec; n=$1; shift
  (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace -d "$O/tr_$n" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" "$@" --no-eval > "$O/tr_$n.json" 2> "$O/tr_$n.err")
  python3 scripts/lab/step_timeline.py "$O/tr_$n" 0 > "$O/tr_$n.windows.jsonl"
  python3 scripts/lab/step_timeline.py "$O/tr_$n" 25 > "$O/tr_$n.last25.jsonl"
  rm -rf "$O/tr_$n"
  echo "trace $n $(grep -o '"ms_per_step": [0-9.]*' "$O/tr_$n.json") $(tail -1 "$O/tr_$n.windows.jsonl")"
done
timeout -k 10 200 python3 -u scripts/lab/dp_graph_repro.py dp engines-first on > "$O/repro_dp.log" 2>&1 || { tail -30 "$O/repro_dp.log"; exit 1; }
tail -4 "$O/repro_dp.log"
