#!/bin/bash
# Kernel traces of the driver's short bench (20/5) under the new and the round-3 harness and of a
# long run; per-step timelines of each run's last 20 steps.  Then ensemble sharding through one RCCL rank.
set -e
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/timeline_ab"
mkdir -p "$O"
T="timeout -k 10 240"
export TMPDIR=/tmp
prof() {  # name, args...
  local n=$1; shift
  (cd /tmp && $T rocprofv3 --kernel-trace -d "$O/$n" -o run --output-format csv -- python3 "$@" > "$O/$n.json" 2> "$O/$n.err")
  python3 "$R/scripts/lab/step_timeline.py" "$O/$n" 20 > "$O/$n.timeline.jsonl"
  rm -rf "$O/$n"
  echo "$n $(tail -1 $O/$n.timeline.jsonl) $(grep -o '"ms_per_step": [0-9.]*' $O/$n.json | head -1)"
}
prof new20 "$R/bench.py" --steps 20 --warmup 5 --no-eval
prof old20 "$R/scripts/lab/bench_r3_harness.py" --steps 20 --warmup 5 --no-eval
prof new200 "$R/bench.py" --steps 200 --warmup 20 --no-eval
cd "$R"
$T python3 bench.py --steps 200 --warmup 20 --no-eval --force-dist --parallelism es --compare-parallelism 0 > $O/es1_200.json 2> $O/es1_200.err
$T python3 bench.py --steps 20 --warmup 5 --no-eval --force-dist --parallelism es --compare-parallelism 0 > $O/es1_20.json 2> $O/es1_20.err
$T python3 bench.py --steps 20 --warmup 5 --no-eval > $O/plain_20.json 2> $O/plain_20.err
for r in es1_200 es1_20 plain_20; do echo "$r $(grep -o '"ms_per_step": [0-9.]*' $O/$r.json | head -1)"; done
