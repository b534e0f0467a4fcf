#!/bin/bash
# DVFS settle: per-step kernel busy time over a long run started from an idle GPU (20-step windows).
set -e
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/settle"; mkdir -p "$O"; export TMPDIR=/tmp
(cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace -d "$O/t" -o run --output-format csv -- python3 "$R/bench.py" --steps 600 --warmup 8 --no-eval > "$O/run.json" 2> "$O/run.err")
python3 "$R/scripts/lab/step_timeline.py" "$O/t" 0 > "$O/windows.jsonl"; rm -rf "$O/t"; cat "$O/windows.jsonl"
