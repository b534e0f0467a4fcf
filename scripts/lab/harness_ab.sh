#!/bin/bash
# Driver command (--steps 20 --warmup 5) vs a long run, fresh process each, new vs round-3 harness.
# Usage (on the GPU box): bash scripts/lab/harness_ab.sh OUTDIR
set -e
OUT=${1:-gpurun_out/harness_ab}
mkdir -p "$OUT"
T="timeout -k 10 240"
$T python3 -u scripts/lab/graph_cold_probe.py > "$OUT/probe.jsonl" 2> "$OUT/probe.err"
for i in 1 2 3; do
  $T python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/new_20_5_$i.json" 2> "$OUT/new_20_5_$i.err"
  $T python3 scripts/lab/bench_r3_harness.py --gpus 1 --steps 20 --warmup 5 > "$OUT/old_20_5_$i.json" 2> "$OUT/old_20_5_$i.err"
done
$T python3 bench.py --gpus 1 --steps 200 --warmup 20 --no-eval > "$OUT/new_200_20.json" 2> "$OUT/new_200_20.err"
$T python3 scripts/lab/bench_r3_harness.py --gpus 1 --steps 200 --warmup 20 --no-eval > "$OUT/old_200_20.json" 2> "$OUT/old_200_20.err"
python3 - "$OUT" <<'EOF'
import json, sys, glob, os
out = sys.argv[1]
for f in sorted(glob.glob(os.path.join(out, "*.json"))):
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            print(os.path.basename(f), d["ms_per_step"], d.get("graph_replays"))
EOF
