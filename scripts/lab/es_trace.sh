#!/bin/bash
# Kernel + memory-copy trace of ensemble sharding through one RCCL rank (multi-step groups).
set -e
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/es_trace"; mkdir -p "$O"; export TMPDIR=/tmp
(cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace -d "$O/t" -o run --output-format csv -- python3 "$R/bench.py" --steps 96 --warmup 16 --no-eval --force-dist --parallelism es --compare-parallelism 0 > "$O/run.json" 2> "$O/run.err")
python3 - "$O/t" > "$O/summary.txt" <<'PY'
import csv, glob, sys
d = sys.argv[1]
k = [r for r in csv.DictReader(open(glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]))]
m = glob.glob(d + "/**/*memory_copy_trace.csv", recursive=True)
mc = [r for r in csv.DictReader(open(m[0]))] if m else []
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][-40:], r.get("Queue_Id", r.get("Stream_Id", ""))) for r in k]
ev += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "COPY " + r.get("Direction", ""), r.get("Queue_Id", "")) for r in mc]
ev.sort()
last = ev[-260:]
t0 = last[0][0]
prev_end = None
for s, e, n, q in last:
    gap = (s - prev_end) / 1000 if prev_end else 0
    print(f"{(s - t0) / 1000:10.1f} {(e - s) / 1000:8.1f} gap={gap:7.1f} q={q} {n}")
    prev_end = max(prev_end or 0, e)
print("kernels", len(k), "copies", len(mc))
PY
grep -o '"ms_per_step": [0-9.]*' "$O/run.json"; rm -rf "$O/t"; tail -5 "$O/summary.txt"
