#!/bin/bash
set -e
mkdir -p gpurun_out/svi
R=$GRAFT_REPO_ROOT
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace -d $R/gpurun_out/svi/prof -o run --output-format csv -- python3 $R/scripts/dbg/step_vs_iso.py > $R/gpurun_out/svi/log 2>&1)
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/svi/prof/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
out = []
for r in rows[-400:]:
    out.append(f"{r['Kernel_Name'][:70]:70s} {(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3:8.2f}")
open("gpurun_out/svi/tail.txt", "w").write("\n".join(out))
PY
