"""Idle gaps between consecutive scamd kernels in a rocprofv3 kernel trace (last N kernels)."""
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "scamd" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
prev, gaps = None, []
for r in rows[-int(sys.argv[2] if len(sys.argv) > 2 else 64):]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if prev is not None:
        gaps.append(((s - prev) / 1000, r["Kernel_Name"].split("(")[0][-28:]))
    prev = e
big = [(round(g, 2), k) for g, k in gaps if g > 1]
print(f"{len(gaps)} gaps, {len(big)} over 1 us: {big}")
