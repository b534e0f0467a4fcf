"""Per-step budget from a rocprofv3 kernel trace of bench.py: median time per kernel kind inside a
step, and the idle gaps between consecutive kernels (what the step spends NOT running kernels).

    python scripts/lab/step_budget.py <rocprof dir> [last_n_kernels]
"""
import csv
import glob
import statistics as st
import sys
from collections import defaultdict

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-int(sys.argv[2] if len(sys.argv) > 2 else 1000):]


def kind(name):
    n = name.split("(")[0]
    for key in ("EPI", "sae_gemm_kernel", "step_tail", "gather", "adam", "topk", "decode", "slot", "sparse"):
        if key in name:
            break
    short = n.split("::")[-1][:40]
    if "sae_gemm_kernel" in name:
        # template args carry the epilogue id: sae_gemm_kernel<S, AK, BKM, EPI, BKT, NST[, P32]> with S itself a
        # template (scamd::Shape<WGM, WGN, WI, WJ>): split at top-level commas only
        inside = n[n.find("<") + 1:n.rfind(">")] if "<" in n else ""
        parts, depth, cur = [], 0, ""
        for ch in inside:
            depth += {"<": 1, ">": -1}.get(ch, 0)
            if ch == "," and depth == 0:
                parts.append(cur.strip())
                cur = ""
            else:
                cur += ch
        parts.append(cur.strip())
        shape = parts[0].split("::")[-1].replace(" ", "") if parts else "?"
        short = f"gemm epi={parts[3] if len(parts) > 3 else '?'} {shape} bk{parts[4] if len(parts) > 4 else '?'}" \
                f"x{parts[5] if len(parts) > 5 else '?'}{' p32' if len(parts) > 6 and parts[6] == 'true' else ''}"
    return short


dur = defaultdict(list)
gaps = []
prev_end = None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    dur[kind(r["Kernel_Name"])].append((e - s) / 1e3)
    if prev_end is not None:
        gaps.append((s - prev_end) / 1e3)
    prev_end = e
span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3
busy = sum(sum(v) for v in dur.values())
print(f"{len(rows)} kernels over {span:.1f} us: busy {busy:.1f} us ({100 * busy / span:.1f} %), "
      f"idle {span - busy:.1f} us")
print(f"gaps: median {st.median(gaps):.2f} us, p90 {sorted(gaps)[int(0.9 * len(gaps))]:.2f} us, "
      f"{sum(1 for g in gaps if g > 2)} over 2 us")
for k, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
    print(f"{k:60s} n={len(v):5d} median {st.median(v):8.2f} us  total {sum(v):9.1f} us")
