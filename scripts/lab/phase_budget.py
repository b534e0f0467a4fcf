"""Per-phase budget of a GEMM launch from gemm_phases' per-workgroup stamps (one CSV per kernel:
start / fill / kloop / epi in us, hw_id, xcc_id).  Reports the medians of each phase, the kernel span,
how full the co-resident slots were (sum of workgroup lifetimes / (span x slots)) and the tail: the
time from the first CU going idle for good to the last workgroup's end.

    python scripts/lab/phase_budget.py gpurun_out/r5b3/phases [slots_per_cu]
"""
import csv
import glob
import os
import statistics as st
import sys

d = sys.argv[1]
for f in sorted(glob.glob(os.path.join(d, "*.csv"))):
    rows = list(csv.DictReader(open(f)))
    if not rows:
        continue
    t = [[int(r[k]) for k in ("t0", "t1", "t2", "t3")] for r in rows]
    # shader clock from s_memtime vs s_memrealtime (100 MHz) over the launch; 2.0 GHz if unusable
    r0, r1 = min(int(r["rt0"]) for r in rows), max(int(r["rt3"]) for r in rows)
    m0, m1 = min(x[0] for x in t), max(x[3] for x in t)
    ghz = (m1 - m0) / ((r1 - r0) * 10.0) if r1 > r0 else 0.0
    if not 0.5 < ghz < 3.5:
        print(f"  (clock from stamps {ghz:.3g} GHz unusable; assuming 2.0)")
        ghz = 2.0
    us = lambda ticks: ticks / ghz / 1e3  # noqa: E731
    start = [us(x[0] - m0) for x in t]
    fill = [us(x[1] - x[0]) for x in t]
    kl = [us(x[2] - x[1]) for x in t]
    ep = [us(x[3] - x[2]) for x in t]
    end = [s + a + b + c for s, a, b, c in zip(start, fill, kl, ep)]
    life = [e - s for s, e in zip(start, end)]
    span = max(end) - min(start)
    # CU identity: HW_ID (SE, SH, CU fields) + XCC
    cu = {}
    for r, s, e in zip(rows, start, end):
        hw = int(r["hw_id"])
        key = (int(r["xcc_id"]) & 0xF, (hw >> 8) & 0xF, (hw >> 13) & 0x7, (hw >> 12) & 0x1)
        cu.setdefault(key, []).append((s, e))
    ncu = len(cu)
    last_end = {k: max(e for _, e in v) for k, v in cu.items()}
    first_idle = min(last_end.values())
    per_cu = [len(v) for v in cu.values()]
    slots = int(sys.argv[2]) if len(sys.argv) > 2 else max(1, round(sum(life) / span / ncu + 0.5))
    eff = sum(life) / (span * ncu * slots)
    name = os.path.basename(f)[:-4]
    print(f"{name:18s} blocks {len(rows):5d} on {ncu:3d} CUs (per CU {min(per_cu)}-{max(per_cu)}), span {span:6.1f} us; "
          f"median fill {st.median(fill):5.2f} kloop {st.median(kl):6.2f} epi {st.median(ep):5.2f} life {st.median(life):6.2f} us; "
          f"slot fill {100 * eff:5.1f} % at {slots}/CU; tail after first idle CU {span - (first_idle - min(start)):5.1f} us")
