"""Per-phase budget of a GEMM launch from gemm_phases' per-workgroup stamps (one CSV per kernel:
raw s_memtime ticks at start / first K-tile landed / K loop done / epilogue done, s_memrealtime at
start and end, hw_id, xcc_id).  Reports the medians of each phase, the kernel span,
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
    rt = [(int(r["rt0"]), int(r["rt3"])) for r in rows]
    # s_memtime is a per-XCD shader-clock counter (the XCDs' counters are not synchronised: never
    # compare them across XCDs); s_memrealtime is the chip-wide 100 MHz clock.  Each block's shader
    # clock is its own memtime span over its realtime span; start / end on the realtime axis.
    ghz_b = [(x[3] - x[0]) / ((b - a) * 10.0) if b > a else 0.0 for x, (a, b) in zip(t, rt)]
    good = [g for g in ghz_b if 0.5 < g < 3.5]
    ghz = st.median(good) if good else 2.0
    if not good:
        print("  (no usable block clock; assuming 2.0 GHz)")
    us = lambda ticks: ticks / ghz / 1e3  # noqa: E731
    r_min = min(a for a, _ in rt)
    start = [(a - r_min) / 100.0 for a, _ in rt]
    fill = [us(x[1] - x[0]) for x in t]
    kl = [us(x[2] - x[1]) for x in t]
    ep = [us(x[3] - x[2]) for x in t]
    end = [(b - r_min) / 100.0 for _, b in rt]
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
    print(f"{name:18s} clock {ghz:4.2f} GHz; blocks {len(rows):5d} on {ncu:3d} CUs (per CU {min(per_cu)}-{max(per_cu)}), span {span:6.1f} us; "
          f"median fill {st.median(fill):5.2f} kloop {st.median(kl):6.2f} epi {st.median(ep):5.2f} life {st.median(life):6.2f} us; "
          f"slot fill {100 * eff:5.1f} % at {slots}/CU; tail after first idle CU {span - (first_idle - min(start)):5.1f} us")
    # epilogue sub-phases (wave 0), when the build stamped them (sae_gemm_kernel.h SC_SUB)
    if rows and "e0" in rows[0] and any(int(r["e0"]) for r in rows):
        def med(a, b):
            v = [us(int(r[b]) - int(r[a])) for r in rows if int(r[a]) and int(r[b])]
            return st.median(v) if v else float("nan")
        parts = [("bias+ring barrier", "t2", "e6"), ("relu/put", "e0", "e1"), ("flush stores", "e1", "e2"),
                 ("cmask stores", "e2", "e3"), ("block sum", "e3", "e4"), ("partials", "e4", "e5"),
                 ("to end", "e5", "t3")]
        print("    epilogue sub-phases (median us): " + ", ".join(f"{n} {med(a, b):.2f}" for n, a, b in parts))
