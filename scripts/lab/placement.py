"""Which workgroups of a launch shared a CU (from gemm_phases' per-block hw_id / xcc_id stamps), for
the masked decoder: the logical tile -> model map of the masked grid (xcd_remap, model index fastest),
the models paired on each CU, and each CU's busy time.

    python scripts/lab/placement.py gpurun_out/r5b28/phases/dec_masked.csv [G] [pair]

``pair``: the launch used the masked decoder's block pairing (model g -> G-1-g on every second run of 32
logical tiles, sae_gemm_kernel.h pair_order).
"""
import collections
import csv
import statistics as st
import sys

f = sys.argv[1]
G = int(sys.argv[2]) if len(sys.argv) > 2 else 8
PAIR = len(sys.argv) > 3 and sys.argv[3] == "pair"
rows = list(csv.DictReader(open(f)))
nwg = len(rows)


def xcd_remap(b, n):
    q, r, x = n >> 3, n & 7, b & 7
    base = x * (q + 1) if x < r else r * (q + 1) + (x - r) * q
    return base + (b >> 3)


cu = collections.defaultdict(list)
xcc_ok = 0
r0 = min(int(r["rt0"]) for r in rows)
for r in rows:
    b = int(r["block"])
    hw, xcc = int(r["hw_id"]), int(r["xcc_id"]) & 0xF
    xcc_ok += xcc == (b & 7)
    key = (xcc, (hw >> 13) & 0x7, (hw >> 12) & 0x1, (hw >> 8) & 0xF)  # xcc, se, sh, cu
    s, e = (int(r["rt0"]) - r0) / 100.0, (int(r["rt3"]) - r0) / 100.0
    rem = xcd_remap(b, nwg)
    g = G - 1 - rem % G if PAIR and (rem >> 5) & 1 else rem % G
    cu[key].append((b, g, s, e))
print(f"{nwg} blocks on {len(cu)} CUs; xcc == block % 8 for {xcc_ok}/{nwg}")
pairs = collections.Counter(tuple(sorted(m for _, m, _, _ in v)) for v in cu.values())
print("models per CU (count):", dict(sorted(pairs.items(), key=lambda kv: -kv[1])[:12]))
busy = sorted((max(e for *_, e in v) - min(s for *_, s, _ in v), k, v) for k, v in cu.items())
print(f"CU busy us: min {busy[0][0]:.1f} median {st.median(b for b, *_ in busy):.1f} max {busy[-1][0]:.1f}")
span = max(e for v in cu.values() for *_, e in v)
print(f"kernel span {span:.1f} us")
# the order blocks reach one CU: block ids of the first XCD's CUs
x0 = sorted((k, v) for k, v in cu.items() if k[0] == 0)
for k, v in x0[:8]:
    print(k, [(b, m, round(s, 1), round(e, 1)) for b, m, s, e in sorted(v)])
# within XCD 0: j = block >> 3 -> CU index (order of first appearance)
order = {}
for k, v in x0:
    for b, *_ in v:
        order[b >> 3] = x0.index((k, v))
print("XCD0 j -> CU#:", [order.get(j) for j in range(min(64, nwg // 8))])
