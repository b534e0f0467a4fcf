"""Per-step timeline of the last N training steps in a rocprofv3 kernel trace.

A step starts at its encoder GEMM.  Prints per step: wall from its gather to the next
step's gather, busy time (sum of kernel durations), idle gaps, and per-kernel durations, so a
short timed region (--steps 20) can be compared with the steady state kernel by kernel.
Usage: python step_timeline.py TRACE_DIR [N_STEPS]   (N_STEPS 0: every step; also prints the busy time
averaged over consecutive windows of 20 steps, with the window's start time in ms)
"""
import collections
import csv
import glob
import json
import sys


def short(name):
    n = name.split("(")[0]
    if "sae_gemm_kernel" in n:
        return "gemm" + name[name.index("Shape"):].split(">")[0][5:] + "," + name.split(">,")[1].split(">")[0]
    return n.split("::")[-1][-30:]


def _epi(name):
    if "sae_gemm_kernel" not in name or "Shape<" not in name:
        return None
    try:
        return int(name.split("Shape<")[1].split(">, ")[1].split(",")[2])
    except (IndexError, ValueError):
        return None


def main():
    f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
    nsteps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    rows = [r for r in csv.DictReader(open(f)) if "scamd" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # a step starts at its encoder GEMM (EPI_ENC 0 / EPI_ENC_CNT 6); the batch gather of a graph's
    # first step (the others run inside the previous step's fused tail) counts to the step before
    starts = [i for i, r in enumerate(rows) if _epi(r["Kernel_Name"]) in (0, 6)]
    sel = starts[-nsteps:] if nsteps > 0 else starts
    out = []
    for k, i0 in enumerate(sel):
        i1 = sel[k + 1] if k + 1 < len(sel) else len(rows)
        seg = rows[i0:i1]
        t0 = int(seg[0]["Start_Timestamp"])
        t1 = int(rows[i1]["Start_Timestamp"]) if i1 < len(rows) else int(seg[-1]["End_Timestamp"])
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg)
        kern = collections.OrderedDict()
        for r in seg:
            kern[short(r["Kernel_Name"])] = round((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000, 1)
        out.append({"step": k, "wall_us": round((t1 - t0) / 1000, 1), "busy_us": round(busy / 1000, 1),
                    "kernels": kern})
    if nsteps > 0:
        for o in out:
            print(json.dumps(o))
    else:
        t_first = int(rows[sel[0]]["Start_Timestamp"])
        for w in range(0, len(out), 20):
            win = out[w:w + 20]
            t = (int(rows[sel[w]]["Start_Timestamp"]) - t_first) / 1e6
            print(json.dumps({"from_step": w, "t_ms": round(t, 2), "busy_us": round(sum(o["busy_us"] for o in win) / len(win), 1),
                              "wall_us": round(sum(o["wall_us"] for o in win) / len(win), 1)}))
    walls = [o["wall_us"] for o in out[:-1]]
    print(json.dumps({"mean_wall_us": round(sum(walls) / max(1, len(walls)), 1),
                      "mean_busy_us": round(sum(o["busy_us"] for o in out) / len(out), 1)}))


if __name__ == "__main__":
    main()
