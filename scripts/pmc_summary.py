"""Summarise rocprofv3 --pmc counter CSVs: mean counter value per (kernel, counter).

  python scripts/pmc_summary.py gpurun_out/pmc > profiles/pmc_step_kernels_r1.md
"""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
vals = collections.defaultdict(list)
meta = {}
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "?")
        short = name.split("(")[0].replace("void ", "").replace("scamd::", "")
        if any(t in name for t in ("sae_gemm_kernel", "adam", "topk", "bias_loss", "step_tail", "fista")):
            key = name[:160] + (f" grid={r.get('Grid_Size')}" if "rowblock" in name else "")
            vals[(key, r["Counter_Name"])].append(float(r["Counter_Value"]))
            meta[key] = (r.get("VGPR_Count"), r.get("Accum_VGPR_Count"), r.get("LDS_Block_Size"), r.get("Grid_Size"),
                         r.get("Workgroup_Size"))
kernels = sorted({k for k, _ in vals})
counters = sorted({c for _, c in vals})
print("| kernel | vgpr/agpr | lds | grid/wg | " + " | ".join(counters) + " |")
print("|---|---|---|---|" + "---|" * len(counters))
for k in kernels:
    m = meta[k]
    row = [f"{sum(vals[(k, c)]) / len(vals[(k, c)]):.4g}" if (k, c) in vals else "" for c in counters]
    print(f"| `{k}` | {m[0]}/{m[1]} | {m[2]} | {m[3]}/{m[4]} | " + " | ".join(row) + " |")
