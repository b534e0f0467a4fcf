import csv, glob, json, sys, statistics
order = json.loads([l for l in open(sys.argv[1]) if l.startswith("[")][-1])
f = glob.glob(sys.argv[2] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "sae_gemm" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
i = 0
for o in order:
    ds = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows[i:i + o["n"]]]
    i += o["n"]
    print(json.dumps({"case": o["case"], "dbg": sys.argv[3], "kernel_us_median": round(statistics.median(ds), 2),
                      "min": round(min(ds), 2)}))
