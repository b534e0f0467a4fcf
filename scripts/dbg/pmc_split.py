import csv, glob, json, sys, statistics, collections
order = json.loads([l for l in open(sys.argv[1]) if l.startswith("[")][-1])
f = glob.glob(sys.argv[2] + "/**/*counter_collection.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "sae_gemm" in r["Kernel_Name"]]
by = collections.defaultdict(dict)
for r in rows:
    by[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
ids = sorted(by)
i = 0
for o in order:
    ds = ids[i:i + o["n"]]
    i += o["n"]
    agg = {k: statistics.median(by[d][k] for d in ds if k in by[d]) for k in by[ds[0]]}
    print(json.dumps({"case": o["case"], **{k: round(v, 1) for k, v in agg.items()}}))
