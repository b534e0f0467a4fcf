cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT
rm -rf gpurun_out/ptk
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ptk -o run --output-format csv -- python3 $R/scripts/bench_configs.py topk --steps 20 --warmup 3 > $R/gpurun_out/ptk.log 2>&1) || { tail -5 gpurun_out/ptk.log; exit 1; }
tail -1 gpurun_out/ptk.log
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/ptk/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:14]:
    print(f"{r['Name'][:100]:100s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:9.2f}us {float(r['Percentage']):6.2f}%")
PY
