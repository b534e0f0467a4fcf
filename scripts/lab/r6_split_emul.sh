set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r6_split; rm -rf $O; mkdir -p $O
for v in "a:512,804,1097,1389,1682,1974,2267,2560" "b:512,804,1097,1389,841,841,987,987,1134,1134,1280,1280" "c:512,804,1097,1389,841,987,1134,1280"; do
  tag=${v%%:*}; s=${v#*:}
  (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/$tag -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/lab/masked_split_emul.py $s > $O/$tag.log 2>&1) || { tail -20 $O/$tag.log; exit 1; }
  python3 - $O/$tag <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "sae_gemm" in r["Name"] or "step_tail" in r["Name"]:
        print(sys.argv[1].split("/")[-1], r["Name"][:110], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2))
PY
done
