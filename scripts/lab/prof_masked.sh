# rocprofv3 kernel stats of the masked config (masked variant only), top kernels.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O="$GRAFT_REPO_ROOT/gpurun_out/prof_masked"
rm -rf "$O"; mkdir -p "$O"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/scripts/bench_configs.py" masked --variant "${VARIANT:-masked}" > "$O/log.txt" 2>&1) || { tail -20 "$O/log.txt"; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/prof_masked/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:14]:
    print(f"{r['Name'][:100]:100s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:9.2f}us")
PY
