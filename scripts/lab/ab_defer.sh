set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab_defer
timeout -k 10 300 python -u -m pytest tests/test_graphs_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "deferred" > gpurun_out/ab_defer/test.log 2>&1 || { tail -30 gpurun_out/ab_defer/test.log; exit 1; }
tail -3 gpurun_out/ab_defer/test.log
for r in 1 2 3; do
  for v in 0 1; do
    timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-eval --defer-decoder-adam $v >> gpurun_out/ab_defer/v$v.jsonl 2>> gpurun_out/ab_defer/err.log || { tail -20 gpurun_out/ab_defer/err.log; exit 1; }
  done
done
for v in 0 1; do timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-eval --defer-decoder-adam $v >> gpurun_out/ab_defer/drv$v.jsonl 2>> gpurun_out/ab_defer/err.log || exit 1; done
python3 - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/ab_defer/*.jsonl")):
    print(f, [json.loads(l)["ms_per_step"] for l in open(f)])
PY
