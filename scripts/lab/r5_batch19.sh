#!/bin/bash
# round 5, GPU batch 19: config-4 sparse / dense weight-gradient split (the cost model's constants
# predate the bf16 select and the top-k tail) and graph group size
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5b19
mkdir -p $O
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "[batch] $name: $*" >&2
  timeout -k 10 "$t" "$@"
  local rc=$?
  echo "[batch] $name rc=$rc" >&2
  if [ $rc -ne 0 ]; then echo "[batch] stopping after $name (rc=$rc)" >&2; exit $rc; fi
  return 0
}
step build 600 python -c "from sparse_coding__amd.ops import build as b; b.build(force=False)"
for r in 1 2 3; do
  step auto 150 python scripts/bench_configs.py topk --steps 200 --warmup 16 >> $O/auto.jsonl
  step sk32 150 python scripts/bench_configs.py topk --steps 200 --warmup 16 --sparse-k 32 >> $O/sk32.jsonl
  step sk48 150 python scripts/bench_configs.py topk --steps 200 --warmup 16 --sparse-k 48 >> $O/sk48.jsonl
  step gs16 150 python scripts/bench_configs.py topk --steps 192 --warmup 32 --graph-steps 16 >> $O/gs16.jsonl
done
python3 -c "
import json, statistics as st
for f in ('auto','sk32','sk48','gs16'):
    rs = [json.loads(l) for l in open('$O/'+f+'.jsonl') if l.startswith('{')]
    ms = [r['ms_per_step'] for r in rs]
    print(f, ms, 'median', st.median(ms), 'sparse models', rs[0]['sparse_wgrad_models'])"
