#!/bin/bash
# round 5, GPU batch 51: top-k scores GEMM on the pipelined 256x128 blocks (SC_GEMM_CFG=4/3:2) vs the
# automatic 256x256 (and 128x128 BK64 x 2, 4/3:1); config 4, 3 alternating runs each
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5b51
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
  step auto 150 env SC_GEMM_CFG= python scripts/bench_configs.py topk --steps 200 --warmup 16 >> $O/auto.jsonl
  step s2 150 env SC_GEMM_CFG=4/3:2 python scripts/bench_configs.py topk --steps 200 --warmup 16 >> $O/s2.jsonl
  step s1 150 env SC_GEMM_CFG=4/3:1 python scripts/bench_configs.py topk --steps 200 --warmup 16 >> $O/s1.jsonl
done
python3 -c "
import json
for f in ('auto', 's2', 's1'):
    rs = [json.loads(l) for l in open('$O/%s.jsonl' % f) if l.startswith('{')]
    print(f, [r['ms_per_step'] for r in rs])"
