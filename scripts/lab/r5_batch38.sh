#!/bin/bash
# round 5, GPU batch 38: one-barrier final reductions in the encoder / decoder epilogues and the masked
# code gradient's activity words fetched before the K loop -- tests, then same-box A/B against the
# previous commit's tree (_abtree, built in-tree beforehand)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5b38
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
step tests 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_headline_grad_gpu.py tests/test_masked_gpu.py -x -q \
  --timeout 120 --timeout-method thread -k "epilogue or layouts or headline or masked or code_grad or decode or encode" > $O/tests.log 2>&1
tail -2 $O/tests.log
for r in 1 2 3 4; do
  step new 120 python bench.py --steps 20 --warmup 5 --no-eval >> $O/new.jsonl
  (cd $R/_abtree && step old 120 python bench.py --steps 20 --warmup 5 --no-eval >> $O/old.jsonl) || exit 1
done
step mk_new 200 python scripts/bench_configs.py masked --steps 200 --warmup 16 >> $O/mk_new.jsonl
(cd $R/_abtree && step mk_old 200 python scripts/bench_configs.py masked --steps 200 --warmup 16 >> $O/mk_old.jsonl) || exit 1
python3 -c "
import json, statistics as st
for f in ('new','old'):
    rs = [json.loads(l) for l in open('$O/'+f+'.jsonl') if l.startswith('{')]
    ms = [r['ms_per_step'] for r in rs]
    print(f, ms, 'median', st.median(ms))
for f in ('mk_new','mk_old'):
    rs = [json.loads(l) for l in open('$O/'+f+'.jsonl') if l.startswith('{')]
    print(f, [(r['masked_ms_per_step'], r['unmasked_ms_per_step'], r['time_ratio']) for r in rs])"
