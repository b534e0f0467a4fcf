#!/bin/bash
# round 5, GPU batch 17: k rotation of the FISTA Gram solver's Gm stream (SC_FISTA_KROT=1), config 5 shapes
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5b17
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
SC_FISTA_KROT=1 step ftest 300 python -u -m pytest tests -m gpu -q -k "fista and not row_tiles" --timeout 200 --timeout-method thread > $O/ftest.log 2>&1
tail -3 $O/ftest.log
for r in 1 2; do
  step base 240 python scripts/bench_configs.py fista --steps 6 --warmup 2 >> $O/base.jsonl
  SC_FISTA_KROT=1 step krot 240 python scripts/bench_configs.py fista --steps 6 --warmup 2 >> $O/krot.jsonl
done
python3 -c "
import json
for f in ('base','krot'):
    print(f, [(json.loads(l)['solve_ms_by_form'], json.loads(l)['ms_per_step']) for l in open('$O/'+f+'.jsonl') if l.startswith('{')])"
