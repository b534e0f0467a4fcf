#!/bin/bash
# round 5, GPU batch 29: masked decoder block pairing (g with G-1-g on one CU): placement probe,
# masked tests, masked-config A/B (SC_PAIR_K=1 default vs 0)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5b29
mkdir -p $O/phases
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
step phases 120 scripts/lab/gemm_phases_masked $O/phases > $O/phases.jsonl
grep dec_ $O/phases.jsonl
python3 scripts/lab/placement.py $O/phases/dec_masked.csv > $O/placement.txt 2>&1
head -4 $O/placement.txt
step masked_test 300 python -u -m pytest tests/test_masked_gpu.py -q --timeout 120 --timeout-method thread > $O/masked_test.log 2>&1
tail -2 $O/masked_test.log
for r in 1 2 3; do
  SC_PAIR_K=1 step pair 200 python scripts/bench_configs.py masked --steps 200 --warmup 16 >> $O/pair.jsonl
  SC_PAIR_K=0 step nopair 200 python scripts/bench_configs.py masked --steps 200 --warmup 16 >> $O/nopair.jsonl
done
python3 -c "
import json
for f in ('pair','nopair'):
    rs = [json.loads(l) for l in open('$O/'+f+'.jsonl') if l.startswith('{')]
    print(f, [(r['masked_ms_per_step'], r['unmasked_ms_per_step'], r['time_ratio']) for r in rs])"
