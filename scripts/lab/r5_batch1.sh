#!/bin/bash
# round 5, GPU batch 1: the new multi-rank / launcher tests, the whole GPU suite, bench 20/5 and the
# one-rank in-graph RCCL modes.  Test failures (rc 1) do not stop the batch; anything else does.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5b1
mkdir -p $O
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "[batch] $name: $*" >&2
  timeout -k 10 "$t" "$@"
  local rc=$?
  echo "[batch] $name rc=$rc" >&2
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[batch] stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step newtests 600 python -u -m pytest tests/test_graphed_multirank_gpu.py tests/test_bench_gpu.py -v --timeout 240 --timeout-method thread > $O/new_tests.log 2>&1
tail -15 $O/new_tests.log
step suite 500 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread --deselect tests/test_graphed_multirank_gpu.py --deselect tests/test_bench_gpu.py > $O/suite.log 2>&1
tail -5 $O/suite.log
step bench 150 python bench.py --steps 20 --warmup 5 > $O/bench_20_5.json 2> $O/bench.err
cat $O/bench_20_5.json | head -c 600; echo
for m in es dp zero1; do
  step fd_$m 150 python bench.py --force-dist --parallelism $m --steps 20 --warmup 5 --no-eval > $O/fd_$m.json 2>> $O/bench.err
  python -c "import json;d=json.load(open('$O/fd_$m.json'));print('$m',d['ms_per_step'],d['collectives']['path'][:40],d['collectives']['rccl_ranks'],d['collectives']['consistency'])"
done
