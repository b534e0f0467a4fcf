#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD FAIL; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1; rc=$?
tail -5 gpurun_out/gputests.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|error" gpurun_out/gputests.log | head -20; exit $rc; }
timeout -k 10 300 python scripts/pipe_bench.py > gpurun_out/pipe_bench.jsonl 2> gpurun_out/pipe_bench.err || { tail -20 gpurun_out/pipe_bench.err; exit 1; }
cat gpurun_out/pipe_bench.jsonl
timeout -k 10 400 python scripts/fvu_curve.py --steps 20000 --out gpurun_out/fvu_curve > gpurun_out/fvu_curve.jsonl 2> gpurun_out/fvu_curve.err || { tail -20 gpurun_out/fvu_curve.err; exit 1; }
cat gpurun_out/fvu_curve.jsonl
