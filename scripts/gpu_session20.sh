#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD FAIL; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1; rc=$?
tail -3 gpurun_out/gputests.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/gputests.log | head; exit $rc; }
timeout -k 10 600 python scripts/bench_configs.py fista --steps 10 --warmup 2 --ring-gb 150 > gpurun_out/config5_fista.json 2> gpurun_out/config5.err || { tail -20 gpurun_out/config5.err; exit 1; }
cat gpurun_out/config5_fista.json
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cut -c1-400 gpurun_out/bench.json
