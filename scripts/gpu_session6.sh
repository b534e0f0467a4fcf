#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD FAIL; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1; rc=$?
tail -4 gpurun_out/gputests.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/gputests.log | head; exit $rc; }
timeout -k 10 300 python scripts/topk_bench.py > gpurun_out/topk_bench.jsonl 2> gpurun_out/topk_bench.err || { tail -20 gpurun_out/topk_bench.err; exit 1; }
cat gpurun_out/topk_bench.jsonl
timeout -k 10 300 python scripts/bench_configs.py topk --steps 50 --warmup 5 > gpurun_out/config4_topk.json 2> gpurun_out/config4.err || { tail -20 gpurun_out/config4.err; exit 1; }
cat gpurun_out/config4_topk.json
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
timeout -k 10 300 python scripts/es_projection.py > gpurun_out/es_projection.jsonl 2> gpurun_out/es_projection.err || { tail -20 gpurun_out/es_projection.err; exit 1; }
cat gpurun_out/es_projection.jsonl
