#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD FAIL; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "topk" > gpurun_out/gputests_topk.log 2>&1; rc=$?
tail -6 gpurun_out/gputests_topk.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/topk_bench.py > gpurun_out/topk_bench.jsonl 2> gpurun_out/topk_bench.err || { tail -20 gpurun_out/topk_bench.err; exit 1; }
cat gpurun_out/topk_bench.jsonl
timeout -k 10 300 python scripts/bench_configs.py topk --steps 50 --warmup 5 > gpurun_out/config4_topk.json 2> gpurun_out/config4.err || { tail -20 gpurun_out/config4.err; exit 1; }
cat gpurun_out/config4_topk.json
