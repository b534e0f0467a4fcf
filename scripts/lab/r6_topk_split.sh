# top-k config 4: scores/select/decode of two model groups on two streams (SC_TOPK_SPLIT=sp) vs one
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_tks; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_graphs_gpu.py -k topk -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
SC_TOPK_SPLIT=4 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_graphs_gpu.py -k topk -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests_split.log 2>&1 || { tail -30 $O/tests_split.log; exit 1; }
tail -1 $O/tests_split.log
for r in 1 2; do
  for sp in 0 4 6 2; do
    SC_TOPK_SPLIT=$sp timeout -k 10 200 python scripts/bench_configs.py topk --steps 200 --warmup 16 >> $O/sp$sp.jsonl 2>> $O/err.log || exit 1
  done
done
python3 -c "
import json
for sp in (0,4,6,2): print(sp, [json.loads(l)['ms_per_step'] for l in open('$O/sp%d.jsonl'%sp)])"
