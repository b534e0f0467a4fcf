# with the fp32 weight-gradient default on cfg 14: the other engines that use it
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_wg14b; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_headline_grad_gpu.py tests/test_masked_gpu.py tests/test_unrolled_gpu.py tests/test_graphs_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for m in "" "--residual"; do
    timeout -k 10 200 python scripts/unrolled_bench.py --only-unrolled $m >> $O/new_u.jsonl 2>> $O/err.log || exit 1
    SC_GEMM_CFG=3/0:0 timeout -k 10 200 python scripts/unrolled_bench.py --only-unrolled $m >> $O/old_u.jsonl 2>> $O/err.log || exit 1
  done
  timeout -k 10 200 python scripts/bench_configs.py masked --steps 200 --warmup 16 >> $O/new_m.jsonl 2>> $O/err.log || exit 1
  SC_GEMM_CFG=3/0:0 timeout -k 10 200 python scripts/bench_configs.py masked --steps 200 --warmup 16 >> $O/old_m.jsonl 2>> $O/err.log || exit 1
done
cat $O/new_u.jsonl; echo; cat $O/old_u.jsonl
python3 -c "
import json
for v in ('new_m','old_m'): print(v, [(json.loads(l)['masked_ms_per_step'], json.loads(l)['unmasked_ms_per_step']) for l in open('$O/'+v+'.jsonl')])"
