# cfg 14 (eight-wave 256x128, BK32 x 3) as the encoder / masked code-gradient default: tests + step A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_w8b; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_headline_grad_gpu.py tests/test_masked_gpu.py tests/test_graphs_gpu.py tests/test_sim_comm_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do
  for v in "new:" "old:0:29,7:29" "cnt:6:14" "dec:1:14"; do
    tag=${v%%:*}; e=${v#*:}
    SC_GEMM_CFG=$e timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-eval >> $O/$tag.jsonl 2>> $O/err.log || exit 1
  done
done
for r in 1 2; do
  timeout -k 10 200 python scripts/bench_configs.py masked --steps 200 --warmup 16 >> $O/m_new.jsonl 2>> $O/err.log || exit 1
  SC_GEMM_CFG=0:29,7:29 timeout -k 10 200 python scripts/bench_configs.py masked --steps 200 --warmup 16 >> $O/m_old.jsonl 2>> $O/err.log || exit 1
done
python3 -c "
import json
for v in ('new','old','cnt','dec'): print(v, [json.loads(l)['ms_per_step'] for l in open('$O/'+v+'.jsonl')])
for v in ('m_new','m_old'): print(v, [(json.loads(l)['masked_ms_per_step'], json.loads(l)['unmasked_ms_per_step'], json.loads(l)['time_ratio']) for l in open('$O/'+v+'.jsonl')])"
