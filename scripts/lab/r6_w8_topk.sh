# top-k config 4: the eight-wave 256x128 BK32 x 3 block (cfg 14) for the scores GEMM (epi 4 layout 3)
# and / or the dense weight gradient (epi 4 layout 0)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_w8t; rm -rf $O; mkdir -p $O
SC_GEMM_CFG=4/3:14,4/0:14 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k topk -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in "def:" "sc:4/3:14" "wg:4/0:14" "both:4/3:14,4/0:14"; do
    tag=${v%%:*}; e=${v#*:}
    SC_GEMM_CFG=$e timeout -k 10 200 python scripts/bench_configs.py topk --steps 200 --warmup 16 >> $O/$tag.jsonl 2>> $O/err.log || exit 1
  done
done
python3 -c "
import json
for v in ('def','sc','wg','both'): print(v, [json.loads(l)['ms_per_step'] for l in open('$O/'+v+'.jsonl')])"
# masked config with the masked fallback in place (both variants in one process)
for r in 1 2; do
  timeout -k 10 200 python scripts/bench_configs.py masked --steps 200 --warmup 16 >> $O/masked.jsonl 2>> $O/err.log || exit 1
done
python3 -c "
import json
print('masked', [(json.loads(l)['masked_ms_per_step'], json.loads(l)['unmasked_ms_per_step'], json.loads(l)['time_ratio']) for l in open('$O/masked.jsonl')])"
