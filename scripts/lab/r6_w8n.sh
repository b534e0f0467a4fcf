# 128x256 blocks of eight 64x64 waves (cfg 10 = shape 2 | pipe 2, lab mapping) vs the 256x128 default (cfg 14)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_w8n; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u - > $O/numerics.log 2>&1 <<'PY' || { tail -30 $O/numerics.log; exit 1; }
import sys
sys.path.insert(0, "tests")
import torch
import test_kernels_gpu as T
from sparse_coding__amd.ops import gemm
with gemm.force_shape(10):
    T._sae_epilogues(3, 512, 256, 512)
torch.cuda.synchronize()
print("cfg 10 epilogues ok")
PY
tail -1 $O/numerics.log
for r in 1 2 3; do
  for v in "def:" "both:0:10,7:10" "enc:0:10"; do
    tag=${v%%:*}; e=${v#*:}
    SC_GEMM_CFG=$e timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-eval >> $O/$tag.jsonl 2>> $O/err.log || exit 1
  done
done
for r in 1 2; do
  for v in "tdef:" "tboth:4/3:10,4/0:10"; do
    tag=${v%%:*}; e=${v#*:}
    SC_GEMM_CFG=$e timeout -k 10 200 python scripts/bench_configs.py topk --steps 200 --warmup 16 >> $O/$tag.jsonl 2>> $O/err.log || exit 1
  done
done
python3 -c "
import json
for v in ('def','both','enc','tdef','tboth'): print(v, [json.loads(l)['ms_per_step'] for l in open('$O/'+v+'.jsonl')])"
