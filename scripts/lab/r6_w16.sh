# 256x256 blocks of SIXTEEN 64x64 waves on BK32 x 3 (cfg 31 = shape 3 | pipe 3 | bit 4), one block / 16
# waves per CU: the weight gradients (epi 3 layout 0) and the top-k bf16 GEMMs
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_w16; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u - > $O/numerics.log 2>&1 <<'PY' || { tail -30 $O/numerics.log; exit 1; }
import sys
sys.path.insert(0, "tests")
import torch
import test_kernels_gpu as T
from sparse_coding__amd.ops import gemm
with gemm.force_shape(31):
    T._sae_epilogues(3, 512, 256, 512)
torch.cuda.synchronize()
print("cfg 31 epilogues ok")
PY
tail -1 $O/numerics.log
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-eval >> $O/def.jsonl 2>> $O/err.log || exit 1
  SC_GEMM_CFG=3/0:31 timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-eval >> $O/w16.jsonl 2>> $O/err.log || exit 1
done
for r in 1 2; do
  for v in "def:" "wg:4/0:31" "sc:4/3:31"; do
    tag=${v%%:*}; e=${v#*:}
    SC_GEMM_CFG=$e timeout -k 10 200 python scripts/bench_configs.py topk --steps 200 --warmup 16 >> $O/tk_$tag.jsonl 2>> $O/err.log || exit 1
  done
done
python3 -c "
import json
for v in ('def','w16','tk_def','tk_wg','tk_sc'): print(v, [json.loads(l)['ms_per_step'] for l in open('$O/'+v+'.jsonl')])"
