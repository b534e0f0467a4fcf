# 256x128 blocks of EIGHT 64x64 waves on the BK32 x 3 ring, two blocks per CU (cfg 14 = shape 2 | pipe 3)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_w8; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u - > $O/numerics.log 2>&1 <<'PY' || { tail -30 $O/numerics.log; exit 1; }
import sys
sys.path.insert(0, "tests")
import torch
import test_kernels_gpu as T
from sparse_coding__amd.ops import gemm
with gemm.force_shape(14):
    T._sae_epilogues(3, 512, 256, 512)
torch.cuda.synchronize()
print("cfg 14 epilogues ok")
PY
cat $O/numerics.log | tail -2
PB_CFGS=29,14 PB_KERNELS=enc,dc timeout -k 10 120 python scripts/pipe_bench.py > $O/pipe.jsonl 2>> $O/err.log || exit 1
cat $O/pipe.jsonl
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-eval >> $O/def.jsonl 2>> $O/err.log || exit 1
  SC_GEMM_CFG=0:14,7:14 timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-eval >> $O/w8.jsonl 2>> $O/err.log || exit 1
  SC_GEMM_CFG=0:14 timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-eval >> $O/w8enc.jsonl 2>> $O/err.log || exit 1
done
python3 -c "
import json
for v in ('def','w8','w8enc'): print(v, [json.loads(l)['ms_per_step'] for l in open('$O/'+v+'.jsonl')])"
