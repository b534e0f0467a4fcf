# decoder on 128x128 blocks of EIGHT 64x32 waves (cfg 17 = shape 1 | bit 4 on the BK64 x 2 ring)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_d8; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u - > $O/numerics.log 2>&1 <<'PY' || { tail -30 $O/numerics.log; exit 1; }
import sys
sys.path.insert(0, "tests")
import torch
import test_kernels_gpu as T
from sparse_coding__amd.ops import gemm
# (cfg 17's 64x32 waves break the 64x64-block activity-bitmask layout: decoder epilogue only)
torch.manual_seed(1)
G, B, d, n = 3, 512, 256, 512
c = torch.relu(torch.randn(G, B, n, device="cuda")).to(torch.bfloat16)
wd = torch.nn.functional.normalize(torch.randn(G, n, d, device="cuda"), dim=-1).to(torch.bfloat16)
x = torch.randn(B, d, device="cuda").to(torch.bfloat16)
r0, r1 = torch.empty(G, B, d, device="cuda", dtype=torch.bfloat16), torch.empty(G, B, d, device="cuda", dtype=torch.bfloat16)
p0, p1 = torch.zeros(G, (B // 128) * (d // 128), device="cuda"), torch.zeros(G, (B // 128) * (d // 128), device="cuda")
gemm.decode_residual(c, wd, x, r0, p0)
with gemm.force_shape(17):
    gemm.decode_residual(c, wd, x, r1, p1)
ref = c.float() @ wd.float() - x.float()
torch.cuda.synchronize()
e0 = ((r0.float() - ref).norm() / ref.norm()).item(); e1 = ((r1.float() - ref).norm() / ref.norm()).item()
print("dec rel err default", e0, "cfg17", e1, "part", ((p1.sum(1) - (ref ** 2).sum((1, 2))).abs() / (ref ** 2).sum((1, 2))).max().item())
assert e1 < 1e-2 and ((p1.sum(1) - (ref ** 2).sum((1, 2))).abs() / (ref ** 2).sum((1, 2))).max().item() < 2e-2
print("cfg 17 decoder ok")
PY
tail -1 $O/numerics.log
PB_CFGS=1,17 PB_KERNELS=dec timeout -k 10 120 python scripts/pipe_bench.py > $O/pipe.jsonl 2>> $O/err.log || exit 1
cat $O/pipe.jsonl
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-eval >> $O/def.jsonl 2>> $O/err.log || exit 1
  SC_GEMM_CFG=1:17 timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-eval >> $O/d8.jsonl 2>> $O/err.log || exit 1
done
for r in 1 2; do
  timeout -k 10 200 python scripts/bench_configs.py masked --steps 200 --warmup 16 >> $O/m_def.jsonl 2>> $O/err.log || exit 1
  SC_GEMM_CFG=1:17 timeout -k 10 200 python scripts/bench_configs.py masked --steps 200 --warmup 16 >> $O/m_d8.jsonl 2>> $O/err.log || exit 1
done
python3 -c "
import json
for v in ('def','d8'): print(v, [json.loads(l)['ms_per_step'] for l in open('$O/'+v+'.jsonl')])
for v in ('m_def','m_d8'): print(v, [(json.loads(l)['masked_ms_per_step'], json.loads(l)['unmasked_ms_per_step'], json.loads(l)['time_ratio']) for l in open('$O/'+v+'.jsonl')])"
