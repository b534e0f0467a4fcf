"""Debug: threshold-activation ramp bits (cmask2) of the persistent vs the tile kernel."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from sparse_coding__amd.ops import gemm

DEV = "cuda"
torch.manual_seed(7)
G, B, d, n = 2, 256, 512, 256
x = ((torch.rand(B, d, device=DEV) * 2 - 1)).to(torch.bfloat16)
w = torch.nn.functional.normalize(torch.randn(G, n, d, device=DEV), dim=-1).to(torch.bfloat16)
gain = torch.randn(G, n, device=DEV) * 0.2
s2 = torch.rand(G, n, device=DEV) * 0.5 + 0.75
l1 = torch.tensor([2e-3, 5e-3], device=DEV)
r = ((torch.rand(G, B, d, device=DEV) * 2 - 1) * 0.3).to(torch.bfloat16)
out = {}
for pers in (True, False):
    with gemm.force_persistent(pers):
        c = torch.empty(G, B, n, device=DEV, dtype=torch.bfloat16)
        part = torch.zeros(G, (B // 128) * (n // 128), 2, device=DEV)
        cmask = torch.zeros(gemm.code_mask_shape(G, B, n), device=DEV, dtype=torch.int64)
        cmask2 = torch.zeros_like(cmask)
        gemm.encode_relu(x, w, gain, c, part, None, None, mask_out=cmask, act=2, ascale=s2, mask2_out=cmask2)
        dpre = torch.empty(G, B, n, device=DEV, dtype=torch.bfloat16)
        colpart = torch.zeros(G, B // 128, n, device=DEV)
        dotpart = torch.zeros(G, B // 128, n, device=DEV)
        gemm.code_grad(r, w, c, l1, dpre, colpart, dotpart=dotpart, mask=cmask, act=2, ascale=s2, mask2=cmask2)
    torch.cuda.synchronize()
    out[pers] = dict(c=c.clone(), cmask=cmask.clone(), cmask2=cmask2.clone(), dpre=dpre.clone(), dot=dotpart.sum(1))
for k in ("c", "cmask", "cmask2", "dpre", "dot"):
    a, b = out[True][k], out[False][k]
    print(k, "equal" if torch.equal(a, b) else f"DIFF maxabs={float((a.float()-b.float()).abs().max())} nbits_a={int(a.ne(0).sum()) if a.dtype==torch.int64 else '-'} nbits_b={int(b.ne(0).sum()) if b.dtype==torch.int64 else '-'}")
pre = x.float() @ w.float().transpose(1, 2) + gain[:, None, :]
u = pre / s2[:, None, :]
cref = (torch.clamp(10 * (u - 0.9), 0, 1) + torch.relu(u - 1)) * s2[:, None, :]
on = cref > 0
ramp = on & (u < 1)
print("ref on", int(on.sum()), "ref ramp", int(ramp.sum()))
for pers in (True, False):
    m2 = out[pers]["cmask2"]
    pc = sum(bin(int(v) & (2**64 - 1)).count("1") for v in m2.flatten().tolist())
    m1 = out[pers]["cmask"]
    pc1 = sum(bin(int(v) & (2**64 - 1)).count("1") for v in m1.flatten().tolist())
    print("persistent" if pers else "tile", "on bits", pc1, "ramp bits", pc)
gdc = r.float() @ w.float().transpose(1, 2) + (l1 * d / 2)[:, None, None]
print("ref dot col0..8", (-9.0 * gdc * ramp).sum(1)[0, :8].tolist())
for pers in (True, False):
    print("persistent" if pers else "tile", out[pers]["dot"][0, :8].tolist())
