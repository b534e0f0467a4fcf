"""Replicates tests/test_gemm_persistent_gpu.py::test_activation_epilogues[act=2] and
localises the elements whose ramp/on bits disagree with the fp32 reference."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from sparse_coding__amd.ops import gemm

DEV = "cuda"
def _bf(*shape, scale=1.0):
    return (torch.randn(*shape, device=DEV) * scale).to(torch.bfloat16)

def bits(m, G, B, n):
    # [G][B/16][n/16][4] uint64, bit l of word r: row 16i + (l&15), col 16j + 4(l>>4) + r
    m = m.view(G, B // 16, n // 16, 4).cpu()
    out = torch.zeros(G, B, n, dtype=torch.bool)
    for l in range(64):
        b = ((m >> l) & 1).bool()  # [G, B/16, n/16, 4]
        for r in range(4):
            out[:, (l & 15)::16, (4 * (l >> 4) + r)::16] = b[..., r]
    return out

for pers, grid in ((True, 0), (True, 2), (False, 0)):
    torch.manual_seed(7)
    G, B, d, n = 2, 256, 512, 256
    x = _bf(B, d)
    w = torch.nn.functional.normalize(torch.randn(G, n, d, device=DEV), dim=-1).to(torch.bfloat16)
    gain = torch.randn(G, n, device=DEV) * 0.2
    s2 = torch.rand(G, n, device=DEV) * 0.5 + 0.75
    l1 = torch.tensor([2e-3, 5e-3], device=DEV)
    with gemm.force_persistent(pers, max_blocks=grid):
        c = torch.empty(G, B, n, device=DEV, dtype=torch.bfloat16)
        part = torch.zeros(G, (B // 128) * (n // 128), 2, device=DEV)
        cmask = torch.zeros(gemm.code_mask_shape(G, B, n), device=DEV, dtype=torch.int64)
        cmask2 = torch.zeros_like(cmask)
        gemm.encode_relu(x, w, gain, c, part, None, None, mask_out=cmask, act=2, ascale=s2, mask2_out=cmask2)
        r = _bf(G, B, d, scale=0.3)
        dpre = torch.empty(G, B, n, device=DEV, dtype=torch.bfloat16)
        colpart = torch.zeros(G, B // 128, n, device=DEV)
        dotpart = torch.zeros(G, B // 128, n, device=DEV)
        gemm.code_grad(r, w, c, l1, dpre, colpart, dotpart=dotpart, mask=cmask, act=2, ascale=s2, mask2=cmask2)
    torch.cuda.synchronize()
    pre = x.float() @ w.float().transpose(1, 2) + gain[:, None, :]
    u = pre / s2[:, None, :]
    on = ((torch.clamp(10 * (u - 0.9), 0, 1) + torch.relu(u - 1)) * s2[:, None, :]) > 0
    ramp = on & (u < 1)
    kon, kramp = bits(cmask, G, B, n), bits(cmask2, G, B, n)
    don = (kon != on.cpu()); dr = (kramp != ramp.cpu())
    print("persistent" if pers else "tile", "grid", grid, "on mismatches", int(don.sum()), "ramp mismatches", int(dr.sum()))
    idx = dr.nonzero()[:8]
    for g_, b_, j_ in idx.tolist():
        print("   ", (g_, b_, j_), "u", float(u[g_, b_, j_]), "k_on", bool(kon[g_, b_, j_]), "k_ramp", bool(kramp[g_, b_, j_]),
              "c", float(c[g_, b_, j_]))
    gdc = r.float() @ w.float().transpose(1, 2) + (l1 * d / 2)[:, None, None]
    ref = (-9.0 * gdc * ramp).sum(1)
    print("    max |dot - ref|", float((dotpart.sum(1) - ref).abs().max()))
