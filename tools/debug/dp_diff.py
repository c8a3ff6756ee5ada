"""Debug: where fused sa_mask_dp differs from perturb-then-mask (GPU)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from sfl_amd import kernels as K, _lib as L
DEV = "cuda:0"
n = 50_003
torch.manual_seed(0)
x = torch.randn(n, device=DEV) * 0.05
out = torch.zeros(1, dtype=torch.float64, device=DEV)
part = torch.empty(L.SA_DP_PARTIALS, dtype=torch.float64, device=DEV)
s = K.sumsq_f32(x, out, part)
mk = lambda: K.make_dp(s, l2_norm_clip=0.3, noise_std=0.01, num_updates=8, key=77, counter0=40)
xp = K.dp_perturb(x, torch.empty_like(x), mk())
m1 = torch.empty(n, dtype=torch.int64, device=DEV)
K.mask(xp, m1, [], weight=3.0)
m2 = torch.empty(n, dtype=torch.int64, device=DEV)
K.mask_dp(x, m2, [], mk(), weight=3.0)
m3 = torch.empty(n, dtype=torch.int64, device=DEV)
K.mask(x, m3, [], weight=3.0)
torch.cuda.synchronize()
d = (m1 != m2).nonzero().flatten().cpu()
print("mismatches", d.numel(), d[:20].tolist())
q = (xp.double() * 3 * 2**18).trunc().long()
print("m1==trunc(xp*w*2^18):", torch.equal(m1.cpu(), q.cpu()), "m3 vs x quant:", torch.equal(m3.cpu(), (x.double()*3*2**18).trunc().long().cpu()))
for j in d[:5].tolist():
    print(j, x[j].item(), xp[j].item(), m1[j].item(), m2[j].item(), m3[j].item())
d1 = torch.zeros(1, dtype=torch.int64, device=DEV)
d2 = torch.zeros(1, dtype=torch.int64, device=DEV)
K.mask(xp, m1, [], weight=3.0, digest=d1)
K.mask_dp(x, m2, [], mk(), weight=3.0, digest=d2)
torch.cuda.synchronize()
import numpy as np
dm1 = np.bitwise_xor.reduce(m1.cpu().numpy().view(np.uint64))
dm2 = np.bitwise_xor.reduce(m2.cpu().numpy().view(np.uint64))
print("digests", hex(d1.item() & (2**64-1)), hex(d2.item() & (2**64-1)), "host xor", hex(int(dm1)), hex(int(dm2)), "m eq", torch.equal(m1, m2))
