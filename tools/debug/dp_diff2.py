"""Debug: find elements where fused sa_mask_dp differs from perturb-then-mask."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from sfl_amd import kernels as K, _lib as L
DEV = "cuda:0"
n = 50_003
for trial in range(30):
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
    torch.cuda.synchronize()
    d = (m1 != m2).nonzero().flatten().cpu().tolist()
    if d:
        print("trial", trial, "mismatches", d[:10])
        for j in d[:4]:
            p = xp[j].item() * 3.0 * 2**18
            print(j, "x", x[j].item(), "xp", repr(xp[j].item()), "xp*w*2^18", repr(p), "m1", m1[j].item(), "m2", m2[j].item())
        break
else:
    print("no mismatch in 30 trials")
