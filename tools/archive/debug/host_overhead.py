"""Host cost per sa_fused_clients call through the Python wrapper (tiny n, so
the GPU time is negligible): the pipelined multi-GPU step makes 8 calls."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from bench import pair_seed
from sfl_amd import _lib, kernels as K
from sfl_amd.parallel_sum import plan_generators, plan_rank
_lib.lib()
dev = torch.device("cuda", 0)
for W in (1, 8):
    names = [f"client{c}" for c in range(8)]
    plan = plan_rank(names, W, 0)
    n = 4096
    xs = [torch.randn(n, device=dev) for _ in plan.clients]
    pg, ps, cross = plan_generators(plan, pair_seed)
    s = torch.empty(n, dtype=torch.int64, device=dev)
    dig = torch.zeros(len(plan.clients), dtype=torch.int64, device=dev)
    for _ in range(20):
        K.fused_clients(xs, [1.0] * len(xs), pg, ps, cross, plan.n_cross, s, digests=dig)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(200):
        K.fused_clients([x[0:n] for x in xs], [1.0] * len(xs), pg, ps, cross, plan.n_cross, s[0:n], digests=dig)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"W={W}: host {1e6 * (t1 - t0) / 200:.1f} us/call (to sync {1e6 * (t2 - t0) / 200:.1f})")
