import sys, numpy as np, torch
sys.path.insert(0, '.')
from oracle import secagg as o
from sfl_amd.device import PYU, reveal as rv
from sfl_amd.security.aggregation import SecureAggregator
names = ["alice", "bob", "carol", "dave"]
seeds = o.seeds_for(names)
pair = {(a, b): seeds[a][b] for a in names for b in names if a != b}
pyus = [PYU(nm, 0) for nm in names]
for fused, keep in [(False, True), (True, True)]:
    agg = SecureAggregator(PYU("server", 0), pyus, seeds=pair, fused=fused, keep_masked=keep)
    rng = np.random.default_rng(4)
    offset = 0
    for rnd in range(3):
        layers = [(rng.standard_normal((3, 5)) * 0.1).astype(np.float32), rng.standard_normal(7).astype(np.float32)]
        data = [[(l_ + 0.01 * i).astype(np.float32) for l_ in layers] for i in range(len(names))]
        objs = [p(lambda d=d: d)() for p, d in zip(pyus, data)]
        w = [10 * (i + 1) for i in range(len(names))]
        got = rv(agg.average(objs, axis=0, weights=w))
        for li in range(2):
            xs = [d[li] for d in data]
            exp, s, masked = o.secure_average(xs, names, weights=w, seeds=seeds, offset=offset)
            ok = np.array_equal(got[li], exp.reshape(xs[0].shape))
            for c in range(4):
                g = agg.last_masked[li][c].cpu().numpy().view(np.uint64)
                e = masked[c].reshape(-1)
                bad = np.nonzero(g != e)[0]
                print(fused, keep, rnd, li, c, "dec_ok", ok, "bad", bad.tolist(), g[:2], e[:2])
            offset += xs[0].size
