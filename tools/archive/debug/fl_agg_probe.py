"""Which SecureAggregator path the FL round (config 4) takes, and where its
aggregation time goes (cProfile of the aggregate calls)."""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import numpy as np
    import torch

    import test_fl_round as T
    from oracle import secagg as o
    from sfl_amd.device import PYU
    from sfl_amd.ml.fl import FLModel, TorchModel, optim_wrapper
    from sfl_amd.security.aggregation import SecureAggregator

    calls = {"fast": 0, "all": 0}
    fast, agg_fn = SecureAggregator._aggregate_host_fused, SecureAggregator._aggregate
    prof = cProfile.Profile()
    times = []

    def fast_wrap(self, *a, **k):
        calls["fast"] += 1
        return fast(self, *a, **k)

    def agg_wrap(self, *a, **k):
        calls["all"] += 1
        t0 = time.perf_counter()
        prof.enable()
        r = agg_fn(self, *a, **k)
        prof.disable()
        times.append(time.perf_counter() - t0)
        return r

    SecureAggregator._aggregate_host_fused = fast_wrap
    SecureAggregator._aggregate = agg_wrap
    names = T.NAMES
    seeds = o.seeds_for(names)
    pair = {(a, b): seeds[a][b] for a in names for b in names if a != b}
    pyus = [PYU(n, 0) for n in names]
    xs, ys = T._data(n_per=960)
    model = TorchModel(model_fn=T.MlpNet, loss_fn=torch.nn.CrossEntropyLoss,
                       optim_fn=optim_wrapper(torch.optim.Adam, lr=5e-3))
    fl = FLModel(device_list=pyus, model=model, aggregator=SecureAggregator(PYU("server", 0), pyus, seeds=pair),
                 random_seed=1234, train_device="cuda")
    fl.fit({p: x for p, x in zip(pyus, xs)}, {p: y for p, y in zip(pyus, ys)}, batch_size=32, epochs=1,
           aggregate_freq=1)
    print(calls, "median aggregate ms", 1e3 * float(np.median(times[1:])))
    pstats.Stats(prof).sort_stats("tottime").print_stats(15)


if __name__ == "__main__":
    main()
