#!/usr/bin/env python3
"""BASELINE config 4: a horizontal-FL round (fed_avg_w, reference MlpNet
4-50-50-3, 8 clients, synthetic data) with the secure aggregator swapped to
the HIP path end-to-end -- the in-process simulation (one fused launch) and
the per-party drop-in (sfl_amd.compat.secretflow) -- against the same loop
on the numpy oracle aggregator.  Reports per-round and per-aggregation wall
time.

usage: python tools/fl_round_bench.py [--epochs 2] [--train-device cuda|cpu] [--hidden 50]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=2)
    ap.add_argument("--train-device", default="cuda")
    ap.add_argument("--rows", type=int, default=960, help="rows per client")
    args = ap.parse_args()
    import numpy as np
    import torch

    import test_fl_round as T
    from oracle import secagg as o
    from sfl_amd.device import PYU
    from sfl_amd.ml.fl import FLModel, TorchModel, optim_wrapper
    from sfl_amd.security.aggregation import SecureAggregator

    names = T.NAMES
    seeds = o.seeds_for(names)
    pair = {(a, b): seeds[a][b] for a in names for b in names if a != b}
    pyus = [PYU(n, 0) for n in names]
    xs, ys = T._data(n_per=args.rows)
    res = {"config": f"8 clients, MlpNet 4-50-50-3 fed_avg_w, {args.rows} rows/client, batch 32, "
                     f"aggregate_freq 1, local training on {args.train_device}"}
    # untimed warm-up fit: the process's first CUDA training and the HIP
    # library's first launches would otherwise land in whichever run is first
    warm = FLModel(device_list=pyus, model=TorchModel(model_fn=T.MlpNet, loss_fn=torch.nn.CrossEntropyLoss,
                                                      optim_fn=optim_wrapper(torch.optim.Adam, lr=5e-3)),
                   aggregator=SecureAggregator(PYU("server", 0), pyus, seeds=pair), random_seed=1234,
                   train_device=args.train_device)
    warm.fit({p: x for p, x in zip(pyus, xs)}, {p: y for p, y in zip(pyus, ys)}, batch_size=32, epochs=1,
             aggregate_freq=1, validation_data=(np.concatenate(xs), np.concatenate(ys)))  # first evaluate too
    from sfl_amd.compat import secretflow as hip_compat

    for label, agg in (("hip", SecureAggregator(PYU("server", 0), pyus, seeds=pair)),
                       # the secretflow-facing drop-in: every party masks by itself (sa_mask on its
                       # device, masked payload to the server, sa_sum_u64 + sa_decode there)
                       ("hip_per_party_drop_in", hip_compat.SecureAggregator(PYU("server", 0), pyus, seeds=pair)),
                       ("oracle_numpy", T.OracleAggregator(names, seeds))):
        model = TorchModel(model_fn=T.MlpNet, loss_fn=torch.nn.CrossEntropyLoss,
                           optim_fn=optim_wrapper(torch.optim.Adam, lr=5e-3))
        fl = FLModel(device_list=pyus, model=model, aggregator=agg, random_seed=1234,
                     train_device=args.train_device)
        t0 = time.perf_counter()
        h = fl.fit({p: x for p, x in zip(pyus, xs)}, {p: y for p, y in zip(pyus, ys)}, batch_size=32,
                   epochs=args.epochs, aggregate_freq=1,
                   validation_data=(np.concatenate(xs), np.concatenate(ys)))
        wall = time.perf_counter() - t0
        agg_s = h["aggregation_s"][1:]  # first aggregation includes one-time setup
        res[label] = {"rounds": len(h["round_s"]), "fit_s": wall, "rounds_s": float(np.sum(h["round_s"])),
                      "round_ms_median": 1e3 * float(np.median(h["round_s"][1:])),
                      "aggregation_ms_median": 1e3 * float(np.median(agg_s)),
                      "first_aggregations_ms": [1e3 * float(v) for v in h["aggregation_s"][:3]],
                      "outside_rounds_s": wall - float(np.sum(h["round_s"])),
                      "init_average_s": h["init_s"], "evaluate_s": h["eval_s"],
                      "aggregation_share": float(np.sum(agg_s) / np.sum(h["round_s"][1:])),
                      "val_accuracy": h["val_accuracy"][-1]}
    n_params = sum(p.numel() for p in T.MlpNet().parameters())
    res["params_per_client"] = n_params
    print(json.dumps(res))


if __name__ == "__main__":
    main()
