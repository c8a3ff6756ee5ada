#!/usr/bin/env python3
"""Probe: does torch.cuda.Event(blocking=True).synchronize() return after a
long GPU job on this box (an interrupt-driven wait), and how long does the
host thread take to wake vs a spinning event?"""
import json
import threading
import time

import torch

dev = torch.device("cuda", 0)
a = torch.randn(8192, 8192, device=dev)
res = {}
for blocking in (False, True):
    for rep in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            b = a @ a
        e = torch.cuda.Event(blocking=blocking)
        e.record()
        t_enq = time.perf_counter()
        c0 = time.thread_time()
        e.synchronize()
        res[f"blocking={blocking} rep{rep}"] = {"wait_s": time.perf_counter() - t_enq,
                                                "wait_cpu_s": time.thread_time() - c0}
# from a second thread, as the loopback server's receive threads do
out = {}


def worker():
    e = torch.cuda.Event(blocking=True)
    for _ in range(20):
        b = a @ a
    e.record()
    t0 = time.perf_counter()
    e.synchronize()
    out["thread_wait_s"] = time.perf_counter() - t0


t = threading.Thread(target=worker)
t.start()
t.join(60)
res["thread"] = out or "HUNG"
print(json.dumps(res), flush=True)
