#!/usr/bin/env python3
"""Host-resident secure aggregation over loopback sockets (BASELINE north
star: "this path starts and ends in host memory"; config 5's H2D/D2H-inclusive
rate).  C client processes + this process as the server on one GPU; every
round moves each client's fp32 gradient H2D, masks it, moves the masked u64
vector D2H, sends it over 127.0.0.1, and the server receives, H2D, sums,
decodes and broadcasts the float64 result.

usage: python tools/loopback_bench.py [--clients 8] [--elems 100000000] [--rounds 3] [--gpus N]

--gpus N places client process g on GPU g % N and the server on GPU 0
(sfl_amd.loopback.placement): on the 8-GPU node config 3 is
`--clients 8 --elems 100000000 --gpus 8` and config 5
`--clients 32 --elems 256000000 --parties-per-process 4 --gpus 8`, so every
GPU's PCIe link carries only its own parties' copies.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _median_stages(reports):
    import numpy as np

    names = sorted({k for r in reports for k in r})
    return {k: {f: float(np.median([r[k][f] for r in reports if k in r])) for f in ("wall_s", "cpu_s", "calls")}
            for k in names}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=8)
    ap.add_argument("--elems", type=int, default=100_000_000)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--parties-per-process", type=int, default=1,
                    help="client parties hosted per OS process (config 5: 32 clients as 8 x 4)")
    ap.add_argument("--gpus", type=int, default=1,
                    help="client process g on GPU g %% N, the server on GPU 0 (one GPU: every party on GPU 0)")
    ap.add_argument("--ab", type=int, default=0,
                    help="A/B passes over the host-path knobs (SFL_LOOPBACK_SEND x SFL_LOOPBACK_WAIT), one line "
                         "per run")
    ap.add_argument("--dump-after", type=float, default=0.0,
                    help="diagnostics: dump every thread's stack (server and client processes) after this many "
                         "seconds")
    args = ap.parse_args()
    import numpy as np

    if args.dump_after > 0:
        import faulthandler

        faulthandler.dump_traceback_later(args.dump_after, exit=False)
        os.environ["SFL_LOOPBACK_DUMP_AFTER"] = str(args.dump_after)

    from sfl_amd.loopback import run_loopback

    names = [f"client{c}" for c in range(args.clients)]
    seeds = {a: {b: (0x5ECA66 << 32) | (min(i, j) << 16) | max(i, j) for j, b in enumerate(names) if b != a}
             for i, a in enumerate(names)}

    def one_run():
        res, timings, stats, _ = run_loopback(names, args.elems, args.rounds, seeds=seeds, timeout=900,
                                              parties_per_process=args.parties_per_process, keep_results=False,
                                              gpus=list(range(args.gpus)))
        # no server-side copy of the results: every client must have received the same bytes
        xors = [{s[r]["result_xor"] for s in stats.values()} for r in range(args.rounds)]
        if any(len(x) != 1 for x in xors):
            raise SystemExit(f"clients received different results: {xors}")
        steady = timings[1:] if len(timings) > 1 else timings
        rs = float(np.median([t["round_s"] for t in steady]))
        # the rate: wall time from the start of round 1 (round 0 warms up) to the
        # end of the last round, per round -- it counts the parties' turnaround
        # between rounds as well as the server's rounds; one round: its time
        if len(timings) > 1:
            span = timings[-1]["t_start"] + timings[-1]["round_s"] - timings[1]["t_start"]
            period = span / (len(timings) - 1)
        else:
            period = rs
        cl = [s for per in stats.values() for s in per[1:] or per]
        return {
            "metric": "host-resident grad elems/s (loopback sockets, H2D/D2H inclusive)",
            "clients": args.clients, "elems_per_client": args.elems, "rounds": args.rounds,
            "period_s": period, "grad_elems_per_s": args.clients * args.elems / period,
            "round_s_median": rs,
            "server": {k: float(np.median([t[k] for t in steady])) for k in steady[0]
                       if k not in ("t_start", "stages", "placement")},
            "placement": timings[0]["placement"], "gpus": args.gpus,
            # host-side profile (sfl_amd.loopback.StageClock): wall and thread-CPU
            # seconds per named copy / wait, summed over the threads that ran it,
            # median over the steady rounds (server) or over clients x rounds
            "server_stages": _median_stages([t["stages"] for t in steady]),
            "client_stages": _median_stages([s["stages"] for s in cl]),
            "client_h2d_mask_s_median": float(np.median([s["h2d_mask_s"] for s in cl])),
            "client_d2h_send_s_median": float(np.median([s["d2h_send_s"] for s in cl])),
            "parties_per_process": args.parties_per_process,
            "wire_bytes_per_round": args.clients * args.elems * 8,
            "send": os.environ.get("SFL_LOOPBACK_SEND", "copy"),
            "wait": os.environ.get("SFL_LOOPBACK_WAIT", "poll"),
            "results_agree_across_clients": True,
        }

    if not args.ab:
        r = one_run()
        r["client_rx"] = os.environ.get("SFL_LOOPBACK_CLIENT_RX", "concurrent")
        print(json.dumps(r), flush=True)
        return
    # same-box A/B of the host-path choices, interleaved passes (boxes differ
    # by +-25 % on this host-bound path, so only same-box runs compare)
    for p in range(args.ab):
        for send, wait, rx in (("sendfile", "poll", "concurrent"), ("copy", "spin", "after"),
                               ("copy", "poll", "concurrent"), ("copy", "spin", "concurrent")):
            os.environ["SFL_LOOPBACK_SEND"], os.environ["SFL_LOOPBACK_WAIT"] = send, wait
            os.environ["SFL_LOOPBACK_CLIENT_RX"] = rx
            r = one_run()
            r["client_rx"] = rx
            r["ab_pass"] = p
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
