#!/usr/bin/env python3
"""Which environment keeps the one-GPU W = 8 rehearsal fast?  Runs
`bench.py --gpus 8 --rehearse-one-gpu` (1M elements, every design) once per
environment variant, in order, and prints one JSON line per run: the wall
time, rank 0's phase timeline and the cgroup CPU counters.  Stops after the
first run that does not exit 0 (a rank watchdog or a failure: nothing more is
started on the GPU after that).  This process never touches the GPU.

usage: python tools/rehearsal_env_probe.py [--variants default,q1,nosdma,q1nosdma] [--out DIR]
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))

VARIANTS = {
    "default": {"GPU_MAX_HW_QUEUES": "2"},
    "q4": {"GPU_MAX_HW_QUEUES": "4"},
    "q1": {"GPU_MAX_HW_QUEUES": "1"},
    "nosdma": {"GPU_MAX_HW_QUEUES": "2", "HSA_ENABLE_SDMA": "0"},
    "q1nosdma": {"GPU_MAX_HW_QUEUES": "1", "HSA_ENABLE_SDMA": "0"},
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="default,q1,nosdma,q1nosdma")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "rehearsal_env_probe"))
    args = ap.parse_args()
    from test_gpu_bench_rehearsal import host_counters

    os.makedirs(args.out, exist_ok=True)
    for i, name in enumerate(args.variants.split(",")):
        env = dict(os.environ)
        for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
            env.pop(k, None)
        env["SFL_BENCH_TRACE"] = "1"
        env.update(VARIANTS[name])
        before, t0 = host_counters(), time.time()
        r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(args.world),
                            "--rehearse-one-gpu", "--elems", "1000003", "--steps", "3", "--warmup", "1",
                            "--variant-steps", "2", "--host-resident-steps", "3", "--cpu-baseline-seconds", "0",
                            "--watchdog-seconds", "150"],
                           capture_output=True, text=True, timeout=200, env=env, cwd=ROOT)
        wall = time.time() - t0
        after = host_counters()
        with open(os.path.join(args.out, f"{i}_{name}.err"), "w") as f:
            f.write(r.stderr)
        phases = [ln.split("phase ", 1)[1] for ln in r.stderr.splitlines() if "rank 0: phase" in ln]
        print(json.dumps({"variant": name, "env": VARIANTS[name], "rc": r.returncode, "wall_s": round(wall, 1),
                          "phases": phases, "cpu": {k: after[k] - before[k] for k in after if k in before}}),
              flush=True)
        if r.returncode != 0:
            break


if __name__ == "__main__":
    main()
