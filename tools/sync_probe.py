#!/usr/bin/env python3
"""How much of bench.py's host-wall step is the host's wait, not the GPU.

The bench's timed region is: synchronize, K launches, synchronize.  With
K = 20 the wall per step exceeds the HIP-event kernel average by ~1.3 us
(~27 us of fixed cost per region: the first launch's latency and the host's
wake-up after the last kernel).  This probe times the same region over the
same GpuRunner two ways, interleaved:

  plain   torch.cuda.synchronize() straight after the launches (bench.py)
  poll    the host polls the launch stream (hipStreamQuery through
          torch's Stream.query) until it drains, then synchronize()

and prints the median wall per step and the kernel average for each K.

  python tools/sync_probe.py [--workload cfg2] [--ks 20,200] [--reps 15]
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cfg2")
    ap.add_argument("--ks", default="20,200")
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--footprint-mib", type=int, default=640)
    args = ap.parse_args()
    import torch
    import bench
    S, L = bench.CONFIG_SHAPES[args.workload]
    R = bench.rotation_batches(S, L, args.footprint_mib)
    run = bench.GpuRunner(torch, 0, S, L, R, 0)
    for i in range(120):
        run.step(i)
    run.sync()
    out = {"workload": args.workload, "rotation_batches": R}
    nxt = 120
    for k in (int(v) for v in args.ks.split(",")):
        res = {"plain": [], "poll": []}
        kern = {"plain": [], "poll": []}
        for rep in range(args.reps):
            for mode in ("plain", "poll") if rep % 2 == 0 else ("poll", "plain"):
                marks = run.make_events(k, 16)
                run.sync()
                t0 = time.perf_counter()
                run.launch_steps(nxt, k, 16, marks)
                if mode == "poll":
                    while not run.stream.query():
                        pass
                run.sync()
                wall = time.perf_counter() - t0
                nxt += k
                res[mode].append(wall / k * 1e6)
                kern[mode].append(statistics.mean(run.segment_ms(k, 16, marks)) * 1e3)
        out[str(k)] = {m: {"wall_us_per_step_med": round(statistics.median(res[m]), 3),
                           "wall_us_per_step_min": round(min(res[m]), 3),
                           "kernel_us_med": round(statistics.median(kern[m]), 3),
                           "fixed_us_med": round(statistics.median(
                               (w - q) * k for w, q in zip(res[m], kern[m])), 2)}
                       for m in res}
        print(k, json.dumps(out[str(k)]), flush=True)
    run.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
