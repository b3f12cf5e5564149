#!/usr/bin/env python3
"""Per-step wall time of the bench loop under different timing instrumentations
(cfg2 by default): events around every launch (bench.py's timed_steps), events
around every Nth launch, and no events (start/end only).  Prints one JSON line.
"""
import argparse
import json
import statistics
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cfg2")
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--rounds", type=int, default=5)
    args = ap.parse_args()
    import torch
    import bench
    S, L = bench.CONFIG_SHAPES[args.workload]
    R = bench.rotation_batches(S, L, 640)
    run = bench.GpuRunner(torch, 0, S, L, R, 0)
    st = run.stream
    for i in range(50):
        run.step(i)
    run.sync()

    def plain(k, first):
        run.sync()
        t0 = time.perf_counter()
        for i in range(k):
            run.step(first + i)
        run.sync()
        return (time.perf_counter() - t0) / k * 1e6

    def every(k, first, n):
        evs = []
        run.sync()
        t0 = time.perf_counter()
        for i in range(k):
            if i % n == 0:
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(st)
                run.step(first + i)
                b.record(st)
                evs.append((a, b))
            else:
                run.step(first + i)
        run.sync()
        wall = (time.perf_counter() - t0) / k * 1e6
        return wall, statistics.mean(a.elapsed_time(b) * 1e3 for a, b in evs)

    def host_only(k, first):
        # host cost of one launch call (GPU kept busy by a long queue ahead of it)
        t0 = time.perf_counter()
        for i in range(k):
            run.step(first + i)
        t = (time.perf_counter() - t0) / k * 1e6
        run.sync()
        return t

    out = {"workload": args.workload, "steps": args.steps}
    res = {"plain_us": [], "ev1_us": [], "ev1_kernel_us": [], "ev8_us": [], "ev8_kernel_us": [],
           "host_enqueue_us": []}
    for r in range(args.rounds):
        res["plain_us"].append(plain(args.steps, 1000))
        w, kern = every(args.steps, 1000, 1)
        res["ev1_us"].append(w); res["ev1_kernel_us"].append(kern)
        w, kern = every(args.steps, 1000, 8)
        res["ev8_us"].append(w); res["ev8_kernel_us"].append(kern)
        res["host_enqueue_us"].append(host_only(args.steps, 1000))
    for k, v in res.items():
        out[k] = round(statistics.median(v), 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
