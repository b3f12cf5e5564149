#!/usr/bin/env python3
"""Do consecutive independent batches gain from running on two HIP streams?

bench.py's cfg2 rotates over R disjoint 4 096-session batches, so step i and
step i + 1 touch different slots and payload.  This times K steps launched on
one stream (the bench) against the same K steps alternating over two streams
(steps i and i + 2 stay ordered on one stream; R is even), wall clock between
two device synchronizes, interleaved repetitions.

  python tools/overlap_probe.py --workload cfg2 --steps 200 --reps 7
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cfg2")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--streams", type=int, default=2)
    args = ap.parse_args()
    import torch
    S, L = bench.CONFIG_SHAPES[args.workload]
    R = bench.rotation_batches(S, L, 640)
    if R % args.streams:
        R += args.streams - R % args.streams
    run = bench.GpuRunner(torch, 0, S, L, R, 0, "range")
    streams = [run.stream] + [torch.cuda.Stream(device=0) for _ in range(args.streams - 1)]
    alt = []
    for i, a in enumerate(run._args):
        alt.append(a[:-1] + (C.c_void_p(streams[i % args.streams].cuda_stream),))
    fn = run._fn

    def timed(argl):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.steps):
            rc = fn(*argl[i % R])
            if rc:
                raise SystemExit(f"crypt failed {rc}")
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / args.steps * 1e6

    for _ in range(3):                       # warm both paths
        timed(run._args)
        timed(alt)
    one, two = [], []
    for _ in range(args.reps):
        one.append(timed(run._args))
        two.append(timed(alt))
    run.check()
    out = {"workload": args.workload, "steps": args.steps, "batches": R, "streams": args.streams,
           "one_stream_us_per_step": round(statistics.median(one), 2),
           f"{args.streams}_streams_us_per_step": round(statistics.median(two), 2),
           "one_all": [round(v, 2) for v in one], "multi_all": [round(v, 2) for v in two]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
