#!/usr/bin/env python3
"""bench.py --host-inclusive over a grid of chunk / stream counts in one
process: which pipelining of pinned H2D -> kernel -> D2H
moves a batch fastest, next to the zero-copy mode.

  python tools/hostinc_sweep.py --workloads cfg2,cfg3,cfg5 --chunks 1,2,4,8,16 --streams 1,2,4
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def pcie_ceiling(mib: int = 256, reps: int = 5) -> dict:
    """Pinned-host copy rates on this box (GB/s): H2D alone, D2H alone, and
    both at once on two streams (the duplex ceiling an in-place host
    round trip can reach)."""
    import statistics
    import time
    import torch
    dev = torch.device("cuda", 0)
    n = mib << 20
    h1 = torch.empty(n, dtype=torch.uint8).pin_memory()
    h2 = torch.empty(n, dtype=torch.uint8).pin_memory()
    d1 = torch.empty(n, dtype=torch.uint8, device=dev)
    d2 = torch.empty(n, dtype=torch.uint8, device=dev)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    out = {}
    for name in ("h2d", "d2h", "both"):
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if name in ("h2d", "both"):
                with torch.cuda.stream(s1):
                    d1.copy_(h1, non_blocking=True)
            if name in ("d2h", "both"):
                with torch.cuda.stream(s2):
                    h2.copy_(d2, non_blocking=True)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        t = statistics.median(ts)
        out[name + "_gbs"] = round((2 if name == "both" else 1) * n / t / 1e9, 2)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workloads", default="cfg2,cfg3,cfg5")
    ap.add_argument("--chunks", default="1,2,4,8,16")
    ap.add_argument("--streams", default="1,2,4")
    ap.add_argument("--steps", type=int, default=15)
    ap.add_argument("--pcie-only", action="store_true")
    a = ap.parse_args()
    print("pcie", json.dumps(pcie_ceiling()), flush=True)
    if a.pcie_only:
        return
    import bench
    for wl in a.workloads.split(","):
        rows = []
        for zc in (True, False):
            for c in ([1] if zc else [int(v) for v in a.chunks.split(",")]):
                for s in ([1] if zc else [int(v) for v in a.streams.split(",")]):
                    args = bench.parse(["--host-inclusive", "--workload", wl, "--chunks", str(c), "--streams", str(s),
                                        "--steps", str(a.steps), "--warmup", "3"] + (["--zero-copy"] if zc else []))
                    r = bench.host_inclusive(args)
                    rows.append({"zero_copy": zc, "chunks": r.get("chunks", 1), "streams": r.get("streams", 1),
                                 "gibs": r["value"], "ms": r["ms_per_pass"]})
                    print(wl, json.dumps(rows[-1]), flush=True)
        best = max((r for r in rows if not r["zero_copy"]), key=lambda r: r["gibs"])
        print(wl, "best_copy", json.dumps(best), flush=True)


if __name__ == "__main__":
    main()
