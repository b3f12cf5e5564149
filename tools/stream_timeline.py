#!/usr/bin/env python3
"""Where a crypt_stream_kernel launch spends its time (diagnostic build).

Builds libzrc4 with ZRC4_TIMING=1: lane 0 of every workgroup's first wave
stamps s_memrealtime (100 MHz) at kernel entry, at the start and end of each
group's keystream, and at exit (zrc4_kernels.hpp, stream_stamp).  The last of
--launches back-to-back launches is read back and summarised per workgroup:

  prologue   first keystream start - entry   (first image + entries + lines)
  chain k    keystream of the k-th group walked (all its messages)
  boundary k start of group k+1 - end of group k (image out, next image in, barriers)
  epilogue   exit - end of the last group (last image store, drained)

  python tools/stream_timeline.py --workloads cfg5,131072x1024
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

SHAPES = {"cfg5": (524288, 1024)}


def q(a):
    a = np.asarray(a, dtype=np.float64)
    if a.size == 0:
        return None
    return {"min": round(float(a.min()), 3), "med": round(float(np.median(a)), 3), "max": round(float(a.max()), 3)}


def summarise(rt: np.ndarray, clk: np.ndarray, wgs: int, K: int) -> dict:
    r = rt[:wgs].astype(np.float64) * 10.0 / 1000.0          # us
    t0 = r[:, 0].min()
    out = {"workgroups": wgs, "span_us": round(float(r[:, 15].max() - t0), 3),
           "entry_skew_us": q(r[:, 0] - t0)}
    out["groups_per_workgroup"] = K
    out["prologue_us"] = q(r[:, 1] - r[:, 0])
    for k in range(K):
        out[f"chain{k}_us"] = q(r[:, 2 + 2 * k] - r[:, 1 + 2 * k])
        if k + 1 < K:
            out[f"boundary{k}_us"] = q(r[:, 3 + 2 * k] - r[:, 2 + 2 * k])
    out["epilogue_us"] = q(r[:, 15] - r[:, 2 + 2 * (K - 1)])
    out["chain_start_skew_us"] = {f"g{k}": q(r[:, 1 + 2 * k] - r[:, 1 + 2 * k].min()) for k in range(K)}
    c = clk[:wgs].astype(np.float64)
    out["clock_ghz"] = q((c[:, 1] - c[:, 0]) / np.maximum(r[:, 15] - r[:, 0], 1e-9) / 1e3)
    return out


def by_place(rt: np.ndarray, hwid: np.ndarray, wgs: int, K: int) -> dict:
    """Mean keystream time per group (us) of the workgroups, split by XCC, by
    shader engine, and by whether the other workgroup on the CU is an even or
    odd one; plus the slowest and fastest CUs."""
    r = rt[:wgs].astype(np.float64) * 10.0 / 1000.0
    chain = np.mean([r[:, 2 + 2 * k] - r[:, 1 + 2 * k] for k in range(K)], axis=0)
    h = hwid[:wgs, 0]
    xcc, se, cu, simd = hwid[:wgs, 1] & 15, (h >> 13) & 7, (h >> 8) & 15, (h >> 4) & 3
    out = {}
    for name, key in (("xcc", xcc), ("se", se), ("simd_of_wave0", simd)):
        out[name] = {int(v): round(float(np.median(chain[key == v])), 2) for v in np.unique(key)}
    cuk = xcc * 1000 + se * 100 + cu
    from collections import Counter
    cnt = Counter(cuk.tolist())
    out["wgs_per_cu"] = dict(Counter(cnt.values()))
    pairs = {}
    for i, k in enumerate(cuk.tolist()):
        pairs.setdefault(k, []).append(i)
    means, diffs, uneq = [], [], []
    for k, ix in pairs.items():
        if len(ix) == 2:
            a, b = ix
            means.append((chain[a] + chain[b]) / 2)
            diffs.append(abs(chain[a] - chain[b]))
            uneq.append((abs(chain[a] - chain[b]), int(simd[a]), int(simd[b]), round(float(chain[a]), 1),
                         round(float(chain[b]), 1)))
    if means:
        two = [ix for ix in pairs.values() if len(ix) == 2]
        out["cu_pairs"] = {"std_of_cu_means": round(float(np.std(means)), 2),
                           "mean_abs_diff_in_pair": round(float(np.mean(diffs)), 2),
                           "most_unequal": [list(u[1:]) for u in sorted(uneq)[-8:]],
                           # which workgroup ids share a CU (for grid-half / parity staggers)
                           "split_by_half": round(sum((a < wgs // 2) != (b < wgs // 2) for a, b in two) / len(two), 3),
                           "split_by_parity": round(sum((a & 1) != (b & 1) for a, b in two) / len(two), 3),
                           "sample": [sorted(ix) for ix in two[:8]]}
    order = np.argsort(chain)
    out["fastest"] = [[int(xcc[i]), int(se[i]), int(cu[i]), round(float(chain[i]), 2)] for i in order[:6]]
    out["slowest"] = [[int(xcc[i]), int(se[i]), int(cu[i]), round(float(chain[i]), 2)] for i in order[-6:]]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workloads", default="cfg5,131072x1024")
    ap.add_argument("--launches", type=int, default=150,
                    help="launches before the recorded one: the clock dips for ~30 cfg5 launches and recovers by ~100 (profiles/r02/cfg5_launch_durations.json)")
    ap.add_argument("--footprint-mib", type=int, default=1200)
    ap.add_argument("--build-only", action="store_true")
    ap.add_argument("--define", action="append", default=[], help="extra -D for the timing build (NAME=V)")
    ap.add_argument("--dump", default="", help="save the raw per-workgroup stamps (npz) under this prefix")
    ap.add_argument("--ids", choices=("range", "grouped"), default="range",
                    help="grouped: zrc4_crypt_grouped, slots permuted inside each group and groups in random order "
                         "(bench.py --ids grouped)")
    args = ap.parse_args()
    from zsummerx_amd import build
    defs = {"ZRC4_TIMING": "1"}
    for d in args.define:
        k, _, v = d.partition("=")
        defs[k] = v or "1"
    name = "timing" + "".join(f"_{k}{v}" for k, v in sorted(defs.items()) if k != "ZRC4_TIMING")
    path = build.build_variant(name, defs)
    if args.build_only:
        print("built", path)
        return
    import torch
    from zsummerx_amd import _capi, synth
    lib = _capi.load(path)
    lib.zrc4_debug_sink.argtypes = [C.c_void_p, C.POINTER(C.c_void_p)]
    hip = C.CDLL("libamdhip64.so.7")
    dev = torch.device("cuda", 0)
    st = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    out = {}
    for wl in args.workloads.split(","):
        S, L = SHAPES[wl] if wl in SHAPES else (int(v) for v in wl.lower().split("x"))
        R = max(1, min(-(-args.footprint_mib * (1 << 20) // (S * (L + 256))), (1 << 24) // S))
        n = S * R
        keys = torch.from_numpy(synth.keys(0, n).reshape(-1)).to(dev)
        klen = torch.full((n,), 16, dtype=torch.int32, device=dev)
        koff = torch.arange(n, dtype=torch.int64, device=dev) * 16
        pay = torch.from_numpy(synth.payload(0, n * L, threads=8)).to(dev)
        off = torch.arange(n, dtype=torch.int64, device=dev) * L
        ln = torch.full((n,), L, dtype=torch.int32, device=dev)
        gids = None
        if args.ids == "grouped":
            rng = np.random.default_rng(77)
            perm = np.empty(n, dtype=np.int64)
            for b in range(R):
                pos = 0
                for g in rng.permutation(-(-S // 256)):
                    lo, hi = b * S + g * 256, min(b * S + (g + 1) * 256, (b + 1) * S)
                    perm[b * S + pos: b * S + pos + (hi - lo)] = lo + rng.permutation(hi - lo)
                    pos += hi - lo
            gids = torch.from_numpy(perm.astype(np.int32)).to(dev)
            off = torch.from_numpy(perm * L).to(dev)
        h = C.c_void_p()
        _capi.check(lib.zrc4_create(C.byref(h), 0, n), "create")
        _capi.check(lib.zrc4_ksa_range(h, 0, C.c_void_p(keys.data_ptr()), C.c_void_p(koff.data_ptr()),
                                       C.c_void_p(klen.data_ptr()), n, st))
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for i in range(args.launches):
            b = i % R
            if i == args.launches - 1:
                ev0.record()
            if gids is None:
                _capi.check(lib.zrc4_crypt_range(h, b * S, C.c_void_p(pay.data_ptr()),
                                                 C.c_void_p(off.data_ptr() + 8 * b * S),
                                                 C.c_void_p(ln.data_ptr() + 4 * b * S), S, st))
            else:
                _capi.check(lib.zrc4_crypt_grouped(h, C.c_void_p(gids.data_ptr() + 4 * b * S),
                                                   C.c_void_p(pay.data_ptr()), C.c_void_p(off.data_ptr() + 8 * b * S),
                                                   C.c_void_p(ln.data_ptr() + 4 * b * S), S, st))
        ev1.record()
        _capi.check(lib.zrc4_sync(h, st))
        torch.cuda.synchronize()
        last_event_us = ev0.elapsed_time(ev1) * 1000.0
        sink = C.c_void_p()
        _capi.check(lib.zrc4_debug_sink(h, C.byref(sink)))
        rt = np.zeros((512, 16), dtype=np.uint64)
        clk = np.zeros((512, 2), dtype=np.uint64)
        hwid = np.zeros((512, 2), dtype=np.uint32)
        for arr, o in ((rt, 0), (clk, 65536), (hwid, 65536 + 8192)):
            rc = hip.hipMemcpy(C.c_void_p(arr.ctypes.data), C.c_void_p(sink.value + o), C.c_size_t(arr.nbytes), 2)
            if rc:
                raise SystemExit(f"hipMemcpy failed {rc}")
        groups = -(-S // 256)
        wgs = min(groups, 512)
        out[wl] = summarise(rt, clk, wgs, min(7, groups // wgs))
        out[wl]["ids"] = args.ids
        out[wl]["last_launch_event_us"] = round(last_event_us, 2)
        out[wl]["by_place"] = by_place(rt, hwid, wgs, min(7, groups // wgs))
        print(wl, json.dumps(out[wl]), flush=True)
        if args.dump:
            np.savez(f"{args.dump}_{wl}.npz", rt=rt[:wgs], clk=clk[:wgs], hwid=hwid[:wgs])
        lib.zrc4_destroy(h)
        del keys, pay, off, ln, klen, koff
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
