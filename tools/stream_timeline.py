#!/usr/bin/env python3
"""Where a crypt_stream_kernel launch spends its time (diagnostic build).

Builds libzrc4 with ZRC4_TIMING=1: lane 0 of the first wave of every wave
pair (waves 0 and 2 of each workgroup) stamps s_memrealtime (100 MHz) at
kernel entry, at the start and end of each group's keystream, and at exit
(zrc4_kernels.hpp, stream_stamp).  The last of --launches back-to-back
launches is read back and summarised per workgroup (its pair 0, as the
pre-r05 timelines) and per pair:

  prologue   first keystream start - entry   (first image + entries + lines)
  chain k    keystream of the k-th group walked (all its messages)
  boundary k start of group k+1 - end of group k (image out, next image in, barriers)
  epilogue   exit - end of the last group (last image store, drained)

and "what_if" replays each pair's own sequence with one component replaced
(every prologue the launch's fastest / median one, every chain the median of
its group index, no boundaries) to bound what removing that component's
spread could give the launch span.

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


def what_if(rt: np.ndarray, rows: int, K: int) -> dict:
    """Launch span (us) if each pair ran its own recorded sequence with one
    component replaced.  Pair p: entry e, prologue P, chains C_k, boundaries
    B_k, epilogue E; end = e + P + sum C + sum B + E (exactly its exit)."""
    r = rt[:rows].astype(np.float64) * 10.0 / 1000.0
    e = r[:, 0]
    t0 = e.min()
    P = r[:, 1] - r[:, 0]
    C = np.stack([r[:, 2 + 2 * k] - r[:, 1 + 2 * k] for k in range(K)], axis=1)
    B = np.stack([r[:, 3 + 2 * k] - r[:, 2 + 2 * k] for k in range(K - 1)], axis=1) if K > 1 else np.zeros((rows, 0))
    E = r[:, 15] - r[:, 2 + 2 * (K - 1)]

    def span(e_, P_, C_, B_, E_):
        return round(float((e_ + P_ + C_.sum(1) + B_.sum(1) + E_).max() - t0), 2)

    end = e + P + C.sum(1) + B.sum(1) + E
    out = {"recorded": span(e, P, C, B, E),
           "prologue_fastest": span(e, np.full_like(P, P.min()), C, B, E),
           "prologue_median": span(e, np.minimum(P, np.median(P)), C, B, E),
           "no_entry_skew": span(np.full_like(e, t0), P, C, B, E),
           "chains_median": span(e, P, np.broadcast_to(np.median(C, 0), C.shape), B, E),
           "chains_fastest_quartile": span(e, P, np.minimum(C, np.percentile(C, 25, axis=0)), B, E),
           "no_boundaries": span(e, P, C, np.zeros_like(B), E),
           "prologue_median_and_chains_median": span(e, np.minimum(P, np.median(P)),
                                                     np.broadcast_to(np.median(C, 0), C.shape), B, E),
           "sum_chain_median": round(float(np.median(C.sum(1))), 2)}
    # which component the 16 latest pairs lose their time in, against the median pair
    late = np.argsort(end)[-16:]
    med = {"entry": np.median(e - t0), "prologue": np.median(P), "chains": np.median(C.sum(1)),
           "boundaries": np.median(B.sum(1)), "epilogue": np.median(E)}
    out["latest16_excess_over_median"] = {
        "entry": round(float(np.mean(e[late] - t0) - med["entry"]), 2),
        "prologue": round(float(np.mean(P[late]) - med["prologue"]), 2),
        "chains": round(float(np.mean(C[late].sum(1)) - med["chains"]), 2),
        "boundaries": round(float(np.mean(B[late].sum(1)) - med["boundaries"]), 2),
        "epilogue": round(float(np.mean(E[late]) - med["epilogue"]), 2)}
    out["corr_end_with"] = {n: round(float(np.corrcoef(end, v)[0, 1]), 3)
                            for n, v in (("entry", e), ("prologue", P), ("chains", C.sum(1)),
                                         ("boundaries", B.sum(1)))}
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
        rt = np.zeros((1024, 16), dtype=np.uint64)     # record 2 wg + pair
        clk = np.zeros((1024, 2), dtype=np.uint64)
        hwid = np.zeros((1024, 2), dtype=np.uint32)
        base = 65536 + 16384                            # zrc4_kernels.hpp kStampBase
        for arr, o in ((rt, base), (clk, base + 131072), (hwid, base + 131072 + 16384)):
            rc = hip.hipMemcpy(C.c_void_p(arr.ctypes.data), C.c_void_p(sink.value + o), C.c_size_t(arr.nbytes), 2)
            if rc:
                raise SystemExit(f"hipMemcpy failed {rc}")
        groups = -(-S // 256)
        wgs = min(groups, 512)
        K = min(7, groups // wgs)
        wrt, wclk, whw = rt[0::2], clk[0::2], hwid[0::2]        # pair 0 of each workgroup
        out[wl] = summarise(wrt, wclk, wgs, K)
        out[wl]["ids"] = args.ids
        out[wl]["last_launch_event_us"] = round(last_event_us, 2)
        out[wl]["by_place"] = by_place(wrt, whw, wgs, K)
        out[wl]["pairs"] = summarise(rt, clk, 2 * wgs, K)
        out[wl]["pairs"]["partner_end_diff_us"] = q(np.abs(rt[0:2 * wgs:2, 15].astype(np.float64) -
                                                           rt[1:2 * wgs:2, 15].astype(np.float64)) / 100.0)
        out[wl]["pairs"]["what_if"] = what_if(rt, 2 * wgs, K)
        print(wl, json.dumps(out[wl]), flush=True)
        if args.dump:
            np.savez(f"{args.dump}_{wl}.npz", rt=rt[:2 * wgs], clk=clk[:2 * wgs], hwid=hwid[:2 * wgs])
        lib.zrc4_destroy(h)
        del keys, pay, off, ln, klen, koff
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
