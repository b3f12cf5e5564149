#!/usr/bin/env python3
"""Where a crypt_kernel / crypt_win_kernel launch spends its time, per wave
(diagnostic build).

Builds libzrc4 with ZRC4_TIMING=1 (zrc4_kernels.hpp, Stamps): lane 0 of every
wave stamps s_memrealtime (100 MHz) and s_memtime (shader clock) at kernel
entry (t0), S-boxes in LDS (t1), keystream done (t2) and state stored (t3).
The last of --launches back-to-back launches (rotating over batches, as
bench.py does) is read back and summarised:

  prologue   t1 - t0   image + entries + LDS fill
  chain      t2 - t1   the message loop (cycles per byte = clock delta / L)
  epilogue   t3 - t2   x/y + image store, drained
  span       max t3 - min t0 over the launch; entry skew = spread of t0

  python tools/kernel_timeline.py --workloads cfg2,cfg3,65536x1024
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import statistics
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

SHAPES = {"cfg2": (4096, 1024), "cfg3": (65536, 256), "cfg4": (1024, 65536)}


def summarise(rec: np.ndarray, waves: int, L: int) -> dict:
    r = rec[:waves, :4].astype(np.float64) * 10.0 / 1000.0     # us (100 MHz ticks)
    c = rec[:waves, 4:].astype(np.float64)
    t0 = r[:, 0].min()
    pro, chain, epi = r[:, 1] - r[:, 0], r[:, 2] - r[:, 1], r[:, 3] - r[:, 2]
    clk = (c[:, 2] - c[:, 1]) / np.maximum(r[:, 2] - r[:, 1], 1e-9) / 1e3     # GHz
    q = lambda a: {"min": round(float(a.min()), 3), "med": round(float(np.median(a)), 3),
                   "max": round(float(a.max()), 3)}
    return {"waves": waves, "span_us": round(float(r[:, 3].max() - t0), 3),
            "entry_skew_us": q(r[:, 0] - t0), "prologue_us": q(pro), "chain_us": q(chain),
            "epilogue_us": q(epi), "end_us": q(r[:, 3] - t0), "clock_ghz": q(clk),
            "chain_cyc_per_byte": q((c[:, 2] - c[:, 1]) / max(L, 1))}


def placement(rec: np.ndarray, hwid: np.ndarray, act: np.ndarray, L: int) -> dict:
    """gfx9 HW_ID fields (wave 3:0, simd 5:4, cu 11:8, sh 12, se 15:13) + XCC_ID;
    chain cycles/byte per wave, and the same split by how many active waves
    ran on the wave's CU, its CU pair (cu >> 1) and its SIMD."""
    c = rec[:, 4:].astype(np.float64)
    cyc = (c[:, 2] - c[:, 1]) / max(L, 1)
    h = hwid[:, 0]
    simd, cu, sh, se = (h >> 4) & 3, (h >> 8) & 15, (h >> 12) & 1, (h >> 13) & 7
    xcc = hwid[:, 1] & 15
    key_cu = [(int(x), int(a), int(b), int(u)) for x, a, b, u in zip(xcc, se, sh, cu)]
    key_pair = [(k[0], k[1], k[2], k[3] >> 1) for k in key_cu]
    key_simd = [k + (int(sd),) for k, sd in zip(key_cu, simd)]
    from collections import Counter
    n_cu = Counter(k for k, a in zip(key_cu, act) if a)
    n_pair = Counter(k for k, a in zip(key_pair, act) if a)
    n_simd = Counter(k for k, a in zip(key_simd, act) if a)
    out = {"by_waves_on_cu": {}, "by_waves_on_cu_pair": {}, "by_waves_on_simd": {}, "slow": []}
    med = float(np.median(cyc[act]))
    for name, keys, cnt in (("by_waves_on_cu", key_cu, n_cu), ("by_waves_on_cu_pair", key_pair, n_pair),
                            ("by_waves_on_simd", key_simd, n_simd)):
        groups = {}
        for i in np.flatnonzero(act):
            groups.setdefault(cnt[keys[i]], []).append(cyc[i])
        out[name] = {str(k): {"waves": len(v), "med": round(float(np.median(v)), 2), "max": round(float(max(v)), 2)}
                     for k, v in sorted(groups.items())}
    for i in np.flatnonzero(act):
        if cyc[i] > med + 2:
            out["slow"].append({"wave": int(i), "cyc": round(float(cyc[i]), 2), "xcc": int(xcc[i]), "se": int(se[i]),
                                "sh": int(sh[i]), "cu": int(cu[i]), "simd": int(simd[i])})
    out["slow"] = out["slow"][:24]
    out["by_xcc"] = {int(x): {"waves": int(((xcc == x) & act).sum()),
                              "med": round(float(np.median(cyc[(xcc == x) & act])), 2),
                              "p90": round(float(np.percentile(cyc[(xcc == x) & act], 90)), 2),
                              "max": round(float(cyc[(xcc == x) & act].max()), 2)}
                     for x in np.unique(xcc[act])}
    out["all"] = [[int(xcc[i]), int(se[i]), int(sh[i]), int(cu[i]), int(simd[i]), round(float(cyc[i]), 1)]
                  for i in np.flatnonzero(act)][:256]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workloads", default="cfg2,cfg3,65536x1024")
    ap.add_argument("--launches", type=int, default=12)
    ap.add_argument("--footprint-mib", type=int, default=640)
    ap.add_argument("--build-only", action="store_true")
    ap.add_argument("--placement", action="store_true",
                    help="per-wave chain cycles/byte against where the wave ran (XCC, SE, SH, CU, SIMD)")
    ap.add_argument("--ids", choices=("range", "grouped", "declared"), default="range",
                    help="grouped: slots permuted inside each group, groups in random order (bench.py --ids grouped) "
                         "through zrc4_crypt_grouped; declared: the same through zrc4_crypt_grouped_declared")
    ap.add_argument("--active-waves", type=int, default=4,
                    help="only the first k waves of every 256-session group get payload (len 0 for the rest): "
                         "the chain rate at k waves per CU")
    ap.add_argument("--define", action="append", default=[], help="extra -D for the timing build (NAME=V)")
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
    hip = C.CDLL("libamdhip64.so.7")          # the runtime torch already mapped (same SONAME)
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    st = C.c_void_p(stream.cuda_stream)
    out = {}
    for wl in args.workloads.split(","):
        S, L = SHAPES[wl] if wl in SHAPES else (int(v) for v in wl.lower().split("x"))
        if S > 65536:
            raise SystemExit("timing records cover at most 256 workgroups (65536 sessions)")
        R = max(1, min(-(-args.footprint_mib * (1 << 20) // (S * (L + 256))), (1 << 24) // S))
        n = S * R
        keys = torch.from_numpy(synth.keys(0, n).reshape(-1)).to(dev)
        adv = torch.from_numpy(synth.advance(0, n).view(np.int32)).to(dev)
        klen = torch.full((n,), 16, dtype=torch.int32, device=dev)
        koff = torch.arange(n, dtype=torch.int64, device=dev) * 16
        pay = torch.from_numpy(synth.payload(0, n * L, threads=8)).to(dev)
        perm = np.arange(n, dtype=np.int64)
        bgroups = []
        if args.ids != "range":
            if S % 256:
                raise SystemExit("grouped modes need whole groups")
            rng = np.random.default_rng(77)
            for b in range(R):
                order = rng.permutation(S // 256)
                bgroups.append(np.ascontiguousarray((b * S // 256 + order).astype(np.uint32)))
                for k, g in enumerate(order):
                    perm[b * S + 256 * k: b * S + 256 * (k + 1)] = b * S + g * 256 + rng.permutation(256)
        ids = torch.from_numpy(perm.astype(np.int32)).to(dev)
        off = torch.from_numpy(perm * L).to(dev)
        lnh = np.full(n, L, dtype=np.int32)
        lnh.reshape(-1, 4, 64)[:, args.active_waves:, :] = 0
        ln = torch.from_numpy(lnh).to(dev)
        h = C.c_void_p()
        _capi.check(lib.zrc4_create(C.byref(h), 0, n), "create")
        _capi.check(lib.zrc4_ksa_range(h, 0, C.c_void_p(keys.data_ptr()), C.c_void_p(koff.data_ptr()),
                                       C.c_void_p(klen.data_ptr()), n, st))
        zoff = torch.zeros(n, dtype=torch.int64, device=dev)
        scratch = torch.zeros(1000, dtype=torch.uint8, device=dev)
        _capi.check(lib.zrc4_crypt(h, None, C.c_void_p(scratch.data_ptr()), C.c_void_p(zoff.data_ptr()),
                                   C.c_void_p(adv.data_ptr()), n, st))
        torch.cuda.synchronize()
        for i in range(args.launches):
            b = i % R
            if args.ids == "declared":
                _capi.check(lib.zrc4_crypt_grouped_declared(h, C.c_void_p(ids.data_ptr() + 4 * b * S),
                                                            C.c_void_p(bgroups[b].ctypes.data),
                                                            C.c_void_p(pay.data_ptr()),
                                                            C.c_void_p(off.data_ptr() + 8 * b * S),
                                                            C.c_void_p(ln.data_ptr() + 4 * b * S), S, None, st))
            elif args.ids == "grouped":
                _capi.check(lib.zrc4_crypt_grouped(h, C.c_void_p(ids.data_ptr() + 4 * b * S),
                                                   C.c_void_p(pay.data_ptr()), C.c_void_p(off.data_ptr() + 8 * b * S),
                                                   C.c_void_p(ln.data_ptr() + 4 * b * S), S, st))
            else:
                _capi.check(lib.zrc4_crypt_range(h, b * S, C.c_void_p(pay.data_ptr()),
                                                 C.c_void_p(off.data_ptr() + 8 * b * S),
                                                 C.c_void_p(ln.data_ptr() + 4 * b * S), S, st))
        _capi.check(lib.zrc4_sync(h, st))
        sink = C.c_void_p()
        _capi.check(lib.zrc4_debug_sink(h, C.byref(sink)))
        rec = np.zeros((1024, 8), dtype=np.uint64)
        rc = hip.hipMemcpy(C.c_void_p(rec.ctypes.data), sink, C.c_size_t(rec.nbytes), 2)
        if rc:
            raise SystemExit(f"hipMemcpy failed {rc}")
        hwid = np.zeros((1024, 2), dtype=np.uint32)
        rc = hip.hipMemcpy(C.c_void_p(hwid.ctypes.data), C.c_void_p(sink.value + 65536), C.c_size_t(hwid.nbytes), 2)
        if rc:
            raise SystemExit(f"hipMemcpy failed {rc}")
        if S <= 32 * 256:        # crypt_win_kernel (<= 32 groups): one record per 4-stream workgroup
            waves = S // 4
            act = np.ones(waves, dtype=bool)
        else:
            waves = (S + 63) // 64
            act = np.array([(w % 4) < args.active_waves for w in range(waves)])
        out[wl] = summarise(rec[:waves][act], int(act.sum()), L)
        out[wl]["active_waves_per_group"] = args.active_waves
        out[wl]["ids"] = args.ids
        if args.placement:
            print(wl, "placement:", json.dumps(placement(rec[:waves], hwid[:waves], act, L)), flush=True)
        print(wl, json.dumps(out[wl]), flush=True)
        lib.zrc4_destroy(h)
        del keys, adv, pay, off, ids, ln, klen, koff, zoff
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
