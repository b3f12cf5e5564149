#!/usr/bin/env python3
"""A/B timing of libzrc4 variants inside ONE process on ONE GPU.

Cross-box numbers for LDS-bound loops move by up to ~12 % between MI355X
devices (MI355X_MICROARCH.md, DVFS give-back item 5), so kernel changes are
judged here: every variant library (built with -D switches by
zsummerx_amd.build.build_variant) gets its own context seeded identically;
outputs of one batch are compared byte-for-byte across variants (they must be
identical); then timed rounds are interleaved and the median per-launch time
(HIP events on the launch stream) is reported per variant.

  python tools/ab_bench.py --variant base: --variant o1:ZRC4_STEP_ORDER=1 \
      --workloads cfg2,cfg3,cfg5 --rounds 7 --launches 20
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

SHAPES = {"cfg2": (4096, 1024), "cfg3": (65536, 256), "cfg4": (1024, 65536), "cfg5": (524288, 1024)}


def parse_variant(v: str):
    """name[@gitrev]:DEF=v,DEF2=v"""
    name, _, defs = v.partition(":")
    d = {}
    for kv in filter(None, defs.split(",")):
        k, _, val = kv.partition("=")
        d[k] = val or "1"
    return name, d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", action="append", required=True, help="name:DEF=v,DEF2=v")
    ap.add_argument("--workloads", default="cfg2,cfg3,cfg5")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--launches", type=int, default=20)
    ap.add_argument("--footprint-mib", type=int, default=640)
    ap.add_argument("--build-only", action="store_true")
    ap.add_argument("--ksa", action="store_true", help="also time zrc4_ksa_range per variant")
    ap.add_argument("--key-len", type=int, default=16, help="key bytes per session (16: the synthetic keys)")
    ap.add_argument("--segment", action="store_true",
                    help="time each round's launches as one back-to-back segment (per-launch average)")
    ap.add_argument("--no-check", action="store_true", help="timing-only ablation builds (outputs differ)")
    ap.add_argument("--ids", default="range",
                    help="comma list of range | grouped | declared; grouped: zrc4_crypt_grouped over the same "
                         "batches with slots permuted inside each group and groups in random order (bench.py "
                         "--ids grouped); declared: the same through zrc4_crypt_grouped_declared.  Every "
                         "variant runs every mode (its own context each), interleaved")
    args = ap.parse_args()

    from zsummerx_amd import build
    variants = []
    for v in args.variant:
        name, defs = parse_variant(v)
        name, _, rev = name.partition("@")
        variants.append((name, build.build_variant(name, defs, rev or None)))
    if args.build_only:
        print("built", [str(p) for _, p in variants])
        return

    import torch  # one HIP runtime for every variant library (see _capi.load)
    from zsummerx_amd import _capi, synth

    modes = args.ids.split(",")
    for m in modes:
        if m not in ("range", "grouped", "declared"):
            raise SystemExit(f"--ids: unknown mode {m}")
    loaded = [(n, _capi.load(p)) for n, p in variants]
    # one run per (variant, mode); names carry the mode when several are compared
    libs = [((n if len(modes) == 1 else f"{n}/{m}"), lib, m) for n, lib in loaded for m in modes]
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    st = C.c_void_p(stream.cuda_stream)
    report = {}
    for wl in args.workloads.split(","):
        if wl in SHAPES:
            S, L = SHAPES[wl]
        else:                                   # custom "SxL"
            S, L = (int(v) for v in wl.lower().split("x"))
        R = max(1, -(-args.footprint_mib * (1 << 20) // (S * (L + 256))))
        R = min(R, (1 << 24) // S)
        n = S * R
        KL = args.key_len
        if KL == 16:
            keys = torch.from_numpy(synth.keys(0, n).reshape(-1)).to(dev)
        else:
            keys = torch.from_numpy(np.random.default_rng(1).integers(0, 256, n * KL, dtype=np.uint8)).to(dev)
        adv = torch.from_numpy(synth.advance(0, n).view(np.int32)).to(dev)
        klen = torch.full((n,), KL, dtype=torch.int32, device=dev)
        koff = torch.arange(n, dtype=torch.int64, device=dev) * KL
        pay = torch.from_numpy(synth.payload(0, n * L, threads=8)).to(dev)
        off = torch.arange(n, dtype=torch.int64, device=dev) * L
        ln = torch.full((n,), L, dtype=torch.int32, device=dev)
        scratch = torch.zeros(1000, dtype=torch.uint8, device=dev)
        zoff = torch.zeros(n, dtype=torch.int64, device=dev)
        gids = goff = None
        bgroups = []
        if any(m != "range" for m in modes):
            # entry e of batch b -> session perm[e] (its slot, key, state and
            # payload); whole groups only (a short group mid-batch would make
            # later buckets straddle two groups)
            if S % 256:
                raise SystemExit(f"{wl}: grouped modes need a multiple of 256 sessions")
            rng = np.random.default_rng(77)
            perm = np.empty(n, dtype=np.int64)
            for b in range(R):
                order = rng.permutation(S // 256)
                bgroups.append(np.ascontiguousarray((b * S // 256 + order).astype(np.uint32)))
                for k, g in enumerate(order):
                    perm[b * S + 256 * k: b * S + 256 * (k + 1)] = b * S + g * 256 + rng.permutation(256)
            gids = torch.from_numpy(perm.astype(np.int32)).to(dev)
            goff = torch.from_numpy(perm * L).to(dev)

        def crypt(lib, mode, h, b, buf=None):
            p = C.c_void_p((pay if buf is None else buf).data_ptr())
            lp = C.c_void_p(ln.data_ptr() + 4 * b * S)
            if mode == "range":
                return lib.zrc4_crypt_range(h, b * S, p, C.c_void_p(off.data_ptr() + 8 * b * S), lp, S, st)
            ip, op = C.c_void_p(gids.data_ptr() + 4 * b * S), C.c_void_p(goff.data_ptr() + 8 * b * S)
            if mode == "declared":
                return lib.zrc4_crypt_grouped_declared(h, ip, C.c_void_p(bgroups[b].ctypes.data), p, op, lp, S,
                                                       None, st)
            return lib.zrc4_crypt_grouped(h, ip, p, op, lp, S, st)
        ctxs = []
        for name, lib, _ in libs:
            h = C.c_void_p()
            _capi.check(lib.zrc4_create(C.byref(h), 0, n), f"{name} create")
            _capi.check(lib.zrc4_ksa_range(h, 0, C.c_void_p(keys.data_ptr()), C.c_void_p(koff.data_ptr()),
                                           C.c_void_p(klen.data_ptr()), n, st))
            _capi.check(lib.zrc4_crypt(h, None, C.c_void_p(scratch.data_ptr()), C.c_void_p(zoff.data_ptr()),
                                       C.c_void_p(adv.data_ptr()), n, st))
            ctxs.append(h)
        torch.cuda.synchronize()
        # identical-output check on batch 0
        ref = None
        for (name, lib, mode), h in zip(libs, ctxs):
            buf = pay[: S * L].clone()
            _capi.check(crypt(lib, mode, h, 0, buf))
            _capi.check(lib.zrc4_sync(h, st))
            if ref is None:
                ref = buf
            elif not args.no_check and not torch.equal(ref, buf):
                raise SystemExit(f"variant {name} output differs from {libs[0][0]} on {wl}")
        if args.ksa:
            # connection-storm KSA timing: the batch-0 sessions re-seeded per launch
            kt = {name: [] for name, _, _ in libs}
            for r in range(args.rounds):
                for (name, lib, _), h in zip(libs, ctxs):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    for i in range(args.launches):
                        _capi.check(lib.zrc4_ksa_range(h, 0, C.c_void_p(keys.data_ptr()), C.c_void_p(koff.data_ptr()),
                                                       C.c_void_p(klen.data_ptr()), S, st), f"{name} ksa")
                    e1.record(stream)
                    torch.cuda.synchronize()
                    kt[name].append(e0.elapsed_time(e1) * 1e3 / args.launches)
            report[wl + "_ksa"] = {name: {"median_us": round(statistics.median(t), 2), "min_us": round(min(t), 2),
                                          "streams_per_s": round(S / (statistics.median(t) * 1e-6), 1)}
                                   for name, t in kt.items()}
            print(wl + "_ksa", json.dumps(report[wl + "_ksa"]), flush=True)
        times = {name: [] for name, _, _ in libs}
        step = 1
        for r in range(args.rounds):
            for (name, lib, mode), h in zip(libs, ctxs):
                evs = []
                if args.segment:               # back-to-back launches, like bench.py (kernel boundaries included)
                    s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s0.record(stream)
                for i in range(args.launches):
                    b = step % R
                    step += 1
                    if not args.segment:
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record(stream)
                    rc = crypt(lib, mode, h, b)
                    if not args.segment:
                        e1.record(stream)
                        evs.append((e0, e1))
                    if rc:
                        raise SystemExit(f"{name}: crypt failed {rc}")
                if args.segment:
                    s1.record(stream)
                torch.cuda.synchronize()
                if args.segment:
                    times[name].append(s0.elapsed_time(s1) * 1e3 / args.launches)
                else:
                    times[name].extend(a.elapsed_time(b_) * 1e3 for a, b_ in evs)
        B = 2 * S * L + 516 * S
        report[wl] = {name: {"median_us": round(statistics.median(t), 2), "min_us": round(min(t), 2),
                             "hbm_frac": round(B / (statistics.median(t) * 1e-6) / 8e12, 4)}
                      for name, t in times.items()}
        print(wl, json.dumps(report[wl]), flush=True)
        for (name, lib, _), h in zip(libs, ctxs):
            lib.zrc4_destroy(h)
        del keys, adv, pay, off, ln, klen, koff, zoff, gids, goff
        torch.cuda.empty_cache()
    print(json.dumps(report))


if __name__ == "__main__":
    main()
