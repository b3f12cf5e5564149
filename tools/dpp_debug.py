#!/usr/bin/env python3
"""Debug aid for the throughput store path: zero payloads (output = keystream)
through one libzrc4 variant, compared with the oracle keystream per 16-byte
chunk.  For every wrong chunk of the first wave, report which (session, chunk)
of the expected output it holds instead -- a transpose or addressing error
shows up as a permutation.

  python tools/dpp_debug.py [--lib zsummerx_amd/libzrc4.so] [--n 70000] [--len 1024]
"""
from __future__ import annotations

import argparse
import ctypes as C
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=str(ROOT / "zsummerx_amd" / "libzrc4.so"))
    ap.add_argument("--n", type=int, default=70000)
    ap.add_argument("--len", type=int, default=1024)
    ap.add_argument("--sessions", type=int, default=64, help="sessions to diagnose")
    args = ap.parse_args()
    import torch
    import pyoracle
    from zsummerx_amd import _capi
    lib = _capi.load(args.lib)
    n, L = args.n, args.len
    rng = np.random.default_rng(5)
    keys = rng.integers(0, 256, 16 * n, dtype=np.uint8)
    koff = np.arange(n, dtype=np.uint64) * 16
    klen = np.full(n, 16, dtype=np.uint32)
    off = np.arange(n, dtype=np.uint64) * L
    ln = np.full(n, L, dtype=np.uint32)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    h = C.c_void_p()
    _capi.check(lib.zrc4_create(C.byref(h), 0, n))
    dk, dko, dkl = T(keys), T(koff.view(np.int64)), T(klen.view(np.int32))
    _capi.check(lib.zrc4_ksa(h, None, C.c_void_p(dk.data_ptr()), C.c_void_p(dko.data_ptr()),
                             C.c_void_p(dkl.data_ptr()), n, st))
    src = np.zeros(n * L, np.uint8)
    pay = T(src)
    do, dl = T(off.view(np.int64)), T(ln.view(np.int32))
    _capi.check(lib.zrc4_crypt(h, None, C.c_void_p(pay.data_ptr()), C.c_void_p(do.data_ptr()),
                               C.c_void_p(dl.data_ptr()), n, st))
    _capi.check(lib.zrc4_sync(h, st))
    got = pay.cpu().numpy()
    ns = min(n, 4096)
    want = src[: ns * L].copy()
    ob = pyoracle.Batch(ns)
    ob.make_sbox(keys[: 16 * ns], koff[:ns], klen[:ns])
    ob.crypt(want, off[:ns], ln[:ns])
    g = got[: ns * L].reshape(ns, L // 16, 16)
    w = want.reshape(ns, L // 16, 16)
    index = {w[s, c].tobytes(): (s, c) for s in range(ns) for c in range(L // 16)}
    bad_total = int((g != w).any(axis=2).sum())
    print(f"wrong 16-B chunks in first {ns} sessions: {bad_total} of {ns * (L // 16)}")
    shown = 0
    for s in range(min(args.sessions, ns)):
        row = []
        for c in range(L // 16):
            if (g[s, c] != w[s, c]).any():
                src = index.get(g[s, c].tobytes())
                zero = not g[s, c].any()
                row.append(f"c{c}<-{'zero' if zero else src}")
        if row:
            print(f"session {s}: " + " ".join(row[:12]) + (" ..." if len(row) > 12 else ""))
            shown += 1
            if shown >= 24:
                break
    # dword-level provenance of the first wrong chunks (4-byte words of the expected output)
    wd = w.reshape(-1).view(np.uint32)
    where = {}
    for k, v in enumerate(wd[: 4096 * (L // 4)]):
        where.setdefault(int(v), k)
    shown = 0
    for s in range(min(4, ns)):
        for c in range(min(10, L // 16)):
            if (g[s, c] != w[s, c]).any():
                dws = g[s, c].view(np.uint32)
                prov = []
                for v in dws:
                    k = where.get(int(v))
                    prov.append("?" if k is None else f"s{(4 * k) // L}+{(4 * k) % L}")
                print(f"s{s} c{c}: got {g[s, c].tobytes().hex()} want {w[s, c].tobytes().hex()} dwords from {prov}")
    lib.zrc4_destroy(h)


if __name__ == "__main__":
    main()
