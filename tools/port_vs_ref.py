#!/usr/bin/env python3
"""Time the CPU restatement (oracle/rc4_oracle.c, the bench's cpu_baseline)
against the REAL reference class (oracle/_ref, compiled from
/root/reference/depends/rc4/rc4_encryption.h) on the same cfg2 sample, one
thread, and check they produce identical bytes (the port must
time within +-5 % of the real header).  Runs in the build container only
(/root/reference does not exist on the GPU box).  Prints one JSON line.

  python tools/port_vs_ref.py [--sessions 4096] [--length 1024]
"""
import argparse
import ctypes as C
import json
import statistics
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "oracle"))
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sessions", type=int, default=4096)
    ap.add_argument("--length", type=int, default=1024)
    ap.add_argument("--min-seconds", type=float, default=0.25)
    ap.add_argument("--runs", type=int, default=7)
    args = ap.parse_args()
    import pyoracle
    from zsummerx_amd import synth
    pyoracle.build()
    R = pyoracle.ref_lib()
    if R is None:
        sys.exit("oracle/_ref/libzrc4_ref.so missing (needs /root/reference; make -C oracle)")
    S, L = args.sessions, args.length
    keys = synth.keys(0, S).reshape(-1)
    key_off = np.arange(S, dtype=np.uint32) * 16
    key_len = np.full(S, 16, dtype=np.uint32)
    payload = synth.payload(0, S * L)
    off = np.arange(S, dtype=np.uint64) * L
    length = np.full(S, L, dtype=np.uint32)

    port = pyoracle.Batch(S)
    port.make_sbox(keys, key_off, key_len)
    size = R.zrc4_ref_state_size()
    ref_states = (C.c_uint8 * (size * S))()
    base = C.addressof(ref_states)
    for i in range(S):
        k = bytes(keys[16 * i:16 * i + 16])
        R.zrc4_ref_make_sbox(C.c_void_p(base + i * size), k, len(k))

    buf_p, buf_r = payload.copy(), payload.copy()

    def run_port():
        t0 = pyoracle.now()
        port.crypt(buf_p, off, length, threads=1)
        return pyoracle.now() - t0

    def run_ref():
        return R.zrc4_ref_crypt_batch(C.c_void_p(base), C.c_void_p(buf_r.ctypes.data),
                                      C.c_void_p(off.ctypes.data), C.c_void_p(length.ctypes.data), S)

    # equal work on both sides: the same number of batch passes, order alternated per run
    reps = 1
    while True:
        t = run_port() + run_ref()
        if t * reps >= 2 * args.min_seconds:
            break
        reps *= 2
    tp, tr = [], []
    for r in range(args.runs):
        order = (run_port, run_ref) if r % 2 == 0 else (run_ref, run_port)
        for fn in order:
            t = sum(fn() for _ in range(reps))
            (tp if fn is run_port else tr).append(t)
    same = bool(np.array_equal(buf_p, buf_r))
    gib = S * L * reps / 2**30
    port_gibs, ref_gibs = gib / statistics.median(tp), gib / statistics.median(tr)
    out = {
        "sample": f"{S} sessions x {L} B (cfg2 shape, synthetic keys/payload), {reps} batch passes per run, "
                  f"median of {args.runs} runs, 1 thread, port/ref order alternated",
        "port_gibs": round(port_gibs, 4), "ref_gibs": round(ref_gibs, 4),
        "port_over_ref": round(port_gibs / ref_gibs, 4),
        "identical_output": same,
        "port": "oracle/rc4_oracle.c (gcc -O3)", "ref": "oracle/_ref/libzrc4_ref.so (g++ -O3, real header)",
        "host": f"build container, {__import__('os').cpu_count()} CPUs",
        "when": time.strftime("%Y-%m-%d"),
    }
    print(json.dumps(out))
    return 0 if same else 1


if __name__ == "__main__":
    sys.exit(main())
