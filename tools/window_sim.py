#!/usr/bin/env python3
"""Lane-parallel speculative RC4 windows: a CPU model of the rules the
`crypt_win_kernel` runs (design tool; checks itself against a plain PRGA).

RC4 (`depends/rc4/rc4_encryption.h:81-89`) is serial per stream, but over a
short window of W steps the serial dependence is rare: step l reads
a_l = S[x+1+l] and b_l = S[j_l] with j_l = y + a_0 + ... + a_l, and those
reads only differ from reads of the window-start state S0 when an earlier step
of the window wrote the same position.  W lanes therefore run W steps at once
from S0 and commit the longest prefix that provably matches the serial order:

  d_l = (j_l - x - 1) mod 256       (j_l's offset among the window's i's)
  d_l <  l, d_l != l  -> j_l hits an earlier step's i: b_l stale   -> cut <= l
  l < d_l < W         -> j_l hits a later step's i: a_{d_l} stale  -> cut <= d_l
  j_k == j_l, k < l   -> b_l stale                                 -> cut <= l
  cut <= remaining message length

Steps 0..cut-1 touch pairwise distinct positions (apart from i_l == j_l, where
a_l == b_l), so their swaps commute and are written in parallel.  The
keystream byte K_l = S_l[t_l], t_l = a_l + b_l, is S_final[t_l] when t_l was
written by a committed step <= l, else S0[t_l] (a later step's write is
invisible to step l, and positions are written at most once).  Neither read
is on the window-to-window path.

Run: python tools/window_sim.py [--w 8] [--streams 64] [--len 4096]
"""
from __future__ import annotations

import argparse
import random


def ksa(key: bytes):
    S = list(range(256))
    j = 0
    for i in range(256):
        j = (j + S[i] + (key[i % len(key)] if key else 0)) & 255
        S[i], S[j] = S[j], S[i]
    return S


def prga_serial(S, x, y, n):
    S = S[:]
    out = []
    for _ in range(n):
        x = (x + 1) & 255
        a = S[x]
        y = (y + a) & 255
        b = S[y]
        S[x], S[y] = b, a
        out.append(S[(a + b) & 255])
    return out, S, x, y


def prga_window(S, x, y, n, W=8):
    """Returns keystream, final S/x/y and the number of windows taken."""
    S = S[:]
    out = []
    windows = 0
    while len(out) < n:
        windows += 1
        S0 = S[:]
        i = [(x + 1 + l) & 255 for l in range(W)]
        a = [S0[p] for p in i]
        j = []
        acc = y
        for l in range(W):
            acc = (acc + a[l]) & 255
            j.append(acc)
        b = [S0[p] for p in j]
        cut = min(W, n - len(out))
        for l in range(W):
            d = (j[l] - x - 1) & 255
            if d < l:
                cut = min(cut, l)
            elif l < d < W:
                cut = min(cut, d)
            for k in range(l):
                if j[k] == j[l]:
                    cut = min(cut, l)
        assert cut >= 1
        for l in range(cut):          # parallel commit (positions disjoint)
            S[i[l]] = b[l]
        for l in range(cut):
            S[j[l]] = a[l]
        for l in range(cut):
            t = (a[l] + b[l]) & 255
            e = (t - x - 1) & 255
            own = e <= l or any(j[k] == t for k in range(l + 1))
            out.append(S[t] if own else S0[t])
        x = (x + cut) & 255
        y = j[cut - 1]
    return out, S, x, y, windows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--w", type=int, default=8)
    ap.add_argument("--streams", type=int, default=64)
    ap.add_argument("--len", type=int, default=4096)
    ap.add_argument("--seed", type=int, default=1)
    args = ap.parse_args()
    rng = random.Random(args.seed)
    tot_bytes = tot_win = 0
    for s in range(args.streams):
        key = bytes(rng.randrange(256) for _ in range(rng.randrange(0, 40)))
        S = ksa(key)
        x = y = 0
        # resume mid-stream too: a few serial bytes first
        pre = rng.randrange(0, 300)
        _, S, x, y = prga_serial(S, x, y, pre)
        want, Sw, xw, yw = prga_serial(S, x, y, args.len)
        got, Sg, xg, yg, nw = prga_window(S, x, y, args.len, args.w)
        assert got == want, f"stream {s}: keystream differs"
        assert (Sg, xg, yg) == (Sw, xw, yw), f"stream {s}: state differs"
        tot_bytes += args.len
        tot_win += nw
    print(f"W={args.w}: bit-exact over {args.streams} streams x {args.len} B; "
          f"{tot_bytes / tot_win:.3f} bytes per window")


if __name__ == "__main__":
    main()
