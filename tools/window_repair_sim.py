#!/usr/bin/env python3
"""Speculative RC4 windows that REPAIR stale b reads instead of cutting
(design model, checked bit-exact against a plain PRGA; not built, DESIGN.md
§3.8 says why).

The product rules (tools/window_sim.py) cut a window at the first lane whose
b_l = S0[j_l] is stale.  Two of those cases have a known true value, because
j_l does not depend on b:
  j_l == j_k for an earlier lane k (duplicate j): b_l = a_k of the last such k;
  j_l == i_m, m < l (d_l < l):                    b_l = b_m (true) of lane m.
Only a stale a (an earlier lane's j is my i) cascades, so the window cuts at:
  - a stale a_l; the middle lane of three equal j's (the marker pair lowest /
    highest lane cannot name it); a d-repair whose source lane was itself
    repaired (a chain); the message end.
Keystream of lane l: the last write <= l to t_l = a_l + b_l (a J-write of
the highest / lowest lane with that j, else the i-write of lane t_l - x - 1,
else S0[t_l]); commit: i-writes with the true b, then J-writes by the last
committed writer of each j.

  python tools/window_repair_sim.py      # bit-exact check + bytes per window, W = 16, 32, 64
"""
from __future__ import annotations

import random


def ksa(key):
    S = list(range(256))
    j = 0
    for i in range(256):
        j = (j + S[i] + key[i % len(key)]) & 255
        S[i], S[j] = S[j], S[i]
    return S


def serial(S, x, y, n):
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


def window_repair(S, x, y, n, W):
    S = S[:]
    out = []
    wins = 0
    while len(out) < n:
        rem = n - len(out)
        wins += 1
        i = [(x + 1 + l) & 255 for l in range(W)]
        a = [S[p] for p in i]
        J, acc = [], y
        for l in range(W):
            acc = (acc + a[l]) & 255
            J.append(acc)
        b = [S[p] for p in J]
        d = [(J[l] - x - 1) & 255 for l in range(W)]
        Mlo, Mhi = {}, {}                       # lowest / highest lane per j (the two marker tables)
        for l in range(W):
            Mlo.setdefault(J[l], l)
            Mhi[J[l]] = l
        dup = [Mlo[J[l]] < l for l in range(W)]
        rep = [dup[l] or d[l] < l for l in range(W)]
        flag = [False] * W
        for l in range(W):
            if l >= rem:
                flag[l] = True
            if i[l] in Mlo and Mlo[i[l]] < l:                 # stale a: cascades
                flag[l] = True
            if Mlo[J[l]] < l < Mhi[J[l]]:                     # middle of three
                flag[l] = True
            if not dup[l] and d[l] < l and rep[d[l]]:         # chain
                flag[l] = True
        cut = next((l for l in range(W) if flag[l]), W)
        bt = [0] * W
        for l in range(cut):
            bt[l] = a[Mlo[J[l]]] if dup[l] else (b[d[l]] if d[l] < l else b[l])
        for l in range(cut):
            t = (a[l] + bt[l]) & 255
            lo, hi, e = Mlo.get(t, W), Mhi.get(t, W), (t - x - 1) & 255
            out.append(a[hi] if hi <= l else a[lo] if lo <= l else bt[e] if e <= l else S[t])
        for l in range(cut):
            S[i[l]] = bt[l]
        for l in range(cut):
            if Mhi[J[l]] == l or Mhi[J[l]] >= cut:
                S[J[l]] = a[l]
        x = (x + cut) & 255
        y = J[cut - 1]
    return out, S, x, y, wins


def main():
    rng = random.Random(5)
    for W in (16, 32, 64):
        for t in range(200):
            key = [rng.randrange(256) for _ in range(16)]
            S = ksa(key)
            x, y, n = rng.randrange(256), rng.randrange(256), rng.choice([1, 5, 100, 1000, 3000])
            assert serial(S, x, y, n) == window_repair(S, x, y, n, W)[:4], (W, t)
        tot = tw = 0
        for t in range(20):
            S = ksa([rng.randrange(256) for _ in range(16)])
            r = window_repair(S, rng.randrange(256), rng.randrange(256), 20000, W)
            tot, tw = tot + 20000, tw + r[4]
        print(f"W={W}: bit-exact; {tot / tw:.2f} bytes per window (long messages)")


if __name__ == "__main__":
    main()
