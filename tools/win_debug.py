"""Debug: the window path on a ragged batch; prints per-stream positions of
wrong bytes (stream, position in message, length, lead)."""
import sys
import numpy as np
sys.path.insert(0, "oracle")
sys.path.insert(0, ".")
import pyoracle
import torch
from zsummerx_amd import Context

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4059
mode = sys.argv[2] if len(sys.argv) > 2 else "mixed"
rng = np.random.default_rng(31 + n)
keys = rng.integers(0, 256, 16 * n, dtype=np.uint8)
koff = np.arange(n, dtype=np.uint64) * 16
klen = np.full(n, 16, dtype=np.uint32)
ob = pyoracle.Batch(n)
ob.make_sbox(keys, koff, klen)
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
edges = [0, 1, 15, 16, 17, 31, 32, 33, 255, 256, 1023, 1024, 1025, 2047, 2048, 2049, 4095, 4096, 4097, 5000]
s = torch.cuda.current_stream()
with Context(0, 16 * 256 + 256) as c:
    c.ksa_range(0, T(klen.view(np.int32)), T(koff.view(np.int64)), T(keys), stream=s)
    L = np.where(rng.random(n) < 0.3, np.resize(edges, n), rng.integers(0, 1500, n)).astype(np.uint32)
    if mode == "equal":
        L[:] = 1024
    rng.shuffle(L)
    lead = np.where(np.arange(n) % 2 == 0, 0, rng.integers(1, 16, n)).astype(np.uint64)
    if mode in ("aligned", "equal"):
        lead[:] = 0
    gap = (rng.integers(0, 4, n) * 16).astype(np.uint64)
    seg = ((L.astype(np.uint64) + 15) // 16) * 16 + 16
    base = np.concatenate([[0], np.cumsum(seg + gap)[:-1]]).astype(np.uint64)
    off = base + lead
    data = rng.integers(0, 256, int(base[-1] + seg[-1] + gap[-1]) + 64, dtype=np.uint8)
    want = data.copy()
    ob.crypt(want, off, L, threads=8)
    pay = T(data)
    c.crypt_range(0, pay, T(off.view(np.int64)), T(L.view(np.int32)), stream=s)
    c.sync(s)
    got = pay.cpu().numpy()
    bad = np.flatnonzero(got != want)
    print("mode", mode, "bad bytes", bad.size)
    streams = np.searchsorted(off, bad, side="right") - 1
    from collections import Counter
    cnt = Counter(streams.tolist())
    for st, k in list(cnt.items())[:25]:
        pos = bad[streams == st] - off[st]
        print(f"stream {st} (wave {st // 4}? entry) L={L[st]} lead={lead[st]} bad={k} pos={pos[:12].tolist()}")
    ok_state = 0
    for i in range(n):
        sb, x, y = c.get_state(i)
        wsb, wx, wy = ob.state(i)
        ok_state += (sb, x, y) == (bytes(wsb), wx, wy)
    print("states ok", ok_state, "of", n)
