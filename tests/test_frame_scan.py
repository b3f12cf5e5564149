"""Device-side proto4z framing: zrc4_frame_scan walks
decrypted session buffers exactly as TcpSession::onRecv's framing loop
(src/frame/session.cpp:329-371) drives HasRawPacket
(depends/proto4z/proto4z.h:704-748).

Pinned by tests/golden/frame.json, generated from the REAL reference
HasRawPacket compiled from /root/reference (oracle/ref_shim.cpp)."""
import random
import struct

import numpy as np
import pytest

import pyoracle
from conftest import soak_seeds

BOUND = 20480



def payload_report(got, want, off, ln):
    """'' when the buffers match; else the count of differing bytes, the
    first offsets and the sessions (entries) they fall in, with each one's
    [off, off + len) span -- enough to tell a stray store from a wrong
    keystream after one failing run (no reruns to reproduce)."""
    bad = np.flatnonzero(got != want)
    if bad.size == 0:
        return ""
    off = np.asarray(off, dtype=np.int64)
    ln = np.asarray(ln, dtype=np.int64)
    order = np.argsort(off, kind="stable")
    ent = order[np.clip(np.searchsorted(off[order], bad[:16], side="right") - 1, 0, len(off) - 1)]
    inside = (bad[:16] >= off[ent]) & (bad[:16] < off[ent] + ln[ent])
    sess = sorted(set(int(e) for e in ent))
    return (f"{bad.size} bytes differ; first offsets {bad[:16].tolist()}; entries {ent.tolist()} "
            f"(inside their span: {inside.tolist()}); {len(np.unique(ent))} distinct among the first 16; "
            f"spans {[(int(off[e]), int(off[e] + ln[e])) for e in sess[:4]]}; "
            f"got {got[bad[:8]].tolist()} want {want[bad[:8]].tolist()}")


def frame_report(w, g, name):
    """'' when a framing output matches; else where it differs."""
    w, g = np.asarray(w), np.asarray(g)
    if np.array_equal(w, g):
        return ""
    rows = np.flatnonzero((w != g).reshape(len(w), -1).any(axis=1))
    return (f"{name}: {rows.size} entries differ, first {rows[:8].tolist()}: "
            f"want {w[rows[:4]].tolist()} got {g[rows[:4]].tolist()}")

def pack_cases(frame_golden):
    cases = frame_golden["cases"]
    datas = [bytes.fromhex(c["data"]) for c in cases]
    off = np.zeros(len(datas), dtype=np.uint64)
    acc = 0
    for i, d in enumerate(datas):
        off[i] = acc
        acc += len(d) + 3                       # odd spacing: headers land at every alignment
    buf = np.zeros(acc + 8, dtype=np.uint8)
    for i, d in enumerate(datas):
        buf[int(off[i]):int(off[i]) + len(d)] = np.frombuffer(d, np.uint8)
    return cases, buf, off, np.array([len(d) for d in datas], dtype=np.uint32)


def packet_streams(n, avg_len, seed, max_pk=4000):
    """n session buffers of proto4z packets, each ending in a partial packet
    or exactly, plus a few corrupt ones."""
    rng = random.Random(seed)
    bufs = []
    for i in range(n):
        out = bytearray()
        target = rng.randint(0, 2 * avg_len)
        while len(out) < target:
            ln = rng.choice([6, 8, 9, 33, 64, 200, 700, rng.randint(6, max_pk)])
            out += struct.pack("<IHH", ln, 0, 7)[: min(8, ln)] + bytes(max(0, ln - 8))
        cut = len(out) - rng.randint(0, 20) if out and rng.random() < 0.7 else len(out)
        b = bytes(out[:max(cut, 0)])
        if rng.random() < 0.05 and len(b) > 10:           # corrupt a length field
            b = struct.pack("<I", rng.choice([0, 3, 5, 30000, 1 << 30])) + b[4:]
        bufs.append(b[:BOUND])
    off = np.zeros(n, dtype=np.uint64)
    acc = 0
    for i, b in enumerate(bufs):
        off[i] = acc
        acc += len(b) + (i % 5)
    buf = np.zeros(acc + 8, dtype=np.uint8)
    for i, b in enumerate(bufs):
        buf[int(off[i]):int(off[i]) + len(b)] = np.frombuffer(b, np.uint8)
    return buf, off, np.array([len(b) for b in bufs], dtype=np.uint32)


@pytest.fixture(scope="module")
def frame_golden():
    import json
    from conftest import GOLDEN
    return json.loads((GOLDEN / "frame.json").read_text())


# ------------------------------------------------------------------ CPU
def test_oracle_scan_matches_reference_fixtures(frame_golden):
    cases, buf, off, ln = pack_cases(frame_golden)
    npk, used, status, pk = pyoracle.frame_scan(buf, off, ln, BOUND, 16)
    for i, c in enumerate(cases):
        if c["bound"] != BOUND:
            continue
        assert (int(npk[i]), int(used[i]), int(status[i])) == (len(c["packets"]), c["used"], c["status"]), c["name"]
        assert list(pk[i][: min(16, len(c["packets"]))]) == c["packets"][:16], c["name"]


def test_py_restatement_matches_reference_fixtures(frame_golden):
    for c in frame_golden["cases"]:
        assert pyoracle.py_frame_scan(bytes.fromhex(c["data"]), c["bound"]) == (c["packets"], c["used"], c["status"])


def test_oracle_scan_matches_real_reference_random():
    if pyoracle.ref_lib() is None:
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    buf, off, ln = packet_streams(300, 1500, seed=3)
    npk, used, status, pk = pyoracle.frame_scan(buf, off, ln, BOUND, 64)
    for i in range(300):
        data = buf[int(off[i]):int(off[i]) + int(ln[i])].tobytes()
        pkts, u, st = pyoracle.ref_frame_scan(data, BOUND)
        assert (int(npk[i]), int(used[i]), int(status[i])) == (len(pkts), u, st)
        assert list(pk[i][: min(64, len(pkts))]) == pkts[:64]


# ------------------------------------------------------------------ GPU
def device_scan(torch, c, buf, off, ln, bound, maxp):
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to("cuda")
    n = ln.size
    npk, used, status = (torch.zeros(n, dtype=torch.int32, device="cuda") for _ in range(3))
    pk = torch.zeros(max(1, n * maxp), dtype=torch.int32, device="cuda")
    c.frame_scan(T(buf), T(off.view(np.int64)), T(ln.view(np.int32)), bound, npk, used, status,
                 pk if maxp else None, maxp)
    c.sync()
    return (npk.cpu().numpy().view(np.uint32), used.cpu().numpy().view(np.uint32),
            status.cpu().numpy().view(np.uint32), pk.cpu().numpy().view(np.uint32)[: n * maxp].reshape(n, maxp))


@pytest.mark.gpu
def test_device_scan_matches_reference_fixtures(built, frame_golden):
    import torch
    from zsummerx_amd import Context
    cases, buf, off, ln = pack_cases(frame_golden)
    with Context(0, 256) as c:
        for bound in sorted({cs["bound"] for cs in cases}):
            idx = [i for i, cs in enumerate(cases) if cs["bound"] == bound]
            npk, used, status, pk = device_scan(torch, c, buf, off[idx], ln[idx], bound, 16)
            for j, i in enumerate(idx):
                cs = cases[i]
                assert (int(npk[j]), int(used[j]), int(status[j])) == (len(cs["packets"]), cs["used"], cs["status"]), cs["name"]
                assert list(pk[j][: min(16, len(cs["packets"]))]) == cs["packets"][:16], cs["name"]


@pytest.mark.gpu
@pytest.mark.parametrize("n,avg,maxp", [(4096, 1024, 8), (65536, 256, 4), (1024, 16384, 64)])
def test_device_scan_matches_oracle_at_baseline_shapes(built, n, avg, maxp):
    import torch
    from zsummerx_amd import Context
    buf, off, ln = packet_streams(n, avg, seed=n)
    want = pyoracle.frame_scan(buf, off, ln, BOUND, maxp)
    with Context(0, 256) as c:
        got = device_scan(torch, c, buf, off, ln, BOUND, maxp)
    for w, g, name in zip(want, got, ["npk", "used", "status", "pkt_len"]):
        msg = frame_report(w, g, name)
        assert not msg, msg


@pytest.mark.gpu
def test_decrypt_then_scan_pipeline(built):
    """Ciphertext (oracle RC4 over packet streams) -> zrc4_crypt on the GPU ->
    zrc4_frame_scan on the GPU, against the oracle doing both on the CPU."""
    import torch
    from zsummerx_amd import Context
    n = 2048
    buf, off, ln = packet_streams(n, 900, seed=11)
    rng = np.random.default_rng(2)
    keys = [rng.integers(0, 256, 16, dtype=np.uint8).tobytes() for _ in range(n)]
    ct = buf.copy()
    for i in range(n):
        a, z = int(off[i]), int(off[i]) + int(ln[i])
        ct[a:z] = np.frombuffer(pyoracle.Rc4(keys[i]).encryption(ct[a:z].tobytes()), np.uint8)
    want = pyoracle.frame_scan(buf, off, ln, BOUND, 8)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to("cuda")
    with Context(0, n) as c:
        c.ksa_host(keys)
        d = T(ct)
        d_off, d_len = T(off.view(np.int64)), T(ln.view(np.int32))
        c.crypt(d, d_off, d_len)
        npk, used, status = (torch.zeros(n, dtype=torch.int32, device="cuda") for _ in range(3))
        pk = torch.zeros(n * 8, dtype=torch.int32, device="cuda")
        c.frame_scan(d, d_off, d_len, BOUND, npk, used, status, pk, 8)
        c.sync()
        msg = payload_report(d.cpu().numpy(), buf, off, ln)
        assert not msg, msg
        got = (npk.cpu().numpy().view(np.uint32), used.cpu().numpy().view(np.uint32),
               status.cpu().numpy().view(np.uint32), pk.cpu().numpy().view(np.uint32).reshape(n, 8))
    for w, g, name in zip(want, got, ["npk", "used", "status", "pkt_len"]):
        msg = frame_report(w, g, name)
        assert not msg, msg


def _fused_case(n, avg, seed, tail_frac=0.5):
    """Receive blocks as onRecv sees them: the first part of each block was
    decrypted by an earlier iteration (plaintext already), the rest is the
    fresh ciphertext tail (session.cpp:315-323).  Returns plaintext blocks,
    the device input, the decrypt spans and the per-session keys."""
    buf, off, ln = packet_streams(n, avg, seed=seed)
    rng = np.random.default_rng(seed)
    keys = [rng.integers(0, 256, 16, dtype=np.uint8).tobytes() for _ in range(n)]
    head = (ln * rng.uniform(0, tail_frac, n)).astype(np.uint32)      # already-decrypted prefix
    inp = buf.copy()
    for i in range(n):
        a, z = int(off[i] + head[i]), int(off[i] + ln[i])
        inp[a:z] = np.frombuffer(pyoracle.Rc4(keys[i]).encryption(inp[a:z].tobytes()), np.uint8)
    return buf, inp, off, ln, off + head, ln - head, keys


@pytest.mark.gpu
@pytest.mark.parametrize("n,avg,mode", [(4096, 900, "range"), (1000, 3000, "grouped"), (70000, 200, "range"),
                                        (150000, 200, "grouped"), (600000, 40, "range"), (600000, 40, "grouped"),
                                        (1000, 3000, "declared"), (25000, 300, "declared"), (40000, 300, "declared"),
                                        (150000, 200, "declared"), (600001, 40, "range"), (333333, 48, "range")])
def test_fused_decrypt_and_frame(built, n, avg, mode):
    """zrc4_crypt_*_frame: decrypt the fresh tail and frame the WHOLE block in
    one launch: the direct kernels' epilogue at <= 1 group per CU, the
    persistent kernel's tail above (70 000 / 150 000 sessions: 274 / 587
    groups, one or two chunks per workgroup; 600 000: 2 344 groups, five
    chunks per workgroup, the tail's four-walk lockstep plus a remainder;
    r06: 600 001 -- the round-5 red shape with other inputs and a last group
    of one session -- and 333 333, 1 303 groups with a 21-session tail).
    declared: zrc4_crypt_grouped_declared with framing, the engine's call --
    6 buckets on the window kernel, ~100 and ~159 on crypt_decl_kernel
    (half- and whole-group), ~587 behind the declared check on the
    persistent kernel.  Plaintext and framing
    against the oracle."""
    _run_fused(n, avg, mode, seed=n + avg)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", soak_seeds())
def test_fused_decrypt_and_frame_soak(built, seed):
    """A random fused decrypt+frame case per seed (one by default;
    scripts/r06_soak.sh runs many through $ZRC4_SOAK_SEEDS): entry point,
    session count on either side of every launch_crypt boundary (window,
    half-group, whole-group, persistent with one to several chunks per
    workgroup, ragged last groups), packet size, and how much of each block
    an earlier iteration already decrypted."""
    rng = np.random.default_rng(7000 + seed)
    mode = ["range", "grouped", "declared"][int(rng.integers(0, 3))]
    cls = int(rng.integers(0, 4))
    n = int(rng.integers(*[(1, 8193), (8193, 32769), (32769, 65537), (65537, 300001)][cls]))
    avg = int(rng.choice([40, 200, 900, 3000]))
    avg = min(avg, max(40, 24_000_000 // n))              # <= ~48 MB of packets
    tail = float(rng.choice([0.0, 0.5, 1.0]))
    _run_fused(n, avg, mode, seed=seed, tail_frac=tail)


def _run_fused(n, avg, mode, seed, tail_frac=0.5):
    import torch
    from zsummerx_amd import Context
    from zsummerx_amd._capi import IDLE_SLOT
    maxp = 8
    buf, inp, off, ln, toff, tlen, keys = _fused_case(n, avg, seed=seed, tail_frac=tail_frac)
    want = pyoracle.frame_scan(buf, off, ln, BOUND, maxp)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to("cuda")
    npk, used, status = (torch.zeros(n, dtype=torch.int32, device="cuda") for _ in range(3))
    pk = torch.zeros(n * maxp, dtype=torch.int32, device="cuda")
    d = T(inp)
    frame = {"off": T(off.view(np.int64)), "len": T(ln.view(np.int32)), "bound": BOUND, "max_packets": maxp,
             "npk": npk, "used": used, "status": status, "pkt_len": pk}
    with Context(0, n + 512) as c:
        if mode == "range":
            c.ksa_host(keys)
            c.crypt_range_frame(0, d, T(toff.view(np.int64)), T(tlen.view(np.int32)), frame)
        else:
            # slots scattered over groups, entries bucketed by group (zrc4_crypt_grouped contract)
            rng = np.random.default_rng(5)
            slots = rng.permutation(n + 512)[:n].astype(np.uint32)
            c.ksa_host(keys, ids=slots)
            order = np.argsort(slots, kind="stable")
            ids, eo, el, fo, fl, back = [], [], [], [], [], []
            cur = None
            for i in order:
                g = int(slots[i]) // 256
                if g != cur:
                    while len(ids) % 256:
                        ids.append(IDLE_SLOT); eo.append(0); el.append(0); fo.append(0); fl.append(0); back.append(-1)
                    cur = g
                ids.append(int(slots[i])); eo.append(int(toff[i])); el.append(int(tlen[i]))
                fo.append(int(off[i])); fl.append(int(ln[i])); back.append(int(i))
            m = len(ids)
            npk, used, status = (torch.zeros(m, dtype=torch.int32, device="cuda") for _ in range(3))
            pk = torch.zeros(m * maxp, dtype=torch.int32, device="cuda")
            frame.update(off=T(np.array(fo, np.uint64).view(np.int64)), len=T(np.array(fl, np.uint32).view(np.int32)),
                         npk=npk, used=used, status=status, pkt_len=pk)
            args = (d, T(np.array(eo, np.uint64).view(np.int64)), T(np.array(el, np.uint32).view(np.int32)),
                    T(np.array(ids, np.uint32).view(np.int32)))
            if mode == "declared":
                ida = np.full(-(-len(ids) // 256) * 256, IDLE_SLOT, np.uint32)    # (the last bucket is short)
                ida[:len(ids)] = ids
                ida = ida.reshape(-1, 256)
                groups = np.where((ida != IDLE_SLOT).any(axis=1), ida.min(axis=1) // 256, IDLE_SLOT).astype(np.uint32)
                c.crypt_grouped_declared(*args, groups, frame=frame)
            else:
                c.crypt_grouped_frame(*args, frame)
        c.sync()
        msg = payload_report(d.cpu().numpy(), buf, toff, tlen)
        assert not msg, f"{mode} n={n}: {msg}"
        got = [npk.cpu().numpy().view(np.uint32), used.cpu().numpy().view(np.uint32),
               status.cpu().numpy().view(np.uint32), pk.cpu().numpy().view(np.uint32).reshape(-1, maxp)]
        if mode != "range":
            back = np.array(back)
            sel = back >= 0
            perm = np.empty(n, dtype=np.int64)
            perm[back[sel]] = np.flatnonzero(sel)
            got = [g[perm] for g in got]
    for w, g, name in zip(want, got, ["npk", "used", "status", "pkt_len"]):
        msg = frame_report(w, g, name)
        assert not msg, f"{mode} n={n}: {msg}"
