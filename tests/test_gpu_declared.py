"""GPU parity of zrc4_crypt_grouped_declared (include/zrc4.h): grouped batches
whose buckets' groups the caller declares from the host, as the session
engine and zrc4_crypt_host do (they bucket the ids on the host).  The
reference runs one RC4Encryption::encryption per session per event-loop
iteration (src/frame/session.cpp:313-323, depends/rc4/rc4_encryption.h:74-93);
the batch must equal those calls byte for byte, and a bucket whose ids
disagree with its declared group must write nothing.  Checked against the
oracle (oracle/rc4_oracle.c), every payload byte and every state."""
import numpy as np
import pytest

import pyoracle
from zsummerx_amd import Context, ZRC4Error
from zsummerx_amd._capi import IDLE_SLOT

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    return torch


def _seeded(torch, rng, cap):
    keys = rng.integers(0, 256, 16 * cap, dtype=np.uint8)
    koff = np.arange(cap, dtype=np.uint64) * 16
    klen = np.full(cap, 16, dtype=np.uint32)
    ob = pyoracle.Batch(cap)
    ob.make_sbox(keys, koff, klen)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    c = Context(0, cap)
    c.ksa_range(0, T(klen.view(np.int32)), T(koff.view(np.int64)), T(keys), stream=torch.cuda.current_stream())
    return c, ob, T


def _buckets(rng, groups, fill=(1, 256)):
    """Bucket b: a random subset of group groups[b]'s slots in random entry
    positions (IDLE_SLOT elsewhere); groups[b] == IDLE_SLOT: an idle bucket."""
    ids = np.full(256 * len(groups), IDLE_SLOT, dtype=np.uint32)
    for b, g in enumerate(groups):
        if g == IDLE_SLOT:
            continue
        k = int(rng.integers(fill[0], fill[1] + 1))
        ids[256 * b + rng.permutation(256)[:k]] = int(g) * 256 + rng.permutation(256)[:k]
    return ids


def _oracle_crypt(ob, data, ids, off, L, skip=()):
    want = data.copy()
    for e in np.flatnonzero(ids != IDLE_SLOT):
        if int(ids[e]) // 256 in skip:
            continue
        pyoracle.lib().oracle_encryption(pyoracle.C.byref(ob.st[int(ids[e])]),
                                         pyoracle.C.c_void_p(want.ctypes.data + int(off[e])), int(L[e]))
    return want


def _check_states(c, ob, cap):
    gsb, gx, gy = c.get_states(0, cap)
    osb, ox, oy = ob.states()
    bad = np.flatnonzero((gsb != osb).any(axis=1) | (gx != ox) | (gy != oy))
    assert bad.size == 0, bad[:8]


@pytest.mark.parametrize("nb,trunc,idle", [(16, 0, 0), (27, 11, 0.2), (32, 0, 0), (100, 0, 0.1), (200, 5, 0.1),
                                           (256, 0, 0), (300, 37, 0), (700, 0, 0.05)])
def test_declared_bit_exact(built, torch_cuda, nb, trunc, idle):
    """nb <= 32: the window kernel with the groups in its arguments (16 and 32
    buckets: every column of a bucket on one XCD; 27: spread); 100: the
    half-group kernel and 200 / 256 the whole-group kernel, the groups in
    their arguments too (crypt_decl_kernel); 300 / 700: the persistent kernel
    behind the declared check.  Idle buckets declared ZRC4_IDLE_SLOT, a truncated last bucket,
    two calls in a row, every state checked (slots outside the calls keep
    theirs)."""
    torch = torch_cuda
    rng = np.random.default_rng(900 + nb + trunc)
    G = max(256, nb + 40)
    cap = 256 * G
    c, ob, T = _seeded(torch, rng, cap)
    s = torch.cuda.current_stream()
    with c:
        for call in range(2):
            groups = rng.permutation(G)[:nb].astype(np.uint32)
            if idle:
                groups[:-1][rng.random(nb - 1) < idle] = IDLE_SLOT
            ids = _buckets(rng, groups)
            if trunc:                                           # a short last bucket
                ids = ids[:ids.size - trunc].copy()
            busy = ids != IDLE_SLOT
            L = np.where(busy, rng.integers(0, 688, ids.size), 0).astype(np.uint32)   # 16 + 688 <= 704: no overlap
            off = np.arange(ids.size, dtype=np.uint64) * 704 + rng.integers(0, 16, ids.size).astype(np.uint64)
            data = rng.integers(0, 256, ids.size * 704 + 64, dtype=np.uint8)
            want = _oracle_crypt(ob, data, ids, off, L)
            pay = T(data)
            c.crypt_grouped_declared(pay, T(off.view(np.int64)), T(L.view(np.int32)), T(ids.view(np.int32)),
                                     groups, stream=s)
            c.sync(s)
            got = pay.cpu().numpy()
            bad = np.flatnonzero(got != want)
            assert bad.size == 0, (call, bad[:8], int(bad.size))
        _check_states(c, ob, cap)


@pytest.mark.parametrize("nb", [20, 100, 200, 700])
def test_declared_mismatch_is_refused(built, torch_cuda, nb):
    """Bucket 2 declares group A but its ids all lie in group H (named by no
    other bucket); bucket 5 is declared idle but holds a busy entry of group
    H2.  Both are refused: ZRC4_ERR_GROUP, no payload byte and no state of
    theirs touched; every other bucket is bit-exact."""
    torch = torch_cuda
    rng = np.random.default_rng(1200 + nb)
    G = max(256, nb + 40)
    cap = 256 * G
    c, ob, T = _seeded(torch, rng, cap)
    s = torch.cuda.current_stream()
    with c:
        perm = rng.permutation(G)
        groups = perm[:nb].astype(np.uint32)
        H, H2 = int(perm[nb]), int(perm[nb + 1])          # groups no bucket declares
        ids = _buckets(rng, groups)
        ids[256 * 2: 256 * 3] = IDLE_SLOT
        ids[256 * 2 + rng.permutation(256)[:50]] = H * 256 + rng.permutation(256)[:50]
        groups[5] = IDLE_SLOT
        ids[256 * 5: 256 * 6] = IDLE_SLOT
        ids[256 * 5 + 9] = H2 * 256 + 3
        busy = ids != IDLE_SLOT
        L = np.where(busy, rng.integers(1, 400, ids.size), 0).astype(np.uint32)
        off = np.arange(ids.size, dtype=np.uint64) * 400
        data = rng.integers(0, 256, ids.size * 400, dtype=np.uint8)
        want = _oracle_crypt(ob, data, ids, off, L, skip=(H, H2))
        pay = T(data)
        c.crypt_grouped_declared(pay, T(off.view(np.int64)), T(L.view(np.int32)), T(ids.view(np.int32)),
                                 groups, stream=s)
        with pytest.raises(ZRC4Error) as ei:
            c.sync(s)
        assert ei.value.code == -7                           # ZRC4_ERR_GROUP
        got = pay.cpu().numpy()
        bad = np.flatnonzero(got != want)
        assert bad.size == 0, (bad[:8], int(bad.size))
        _check_states(c, ob, cap)                            # H, H2 states unchanged (oracle skipped them)


@pytest.mark.parametrize("nb", [20, 100, 200, 700])
def test_declared_mismatch_blocks_named_group_above_window(built, torch_cuda, nb):
    """A bucket declared A whose ids lie in group B, while another bucket
    legitimately declares B.  Launches of at most 256 buckets (the groups in
    the kernel arguments) refuse only the disagreeing bucket; larger launches
    (the declared check before the crypt launch) refuse both, as for two
    buckets naming one group (include/zrc4.h).  Nothing is half-crypted
    either way."""
    torch = torch_cuda
    rng = np.random.default_rng(1300 + nb)
    G = max(256, nb + 40)
    cap = 256 * G
    c, ob, T = _seeded(torch, rng, cap)
    s = torch.cuda.current_stream()
    with c:
        groups = rng.permutation(G)[:nb].astype(np.uint32)
        ids = _buckets(rng, groups, fill=(100, 200))
        B = int(groups[7])
        ids[256 * 3: 256 * 4] = IDLE_SLOT                     # bucket 3 (declared groups[3]) names B's slots
        used7 = set(int(v) for v in ids[256 * 7: 256 * 8] if v != IDLE_SLOT)
        free = [B * 256 + k for k in range(256) if B * 256 + k not in used7][:40]
        ids[256 * 3: 256 * 3 + len(free)] = free
        busy = ids != IDLE_SLOT
        L = np.where(busy, rng.integers(1, 300, ids.size), 0).astype(np.uint32)
        off = np.arange(ids.size, dtype=np.uint64) * 300
        data = rng.integers(0, 256, ids.size * 300, dtype=np.uint8)
        pay = T(data)
        c.crypt_grouped_declared(pay, T(off.view(np.int64)), T(L.view(np.int32)), T(ids.view(np.int32)),
                                 groups, stream=s)
        with pytest.raises(ZRC4Error) as ei:
            c.sync(s)
        assert ei.value.code == -7
        got = pay.cpu().numpy()
        # bucket 3 never runs; bucket 7 runs unless the launch is checked up front
        skip_entries = set(range(256 * 3, 256 * 4)) | (set() if nb <= 256 else set(range(256 * 7, 256 * 8)))
        keep = ids.copy()
        keep[list(skip_entries)] = IDLE_SLOT
        want = _oracle_crypt(ob, data, keep, off, L)
        bad = np.flatnonzero(got != want)
        assert bad.size == 0, (bad[:8], int(bad.size))
        _check_states(c, ob, cap)


def test_declared_argument_checks(built, torch_cuda):
    """A declared group past the arena is refused on the host (nothing
    launched); a NULL group array is refused."""
    torch = torch_cuda
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    with Context(0, 1024) as c:
        ids = T(np.arange(256, dtype=np.int32))
        pay = T(np.zeros(256 * 8, dtype=np.uint8))
        off = T(np.arange(256, dtype=np.int64) * 8)
        ln = T(np.full(256, 8, dtype=np.int32))
        with pytest.raises(ZRC4Error) as ei:
            c.crypt_grouped_declared(pay, off, ln, ids, np.array([4], dtype=np.uint32))
        assert ei.value.code == -1
        assert not pay.cpu().numpy().any()
        rc = c._lib.zrc4_crypt_grouped_declared(c._h, None, None, None, None, None, 256, None, None)
        assert rc == -1
        c.crypt_grouped_declared(pay, off, ln, ids, np.array([0], dtype=np.uint32))
        c.sync()
        ks = pyoracle.Rc4(b"").encryption(bytes(8))           # fresh slots: the empty-key state
        assert pay.cpu().numpy()[:8].tobytes() == ks


def _claim_part(nb, cus, j):
    """The part of a group a declared launch of nb buckets claims for group
    lane j (zrc4_kernels.hpp Claim): the window kernel (nb <= 32) claims the
    dword column q = col(j) >> 2, the half-group kernel (2 nb <= CUs) and the
    persistent kernel (nb > CUs, wave-pair halves) the half j >> 7, the
    whole-group kernel the whole group (part 0)."""
    if nb <= 32:
        return (j & 31) | ((j >> 7) << 5)
    if 2 * nb <= cus or nb > cus:
        return j >> 7
    return 0


@pytest.mark.parametrize("nb", [20, 100, 200, 700])
def test_declared_two_buckets_one_group(built, torch_cuda, nb):
    """two buckets of one declared launch both (correctly) declare
    group A, with disjoint slots of it.  The claims (one per part of the
    group, include/zrc4.h) let exactly one of the two buckets run each part:
    every entry of the pair is crypted whole or not at all, no part has
    crypted entries of both buckets, and ZRC4_ERR_GROUP is latched.  Above
    256 buckets the declared check before the crypt passes both (they agree
    with their declarations) and the persistent kernel's claims decide, per
    wave-pair half.  Every other bucket, and every state, matches the
    oracle."""
    torch = torch_cuda
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    rng = np.random.default_rng(1400 + nb)
    G = max(256, nb + 40)
    cap = 256 * G
    c, ob, T = _seeded(torch, rng, cap)
    s = torch.cuda.current_stream()
    with c:
        groups = rng.permutation(G)[:nb].astype(np.uint32)
        A = int(groups[4])
        groups[9] = A                                          # bucket 9 declares A too
        ids = _buckets(rng, groups)
        lanes = rng.permutation(256)
        for b, half in ((4, lanes[:128]), (9, lanes[128:])):  # disjoint slots of A, spread over every part
            ids[256 * b: 256 * (b + 1)] = IDLE_SLOT
            ids[256 * b + rng.permutation(256)[:half.size]] = A * 256 + half
        busy = ids != IDLE_SLOT
        L = np.where(busy, rng.integers(8, 300, ids.size), 0).astype(np.uint32)
        off = np.arange(ids.size, dtype=np.uint64) * 300
        data = rng.integers(0, 256, ids.size * 300, dtype=np.uint8)
        allc = _oracle_crypt(pyoracle_batch_copy(ob, cap), data, ids, off, L)   # every entry crypted
        pay = T(data)
        c.crypt_grouped_declared(pay, T(off.view(np.int64)), T(L.view(np.int32)), T(ids.view(np.int32)),
                                 groups, stream=s)
        with pytest.raises(ZRC4Error) as ei:
            c.sync(s)
        assert ei.value.code == -7                           # ZRC4_ERR_GROUP
        got = pay.cpu().numpy()
        ran = {}
        for b in (4, 9):
            for e in range(256 * b, 256 * (b + 1)):
                if ids[e] == IDLE_SLOT:
                    continue
                a, z = int(off[e]), int(off[e] + L[e])
                if np.array_equal(got[a:z], allc[a:z]):
                    ran[e] = True
                elif np.array_equal(got[a:z], data[a:z]):
                    ran[e] = False
                else:
                    raise AssertionError(f"entry {e} (bucket {b}) half-crypted")
        parts = {}
        for e, r in ran.items():
            if r:
                parts.setdefault(_claim_part(nb, cus, int(ids[e]) & 255), set()).add(e // 256)
        both = {p: bs for p, bs in parts.items() if len(bs) > 1}
        assert not both, f"parts crypted by both buckets: {both}"
        assert any(ran.values()), "one bucket runs each part it wins"
        keep = ids.copy()
        for e, r in ran.items():
            if not r:
                keep[e] = IDLE_SLOT
        want = _oracle_crypt(ob, data, keep, off, L)
        bad = np.flatnonzero(got != want)
        assert bad.size == 0, (bad[:8], int(bad.size))
        _check_states(c, ob, cap)


def pyoracle_batch_copy(ob, cap):
    """A second oracle batch with the same states (the all-crypted reference
    must not advance the states the final check compares against)."""
    cp = pyoracle.Batch(cap)
    pyoracle.C.memmove(cp.st, ob.st, pyoracle.C.sizeof(ob.st))
    return cp


@pytest.mark.parametrize("nb", [20, 100, 200, 700])
def test_declared_refused_bucket_frames_nothing(built, torch_cuda, nb):
    """with framing, a refused declared bucket decrypts nothing
    and never frames a busy entry over its undecrypted bytes, whether it is
    refused for ids outside its declared group (bucket 2) or for a busy
    entry in a bucket declared idle (bucket 5; on the declared kernels that
    one reached the idle-bucket branch, which framed every entry).  The rest
    of a refused bucket's framing outputs is unspecified (include/zrc4.h).
    Every other entry, idle ones included, is framed as the oracle frames
    the expected buffer.  700 buckets run the persistent kernel, whose tail
    walks every chunk: there only the other buckets are checked."""
    torch = torch_cuda
    rng = np.random.default_rng(1500 + nb)
    G = max(256, nb + 40)
    cap = 256 * G
    c, ob, T = _seeded(torch, rng, cap)
    s = torch.cuda.current_stream()
    with c:
        perm = rng.permutation(G)
        groups = perm[:nb].astype(np.uint32)
        H, H2 = int(perm[nb]), int(perm[nb + 1])
        ids = _buckets(rng, groups)
        ids[256 * 2: 256 * 3] = IDLE_SLOT
        ids[256 * 2 + rng.permutation(256)[:50]] = H * 256 + rng.permutation(256)[:50]
        groups[5] = IDLE_SLOT
        ids[256 * 5: 256 * 6] = IDLE_SLOT
        ids[256 * 5 + 9] = H2 * 256 + 3
        groups[11] = IDLE_SLOT                            # a genuinely idle bucket: framed raw
        ids[256 * 11: 256 * 12] = IDLE_SLOT
        busy = ids != IDLE_SLOT
        L = np.where(busy, rng.integers(1, 400, ids.size), rng.integers(0, 40, ids.size)).astype(np.uint32)
        off = np.arange(ids.size, dtype=np.uint64) * 400
        data = rng.integers(0, 256, ids.size * 400, dtype=np.uint8)
        # proto4z-looking headers at the span starts, so walks go past the first packet
        for e in range(0, ids.size, 3):
            data[int(off[e]): int(off[e]) + 4] = np.frombuffer(int(rng.integers(6, 120)).to_bytes(4, "little"), np.uint8)
        want = _oracle_crypt(ob, data, ids, off, L, skip=(H, H2))
        maxp = 4
        sentinel = np.uint32(0xFFFFFFFF)
        npk, used, status = (T(np.full(ids.size, sentinel, dtype=np.uint32).view(np.int32)) for _ in range(3))
        pk = T(np.zeros(ids.size * maxp, dtype=np.int32))
        frame = {"off": T(off.view(np.int64)), "len": T(L.view(np.int32)), "bound": 20480, "max_packets": maxp,
                 "npk": npk, "used": used, "status": status, "pkt_len": pk}
        pay = T(data)
        c.crypt_grouped_declared(pay, T(off.view(np.int64)), T(L.view(np.int32)), T(ids.view(np.int32)),
                                 groups, frame=frame, stream=s)
        with pytest.raises(ZRC4Error) as ei:
            c.sync(s)
        assert ei.value.code == -7
        got = pay.cpu().numpy()
        bad = np.flatnonzero(got != want)
        assert bad.size == 0, (bad[:8], int(bad.size))
        g_npk, g_used, g_st = (t.cpu().numpy().view(np.uint32) for t in (npk, used, status))
        refused = np.zeros(ids.size, dtype=bool)
        refused[256 * 2: 256 * 3] = True
        refused[256 * 5: 256 * 6] = True
        if nb <= 256:
            rb = refused & busy                           # the refused buckets' busy entries
            assert rb.sum() == 51
            assert (g_npk[rb] == sentinel).all() and (g_used[rb] == sentinel).all() \
                and (g_st[rb] == sentinel).all(), "a refused bucket framed a busy entry over raw bytes"
        w_npk, w_used, w_st, _ = pyoracle.frame_scan(want, off, L, 20480, maxp)
        keep = ~refused
        for name, w, g in (("npk", w_npk, g_npk), ("used", w_used, g_used), ("status", w_st, g_st)):
            diff = np.flatnonzero(keep & (w != g))
            assert diff.size == 0, (name, diff[:8].tolist(), w[diff[:4]].tolist(), g[diff[:4]].tolist())
        _check_states(c, ob, cap)
