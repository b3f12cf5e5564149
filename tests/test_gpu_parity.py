"""GPU parity tests: the HIP path (through the C-ABI) against the golden
fixtures made by the real reference header, against the oracle on seeded
inputs, and at BASELINE.json's full sizes against the reference's SHA-256
digests.  Bit-exact everywhere (integer/byte work).  Run with -m gpu on a
MI355X."""
import hashlib

import numpy as np
import pytest

import pyoracle
from zsummerx_amd import Context, RC4Encryption, ZRC4Error, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    return torch


@pytest.fixture(scope="module")
def ctx(built):
    c = Context(0, 4096)
    yield c
    c.close()


def state_of(ctx, slot):
    sb, x, y = ctx.get_state(slot)
    return sb.hex(), x, y


# ---------------------------------------------------------------- KATs / edges
def test_kats_single_stream(ctx, kat):
    for i, v in enumerate(kat["wikipedia"]):
        ctx.make_sbox(i, bytes.fromhex(v["key"]))
        data = bytearray.fromhex(v["plaintext"])
        ctx.encryption(i, data, len(data))
        assert data.hex() == v["ciphertext"]
    for i, v in enumerate(kat["rfc6229"]):
        ctx.make_sbox(10 + i, bytes.fromhex(v["key"]))
        ks = bytearray(4112)
        ctx.encryption(10 + i, ks, len(ks))
        for o, want in v["offsets"].items():
            assert ks[int(o):int(o) + 16].hex() == want


def test_edge_cases(ctx, edge):
    for i, c in enumerate(edge):
        slot = 100 + i
        ctx.make_sbox(slot, bytes.fromhex(c["key"]))
        data = bytearray.fromhex(c["data"])
        if "length" in c:
            ctx.encryption(slot, data, c["length"])
        elif c["splits"]:
            pos = 0
            for s in c["splits"]:
                part = bytearray(data[pos:pos + s])
                ctx.encryption(slot, part, len(part))
                data[pos:pos + s] = part
                pos += s
            data = data[:pos]
        else:
            ctx.encryption(slot, data, len(data))
        assert data.hex() == c["out"], c["name"]
        assert state_of(ctx, slot) == (c["state"]["sbox"], c["state"]["x"], c["state"]["y"]), c["name"]


def test_ksa_key_lengths_batched(built, torch_cuda):
    """Batched makeSBox over key lengths 0..50, 63, 64, 65, 128, 255, 256,
    257, 300: the 16-byte register pattern takes lengths 1, 2, 4, 8, 16, the
    64-byte register pattern 32 and 64, the LDS window path every other
    length up to 48 (49 and 50 pin its edge), the rest fetch key bytes per
    step (65 and 128 pin the edges of the 64-byte branch); NUL bytes
    included, keys at every alignment; whole groups (range) and scattered
    ids; states against the oracle."""
    torch = torch_cuda
    rng = np.random.default_rng(31)
    lens = list(range(0, 51)) + [63, 64, 65, 128, 255, 256, 257, 300]
    n = 512
    klen = np.array([lens[i % len(lens)] for i in range(n)], dtype=np.uint32)
    koff = (np.concatenate([[3], np.cumsum(klen[:-1] + 1) + 3])).astype(np.uint64)
    keys = rng.integers(0, 256, int(koff[-1] + klen[-1]) + 8, dtype=np.uint8)
    keys[::7] = 0
    ob = pyoracle.Batch(n)
    ob.make_sbox(keys, koff, klen)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    s = torch.cuda.current_stream()
    for ids in (None, rng.permutation(2 * n)[:n].astype(np.uint32)):
        with Context(0, 2 * n) as c:
            c.ksa(T(klen.view(np.int32)), T(koff.view(np.int64)), T(keys),
                  ids=None if ids is None else T(ids.view(np.int32)), stream=s)
            c.sync(s)
            for i in range(n):
                slot = i if ids is None else int(ids[i])
                sb, x, y = c.get_state(slot)
                want_sb, wx, wy = ob.state(i)
                assert (sb, x, y) == (bytes(want_sb), wx, wy), (i, int(klen[i]))


def test_rc4encryption_mirror_class(built, kat):
    v = kat["wikipedia"][2]
    r = RC4Encryption()
    r.makeSBox(bytes.fromhex(v["key"]).decode())
    data = bytearray.fromhex(v["plaintext"])
    r.encryption(data, len(data))
    assert data.hex() == v["ciphertext"]
    r.encryption(data, 0)            # no-op
    r.encryption(data, -3)           # no-op (reference: length <= 0)


def test_rc4encryption_mirror_recycles_slots(built):
    """Instances give their slot back (per-context free list): a 256-slot
    context serves 1 000 short-lived instances, a recycled slot starts from
    the empty-key state, and live instances never share a slot."""
    with Context(0, 256) as c:
        live = [RC4Encryption(c) for _ in range(200)]
        assert len({r.slot for r in live}) == 200
        for _ in range(1000):
            r = RC4Encryption(c)
            r.makeSBox("temporary")
            r.encryption(bytearray(64), 64)
            r.close()
        r = RC4Encryption(c)
        assert c.get_state(r.slot) == (bytes(range(256)), 0, 0)
        with pytest.raises(ZRC4Error):
            _ = [RC4Encryption(c) for _ in range(100)]      # 200 + 1 + 100 > 256 live
        del live


# ----------------------------------------------------------- batched, ragged
def _seed_batch(ctx, b, ids):
    n = b["key_len"].size
    ctx.ksa_host([b["keys"][int(o):int(o) + int(l)].tobytes() for o, l in zip(b["key_off"], b["key_len"])],
                 ids=ids)
    scratch = np.zeros(1000 * n, dtype=np.uint8)
    ctx.crypt_host(scratch, np.arange(n, dtype=np.uint64) * 1000, b["adv"], ids=ids)


def _check_batch(ctx, b, ids, pay):
    assert np.array_equal(pay, b["payload_out"])
    for i in range(b["key_len"].size):
        sb, x, y = ctx.get_state(int(ids[i]) if ids is not None else i)
        assert sb == b["states"][i, :256].tobytes() and (x, y) == tuple(b["states"][i, 256:]), i


def test_batch_small_identity_ids(ctx, batch_small):
    b = batch_small
    _seed_batch(ctx, b, None)
    pay = b["payload_in"].copy()
    ctx.crypt_host(pay, b["off"], b["length"])
    _check_batch(ctx, b, None, pay)


def test_batch_small_scattered_ids(ctx, batch_small):
    """Arbitrary slot ids (gather/scatter path): a permutation across groups."""
    b = batch_small
    n = b["key_len"].size
    ids = (np.random.default_rng(3).permutation(4096)[:n]).astype(np.uint32)
    _seed_batch(ctx, b, ids)
    pay = b["payload_in"].copy()
    ctx.crypt_host(pay, b["off"], b["length"], ids=ids)
    _check_batch(ctx, b, ids, pay)


def test_crypt_host_scattered_ids_grouped(built, torch_cuda):
    """zrc4_crypt_host with many arbitrary ids buckets them by group (the
    grouped kernel; > 128 buckets: whole-group workgroups); entry order and
    payload layout stay the caller's; two calls continue the keystream.  A
    repeated slot is refused and crypts nothing."""
    rng = np.random.default_rng(123)
    cap = 65536
    n = 3000
    ids = rng.permutation(cap)[:n].astype(np.uint32)
    keys = [rng.integers(0, 256, 1 + int(rng.integers(0, 20)), dtype=np.uint8).tobytes() for _ in range(n)]
    ref = [pyoracle.Rc4(k) for k in keys]
    L = rng.integers(0, 300, n).astype(np.uint32)
    off = np.concatenate([[0], np.cumsum(L[:-1] + 3)]).astype(np.uint64)
    data = rng.integers(0, 256, int(off[-1] + L[-1]) + 8, dtype=np.uint8)
    with Context(0, cap) as c:
        c.ksa_host(keys, ids=ids)
        for call in range(2):
            want = data.copy()
            for i in range(n):
                a, z = int(off[i]), int(off[i] + L[i])
                want[a:z] = np.frombuffer(ref[i].encryption(want[a:z].tobytes()), np.uint8)
            got = data.copy()
            c.crypt_host(got, off, L, ids=ids)
            assert np.array_equal(got, want), call
            data = got
        dup = ids[:10].copy()
        dup[5] = dup[2]
        before = c.get_state(int(dup[2]))
        buf = np.zeros(10 * 16, dtype=np.uint8)
        with pytest.raises(ZRC4Error) as ei:
            c.crypt_host(buf, np.arange(10, dtype=np.uint64) * 16, np.full(10, 16, dtype=np.uint32), ids=dup)
        assert ei.value.code == -1                 # ZRC4_ERR_INVALID_ARG
        assert c.get_state(int(dup[2])) == before and not buf.any()
        # an id past the arena -- ZRC4_IDLE_SLOT (0xFFFFFFFF) included, which
        # the kernels would skip as padding -- is refused, nothing crypted
        for bad in (cap, 0xFFFFFFFF):
            bid = ids[:10].copy()
            bid[7] = bad
            before = c.get_state(int(bid[2]))
            with pytest.raises(ZRC4Error) as ei:
                c.crypt_host(buf, np.arange(10, dtype=np.uint64) * 16, np.full(10, 16, dtype=np.uint32), ids=bid)
            assert ei.value.code == -5             # ZRC4_ERR_SLOT_RANGE
            assert c.get_state(int(bid[2])) == before and not buf.any()


@pytest.mark.parametrize("ids_mode", ["range", "ids"])
def test_crypt_host_large_batch_pipelined(built, torch_cuda, ids_mode):
    """zrc4_crypt_host above 32 MiB of payload moves it in 16 MiB chunks
    (host copy of chunk k+1 overlapping the DMA of chunk k, both ways) and
    buckets ids by a counting pass (r06): 45 000 sessions of 0-1 800 bytes
    (~40 MiB, a ragged last chunk), ids in random order, two calls, against
    the oracle; states of a sample of slots checked too."""
    rng = np.random.default_rng(321)
    n, cap = 45000, 65536
    ids = rng.permutation(cap)[:n].astype(np.uint32) if ids_mode == "ids" else None
    slots = ids if ids is not None else np.arange(n, dtype=np.uint32)
    keys = rng.integers(0, 256, 16 * n, dtype=np.uint8)
    ob = pyoracle.Batch(cap)
    koff = np.zeros(cap, dtype=np.uint64)
    klen = np.zeros(cap, dtype=np.uint32)
    koff[slots] = np.arange(n, dtype=np.uint64) * 16
    klen[slots] = 16
    ob.make_sbox(keys, koff, klen)
    L = rng.integers(0, 1800, n).astype(np.uint32)
    off = np.concatenate([[0], np.cumsum(L[:-1] + 1)]).astype(np.uint64)
    data = rng.integers(0, 256, int(off[-1] + L[-1]) + 5, dtype=np.uint8)
    assert data.nbytes > 32 << 20
    with Context(0, cap) as c:
        c.ksa_host([keys[16 * i:16 * i + 16].tobytes() for i in range(n)], ids=slots)
        for call in range(2):
            want = data.copy()
            sl_off = np.zeros(cap, dtype=np.uint64)
            sl_len = np.zeros(cap, dtype=np.uint32)
            sl_off[slots] = off
            sl_len[slots] = L
            ob.crypt(want, sl_off, sl_len, threads=8)
            got = data.copy()
            c.crypt_host(got, off, L, ids=ids)
            bad = np.flatnonzero(got != want)
            assert bad.size == 0, (call, bad[:8].tolist(), int(bad.size))
            data = got
        for s in slots[rng.permutation(n)[:64]]:
            sb, x, y = c.get_state(int(s))
            osb, ox, oy = ob.state(int(s))
            assert (bytes(sb), x, y) == (bytes(osb), ox, oy), int(s)


def test_batch_whole_group_ids(ctx, batch_small):
    """ids given but exactly an aligned 256-slot group -> coalesced fast path."""
    rng = np.random.default_rng(9)
    keys = [rng.integers(0, 256, 16, dtype=np.uint8).tobytes() for _ in range(256)]
    ids = np.arange(512, 768, dtype=np.uint32)
    ctx.ksa_host(keys, ids=ids)
    L = np.array([int(v) for v in rng.integers(0, 700, 256)], dtype=np.uint32)
    off = np.concatenate([[0], np.cumsum(L[:-1])]).astype(np.uint64)
    pay = rng.integers(0, 256, int(L.sum()) + 1, dtype=np.uint8)
    want = pay.copy()
    ctx.crypt_host(pay, off, L, ids=ids)
    for i in range(256):
        a, z = int(off[i]), int(off[i] + L[i])
        want[a:z] = np.frombuffer(pyoracle.Rc4(keys[i]).encryption(want[a:z].tobytes()), np.uint8)
    assert np.array_equal(pay, want)


@pytest.mark.parametrize("first_slot", [512, 300])
def test_crypt_range(ctx, torch_cuda, first_slot):
    """Contiguous-slot entry: aligned first_slot (whole-group image path) and
    unaligned first_slot (per-lane gather path), ragged lengths."""
    torch = torch_cuda
    rng = np.random.default_rng(first_slot)
    n = 600
    keys = [rng.integers(0, 256, 16, dtype=np.uint8).tobytes() for _ in range(n)]
    kblob = torch.from_numpy(np.frombuffer(b"".join(keys), dtype=np.uint8).copy()).cuda()
    koff = torch.arange(n, dtype=torch.int64, device="cuda") * 16
    klen = torch.full((n,), 16, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    ctx.ksa_range(first_slot, klen, koff, kblob, stream=s)
    L = rng.integers(0, 1500, n).astype(np.uint32)
    off = np.concatenate([[0], np.cumsum(L[:-1])]).astype(np.uint64)
    data = rng.integers(0, 256, int(L.sum()) + 1, dtype=np.uint8)
    want = data.copy()
    for i in range(n):
        a, z = int(off[i]), int(off[i] + L[i])
        want[a:z] = np.frombuffer(pyoracle.Rc4(keys[i]).encryption(want[a:z].tobytes()), np.uint8)
    pay = torch.from_numpy(data).cuda()
    ctx.crypt_range(first_slot, pay, torch.from_numpy(off.view(np.int64)).cuda(),
                    torch.from_numpy(L.view(np.int32)).cuda(), stream=s)
    ctx.sync(s)
    assert np.array_equal(pay.cpu().numpy(), want)
    with pytest.raises(ZRC4Error):
        ctx.crypt_range(ctx.capacity - 10, pay, torch.from_numpy(off.view(np.int64)).cuda(),
                        torch.from_numpy(L.view(np.int32)).cuda(), stream=s)


def test_split_invariance_batched(ctx):
    """N calls of a few bytes == one call of the sum (keystream continues)."""
    rng = np.random.default_rng(4)
    n = 300
    keys = [rng.integers(0, 256, 16, dtype=np.uint8).tobytes() for _ in range(n)]
    ctx.ksa_host(keys)
    total = 777
    data = rng.integers(0, 256, n * total, dtype=np.uint8)
    want = data.copy()
    for i in range(n):
        want[i * total:(i + 1) * total] = np.frombuffer(
            pyoracle.Rc4(keys[i]).encryption(data[i * total:(i + 1) * total].tobytes()), np.uint8)
    pos = 0
    for step in [1, 3, 16, 17, 64, 100, 0, 200, 376]:
        off = (np.arange(n, dtype=np.uint64) * total + pos).astype(np.uint64)
        ctx.crypt_host(data, off, np.full(n, step, dtype=np.uint32))
        pos += step
    assert pos == total
    assert np.array_equal(data, want)


def test_state_roundtrip_and_import(ctx):
    r = pyoracle.Rc4(b"roundtrip")
    r.encryption(bytes(333))
    sb, x, y = r.state()
    ctx.set_state(7, sb, x, y)
    assert ctx.get_state(7) == (sb, x, y)
    data = bytearray(range(200))
    want = r.encryption(bytes(data))
    ctx.encryption(7, data, len(data))
    assert bytes(data) == want


def test_slot_out_of_range_is_reported(ctx, torch_cuda):
    torch = torch_cuda
    with pytest.raises(ZRC4Error):
        ctx.make_sbox(ctx.capacity, b"k")
    ids = torch.tensor([0, ctx.capacity + 5], dtype=torch.int32, device="cuda")
    pay = torch.zeros(32, dtype=torch.uint8, device="cuda")
    off = torch.tensor([0, 16], dtype=torch.int64, device="cuda")
    ln = torch.tensor([16, 16], dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    ctx.crypt(pay, off, ln, ids=ids, stream=s)
    with pytest.raises(ZRC4Error) as ei:
        ctx.sync(s)
    assert ei.value.code == -5
    ctx.sync(s)  # latch cleared


# ------------------------------------- throughput (staged) store path, ragged
@pytest.mark.parametrize("ids_kind", ["range", "scattered"])
def test_staged_path_ragged(built, torch_cuda, ids_kind):
    """More than one workgroup per CU selects the throughput path
    (crypt_stream_kernel: persistent over groups, DPP line loop).  Ragged
    lengths 0..699 (head bytes, lines cut mid-way, 16-byte chunks and tail
    bytes), unaligned offsets with gaps that must stay untouched, two calls
    in a row (state write-back), whole-group images with prefetch ("range")
    and per-lane gathers ("scattered" ids).  300 000 sessions = 1 172 groups,
    so every workgroup of the 2-per-CU grid walks 2-3 groups."""
    torch = torch_cuda
    n = 300000
    rng = np.random.default_rng(11 if ids_kind == "range" else 12)
    keys = rng.integers(0, 256, 16 * n, dtype=np.uint8)
    koff = np.arange(n, dtype=np.uint64) * 16
    klen = np.full(n, 16, dtype=np.uint32)
    ob = pyoracle.Batch(n)
    ob.make_sbox(keys, koff, klen)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    ids = None if ids_kind == "range" else rng.permutation(n + 4000)[:n].astype(np.uint32)
    s = torch.cuda.current_stream()
    with Context(0, n + 4000) as c:
        c.ksa(T(klen.view(np.int32)), T(koff.view(np.int64)), T(keys),
              ids=None if ids is None else T(ids.view(np.int32)), stream=s)
        for call in range(2):
            L = rng.integers(0, 700, n).astype(np.uint32)
            gaps = rng.integers(0, 40, n)
            off = np.cumsum(np.concatenate([[gaps[0]], L[:-1] + gaps[1:]])).astype(np.uint64)
            data = rng.integers(0, 256, int(off[-1] + L[-1]) + 64, dtype=np.uint8)
            want = data.copy()
            ob.crypt(want, off, L, threads=8)
            pay = T(data)
            c.crypt(pay, T(off.view(np.int64)), T(L.view(np.int32)),
                    ids=None if ids is None else T(ids.view(np.int32)), stream=s)
            c.sync(s)
            got = pay.cpu().numpy()
            bad = np.flatnonzero(got != want)
            assert bad.size == 0, (call, bad[:8], int(bad.size))
        for i in (0, 1, n // 2, n - 1):
            slot = i if ids is None else int(ids[i])
            sb, x, y = c.get_state(slot)
            want_sb, wx, wy = ob.state(i)
            assert (sb, x, y) == (bytes(want_sb), wx, wy), i


# ------------------------------- direct (chain-bound) path, block-loop edges
@pytest.mark.parametrize("first_slot", [0, 256])
def test_direct_path_block_edges(built, torch_cuda, first_slot):
    """One workgroup per CU selects crypt_kernel's direct block loop (lead
    block, static-count prefetch).  Group 0: every lane exactly one 64-byte
    block (the first block's prefetch re-reads it for every lane of every
    wave); group 1: exactly two; group 2: lengths cycling through the block
    edges with zeros mixed in; group 3: 16-byte aligned messages that start
    mid-line.  Gaps between messages must stay untouched; three calls in a
    row continue the keystream (state write-back)."""
    torch = torch_cuda
    n = 4 * 256
    rng = np.random.default_rng(21 + first_slot)
    keys = rng.integers(0, 256, 16 * n, dtype=np.uint8)
    koff = np.arange(n, dtype=np.uint64) * 16
    klen = np.full(n, 16, dtype=np.uint32)
    ob = pyoracle.Batch(n)
    ob.make_sbox(keys, koff, klen)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    edges = [0, 1, 15, 16, 17, 63, 64, 65, 127, 128, 129, 191, 192, 193, 255, 256, 320, 1000, 1024, 0]
    s = torch.cuda.current_stream()
    with Context(0, first_slot + n) as c:
        c.ksa_range(first_slot, T(klen.view(np.int32)), T(koff.view(np.int64)), T(keys), stream=s)
        for call in range(3):
            L = np.concatenate([np.full(256, 64), np.full(256, 128),
                                np.resize(edges, 256), rng.integers(0, 400, 256)]).astype(np.uint32)
            rng.shuffle(L[512:768])
            stride = 1536
            off = np.arange(n, dtype=np.uint64) * stride
            off[768:] += (rng.integers(0, 8, 256) * 16).astype(np.uint64)   # aligned, mid-line
            data = rng.integers(0, 256, n * stride + 256, dtype=np.uint8)
            want = data.copy()
            ob.crypt(want, off, L, threads=8)
            pay = T(data)
            c.crypt_range(first_slot, pay, T(off.view(np.int64)), T(L.view(np.int32)), stream=s)
            c.sync(s)
            got = pay.cpu().numpy()
            bad = np.flatnonzero(got != want)
            assert bad.size == 0, (call, bad[:8], int(bad.size))
        for i in (0, 255, 256, 511, 600, 767, 800, n - 1):
            sb, x, y = c.get_state(first_slot + i)
            want_sb, wx, wy = ob.state(i)
            assert (sb, x, y) == (bytes(want_sb), wx, wy), i


# ------------------------- speculative-window path (crypt_win_kernel, <= 32 groups)
@pytest.mark.parametrize("first_slot,n", [(0, 16 * 256 - 37), (768, 5), (256, 32 * 256 - 100)])
def test_window_path_ragged(built, torch_cuda, first_slot, n):
    """Aligned range batches of at most 32 groups run 16 lanes per stream
    (zsummerx_amd/csrc/zrc4_win.hpp).  Lengths 0..5000 including every
    16-byte edge and messages longer than the 2 KiB keystream chunk (2-3
    chunks), 16-byte aligned and unaligned message starts (the byte path),
    untouched gaps, a partial last group (the dword columns of the missing
    slots must keep their state), three calls in a row (x/y and image
    write-back), and states checked against the oracle afterwards."""
    torch = torch_cuda
    rng = np.random.default_rng(31 + n)
    keys = rng.integers(0, 256, 16 * n, dtype=np.uint8)
    koff = np.arange(n, dtype=np.uint64) * 16
    klen = np.full(n, 16, dtype=np.uint32)
    ob = pyoracle.Batch(n)
    ob.make_sbox(keys, koff, klen)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    edges = [0, 1, 15, 16, 17, 31, 32, 33, 255, 256, 1023, 1024, 1025, 2047, 2048, 2049, 4095, 4096, 4097, 5000]
    s = torch.cuda.current_stream()
    cap = first_slot + -(-n // 256) * 256 + 256
    with Context(0, cap) as c:
        c.ksa_range(first_slot, T(klen.view(np.int32)), T(koff.view(np.int64)), T(keys), stream=s)
        # a slot outside the batch that shares its image dword with batch slots
        nslot = first_slot + (n if n > 64 else 33)
        neighbour = c.get_state(nslot)
        for call in range(3):
            L = np.where(rng.random(n) < 0.3, np.resize(edges, n), rng.integers(0, 1500, n)).astype(np.uint32)
            rng.shuffle(L)
            lead = np.where(np.arange(n) % 2 == 0, 0, rng.integers(1, 16, n)).astype(np.uint64)
            gap = (rng.integers(0, 4, n) * 16).astype(np.uint64)
            seg = ((L.astype(np.uint64) + 15) // 16) * 16 + 16
            base = np.concatenate([[0], np.cumsum(seg + gap)[:-1]]).astype(np.uint64)
            off = base + lead
            data = rng.integers(0, 256, int(base[-1] + seg[-1] + gap[-1]) + 64, dtype=np.uint8)
            want = data.copy()
            ob.crypt(want, off, L, threads=8)
            pay = T(data)
            c.crypt_range(first_slot, pay, T(off.view(np.int64)), T(L.view(np.int32)), stream=s)
            c.sync(s)
            got = pay.cpu().numpy()
            bad = np.flatnonzero(got != want)
            assert bad.size == 0, (call, bad[:8], int(bad.size))
        for i in sorted({0, 1, n // 2, n - 1}):
            sb, x, y = c.get_state(first_slot + i)
            want_sb, wx, wy = ob.state(i)
            assert (sb, x, y) == (bytes(want_sb), wx, wy), i
        assert c.get_state(nslot) == neighbour


# ----------------------------------- every kernel-choice boundary of launch_crypt
@pytest.mark.parametrize("first_slot,n", [
    (0, 32 * 256), (0, 32 * 256 + 1),          # last window batch / first half-group batch
    (0, 128 * 256), (0, 128 * 256 + 1),        # last half-group batch (2G <= 256 CUs) / first whole-group
    (0, 256 * 256), (0, 256 * 256 + 1),        # last one-group-per-CU batch / first throughput batch
    (100, 20 * 256),                           # few groups but unaligned: no window kernel
    (0, 200 * 256 - 7),                        # whole-group kernel: 3 XCD-run blocks of 64 + a tail of 8
    (37, 150 * 256),                           # unaligned range over 151 groups (gathered columns, runs + tail)
])
def test_dispatch_boundaries_bit_exact(built, torch_cuda, first_slot, n):
    """zrc4.hip launch_crypt picks the kernel from the batch's group count
    and alignment (window <= 32 aligned groups, half-group while 2G <= CUs,
    whole-group while G <= CUs, the persistent throughput kernel above).
    Each side of every boundary, with ragged lengths (0..1 500, unaligned
    starts, untouched gaps), two calls in a row and states checked after."""
    torch = torch_cuda
    rng = np.random.default_rng(41 + n + first_slot)
    keys = rng.integers(0, 256, 16 * n, dtype=np.uint8)
    koff = np.arange(n, dtype=np.uint64) * 16
    klen = np.full(n, 16, dtype=np.uint32)
    ob = pyoracle.Batch(n)
    ob.make_sbox(keys, koff, klen)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    s = torch.cuda.current_stream()
    with Context(0, first_slot + n + 256) as c:
        c.ksa_range(first_slot, T(klen.view(np.int32)), T(koff.view(np.int64)), T(keys), stream=s)
        for call in range(2):
            L = rng.integers(0, 1500, n).astype(np.uint32)
            L[rng.random(n) < 0.05] = 0
            gaps = rng.integers(0, 24, n)
            off = np.cumsum(np.concatenate([[gaps[0]], L[:-1] + gaps[1:]])).astype(np.uint64)
            data = rng.integers(0, 256, int(off[-1] + L[-1]) + 64, dtype=np.uint8)
            want = data.copy()
            ob.crypt(want, off, L, threads=8)
            pay = T(data)
            c.crypt_range(first_slot, pay, T(off.view(np.int64)), T(L.view(np.int32)), stream=s)
            c.sync(s)
            bad = np.flatnonzero(pay.cpu().numpy() != want)
            assert bad.size == 0, (call, bad[:8], int(bad.size))
        for i in sorted({0, 255, n // 2, n - 2, n - 1}):
            sb, x, y = c.get_state(first_slot + i)
            want_sb, wx, wy = ob.state(i)
            assert (sb, x, y) == (bytes(want_sb), wx, wy), i


# ------------------------------------------ grouped ids (zrc4_crypt_grouped)
def grouped_batch(rng, n_groups, groups_total, fill=(1, 256)):
    """Buckets of 256 entries: bucket b takes a random subset (random order)
    of group g_b's slots, groups drawn without repetition; padding entries
    are ZRC4_IDLE_SLOT.  Returns (ids[n], member_index[n] or -1)."""
    from zsummerx_amd._capi import IDLE_SLOT
    groups = rng.permutation(groups_total)[:n_groups]
    ids = np.full(256 * n_groups, IDLE_SLOT, dtype=np.uint32)
    for b, g in enumerate(groups):
        k = int(rng.integers(fill[0], fill[1] + 1))
        slots = g * 256 + rng.permutation(256)[:k]
        pos = rng.permutation(256)[:k]
        ids[256 * b + pos] = slots
    return ids


@pytest.mark.parametrize("fill,nb,trunc,idle", [
    ((256, 256), 64, 0, 0), ((1, 256), 64, 0, 0), ((1, 256), 200, 0, 0),
    ((1, 200), 64, 100, 0), ((1, 256), 200, 37, 0), ((1, 256), 27, 11, 0),
    # more buckets than CUs: the persistent kernel's grouped form
    ((1, 256), 600, 0, 0.1), ((256, 256), 1100, 0, 0), ((1, 200), 700, 100, 0.05), ((1, 64), 513, 255, 0.3)])
def test_grouped_ids_bit_exact(built, torch_cuda, fill, nb, trunc, idle):
    """zrc4_crypt_grouped: each bucket a subset of ONE group, in any order,
    groups in random order, idle padding; two calls in a row continue the
    keystream.  nb = 27 buckets runs the speculative-window kernel (at most 32
    buckets, workgroup columns spread over the XCDs: 27 is no multiple of 8),
    64 half-group workgroups, 200 whole-group ones, 513-1 100 the persistent
    kernel (2 workgroups per CU walking 1-3 buckets each: tables built a
    bucket ahead, claims, gathered entries); trunc drops the last entries of
    the batch (a short last bucket whose slots still fall in both halves of
    its group); idle empties that share of the buckets (all ZRC4_IDLE_SLOT).
    Checked against the oracle, every session that ran and every state;
    slots outside the batch keep their state."""
    torch = torch_cuda
    from zsummerx_amd._capi import IDLE_SLOT
    rng = np.random.default_rng(41 + fill[0] + nb + trunc)
    G = max(256, nb + 64)                          # groups in the arena
    cap = 256 * G
    keys = rng.integers(0, 256, 16 * cap, dtype=np.uint8)
    koff = np.arange(cap, dtype=np.uint64) * 16
    klen = np.full(cap, 16, dtype=np.uint32)
    ob = pyoracle.Batch(cap)
    ob.make_sbox(keys, koff, klen)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    s = torch.cuda.current_stream()
    with Context(0, cap) as c:
        c.ksa_range(0, T(klen.view(np.int32)), T(koff.view(np.int64)), T(keys), stream=s)
        touched = set()
        for call in range(2):
            ids = grouped_batch(rng, nb, G, fill)
            if idle:
                for b in np.flatnonzero(rng.random(nb - 1) < idle):
                    ids[256 * b: 256 * (b + 1)] = IDLE_SLOT
            if trunc:   # the short bucket keeps an upper-half slot of its group (entry 0)
                last = ids[256 * (nb - 1):]
                used = [int(v) for v in last[last != IDLE_SLOT]]
                g = used[0] // 256
                up = [v for v in used if v % 256 >= 128]
                slot = up[0] if up else next(g * 256 + k for k in range(128, 256) if g * 256 + k not in used)
                last[last == slot] = IDLE_SLOT
                last[0] = slot
                ids = ids[:ids.size - trunc].copy()
            busy = ids != IDLE_SLOT
            L = np.where(busy, rng.integers(0, 600, ids.size), 0).astype(np.uint32)
            if trunc:
                L[256 * (nb - 1)] = 333
            off = (np.arange(ids.size, dtype=np.uint64) * 640 + rng.integers(0, 16, ids.size).astype(np.uint64))
            data = rng.integers(0, 256, ids.size * 640 + 64, dtype=np.uint8)
            # oracle: per slot, in batch order (each slot once per call)
            want = data.copy()
            for e in np.flatnonzero(busy):
                st = ob.st[int(ids[e])]
                pyoracle.lib().oracle_encryption(pyoracle.C.byref(st),
                                                 pyoracle.C.c_void_p(want.ctypes.data + int(off[e])), int(L[e]))
            touched.update(int(v) for v in ids[busy])
            pay = T(data)
            c.crypt_grouped(pay, T(off.view(np.int64)), T(L.view(np.int32)), T(ids.view(np.int32)), stream=s)
            c.sync(s)
            got = pay.cpu().numpy()
            bad = np.flatnonzero(got != want)
            assert bad.size == 0, (call, bad[:8], int(bad.size))
        for slot in list(touched)[:40] + [v for v in range(0, cap, 997) if v not in touched][:20]:
            sb, x, y = c.get_state(slot)
            want_sb, wx, wy = ob.state(slot)
            assert (sb, x, y) == (bytes(want_sb), wx, wy), slot


def test_grouped_ids_mixed_bucket_is_refused(built, torch_cuda):
    """A bucket whose busy entries span two groups is skipped whole (no byte
    or state touched) and reported as ZRC4_ERR_GROUP; other buckets run."""
    torch = torch_cuda
    from zsummerx_amd._capi import IDLE_SLOT
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    s = torch.cuda.current_stream()
    with Context(0, 1024) as c:
        c.ksa_host([b"key-%d" % i for i in range(1024)], ids=np.arange(1024, dtype=np.uint32))
        ids = np.full(512, IDLE_SLOT, dtype=np.uint32)
        ids[0], ids[1] = 5, 300                      # bucket 0: groups 0 and 1 -> refused
        ids[256], ids[257] = 700, 701                # bucket 1: group 2 -> runs
        L = np.where(ids != IDLE_SLOT, 32, 0).astype(np.uint32)
        off = np.arange(512, dtype=np.uint64) * 32
        pay = T(np.zeros(512 * 32, dtype=np.uint8))
        before = [c.get_state(v) for v in (5, 300)]
        c.crypt_grouped(pay, T(off.view(np.int64)), T(L.view(np.int32)), T(ids.view(np.int32)), stream=s)
        with pytest.raises(ZRC4Error) as ei:
            c.sync(s)
        assert ei.value.code == -7
        got = pay.cpu().numpy()
        assert not got[:2 * 32].any()                # refused bucket: payload untouched
        assert got[256 * 32: 258 * 32].any()          # bucket 1 ran
        assert [c.get_state(v) for v in (5, 300)] == before
        ks = pyoracle.Rc4(b"key-700").encryption(bytes(32))
        assert got[256 * 32: 257 * 32].tobytes() == ks


@pytest.mark.parametrize("nb,variant", [(20, None), (100, None), (200, None), (700, None), (1600, None),
                                        (1600, "preclaim1"), (5000, None)])
def test_grouped_cross_bucket_conflict_is_refused(built, torch_cuda, nb, variant):
    """The cross-bucket half of the zrc4_crypt_grouped contract: two buckets
    of one call name the same group (disjoint slots of it).  The call reports
    ZRC4_ERR_GROUP; every other bucket is bit-exact (payload and states); in
    the contested group every entry is all-or-nothing -- crypted exactly as
    the oracle does with its state advanced, or untouched with its state
    unchanged -- never raced.  nb = 20: the window kernel (one claim per
    dword column), 100: half-group workgroups, 200: whole-group workgroups,
    700 / 1600: the persistent kernel (each pair claims its half of every
    bucket's group a group ahead; from 3 buckets per workgroup (1600) the
    first 64 of a workgroup in its prologue instead -- the preclaim1 test
    build pre-claims only the first, so the contested buckets meet across
    both paths).  5000 short buckets (1-6 entries): about 10 buckets per
    workgroup, so the prologue pre-claims in two rounds of 8 and the second
    contested bucket (4998, the 10th of its workgroup) is claimed in the
    second round.  Every entry is checked (states read back in
    one copy)."""
    torch = torch_cuda
    from zsummerx_amd._capi import IDLE_SLOT
    rng = np.random.default_rng(500 + nb)
    G = max(256, nb + 8)
    cap = 256 * G
    keys = rng.integers(0, 256, 16 * cap, dtype=np.uint8)
    koff = np.arange(cap, dtype=np.uint64) * 16
    klen = np.full(cap, 16, dtype=np.uint32)
    ob = pyoracle.Batch(cap)
    ob.make_sbox(keys, koff, klen)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    s = torch.cuda.current_stream()
    groups = rng.permutation(G)[:nb - 1]
    dup_a, dup_b = 3, nb - 2                           # buckets dup_a and dup_b both take group groups[dup_a]
    ids = np.full(256 * nb, IDLE_SLOT, dtype=np.uint32)
    contested = int(groups[dup_a])
    half = rng.permutation(256)
    for b in range(nb):
        if b == dup_b:
            ids[256 * b: 256 * b + 128] = contested * 256 + half[128:]
        elif b == dup_a:
            ids[256 * b: 256 * b + 128] = contested * 256 + half[:128]
        else:
            g = int(groups[b if b < dup_b else b - 1])
            k = int(rng.integers(1, 257 if nb <= 2000 else 7))
            ids[256 * b + rng.permutation(256)[:k]] = g * 256 + rng.permutation(256)[:k]
    busy = ids != IDLE_SLOT
    span = 512 if nb <= 2000 else 64
    L = np.where(busy, rng.integers(1, span - 12, ids.size), 0).astype(np.uint32)
    off = np.arange(ids.size, dtype=np.uint64) * span
    data = rng.integers(0, 256, ids.size * span, dtype=np.uint8)
    from zsummerx_amd import build
    with Context(0, cap, lib=None if variant is None else build.PKG / f"libzrc4_{variant}.so") as c:
        c.ksa_range(0, T(klen.view(np.int32)), T(koff.view(np.int64)), T(keys), stream=s)
        pay = T(data)
        c.crypt_grouped(pay, T(off.view(np.int64)), T(L.view(np.int32)), T(ids.view(np.int32)), stream=s)
        with pytest.raises(ZRC4Error) as ei:
            c.sync(s)
        assert ei.value.code == -7                      # ZRC4_ERR_GROUP
        got = pay.cpu().numpy()
        gsb, gx, gy = c.get_states(0, cap)             # every device state in one copy
        crypted = untouched = 0
        for e in np.flatnonzero(busy):
            slot, a, z = int(ids[e]), int(off[e]), int(off[e] + L[e])
            before = ob.state(slot)
            want = data[a:z].copy()
            st = ob.st[slot]
            saved = pyoracle.C.create_string_buffer(bytes(st), pyoracle.C.sizeof(st))
            pyoracle.lib().oracle_encryption(pyoracle.C.byref(st), pyoracle.C.c_void_p(want.ctypes.data), int(L[e]))
            after = ob.state(slot)
            sb, x, y = gsb[slot].tobytes(), int(gx[slot]), int(gy[slot])
            if slot // 256 != contested:
                assert np.array_equal(got[a:z], want), (e, slot)
                assert (sb, x, y) == (bytes(after[0]), after[1], after[2]), slot
                continue
            if np.array_equal(got[a:z], want):
                assert (sb, x, y) == (bytes(after[0]), after[1], after[2]), slot
                crypted += 1
            else:
                assert np.array_equal(got[a:z], data[a:z]), (e, slot)           # untouched, not half-crypted
                assert (sb, x, y) == (bytes(before[0]), before[1], before[2]), slot
                pyoracle.C.memmove(pyoracle.C.byref(st), saved, pyoracle.C.sizeof(st))
                untouched += 1
        assert untouched >= 1 and crypted + untouched == 256


@pytest.mark.parametrize("variant", [None, "preclaim1"])
def test_grouped_stream_refusals(built, torch_cuda, variant):
    """The persistent kernel's grouped form (600 buckets > 256 CUs) with every
    refusal at once: a bucket whose busy entries span two groups, a bucket
    naming one slot twice, a bucket with an id past the arena (that entry is
    skipped, ZRC4_ERR_SLOT_RANGE, the rest of the bucket runs), idle buckets,
    and a slot listed twice with length 0 once (not busy: allowed).  The call
    reports ZRC4_ERR_GROUP; refused buckets leave payload and states
    untouched; every other entry is bit-exact against the oracle.  A second
    call afterwards (no faults) continues every keystream.  preclaim1: the
    test build whose workgroups claim only their first bucket up front."""
    torch = torch_cuda
    from zsummerx_amd._capi import IDLE_SLOT
    rng = np.random.default_rng(77)
    nb = 600
    G = nb + 64
    cap = 256 * G
    keys = rng.integers(0, 256, 16 * cap, dtype=np.uint8)
    koff = np.arange(cap, dtype=np.uint64) * 16
    klen = np.full(cap, 16, dtype=np.uint32)
    ob = pyoracle.Batch(cap)
    ob.make_sbox(keys, koff, klen)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    s = torch.cuda.current_stream()
    mixed, twice, past, zero_dup = 5, 301, 450, 77
    from zsummerx_amd import build
    with Context(0, cap, lib=None if variant is None else build.PKG / f"libzrc4_{variant}.so") as c:
        c.ksa_range(0, T(klen.view(np.int32)), T(koff.view(np.int64)), T(keys), stream=s)
        for call in range(2):
            ids = grouped_batch(rng, nb, G, (2, 256))
            for b in (13, 14, 299, 599):
                ids[256 * b: 256 * (b + 1)] = IDLE_SLOT
            refused = set()
            if call == 0:
                bm = ids[256 * mixed: 256 * (mixed + 1)]
                k = int(np.flatnonzero(bm != IDLE_SLOT)[0])
                other = int(ids[256 * 7 + int(np.flatnonzero(ids[256 * 7: 256 * 8] != IDLE_SLOT)[0])])
                spare = next(v for v in range((other // 256) * 256, (other // 256 + 1) * 256) if v not in set(ids.tolist()))
                free = [p for p in range(256) if bm[p] == IDLE_SLOT] or [k ^ 1]
                bm[free[0]] = spare                       # a slot of another bucket's group
                bt = ids[256 * twice: 256 * (twice + 1)]
                used = np.flatnonzero(bt != IDLE_SLOT)
                dst = [p for p in range(256) if bt[p] == IDLE_SLOT]
                bt[dst[0]] = bt[used[0]]                  # the same slot twice
                refused = {mixed, twice}
                bp = ids[256 * past: 256 * (past + 1)]
                pos = [p for p in range(256) if bp[p] == IDLE_SLOT][0]
                bp[pos] = cap + 1000                      # past the arena: skipped, bucket runs
            bz = ids[256 * zero_dup: 256 * (zero_dup + 1)]
            u = np.flatnonzero(bz != IDLE_SLOT)
            zpos = [p for p in range(256) if bz[p] == IDLE_SLOT][0]
            bz[zpos] = bz[u[0]]                           # listed twice, once with length 0
            busy = (ids != IDLE_SLOT) & (ids < cap)
            L = np.where(busy, rng.integers(1, 680, ids.size), 0).astype(np.uint32)
            L[256 * zero_dup + zpos] = 0
            busy &= L > 0
            off = np.arange(ids.size, dtype=np.uint64) * 704 + rng.integers(0, 16, ids.size).astype(np.uint64)
            data = rng.integers(0, 256, ids.size * 704 + 64, dtype=np.uint8)
            want = data.copy()
            before = {}
            for e in np.flatnonzero(busy):
                if e // 256 in refused:
                    before[int(ids[e])] = ob.state(int(ids[e]))
                    continue
                st = ob.st[int(ids[e])]
                pyoracle.lib().oracle_encryption(pyoracle.C.byref(st),
                                                 pyoracle.C.c_void_p(want.ctypes.data + int(off[e])), int(L[e]))
            pay = T(data)
            c.crypt_grouped(pay, T(off.view(np.int64)), T(L.view(np.int32)), T(ids.view(np.int32)), stream=s)
            if call == 0:
                with pytest.raises(ZRC4Error) as ei:
                    c.sync(s)
                assert ei.value.code == -7                # ZRC4_ERR_GROUP (reported before SLOT_RANGE)
            else:
                c.sync(s)
            got = pay.cpu().numpy()
            bad = np.flatnonzero(got != want)
            assert bad.size == 0, (call, bad[:8], int(bad.size), sorted({int(b) // 704 // 256 for b in bad[:50]}))
            for slot, st0 in list(before.items())[:30]:
                sb, x, y = c.get_state(slot)
                assert (sb, x, y) == (bytes(st0[0]), st0[1], st0[2]), slot
        for slot in [int(v) for v in ids[busy][:40]]:
            sb, x, y = c.get_state(slot)
            want_sb, wx, wy = ob.state(slot)
            assert (sb, x, y) == (bytes(want_sb), wx, wy), slot


# ------------------------------------------------ full BASELINE-size configs
def _device_workload(ctx, w, torch, ids_mode="range"):
    """Seed, pre-advance and crypt the synthetic workload once.  range: entry
    i = slot i (zrc4_crypt, identity ids); grouped / declared: the engine's
    shape -- groups in random order, slots permuted inside each group, entry
    e crypting session perm[e]'s payload (zrc4_crypt_grouped /
    zrc4_crypt_grouped_declared).  Every session is crypted once either way,
    so the ciphertext and the states are the same."""
    dev = "cuda"
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    s = torch.cuda.current_stream()
    ctx.ksa(t(w.key_len.view(np.int32)), t(w.key_off.view(np.int64)), t(w.keys), stream=s)
    scratch = torch.zeros(1000, dtype=torch.uint8, device=dev)
    zero = torch.zeros(w.n, dtype=torch.int64, device=dev)
    ctx.crypt(scratch, zero, t(w.adv.view(np.int32)), stream=s)   # pre-advance
    pay = t(w.payload)
    if ids_mode == "range":
        ctx.crypt(pay, t(w.off.view(np.int64)), t(w.length.view(np.int32)), stream=s)
    else:
        assert w.n % 256 == 0
        rng = np.random.default_rng(2024)
        order = rng.permutation(w.n // 256)
        perm = (order[:, None] * 256 + np.stack([rng.permutation(256) for _ in order])).reshape(-1)
        ids, off, ln = t(perm.astype(np.uint32).view(np.int32)), t(w.off[perm].view(np.int64)), \
            t(w.length[perm].view(np.int32))
        if ids_mode == "grouped":
            ctx.crypt_grouped(pay, off, ln, ids, stream=s)
        else:
            ctx.crypt_grouped_declared(pay, off, ln, ids, order.astype(np.uint32), stream=s)
    ctx.sync(s)
    return pay.cpu().numpy()


def _states_digest(ctx, n):
    """sha256 over slots 0..n-1 of sbox + x + y (zrc4_get_states: one copy)."""
    sb, x, y = ctx.get_states(0, n)
    return hashlib.sha256(np.concatenate([sb, x[:, None], y[:, None]], axis=1).tobytes()).hexdigest()


@pytest.mark.parametrize("cfg,ids_mode", [("cfg2", "range"), ("cfg3", "range"), ("cfg4", "range"),
                                          ("cfg5", "range"), ("cfg2", "grouped"), ("cfg2", "declared"),
                                          ("cfg3", "declared"), ("cfg5", "grouped"), ("cfg5", "declared")])
def test_baseline_configs_bit_exact(cfg, ids_mode, synth_digests, torch_cuda, built):
    """BASELINE configs[1..4] at full size against SHA-256 digests made by the
    real reference header (tests/golden/make_golden.py): the range path, and
    the engine's grouped paths (zrc4_crypt_grouped, and _declared: the window
    kernel with declared groups at cfg2, the declared check + persistent
    kernel at cfg3 / cfg5)."""
    S, L = synth.CONFIGS[cfg]
    d = synth_digests[cfg]
    w = synth.make(0, S, L, threads=8)
    with Context(0, S) as c:
        out = _device_workload(c, w, torch_cuda, ids_mode)
        assert hashlib.sha256(out.tobytes()).hexdigest() == d["ciphertext_sha256"], cfg
        if S <= 65536:
            assert _states_digest(c, S) == d["states_sha256"], cfg
        else:
            sb, x, y = c.get_state(S - 1)
            assert (sb + bytes([x, y])).hex() == d["last_session_state"]


# ------------------------------------------------- keystream reservoirs
def test_xor_ring_matches_numpy(ctx, torch_cuda):
    """zrc4_xor_ring on ragged, unaligned spans with wrapping ring positions:
    payload ^= ring bytes (mod cap) and exactly the used ring bytes become 0."""
    torch = torch_cuda
    rng = np.random.default_rng(11)
    cap, R, n = 4096, 64, 200
    ring = rng.integers(0, 256, R * cap, dtype=np.uint8)
    rid = rng.permutation(R)[: min(R, n)].astype(np.uint32)
    rid = np.concatenate([rid, rng.integers(0, R, n - rid.size).astype(np.uint32)])[:n]
    # distinct rings per entry would be required for a real reservoir; here
    # entries sharing a ring use disjoint windows, so give each entry its own ring slice
    rid = (np.arange(n) % R).astype(np.uint32)
    lens = rng.integers(0, cap // 4, n).astype(np.uint32)
    lens[:5] = [0, 1, 2, 3, cap // 4]
    pos = (rng.integers(0, cap, n)).astype(np.uint32)
    pos[(np.arange(n) // R) > 0] = 0
    # entries that share a ring (n > R) take consecutive windows
    for i in range(R, n):
        prev = i - R
        pos[i] = (int(pos[prev]) + int(lens[prev])) % cap
    off = np.zeros(n, dtype=np.uint64)
    acc = 3
    for i in range(n):
        off[i] = acc
        acc += int(lens[i]) + int(rng.integers(0, 7))
    pay = rng.integers(0, 256, acc + 8, dtype=np.uint8)
    want_pay, want_ring = pay.copy(), ring.copy()
    for i in range(n):
        for k in range(int(lens[i])):
            q = int(rid[i]) * cap + (int(pos[i]) + k) % cap
            want_pay[int(off[i]) + k] ^= want_ring[q]
            want_ring[q] = 0
    T = lambda a: torch.from_numpy(a).to("cuda")
    d_ring, d_pay = T(ring), T(pay)
    d_rid, d_pos, d_off, d_len = T(rid.view(np.int32)), T(pos.view(np.int32)), T(off.view(np.int64)), T(lens.view(np.int32))
    # one launch per ring generation (entries sharing a ring must not run in one launch)
    for g in range(0, n, R):
        sl = slice(g, min(n, g + R))
        ctx.xor_ring(d_ring, cap, d_rid[sl], d_pos[sl], d_pay, d_off[sl], d_len[sl])
    ctx.sync()
    assert np.array_equal(d_pay.cpu().numpy(), want_pay)
    assert np.array_equal(d_ring.cpu().numpy(), want_ring)


@pytest.mark.parametrize("where", ["device", "pinned"])
def test_reservoir_round_trip(built, torch_cuda, where):
    """The engine's reservoir protocol through the C-ABI: seed, fill zeroed
    rings with zrc4_crypt (pure keystream), consume them with zrc4_xor_ring in
    pieces that wrap, refill the consumed bytes, and compare the whole
    ciphertext with the oracle's RC4 over the same data."""
    torch = torch_cuda
    rng = np.random.default_rng(5)
    S, cap, total = 300, 2048, 9000
    keys = [rng.integers(0, 256, int(rng.integers(1, 40)), dtype=np.uint8).tobytes() for _ in range(S)]
    data = rng.integers(0, 256, (S, total), dtype=np.uint8)
    want = np.stack([np.frombuffer(pyoracle.Rc4(keys[s]).encryption(data[s].tobytes()), np.uint8) for s in range(S)])
    if where == "device":
        T = lambda a: torch.from_numpy(a).to("cuda")
    else:       # the session engine's layout: tables and payload in pinned host memory
        T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).pin_memory()
    with Context(0, S) as c:
        c.ksa_host(keys)
        ring = torch.zeros(S * cap, dtype=torch.uint8, device="cuda")
        pay = T(data.reshape(-1).copy())
        gen = np.zeros(S, dtype=np.int64)
        use = np.zeros(S, dtype=np.int64)
        ids = np.arange(S, dtype=np.uint32)
        while (use < total).any():
            # refill every ring to full, in at most two pieces (ring end, ring start)
            for _ in range(2):
                at = gen % cap
                amt = np.minimum(use + cap - gen, cap - at).astype(np.uint32)
                m = amt > 0
                if not m.any():
                    break
                c.crypt(ring, T((ids[m].astype(np.int64) * cap + at[m]).astype(np.int64)), T(amt[m].view(np.int32)),
                        ids=T(ids[m].view(np.int32)))
                c.sync()          # pinned tables are reused next round
                gen[m] += amt[m]
            # consume a random amount per stream (<= what is there)
            take = np.minimum(rng.integers(0, cap + 1, S), np.minimum(gen - use, total - use)).astype(np.uint32)
            if where == "pinned":
                take = np.minimum(take, rng.integers(0, 40, S)).astype(np.uint32)   # small, unaligned pieces
            c.xor_ring(ring, cap, T(ids.view(np.int32)), T((use % cap).astype(np.uint32).view(np.int32)), pay,
                       T((np.arange(S, dtype=np.int64) * total + use).astype(np.int64)), T(take.view(np.int32)))
            c.sync()
            use += take
        c.sync()
        got = pay.cpu().numpy().reshape(S, total)
    assert np.array_equal(got, want)


def test_window_tag_restart(built, torch_cuda):
    """The window kernel's marker tags (24 bits) restart, with the markers
    cleared, long before they could wrap.  A build that restarts them at
    every chunk (ZRC4_WIN_TAG_LIMIT=4) stays bit-exact over multi-chunk
    messages, range and grouped."""
    from zsummerx_amd import build
    torch = torch_cuda
    var = build.build_variant("wintag4", build.TEST_VARIANTS["wintag4"])
    rng = np.random.default_rng(77)
    n = 600
    keys = rng.integers(0, 256, 16 * n, dtype=np.uint8)
    koff = np.arange(n, dtype=np.uint64) * 16
    klen = np.full(n, 16, dtype=np.uint32)
    ob = pyoracle.Batch(n)
    ob.make_sbox(keys, koff, klen)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    s = torch.cuda.current_stream()
    with Context(0, 1024, lib=var) as c:
        c.ksa_range(0, T(klen.view(np.int32)), T(koff.view(np.int64)), T(keys), stream=s)
        for call in range(2):
            L = rng.integers(2000, 9000, n).astype(np.uint32)
            off = (np.concatenate([[0], np.cumsum((L.astype(np.uint64) + 15) // 16 * 16)[:-1]])).astype(np.uint64)
            data = rng.integers(0, 256, int(off[-1] + L[-1]) + 16, dtype=np.uint8)
            want = data.copy()
            ob.crypt(want, off, L, threads=8)
            pay = T(data)
            if call == 0:
                c.crypt_range(0, pay, T(off.view(np.int64)), T(L.view(np.int32)), stream=s)
            else:
                ids = np.arange(n, dtype=np.uint32)
                got = data.copy()
                c.crypt_host(got, off, L, ids=ids)
                pay = T(got)
            c.sync(s)
            bad = np.flatnonzero(pay.cpu().numpy() != want)
            assert bad.size == 0, (call, bad[:8], int(bad.size))


def test_reservoir_failed_tail_loses_position_until_reseeded(built, monkeypatch):
    """a reservoir tail crypt that fails must not let the slot go
    on from an unknown keystream position.  With the test hook
    ZRC4_KS_FAIL_TAIL_AFTER=2 (read only by the ZRC4_TEST_HOOKS build,
    libzrc4_testhooks.so) the second tail crypt of the reservoir fails:
    that call returns the error, every later call on the slot returns
    ZRC4_ERR_STATE (-9) and touches nothing, another slot is unaffected, and
    zrc4_ks_make_sbox reseeds it back to reference bytes."""
    import ctypes as C
    from zsummerx_amd import _capi, build
    lib = _capi.load(build.PKG / "libzrc4_testhooks.so")
    monkeypatch.setenv("ZRC4_KS_FAIL_TAIL_AFTER", "2")
    ctx, ks = C.c_void_p(), C.c_void_p()
    assert lib.zrc4_create(C.byref(ctx), 0, 256) == 0
    try:
        assert lib.zrc4_ks_create(ctx, 4096, C.byref(ks)) == 0
        for slot, key in ((0, b"lost-slot"), (1, b"other-slot")):
            assert lib.zrc4_ks_make_sbox(ks, slot, key, len(key)) == 0

        def call(slot, n):
            buf = (C.c_uint8 * n)()
            ids = (C.c_uint32 * 1)(slot)
            ptrs = (C.c_void_p * 1)(C.cast(buf, C.c_void_p))
            lens = (C.c_uint32 * 1)(n)
            return lib.zrc4_ks_crypt(ks, ids, ptrs, lens, 1), bytes(buf)

        ref1 = pyoracle.Rc4(b"other-slot")
        rc, out = call(1, 64)                          # tail 1: fine
        assert rc == 0 and out == ref1.encryption(bytes(64))
        rc, _ = call(0, 64)                            # tail 2: injected failure
        assert rc != 0
        for _ in range(3):
            rc, out = call(0, 32)
            assert rc == -9 and out == bytes(32)       # ZRC4_ERR_STATE, nothing crypted
        assert lib.zrc4_ks_make_sbox(ks, 0, b"lost-slot", 9) == 0
        rc, out = call(0, 100)                         # reseeded: reference bytes again
        assert rc == 0 and out == pyoracle.Rc4(b"lost-slot").encryption(bytes(100))
        rc, out = call(1, 50)
        assert rc == 0 and out == ref1.encryption(bytes(50))
    finally:
        if ks:
            lib.zrc4_ks_destroy(ks)
        lib.zrc4_destroy(ctx)


def test_reservoir_failed_tail_loses_every_slot_of_the_call(built, monkeypatch):
    """a failed tail marks EVERY slot with len > 0 of the call
    lost, including one served entirely from its ring (its span was already
    crypted on the host when the tail failed).  Slot A's first call is a tail
    (tail 1) and queues its refill; the two-slot call [A: 16 bytes, B: 64]
    serves A from its ring and needs a tail for B (tail 2, injected failure).
    Afterwards both A and B return ZRC4_ERR_STATE until reseeded; reseeded,
    both give the reference bytes again."""
    import ctypes as C
    from zsummerx_amd import _capi, build
    lib = _capi.load(build.PKG / "libzrc4_testhooks.so")
    monkeypatch.setenv("ZRC4_KS_FAIL_TAIL_AFTER", "2")
    ctx, ks = C.c_void_p(), C.c_void_p()
    assert lib.zrc4_create(C.byref(ctx), 0, 256) == 0
    try:
        assert lib.zrc4_ks_create(ctx, 4096, C.byref(ks)) == 0
        for slot, key in ((0, b"slot-a"), (1, b"slot-b")):
            assert lib.zrc4_ks_make_sbox(ks, slot, key, len(key)) == 0

        def call(slots, lens):
            bufs = [(C.c_uint8 * n)() for n in lens]
            ids = (C.c_uint32 * len(slots))(*slots)
            ptrs = (C.c_void_p * len(slots))(*[C.cast(b, C.c_void_p) for b in bufs])
            ln = (C.c_uint32 * len(slots))(*lens)
            return lib.zrc4_ks_crypt(ks, ids, ptrs, ln, len(slots)), [bytes(b) for b in bufs]

        def ring_bytes():
            st = (C.c_uint64 * 6)()
            assert lib.zrc4_ks_stats(ks, st) == 0
            return st[0]

        refa = pyoracle.Rc4(b"slot-a")
        rc, (out,) = call([0], [64])                   # tail 1; A's refill is queued
        assert rc == 0 and out == refa.encryption(bytes(64))
        r0 = ring_bytes()
        rc, _ = call([0, 1], [16, 64])                 # A from its ring, B's tail fails (tail 2)
        assert rc != 0
        assert ring_bytes() - r0 == 16                 # A was served from its ring
        for slot in (0, 1):
            rc, (out,) = call([slot], [32])
            assert rc == -9 and out == bytes(32), slot  # ZRC4_ERR_STATE, nothing crypted
        for slot, key in ((0, b"slot-a"), (1, b"slot-b")):
            assert lib.zrc4_ks_make_sbox(ks, slot, key, len(key)) == 0
            rc, (out,) = call([slot], [100])
            assert rc == 0 and out == pyoracle.Rc4(key).encryption(bytes(100)), slot
    finally:
        if ks:
            lib.zrc4_ks_destroy(ks)
        lib.zrc4_destroy(ctx)
