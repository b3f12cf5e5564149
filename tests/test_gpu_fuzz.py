"""Randomised GPU parity sweep over the whole C-ABI crypt surface.

One context and one oracle arena (oracle/rc4_oracle.c, pinned to the real
reference header, rc4_encryption.h:74-93) live through a seeded sequence of
calls; every call is drawn at random from
  range     zrc4_crypt_range, aligned or unaligned first slot;
  ids       zrc4_crypt with distinct slots anywhere (per-lane gathers);
  grouped   zrc4_crypt_grouped, buckets of random subsets of distinct groups;
  declared  zrc4_crypt_grouped_declared, the same with the groups declared;
with 1..360 groups on both sides of every kernel boundary launch_crypt
knows (the window kernel, half-group, whole-group and persistent kernels), ragged
lengths of a random scale (including 0 and multi-chunk messages),
unaligned offsets and gaps.  The reference runs each session's
RC4Encryption::encryption in call order (src/frame/session.cpp:313-323);
after every call the payload must match the oracle byte for byte, and at
the end every one of the arena's states must too.  Parity: bit-exact."""
import ctypes as C

import numpy as np
import pytest

import pyoracle
from conftest import soak_seeds
from zsummerx_amd import Context
from zsummerx_amd._capi import IDLE_SLOT

pytestmark = pytest.mark.gpu

GROUPS = 400                       # arena: 102 400 slots
CALLS = 84


def _oracle_ids(ob, data, slots, off, L):
    enc = pyoracle.lib().oracle_encryption
    for e in np.flatnonzero((slots != IDLE_SLOT) & (L > 0)):
        enc(C.byref(ob.st[int(slots[e])]), C.c_void_p(data.ctypes.data + int(off[e])), int(L[e]))


def _layout(rng, n, scale):
    L = rng.integers(0, scale + 1, n).astype(np.uint32)
    L[rng.random(n) < 0.08] = 0
    gaps = rng.integers(0, 20, n)
    off = np.cumsum(np.concatenate([[gaps[0]], L[:-1].astype(np.int64) + gaps[1:]])).astype(np.uint64)
    return L, off, int(off[-1] + L[-1]) + 64


def test_random_call_sequence(built):
    _run_sequence(20260518)


@pytest.mark.parametrize("seed", soak_seeds())
def test_random_call_sequence_soak(built, seed):
    """The same sweep from other seeds (one by default; scripts/r06_soak.sh
    runs many in one process through $ZRC4_SOAK_SEEDS)."""
    _run_sequence(1000 + seed)


def _run_sequence(seed):
    import torch
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    rng = np.random.default_rng(seed)
    cap = 256 * GROUPS
    keys = rng.integers(0, 256, 16 * cap, dtype=np.uint8)
    koff = np.arange(cap, dtype=np.uint64) * 16
    klen = rng.integers(1, 17, cap).astype(np.uint32)
    ob = pyoracle.Batch(cap)
    ob.make_sbox(keys, koff, klen)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    s = torch.cuda.current_stream()
    seen = []
    with Context(0, cap) as c:
        c.ksa_range(0, T(klen.view(np.int32)), T(koff.view(np.int64)), T(keys), stream=s)
        # group counts on both sides of every launch_crypt boundary (32: window;
        # 128: half-group; 256: whole-group; above: persistent), shuffled
        classes = [1, 5, 17, 32, 33, 90, 128, 129, 200, 256, 257, 300, 360, 3]
        plan = [int(v) for v in rng.permutation(classes * 6)][:CALLS]
        for call in range(CALLS):
            mode = ["range", "ids", "grouped", "declared"][call % 4]
            ng = plan[call]
            scale = int(rng.choice([40, 300, 1500, 5000]))
            if ng > 64:
                scale = min(scale, 1500)
            if mode == "range":
                n = max(1, ng * 256 - int(rng.integers(0, 200)))
                aligned = rng.random() < 0.7
                first = int(rng.integers(0, GROUPS - ng)) * 256 + (0 if aligned else int(rng.integers(1, 256)))
                n = min(n, cap - first)
                L, off, size = _layout(rng, n, scale)
                data = rng.integers(0, 256, size, dtype=np.uint8)
                want = data.copy()
                pyoracle.lib().oracle_crypt_batch(C.byref(ob.st, first * C.sizeof(pyoracle.OracleState)),
                                                  C.c_void_p(want.ctypes.data), C.c_void_p(off.ctypes.data),
                                                  C.c_void_p(L.ctypes.data), n, 8)
                pay = T(data)
                c.crypt_range(first, pay, T(off.view(np.int64)), T(L.view(np.int32)), stream=s)
            elif mode == "ids":
                n = min(ng * 256, 20000)
                slots = rng.permutation(cap)[:n].astype(np.uint32)
                L, off, size = _layout(rng, n, scale)
                data = rng.integers(0, 256, size, dtype=np.uint8)
                want = data.copy()
                _oracle_ids(ob, want, slots, off, L)
                pay = T(data)
                c.crypt(pay, T(off.view(np.int64)), T(L.view(np.int32)), ids=T(slots.view(np.int32)), stream=s)
            else:
                groups = rng.permutation(GROUPS)[:ng].astype(np.uint32)
                fill = int(rng.choice([256, 128, 16]))
                ids = np.full(256 * ng, IDLE_SLOT, dtype=np.uint32)
                for b, g in enumerate(groups):
                    k = int(rng.integers(1, fill + 1))
                    ids[256 * b + rng.permutation(256)[:k]] = g * 256 + rng.permutation(256)[:k]
                idle = rng.random(ng) < 0.1
                idle[-1] = False
                for b in np.flatnonzero(idle):
                    ids[256 * b: 256 * (b + 1)] = IDLE_SLOT
                decl = np.where(idle, IDLE_SLOT, groups).astype(np.uint32)
                L, off, size = _layout(rng, ids.size, scale)
                L[ids == IDLE_SLOT] = 0
                data = rng.integers(0, 256, size, dtype=np.uint8)
                want = data.copy()
                _oracle_ids(ob, want, ids, off, L)
                pay = T(data)
                if mode == "grouped":
                    c.crypt_grouped(pay, T(off.view(np.int64)), T(L.view(np.int32)), T(ids.view(np.int32)),
                                    stream=s)
                else:
                    c.crypt_grouped_declared(pay, T(off.view(np.int64)), T(L.view(np.int32)),
                                             T(ids.view(np.int32)), decl, stream=s)
            c.sync(s)
            got = pay.cpu().numpy()
            bad = np.flatnonzero(got != want)
            seen.append((mode, ng, scale))
            assert bad.size == 0, (call, mode, ng, scale, bad[:8], int(bad.size))
        gsb, gx, gy = c.get_states(0, cap)
        osb, ox, oy = ob.states()
        bad = np.flatnonzero((gsb != osb).any(axis=1) | (gx != ox) | (gy != oy))
        assert bad.size == 0, (bad[:8], int(bad.size))
    # the sweep reached the window and the persistent kernels with grouped ids
    assert any(m in ("grouped", "declared") and g <= 32 for m, g, _ in seen), seen
    assert any(m in ("grouped", "declared") and g > 256 for m, g, _ in seen), seen


@pytest.mark.parametrize("seed", soak_seeds())
def test_ksa_soak(built, seed):
    """Batched makeSBox (rc4_encryption.h:46-72) from random seeds (one by
    default; scripts/r06_soak.sh runs many through $ZRC4_SOAK_SEEDS): 1-6 000
    keys whose lengths hit every ksa_kernel path half the time (0, the
    register patterns 1-64, the LDS window's edges 48-50, the per-step fetch
    up to 300) and are uniform in 0..300 otherwise, NUL-rich, at random
    alignments, through zrc4_ksa_range at a random (often unaligned) first
    slot or zrc4_ksa with random ids; every state against the oracle."""
    import torch
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    rng = np.random.default_rng(5000 + seed)
    n = int(rng.integers(1, 6001))
    edges = np.array([0, 1, 2, 4, 8, 16, 31, 32, 33, 48, 49, 50, 63, 64, 65, 128, 255, 256, 257, 300])
    klen = np.where(rng.random(n) < 0.5, rng.choice(edges, n), rng.integers(0, 301, n)).astype(np.uint32)
    gaps = rng.integers(0, 17, n)
    koff = np.cumsum(np.concatenate([[gaps[0]], klen[:-1].astype(np.int64) + gaps[1:]])).astype(np.uint64)
    keys = rng.integers(0, 256, int(koff[-1] + klen[-1]) + 8, dtype=np.uint8)
    keys[rng.random(keys.size) < 0.1] = 0
    cap = 256 * (-(-n // 256) + 2)
    ob = pyoracle.Batch(n)
    ob.make_sbox(keys, koff, klen)
    osb, ox, oy = ob.states()
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    s = torch.cuda.current_stream()
    with Context(0, cap) as c:
        if rng.random() < 0.5:
            first = int(rng.integers(0, cap - n + 1))
            slots = first + np.arange(n)
            c.ksa_range(first, T(klen.view(np.int32)), T(koff.view(np.int64)), T(keys), stream=s)
        else:
            slots = rng.permutation(cap)[:n]
            c.ksa(T(klen.view(np.int32)), T(koff.view(np.int64)), T(keys),
                  ids=T(slots.astype(np.uint32).view(np.int32)), stream=s)
        c.sync(s)
        gsb, gx, gy = c.get_states(0, cap)
    bad = np.flatnonzero((gsb[slots] != osb).any(axis=1) | (gx[slots] != ox) | (gy[slots] != oy))
    assert bad.size == 0, (n, bad[:8].tolist(), klen[bad[:8]].tolist(), int(bad.size))
