"""zsummerx_amd -- MI355X-native RC4 payload-encryption path for zsummerX.

Host-side mirror of the reference interface for this path:

  class RC4Encryption                    depends/rc4/rc4_encryption.h:43-99
      makeSBox(obscure)                  :46-72
      encryption(data, length)           :74-93   (in place; length <= 0 no-op)

backed by the C-ABI library libzrc4.so (include/zrc4.h), whose kernels run on
gfx950.  `Context` exposes the batched, device-resident entry points used by
the session hooks (src/frame/session.cpp:110-111, 313-323, 496-499, 535-538,
603-606), the bench and the parity tests.  There is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import threading

import numpy as np

from ._capi import FrameArgs, ZRC4Error, check, load

__all__ = ["Context", "RC4Encryption", "ZRC4Error", "load", "default_context"]

GROUP_SLOTS = 256
STATE_BYTES = 258
_IDENTITY = bytes(range(256))


def _ptr(a) -> C.c_void_p | None:
    if a is None:
        return None
    if isinstance(a, int):
        return C.c_void_p(a)
    if hasattr(a, "data_ptr"):          # torch tensor (device memory)
        return C.c_void_p(a.data_ptr())
    if isinstance(a, np.ndarray):
        if not a.flags["C_CONTIGUOUS"]:
            raise ValueError("array must be C-contiguous")
        return C.c_void_p(a.ctypes.data)
    raise TypeError(f"cannot take a pointer of {type(a)!r}")


def _stream(s) -> C.c_void_p | None:
    if s is None:
        return None
    if isinstance(s, int):
        return C.c_void_p(s)
    return C.c_void_p(s.cuda_stream)     # torch.cuda.Stream


class Context:
    """One device, one arena of `capacity` RC4 streams (slots).  `lib`: an
    A/B build of the same C-ABI (zsummerx_amd.build.build_variant), default the
    product libzrc4.so."""

    def __init__(self, device: int = 0, capacity: int = GROUP_SLOTS, lib=None):
        self._lib = load(lib) if lib is not None else load()
        h = C.c_void_p()
        check(self._lib.zrc4_create(C.byref(h), int(device), int(capacity)), "zrc4_create")
        self._h = h
        self.device = int(device)
        self.capacity = int(self._lib.zrc4_capacity(h))
        # slot allocator of the RC4Encryption mirror: per context, with a free list
        self._slot_lock = threading.Lock()
        self._free_slots: list[int] = []
        self._next_slot = 0

    # -- slot allocation (RC4Encryption instances) ---------------------------
    def acquire_slot(self) -> int:
        with self._slot_lock:
            if self._free_slots:
                return self._free_slots.pop()
            if self._next_slot >= self.capacity:
                raise ZRC4Error(-5, "RC4Encryption: context out of slots")
            self._next_slot += 1
            return self._next_slot - 1

    def release_slot(self, slot: int) -> None:
        """Give a slot back; it is reset to the empty-key state (identity box,
        x = y = 0: what makeSBox("") leaves, rc4_encryption.h:48-56) so a
        later owner never sees the previous owner's stream."""
        if not getattr(self, "_h", None):
            return
        self.set_state(slot, _IDENTITY, 0, 0)
        with self._slot_lock:
            self._free_slots.append(int(slot))

    # -- lifetime ---------------------------------------------------------
    def close(self) -> None:
        if getattr(self, "_h", None):
            check(self._lib.zrc4_destroy(self._h), "zrc4_destroy")
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- device-pointer batch API (torch tensors, ints or None) ------------
    def ksa(self, key_len, key_off, keys, ids=None, n=None, stream=None) -> None:
        n = int(key_len.numel() if n is None else n)
        check(self._lib.zrc4_ksa(self._h, _ptr(ids), _ptr(keys), _ptr(key_off), _ptr(key_len),
                                 n, _stream(stream)), "zrc4_ksa")

    def crypt(self, payload, off, length, ids=None, n=None, stream=None) -> None:
        n = int(length.numel() if n is None else n)
        check(self._lib.zrc4_crypt(self._h, _ptr(ids), _ptr(payload), _ptr(off), _ptr(length),
                                   n, _stream(stream)), "zrc4_crypt")

    def ksa_range(self, first_slot: int, key_len, key_off, keys, n=None, stream=None) -> None:
        n = int(key_len.numel() if n is None else n)
        check(self._lib.zrc4_ksa_range(self._h, int(first_slot), _ptr(keys), _ptr(key_off),
                                       _ptr(key_len), n, _stream(stream)), "zrc4_ksa_range")

    def crypt_range(self, first_slot: int, payload, off, length, n=None, stream=None) -> None:
        n = int(length.numel() if n is None else n)
        check(self._lib.zrc4_crypt_range(self._h, int(first_slot), _ptr(payload), _ptr(off),
                                         _ptr(length), n, _stream(stream)), "zrc4_crypt_range")

    def crypt_grouped(self, payload, off, length, ids, n=None, stream=None) -> None:
        """zrc4_crypt_grouped: 256-entry buckets, each within one slot group."""
        n = int(length.numel() if n is None else n)
        check(self._lib.zrc4_crypt_grouped(self._h, _ptr(ids), _ptr(payload), _ptr(off), _ptr(length),
                                           n, _stream(stream)), "zrc4_crypt_grouped")

    def crypt_grouped_declared(self, payload, off, length, ids, bucket_group, frame: dict | None = None, n=None,
                               stream=None) -> None:
        """zrc4_crypt_grouped_declared: zrc4_crypt_grouped with each bucket's
        group given from the host (bucket_group: ceil(n/256) ints, IDLE_SLOT
        for an idle bucket); optional framing as crypt_grouped_frame."""
        n = int(length.numel() if n is None else n)
        bg = np.ascontiguousarray(bucket_group, dtype=np.uint32)
        if bg.size < -(-n // GROUP_SLOTS):
            raise ValueError("bucket_group needs one entry per 256-entry bucket")
        fa = self._frame(frame) if frame is not None else None
        check(self._lib.zrc4_crypt_grouped_declared(self._h, _ptr(ids), _ptr(bg), _ptr(payload), _ptr(off),
                                                    _ptr(length), n, C.byref(fa) if fa is not None else None,
                                                    _stream(stream)), "zrc4_crypt_grouped_declared")

    @staticmethod
    def _frame(frame: dict) -> FrameArgs:
        return FrameArgs(_ptr(frame["off"]), _ptr(frame["len"]), int(frame["bound"]), int(frame.get("max_packets", 0)),
                         _ptr(frame["npk"]), _ptr(frame["used"]), _ptr(frame["status"]), _ptr(frame.get("pkt_len")))

    def crypt_range_frame(self, first_slot: int, payload, off, length, frame: dict, n=None, stream=None) -> None:
        """zrc4_crypt_range_frame: decrypt + proto4z framing in one launch.
        frame = {off, len, bound, npk, used, status[, pkt_len, max_packets]}."""
        n = int(length.numel() if n is None else n)
        fa = self._frame(frame)
        check(self._lib.zrc4_crypt_range_frame(self._h, int(first_slot), _ptr(payload), _ptr(off), _ptr(length), n,
                                               C.byref(fa), _stream(stream)), "zrc4_crypt_range_frame")

    def crypt_grouped_frame(self, payload, off, length, ids, frame: dict, n=None, stream=None) -> None:
        n = int(length.numel() if n is None else n)
        fa = self._frame(frame)
        check(self._lib.zrc4_crypt_grouped_frame(self._h, _ptr(ids), _ptr(payload), _ptr(off), _ptr(length), n,
                                                 C.byref(fa), _stream(stream)), "zrc4_crypt_grouped_frame")

    def xor_ring(self, ring, ring_cap: int, rid, pos, payload, off, length, n=None, stream=None) -> None:
        """zrc4_xor_ring: payload spans ^= keystream rings (consumed bytes zeroed)."""
        n = int(length.numel() if n is None else n)
        check(self._lib.zrc4_xor_ring(self._h, _ptr(ring), int(ring_cap), _ptr(rid), _ptr(pos), _ptr(payload),
                                      _ptr(off), _ptr(length), n, _stream(stream)), "zrc4_xor_ring")

    def frame_scan(self, buf, off, length, bound: int, npk, used, status, pkt_len=None, max_packets: int = 0,
                   n=None, stream=None) -> None:
        """zrc4_frame_scan: proto4z framing of decrypted buffers (device pointers)."""
        n = int(length.numel() if n is None else n)
        check(self._lib.zrc4_frame_scan(self._h, _ptr(buf), _ptr(off), _ptr(length), int(bound), n,
                                        int(max_packets), _ptr(npk), _ptr(used), _ptr(status), _ptr(pkt_len),
                                        _stream(stream)), "zrc4_frame_scan")

    def sync(self, stream=None) -> None:
        check(self._lib.zrc4_sync(self._h, _stream(stream)), "zrc4_sync")

    # -- host-pointer batch API (numpy) -------------------------------------
    def ksa_host(self, keys, ids=None) -> None:
        """keys: list of bytes, one per entry (slot ids[i] or i)."""
        n = len(keys)
        blob = np.frombuffer(b"".join(keys) or b"\0", dtype=np.uint8).copy()
        lens = np.array([len(k) for k in keys], dtype=np.uint32)
        offs = np.zeros(n, dtype=np.uint64)
        if n > 1:
            offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
        idv = None if ids is None else np.ascontiguousarray(ids, dtype=np.uint32)
        check(self._lib.zrc4_ksa_host(self._h, _ptr(idv), _ptr(blob), int(lens.sum()), _ptr(offs),
                                      _ptr(lens), n), "zrc4_ksa_host")

    def crypt_host(self, payload: np.ndarray, off, length, ids=None) -> None:
        """In-place crypt of a uint8 numpy buffer."""
        if payload.dtype != np.uint8 or not payload.flags["C_CONTIGUOUS"]:
            raise ValueError("payload must be a C-contiguous uint8 array")
        offv = np.ascontiguousarray(off, dtype=np.uint64)
        lenv = np.ascontiguousarray(length, dtype=np.uint32)
        if offv.shape != lenv.shape:
            raise ValueError("off and length must have the same shape")
        idv = None if ids is None else np.ascontiguousarray(ids, dtype=np.uint32)
        check(self._lib.zrc4_crypt_host(self._h, _ptr(idv), _ptr(payload), payload.nbytes,
                                        _ptr(offv), _ptr(lenv), lenv.size), "zrc4_crypt_host")

    # -- single-stream drop-ins --------------------------------------------
    def make_sbox(self, slot: int, key) -> None:
        kb = key.encode() if isinstance(key, str) else bytes(key)
        buf = (C.c_uint8 * max(1, len(kb))).from_buffer_copy(kb or b"\0")
        check(self._lib.zrc4_make_sbox(self._h, int(slot), buf, len(kb)), "zrc4_make_sbox")

    def encryption(self, slot: int, data, length: int) -> None:
        if isinstance(data, np.ndarray):
            if data.dtype != np.uint8 or not data.flags["C_CONTIGUOUS"]:
                raise ValueError("data must be a C-contiguous uint8 array")
            if length > data.nbytes:
                raise ValueError("length exceeds buffer")
            p = _ptr(data)
        else:  # bytearray
            if length > len(data):
                raise ValueError("length exceeds buffer")
            p = C.cast((C.c_uint8 * len(data)).from_buffer(data), C.c_void_p) if len(data) else None
        check(self._lib.zrc4_encryption(self._h, int(slot), p, int(length)), "zrc4_encryption")

    def get_state(self, slot: int):
        sbox = (C.c_uint8 * 256)()
        x, y = C.c_uint8(), C.c_uint8()
        check(self._lib.zrc4_get_state(self._h, int(slot), sbox, C.byref(x), C.byref(y)),
              "zrc4_get_state")
        return bytes(sbox), x.value, y.value

    def get_states(self, first_slot: int, n: int):
        """zrc4_get_states: (sbox uint8[n, 256], x uint8[n], y uint8[n]) of
        slots first_slot .. first_slot + n - 1 in one copy."""
        sb = np.empty((n, 256), dtype=np.uint8)
        x = np.empty(n, dtype=np.uint8)
        y = np.empty(n, dtype=np.uint8)
        check(self._lib.zrc4_get_states(self._h, int(first_slot), int(n), _ptr(sb), _ptr(x), _ptr(y)),
              "zrc4_get_states")
        return sb, x, y

    def set_state(self, slot: int, sbox: bytes, x: int, y: int) -> None:
        if len(sbox) != 256:
            raise ValueError("sbox must be 256 bytes")
        buf = (C.c_uint8 * 256).from_buffer_copy(bytes(sbox))
        check(self._lib.zrc4_set_state(self._h, int(slot), buf, int(x), int(y)), "zrc4_set_state")


_default = None
_default_lock = threading.Lock()


def default_context(capacity: int = 1 << 16) -> Context:
    global _default
    with _default_lock:
        if _default is None:
            _default = Context(0, capacity)
        return _default


class RC4Encryption:
    """Drop-in mirror of the reference class (rc4_encryption.h:43-99).

    Each instance owns one slot of a context (the process-wide default one
    unless `ctx` is given) and gives it back when it is closed or collected,
    so instances can come and go like the reference's value objects (two per
    TcpSession, session.h:115-116).  Like the reference, a fresh instance must
    be seeded with makeSBox before use (the reference leaves the state
    indeterminate; here a fresh or recycled slot is the empty-key identity
    state)."""

    def __init__(self, ctx: Context | None = None):
        self._ctx = ctx or default_context()
        self._slot = self._ctx.acquire_slot()

    def makeSBox(self, obscure) -> None:  # noqa: N802  (reference name)
        self._ctx.make_sbox(self._slot, obscure)

    def encryption(self, data, length: int) -> None:
        self._ctx.encryption(self._slot, data, length)

    @property
    def slot(self) -> int:
        return self._slot

    def close(self) -> None:
        """Return the slot to the context (idempotent)."""
        slot, self._slot = getattr(self, "_slot", None), None
        if slot is not None:
            self._ctx.release_slot(slot)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
