"""oracle/pyoracle.py -- TEST INFRASTRUCTURE ONLY.

ctypes access to
  * oracle/liboracle.so       -- the C restatement (rc4_oracle.c), and
  * oracle/_ref/libzrc4_ref.so -- the REAL reference header compiled by
                                  oracle/Makefile (present only where it was
                                  built; used to pin the restatement),
plus a tiny pure-Python RC4 (for very small cases only), each citing
/root/reference/depends/rc4/rc4_encryption.h.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module.  The product path (zsummerx_amd) never does.
"""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "liboracle.so"
REF_LIB = HERE / "_ref" / "libzrc4_ref.so"

_P = C.c_void_p


class OracleState(C.Structure):
    # int x, y, box[256] -- the reference member layout (rc4_encryption.h:96-98)
    _fields_ = [("x", C.c_int), ("y", C.c_int), ("box", C.c_int * 256)]


_lib = None
_ref = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)


def lib():
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        L = C.CDLL(str(LIB))
        L.oracle_make_sbox.argtypes = [_P, _P, C.c_size_t]
        L.oracle_encryption.argtypes = [_P, _P, C.c_long]
        L.oracle_make_sbox_batch.argtypes = [_P, _P, _P, _P, C.c_uint32]
        L.oracle_crypt_batch.argtypes = [_P, _P, _P, _P, C.c_uint32, C.c_int]
        L.oracle_state_to_bytes.argtypes = [_P, _P, _P, _P]
        L.oracle_state_from_bytes.argtypes = [_P, _P, C.c_uint8, C.c_uint8]
        L.oracle_now.restype = C.c_double
        L.oracle_crypt_rate.argtypes = [_P, _P, _P, _P, C.c_uint32, C.c_int, C.c_double]
        L.oracle_crypt_rate.restype = C.c_double
        L.oracle_frame_scan.argtypes = [_P, _P, _P, C.c_uint32, C.c_uint32, C.c_uint32, _P, _P, _P, _P]
        _lib = L
    return _lib


def ref_lib():
    """The real reference RC4 (compiled from /root/reference), or None."""
    global _ref
    if _ref is None and REF_LIB.exists():
        R = C.CDLL(str(REF_LIB))
        R.zrc4_ref_state_size.restype = C.c_int
        R.zrc4_ref_make_sbox.argtypes = [_P, _P, C.c_size_t]
        R.zrc4_ref_encryption.argtypes = [_P, _P, C.c_int]
        R.zrc4_ref_get_state.argtypes = [_P, _P, _P, _P]
        R.zrc4_ref_crypt_batch.argtypes = [_P, _P, _P, _P, C.c_uint32]
        R.zrc4_ref_crypt_batch.restype = C.c_double
        R.zrc4_ref_crypt_rate.argtypes = [_P, _P, _P, _P, C.c_uint32, C.c_int, C.c_double]
        R.zrc4_ref_crypt_rate.restype = C.c_double
        R.zrc4_ref_has_raw_packet.argtypes = [_P, C.c_uint32, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint32)]
        _ref = R
    return _ref


def _buf(b: bytes):
    return (C.c_uint8 * max(1, len(b))).from_buffer_copy(b or b"\0")


class Rc4:
    """One oracle stream: makeSBox / encryption with the reference's semantics."""

    def __init__(self, key: bytes | None = None):
        self.st = OracleState()
        if key is not None:
            self.make_sbox(key)

    def make_sbox(self, key: bytes) -> None:
        lib().oracle_make_sbox(C.byref(self.st), _buf(key), len(key))

    def encryption(self, data, length: int | None = None) -> bytes | None:
        """Crypt in place if `data` is a bytearray/np.ndarray, else return bytes."""
        if isinstance(data, (bytes, memoryview)):
            arr = bytearray(data)
            self.encryption(arr, length if length is not None else len(arr))
            return bytes(arr)
        n = len(data) if length is None else length
        if isinstance(data, np.ndarray):
            lib().oracle_encryption(C.byref(self.st), C.c_void_p(data.ctypes.data), n)
        else:
            cbuf = (C.c_uint8 * max(1, len(data))).from_buffer(data) if len(data) else _buf(b"")
            lib().oracle_encryption(C.byref(self.st), cbuf, n)
        return None

    def state(self):
        sb = (C.c_uint8 * 256)()
        x, y = C.c_uint8(), C.c_uint8()
        lib().oracle_state_to_bytes(C.byref(self.st), sb, C.byref(x), C.byref(y))
        return bytes(sb), x.value, y.value

    def set_state(self, sbox: bytes, x: int, y: int) -> None:
        lib().oracle_state_from_bytes(C.byref(self.st), _buf(sbox), x, y)


class RefRc4:
    """One stream of the REAL reference class RC4Encryption (oracle/_ref)."""

    def __init__(self, key: bytes | None = None):
        R = ref_lib()
        if R is None:
            raise FileNotFoundError(f"{REF_LIB} not built (needs /root/reference)")
        self.R = R
        self.mem = (C.c_uint8 * R.zrc4_ref_state_size())()
        if key is not None:
            self.make_sbox(key)

    def make_sbox(self, key: bytes) -> None:
        self.R.zrc4_ref_make_sbox(self.mem, _buf(key), len(key))

    def encryption(self, data: bytes, length: int | None = None) -> bytes:
        arr = bytearray(data)
        n = len(arr) if length is None else length
        cbuf = (C.c_uint8 * max(1, len(arr))).from_buffer(arr) if arr else _buf(b"")
        self.R.zrc4_ref_encryption(self.mem, cbuf, n)
        return bytes(arr)

    def state(self):
        sb = (C.c_uint8 * 256)()
        x, y = C.c_uint8(), C.c_uint8()
        self.R.zrc4_ref_get_state(self.mem, sb, C.byref(x), C.byref(y))
        return bytes(sb), x.value, y.value


class RefBatch:
    """n streams of the REAL reference class in one array (oracle/_ref), for
    the CPU baseline (bench.py cpu_baseline, kind "reference")."""

    def __init__(self, n: int):
        R = ref_lib()
        if R is None:
            raise FileNotFoundError(f"{REF_LIB} not built (needs /root/reference)")
        self.R, self.n, self.sz = R, n, R.zrc4_ref_state_size()
        self.mem = (C.c_uint8 * (self.sz * n))()
        self.base = C.addressof(self.mem)

    def make_sbox(self, keys: np.ndarray, key_off: np.ndarray, key_len: np.ndarray) -> None:
        keys = np.ascontiguousarray(keys, dtype=np.uint8)
        for i in range(self.n):
            o = int(key_off[i])
            self.R.zrc4_ref_make_sbox(C.c_void_p(self.base + i * self.sz), C.c_void_p(keys.ctypes.data + o),
                                      int(key_len[i]))

    def advance(self, adv: np.ndarray) -> None:
        """Pre-advance stream i by adv[i] keystream bytes (encryption over zeros)."""
        scratch = np.zeros(int(np.max(adv)) if len(adv) else 1, dtype=np.uint8)
        for i in range(self.n):
            if adv[i]:
                self.R.zrc4_ref_encryption(C.c_void_p(self.base + i * self.sz), C.c_void_p(scratch.ctypes.data),
                                           int(adv[i]))

    def crypt_rate(self, payload: np.ndarray, off: np.ndarray, length: np.ndarray, threads: int,
                   seconds: float) -> float:
        off = np.ascontiguousarray(off, dtype=np.uint64)
        length = np.ascontiguousarray(length, dtype=np.uint32)
        r = self.R.zrc4_ref_crypt_rate(C.c_void_p(self.base), C.c_void_p(payload.ctypes.data),
                                       C.c_void_p(off.ctypes.data), C.c_void_p(length.ctypes.data), self.n,
                                       int(threads), float(seconds))
        if r <= 0:
            raise RuntimeError("zrc4_ref_crypt_rate failed")
        return r


def py_rc4(key: bytes, data: bytes, skip: int = 0) -> bytes:
    """Pure-Python RC4, small cases only (rc4_encryption.h:46-93)."""
    S = list(range(256))
    if key:
        j = 0
        for i in range(256):
            j = (j + S[i] + key[i % len(key)]) & 255
            S[i], S[j] = S[j], S[i]
    x = y = 0
    out = bytearray()
    for n in range(skip + len(data)):
        x = (x + 1) & 255
        a = S[x]
        y = (y + a) & 255
        b = S[y]
        S[x], S[y] = b, a
        if n >= skip:
            out.append(data[n - skip] ^ S[(a + b) & 255])
    return bytes(out)


class Batch:
    """n oracle streams in one contiguous array (for batch crypt and timing)."""

    def __init__(self, n: int):
        self.n = n
        self.st = (OracleState * max(1, n))()

    def make_sbox(self, keys: np.ndarray, key_off: np.ndarray, key_len: np.ndarray) -> None:
        keys = np.ascontiguousarray(keys, dtype=np.uint8)
        key_off = np.ascontiguousarray(key_off, dtype=np.uint64)
        key_len = np.ascontiguousarray(key_len, dtype=np.uint32)
        lib().oracle_make_sbox_batch(self.st, C.c_void_p(keys.ctypes.data),
                                     C.c_void_p(key_off.ctypes.data),
                                     C.c_void_p(key_len.ctypes.data), self.n)

    def crypt(self, payload: np.ndarray, off: np.ndarray, length: np.ndarray, threads: int = 1) -> None:
        off = np.ascontiguousarray(off, dtype=np.uint64)
        length = np.ascontiguousarray(length, dtype=np.uint32)
        lib().oracle_crypt_batch(self.st, C.c_void_p(payload.ctypes.data),
                                 C.c_void_p(off.ctypes.data), C.c_void_p(length.ctypes.data),
                                 self.n, int(threads))

    def crypt_rate(self, payload: np.ndarray, off: np.ndarray, length: np.ndarray, threads: int,
                   seconds: float) -> float:
        """Bytes/s of `threads` workers re-crypting their share for `seconds`."""
        off = np.ascontiguousarray(off, dtype=np.uint64)
        length = np.ascontiguousarray(length, dtype=np.uint32)
        r = lib().oracle_crypt_rate(self.st, C.c_void_p(payload.ctypes.data), C.c_void_p(off.ctypes.data),
                                    C.c_void_p(length.ctypes.data), self.n, int(threads), float(seconds))
        if r < 0:
            raise RuntimeError("oracle_crypt_rate: thread setup failed")
        return r

    def state(self, i: int):
        sb = (C.c_uint8 * 256)()
        x, y = C.c_uint8(), C.c_uint8()
        lib().oracle_state_to_bytes(C.byref(self.st[i]), sb, C.byref(x), C.byref(y))
        return bytes(sb), x.value, y.value

    def states(self):
        """Every stream's (box uint8[n, 256], x uint8[n], y uint8[n]) at once
        (the int fields narrowed to bytes, as oracle_state_to_bytes does)."""
        a = np.frombuffer(self.st, dtype=np.int32).reshape(-1, 258)[: self.n]
        return a[:, 2:].astype(np.uint8), a[:, 0].astype(np.uint8), a[:, 1].astype(np.uint8)


def now() -> float:
    return lib().oracle_now()


def frame_scan(buf: np.ndarray, off: np.ndarray, length: np.ndarray, bound: int, max_packets: int):
    """oracle_frame_scan: (npk, used, status, pkt_len[n, max_packets])."""
    n = int(length.size)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    length = np.ascontiguousarray(length, dtype=np.uint32)
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    npk, used, status = (np.zeros(n, dtype=np.uint32) for _ in range(3))
    pk = np.zeros((n, max(1, max_packets)), dtype=np.uint32)
    p = lambda a: C.c_void_p(a.ctypes.data)
    lib().oracle_frame_scan(p(buf), p(off), p(length), int(bound), n, int(max_packets), p(npk), p(used),
                            p(status), p(pk))
    return npk, used, status, pk


def py_frame_scan(data: bytes, bound: int):
    """Pure-Python restatement for tiny cases (session.cpp:329-371 +
    proto4z.h:704-748): list of packet lengths, used, status."""
    used, out = 0, []
    while True:
        cur, bl = len(data) - used, bound - used
        if bl < cur or bound < bl:
            return out, used, 2
        if cur < 6:
            return out, used, 1
        pl = int.from_bytes(data[used:used + 4], "little")
        if pl < 6:
            return out, used, 2
        if pl > bl:
            return out, used, (2 if pl > bound else 1)
        if pl > bound:
            return out, used, 2
        if pl > cur:
            return out, used, 1
        out.append(pl)
        used += pl


def ref_frame_scan(data: bytes, bound: int):
    """The onRecv framing loop (src/frame/session.cpp:329-371) driven by the
    REAL reference HasRawPacket (oracle/_ref): (packet lengths, used, status)."""
    R = ref_lib()
    if R is None:
        raise FileNotFoundError(f"{REF_LIB} not built (needs /root/reference)")
    buf = _buf(data)
    base = C.addressof(buf)
    used, out = 0, []
    while True:
        second = C.c_uint32()
        st = R.zrc4_ref_has_raw_packet(C.c_void_p(base + used), len(data) - used, bound - used, bound,
                                       C.byref(second))
        if st != 0:
            return out, used, st
        out.append(second.value)
        used += second.value
