"""Synthetic RC4 workloads, shared by bench.py and the tests.

  keys     session s: 16 bytes from std::mt19937_64(seed=1), 2 outputs/session
  payload  bytes of std::mt19937_64(seed=42) filling the contiguous [S][L] buffer
  advance  session s is pre-advanced (s*37) % 1000 bytes before timing

Session ids are GLOBAL: a shard of sessions [first, first+n) gets exactly the
keys/payload/advance the whole batch would give those sessions.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from .build import SYNTH, build_synth

CONFIGS = {
    # name: (sessions, payload bytes per session)   -- BASELINE.json configs[1..4]
    "cfg2": (4096, 1024),
    "cfg3": (65536, 256),
    "cfg4": (1024, 65536),
    "cfg5": (524288, 1024),
}

_lib = None


def lib():
    global _lib
    if _lib is None:
        build_synth()
        L = C.CDLL(str(SYNTH))
        L.zrc4_synth_keys.argtypes = [C.c_uint64, C.c_uint64, C.c_void_p]
        L.zrc4_synth_payload.argtypes = [C.c_uint64, C.c_uint64, C.c_void_p, C.c_int]
        L.zrc4_synth_payload.restype = C.c_int
        L.zrc4_synth_advance.argtypes = [C.c_uint64, C.c_uint64, C.c_void_p]
        _lib = L
    return _lib


def keys(first: int, n: int) -> np.ndarray:
    out = np.empty((n, 16), dtype=np.uint8)
    lib().zrc4_synth_keys(first, n, out.ctypes.data)
    return out


def payload(byte_first: int, nbytes: int, threads: int = 1) -> np.ndarray:
    out = np.empty(nbytes, dtype=np.uint8)
    rc = lib().zrc4_synth_payload(byte_first, nbytes, out.ctypes.data, threads)
    if rc:
        raise ValueError("payload byte_first must be a multiple of 8")
    return out


def advance(first: int, n: int) -> np.ndarray:
    out = np.empty(n, dtype=np.uint32)
    lib().zrc4_synth_advance(first, n, out.ctypes.data)
    return out


@dataclass
class Workload:
    first: int          # global id of the first session
    n: int              # sessions
    L: int              # payload bytes per session
    keys: np.ndarray    # (n,16) u8
    key_off: np.ndarray  # (n,) u64
    key_len: np.ndarray  # (n,) u32
    adv: np.ndarray     # (n,) u32 pre-advance lengths
    payload: np.ndarray  # (n*L,) u8
    off: np.ndarray     # (n,) u64 = i*L
    length: np.ndarray  # (n,) u32 = L


def make(first: int, n: int, L: int, threads: int = 1) -> Workload:
    k = keys(first, n)
    return Workload(
        first=first, n=n, L=L, keys=k.reshape(-1),
        key_off=(np.arange(n, dtype=np.uint64) * 16), key_len=np.full(n, 16, dtype=np.uint32),
        adv=advance(first, n), payload=payload(first * L, n * L, threads),
        off=np.arange(n, dtype=np.uint64) * np.uint64(L), length=np.full(n, L, dtype=np.uint32))
