"""ctypes binding of include/zrc4.h (the C-ABI a maintainer's FFI would bind).

No fallback: if libzrc4.so is missing or no gfx950 device is present, the
calls fail loudly (ZRC4Error), they never drop to a CPU path.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

_PKG = Path(__file__).resolve().parent
LIB_PATH = _PKG / "libzrc4.so"
# A/B validation only: run the suite against an in-tree variant build
# (zsummerx_amd/libzrc4_<name>.so from zsummerx_amd.build.build_variant)
if os.environ.get("ZSX_ZRC4_VARIANT"):
    LIB_PATH = _PKG / f"libzrc4_{os.environ['ZSX_ZRC4_VARIANT']}.so"

ZRC4_OK = 0
ERRORS = {
    -1: "ZRC4_ERR_INVALID_ARG",
    -2: "ZRC4_ERR_NO_DEVICE",
    -3: "ZRC4_ERR_OUT_OF_MEMORY",
    -4: "ZRC4_ERR_LAUNCH",
    -5: "ZRC4_ERR_SLOT_RANGE",
    -6: "ZRC4_ERR_HIP",
    -7: "ZRC4_ERR_GROUP",
    -8: "ZRC4_ERR_INTERNAL",
    -9: "ZRC4_ERR_STATE",
}
IDLE_SLOT = 0xFFFFFFFF

# (name, restype, argtypes) for every symbol declared in include/zrc4.h
_P = C.c_void_p
_U8P = C.POINTER(C.c_uint8)
SIGNATURES = [
    ("zrc4_create", C.c_int, [C.POINTER(_P), C.c_int, C.c_uint32]),
    ("zrc4_destroy", C.c_int, [_P]),
    ("zrc4_capacity", C.c_uint32, [_P]),
    ("zrc4_ksa", C.c_int, [_P, _P, _P, _P, _P, C.c_uint32, _P]),
    ("zrc4_crypt", C.c_int, [_P, _P, _P, _P, _P, C.c_uint32, _P]),
    ("zrc4_ksa_range", C.c_int, [_P, C.c_uint32, _P, _P, _P, C.c_uint32, _P]),
    ("zrc4_crypt_range", C.c_int, [_P, C.c_uint32, _P, _P, _P, C.c_uint32, _P]),
    ("zrc4_crypt_grouped", C.c_int, [_P, _P, _P, _P, _P, C.c_uint32, _P]),
    ("zrc4_crypt_grouped_declared", C.c_int, [_P, _P, _P, _P, _P, _P, C.c_uint32, _P, _P]),
    ("zrc4_crypt_range_frame", C.c_int, [_P, C.c_uint32, _P, _P, _P, C.c_uint32, _P, _P]),
    ("zrc4_crypt_grouped_frame", C.c_int, [_P, _P, _P, _P, _P, C.c_uint32, _P, _P]),
    ("zrc4_ksa_host", C.c_int, [_P, _P, _P, C.c_size_t, _P, _P, C.c_uint32]),
    ("zrc4_crypt_host", C.c_int, [_P, _P, _P, C.c_size_t, _P, _P, C.c_uint32]),
    ("zrc4_make_sbox", C.c_int, [_P, C.c_uint32, _P, C.c_size_t]),
    ("zrc4_encryption", C.c_int, [_P, C.c_uint32, _P, C.c_int]),
    ("zrc4_xor_ring", C.c_int, [_P, _P, C.c_uint32, _P, _P, _P, _P, _P, C.c_uint32, _P]),
    ("zrc4_frame_scan", C.c_int, [_P, _P, _P, _P, C.c_uint32, C.c_uint32, C.c_uint32, _P, _P, _P, _P, _P]),
    ("zrc4_ks_create", C.c_int, [_P, C.c_uint32, C.POINTER(_P)]),
    ("zrc4_ks_destroy", C.c_int, [_P]),
    ("zrc4_ks_crypt", C.c_int, [_P, _P, _P, _P, C.c_uint32]),
    ("zrc4_ks_make_sbox", C.c_int, [_P, C.c_uint32, _P, C.c_size_t]),
    ("zrc4_ks_copy", C.c_int, [_P, C.c_uint32, _P, C.c_uint32]),
    ("zrc4_ks_stats", C.c_int, [_P, C.POINTER(C.c_uint64)]),
    ("zrc4_sync", C.c_int, [_P, _P]),
    ("zrc4_poll_faults", C.c_int, [_P]),
    ("zrc4_get_state", C.c_int, [_P, C.c_uint32, _U8P, _U8P, _U8P]),
    ("zrc4_set_state", C.c_int, [_P, C.c_uint32, _U8P, C.c_uint8, C.c_uint8]),
    ("zrc4_get_states", C.c_int, [_P, C.c_uint32, C.c_uint32, _P, _P, _P]),
    ("zrc4_strerror", C.c_char_p, [C.c_int]),
    ("zrc4_version", C.c_char_p, []),
]


class FrameArgs(C.Structure):
    """struct zrc4_frame_args (include/zrc4.h)."""
    _fields_ = [("off", _P), ("len", _P), ("bound", C.c_uint32), ("max_packets", C.c_uint32),
                ("npk", _P), ("used", _P), ("status", _P), ("pkt_len", _P)]


class ZRC4Error(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        self.code = code
        name = ERRORS.get(code, str(code))
        msg = f"{name}: {_strerror(code)}"
        super().__init__(f"{what}: {msg}" if what else msg)


_lib = None


def load(path: Path | str | None = None) -> C.CDLL:
    """Load libzrc4.so and declare every prototype.  Raises if absent."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = Path(path) if path else LIB_PATH
    # One HIP runtime per process: torch ships its own libamdhip64 (same SONAME
    # libamdhip64.so.7 as /opt/rocm's).  If libzrc4 were loaded first, a later
    # `import torch` would map a SECOND runtime and torch.cuda would see no
    # device.  Importing torch first makes libzrc4 bind to the runtime torch
    # already mapped.  Plain C/C++ users (no torch) get /opt/rocm's via RUNPATH.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not p.exists():
        raise FileNotFoundError(
            f"{p} not built: run `python -m zsummerx_amd.build` (hipcc --offload-arch=gfx950); "
            "there is no CPU fallback for the RC4 path")
    lib = C.CDLL(str(p))
    for name, res, args in SIGNATURES:
        # an explicitly named A/B library from an older revision may predate
        # an entry point; the product library must export every one
        if path is not None and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


def _strerror(code: int) -> str:
    try:
        return load().zrc4_strerror(code).decode()
    except Exception:  # library itself missing
        return "unknown"


def check(code: int, what: str = "") -> None:
    if code != ZRC4_OK:
        raise ZRC4Error(code, what)
