"""CPU tests of the C-ABI boundary: the library builds for gfx950, loads, and
exports every symbol include/zrc4.h declares; the no-GPU behaviour is a loud
error, never a CPU fallback.  No compute calls here."""
import ctypes as C
import re
import subprocess

import pytest

from conftest import ROOT


def declared_symbols():
    text = (ROOT / "include" / "zrc4.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(zrc4_[a-z_]+)\s*\(", text)))


def test_header_declares_expected_api():
    syms = declared_symbols()
    for s in ["zrc4_create", "zrc4_destroy", "zrc4_ksa", "zrc4_crypt", "zrc4_crypt_host",
              "zrc4_make_sbox", "zrc4_encryption", "zrc4_sync", "zrc4_get_state",
              "zrc4_set_state", "zrc4_strerror"]:
        assert s in syms


def test_library_exports_every_declared_symbol(built):
    from zsummerx_amd import _capi
    lib = C.CDLL(str(_capi.LIB_PATH))
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    # the ctypes binding covers exactly the header
    assert sorted(n for n, _, _ in _capi.SIGNATURES) == declared_symbols()


def test_library_contains_gfx950_code_object(built):
    from zsummerx_amd import _capi
    out = subprocess.run(["/opt/rocm/bin/roc-obj-ls", str(_capi.LIB_PATH)], capture_output=True,
                         text=True)
    if out.returncode != 0:
        pytest.skip("roc-obj-ls unavailable")
    assert "gfx950" in out.stdout


def test_exported_symbols_are_c_abi(built):
    from zsummerx_amd import _capi
    nm = subprocess.run(["nm", "-D", "--defined-only", str(_capi.LIB_PATH)], capture_output=True,
                        text=True, check=True).stdout
    exported = set(re.findall(r"\bT (zrc4_\w+)", nm))
    assert set(declared_symbols()) <= exported  # unmangled names


def test_strerror_and_version(built):
    from zsummerx_amd import _capi
    lib = _capi.load()
    assert lib.zrc4_strerror(0) == b"ok"
    assert b"gfx950" in lib.zrc4_strerror(-2)
    assert b"gfx950" in lib.zrc4_version()


def test_no_device_is_a_loud_error(built):
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip("a GPU is visible")
    from zsummerx_amd import Context, ZRC4Error
    with pytest.raises(ZRC4Error) as ei:
        Context(0, 256)
    assert ei.value.code == -2


def _build_cpp_test(tmp_path):
    exe = tmp_path / "test_rc4_mirror"
    lib_dir = ROOT / "zsummerx_amd"
    orc = ROOT / "oracle"
    cmd = ["g++", "-O2", "-std=c++17", f"-I{ROOT / 'include'}", f"-I{orc}",
           str(ROOT / "tests" / "cpp" / "test_rc4_mirror.cpp"), f"-L{lib_dir}", "-lzrc4", f"-Wl,-rpath,{lib_dir}",
           f"-L{orc}", "-loracle", f"-Wl,-rpath,{orc}", "-o", str(exe)]
    subprocess.run(cmd, check=True)
    return exe


def test_cpp_mirror_header_compiles_and_links(built, tmp_path):
    """The reference-shaped C++ header compiles against the C-ABI and links."""
    assert _build_cpp_test(tmp_path).exists()


@pytest.mark.gpu
def test_cpp_mirror_runs_on_gpu(built, tmp_path):
    exe = _build_cpp_test(tmp_path)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "ok" in out.stdout
