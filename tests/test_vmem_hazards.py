"""Static guards on the shipped gfx950 machine code (CPU only).

1. The asm-issued-load discipline: no instruction may read
   or write a VGPR while a full-EXEC VMEM load into it can still be in
   flight (on the prefetching persistent kernels and the grouped window
   kernels: any VMEM load, whatever the EXEC mask -- the grouped claim is
   issued by lane 0 alone).  tools/vmem_hazard_check.py proves it on the product library's
   code object, and must flag the removed round-2 "sink load in place of each
   store" line loop (the variant that faulted the GPU in round 3), which
   tools/gen_line_loop.py --hazard-demo regenerates into a scratch directory.
   That variant is only compiled here, never run.  The analysis is
   path-sensitive on the kernels' uniform control flow (difference
   constraints between SGPRs, the compiler's uniform booleans), so the
   counted waits of the line loop are proved, not assumed.
2. No product kernel spills: the persistent kernel's grouped form sits at
   exactly 256 VGPRs, and a spill there would put a scratch load plus a
   vmcnt(0) drain into every group boundary.
"""
import os
import shutil
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tools"))

import vmem_hazard_check as vh  # noqa: E402

LLVM_OK = all((vh.LLVM / t).exists() for t in ("llvm-objdump", "llvm-objcopy", "clang-offload-bundler"))
pytestmark = pytest.mark.skipif(not LLVM_OK, reason="ROCm LLVM tools not found")


PINNED = set(range(40, 104)) | set(range(148, 152)) | set(range(160, 224))
PREFETCHING = ("crypt_stream_kernelILb1ELb0ELb0E", "crypt_stream_kernelILb1ELb1ELb0E",   # range / grouped
               "crypt_stream_kernelILb1ELb0ELb1E", "crypt_stream_kernelILb1ELb1ELb1E")   # framed
WIN_GROUPED = ("crypt_win_kernelILi2E",)      # the window kernel's claim, issued from asm by lane 0 (r05)
DECL = ("crypt_decl_kernel",)                 # the declared kernels' claim, lane 0 under an in-asm predicate (r06)


def _check_one(item):
    name, insns = item
    dbg = {}
    # the prefetching persistent kernels, the grouped window kernels and the
    # declared kernels issue the grouped claim from asm with lane 0 alone:
    # there every load is tracked, whatever the EXEC mask,
    # so a compiler copy of the claim's register before its wait would be
    # flagged too
    partial = any(k in name for k in PREFETCHING + WIN_GROUPED + DECL)
    hz, _ = vh.check_function(name, insns, debug=dbg, track_partial=partial, max_states=1500000)
    idx = {i.addr: i for i in insns}
    pinned = [a for a in dbg.get("loads", {}) if vh.vmem_dest(idx[a]) & PINNED]
    tracked = [a for a in pinned if True in dbg["loads"][a]]
    return name, (hz, pinned, tracked)


def _check(lib: Path, only=None):
    """Every (selected) kernel analysed in its own process: the persistent
    kernels take minutes each, the rest seconds."""
    from concurrent.futures import ProcessPoolExecutor
    funcs = vh.parse(vh.disassemble(lib))
    items = [(n, i) for n, i in funcs.items() if not only or any(o in n for o in only)]
    items.sort(key=lambda it: -len(it[1]))              # longest first
    workers = max(1, min(len(items), len(os.sched_getaffinity(0)), 8))
    with ProcessPoolExecutor(max_workers=workers) as ex:
        return dict(ex.map(_check_one, items))


def test_product_library_has_no_vmem_hazards(built):
    res = _check(ROOT / "zsummerx_amd" / "libzrc4.so")
    crypt = [n for n in res if "crypt" in n]
    assert len(crypt) >= 15, sorted(res)                # every product crypt kernel was analysed
    bad = {n: [(hex(i.addr), i.text) for i, _, _ in hz[:3]] for n, (hz, _, _) in res.items() if hz}
    assert not bad, bad
    # Not vacuous for the prefetching throughput kernels: every load into a
    # pinned range is issued with the whole wave in EXEC on some path, so the
    # analysis tracks it.  (The scattered-ids form keeps per-lane EXEC state
    # the analysis does not resolve; it is checked where EXEC is known.  The
    # framed forms add the tail's framing walk: compiler byte loads under
    # per-lane EXEC, some of them allocated into those register numbers.)
    for key in PREFETCHING[:2]:
        (name,) = [n for n in res if key in n]
        _, pinned, tracked = res[name]
        assert len(pinned) >= 40 and set(pinned) == set(tracked), (name, len(pinned), len(tracked))


def test_product_kernels_do_not_spill(built):
    """No VGPR spills and no scratch memory in any product kernel.  An SGPR
    spill into a VGPR lane (v_writelane / v_readlane, no memory) is allowed:
    the framed non-prefetching persistent kernel keeps one of its kernel
    arguments there."""
    res = vh.kernel_resources(ROOT / "zsummerx_amd" / "libzrc4.so")
    assert any("crypt_stream_kernelILb1ELb1E" in n for n in res)
    assert all("private_segment_fixed_size" in r for r in res.values())
    spills = {n: (r.get("vgpr_spill_count"), r.get("private_segment_fixed_size")) for n, r in res.items()
              if r.get("vgpr_spill_count") or r.get("private_segment_fixed_size")}
    assert not spills, spills


def test_removed_sink_load_variant_is_flagged(tmp_path):
    """The round-3 fault, reproduced as code only: loads into the line loop's
    store-address temporaries v[148:151] left in flight across the next
    statement's address writes.  The checker must report it (checked on the
    range persistent kernel; the grouped one runs the same generated loop)."""
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not Path(hipcc).exists():
        pytest.skip("hipcc not found")
    src = ROOT / "zsummerx_amd" / "csrc"
    for f in ("zrc4.hip", "zrc4_kernels.hpp", "zrc4_win.hpp", "zrc4_ks.inc"):
        shutil.copy(src / f, tmp_path / f)
    subprocess.run([sys.executable, str(ROOT / "tools" / "gen_line_loop.py"), "--hazard-demo", str(tmp_path)],
                   check=True, capture_output=True)
    lib = tmp_path / "libzrc4_hazard_demo.so"
    subprocess.run([hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                    f"-I{ROOT / 'include'}", "-o", str(lib), str(tmp_path / "zrc4.hip")],
                   check=True, capture_output=True, cwd=tmp_path)
    res = _check(lib, only=PREFETCHING[:1])             # the range form (the grouped one shares the loop)
    assert len(res) == 1 and all(hz for hz, _, _ in res.values()), {n: len(r[0]) for n, r in res.items()}
    for hz, _, _ in res.values():
        regs = {r for _, rr, _ in hz for r in rr}
        assert regs & set(range(148, 152)), sorted(regs)
