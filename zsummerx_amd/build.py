"""In-tree build of the native pieces (no JIT cache, so the .so files travel to
the GPU box with the repo snapshot).

  libzrc4.so        C-ABI product library: HIP kernels for gfx950 + host side
  libzrc4_synth.so  synthetic workload generator (bench/tests input data)
  libzsx_frame.so   batched session engine (include/zsummerx_amd/frame.h) with
                    the gfx950 RC4 hooks over libzrc4.so
  bin/frame_stress  BASELINE config-1 driver (example/frameStressTest analogue)
  oracle/           CPU restatement (+ oracle/_ref when /root/reference exists)
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
BUILD = ROOT / "build"
ARCH = "gfx950"

LIB = PKG / "libzrc4.so"
SYNTH = PKG / "libzrc4_synth.so"

FRAME = PKG / "libzsx_frame.so"
STRESS = PKG / "bin" / "frame_stress"
ENGINE = PKG / "engine"
FRAME_SOURCES = [ENGINE / "frame.cpp", ENGINE / "rc4_hooks_device.cpp"]
FRAME_DEPS = FRAME_SOURCES + [ROOT / "include" / "zsummerx_amd" / "frame.h",
                              ROOT / "include" / "zsummerx_amd" / "rc4_hooks.h", ROOT / "include" / "zrc4.h"]
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))

HIP_SOURCES = [CSRC / "zrc4.hip"]
HIP_DEPS = HIP_SOURCES + [CSRC / "zrc4_kernels.hpp", CSRC / "zrc4_win.hpp", CSRC / "zrc4_line_loop.inc", CSRC / "zrc4_ks.inc",
                         ROOT / "include" / "zrc4.h"]


def _hipcc() -> str:
    for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the zrc4 HIP library cannot be built")


def _stale(out: Path, deps) -> bool:
    if not out.exists():
        return True
    t = out.stat().st_mtime
    return any(Path(d).stat().st_mtime > t for d in deps)


def build_lib(force: bool = False, extra_flags=()) -> Path:
    if force or _stale(LIB, HIP_DEPS):
        BUILD.mkdir(exist_ok=True)
        cmd = [_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
               "-Wall", f"-I{ROOT / 'include'}", f"-save-temps={BUILD}/", *extra_flags,
               "-o", str(LIB), *map(str, HIP_SOURCES)]
        subprocess.run(cmd, check=True, cwd=BUILD)
    return LIB


def build_variant(name: str, defines: dict, rev: str | None = None) -> Path:
    """A/B builds: the same library under another name with -D switches, or
    the sources of git revision `rev` (tools/ab_bench.py loads several side by
    side in one process)."""
    out = PKG / f"libzrc4_{name}.so"
    srcs, inc, deps = HIP_SOURCES, ROOT / "include", HIP_DEPS
    ab_inc = PKG / "csrc" / "ab" / "zrc4_line_loop_ab.inc"
    if defines.get("ZRC4_LL_AB") and not rev and not ab_inc.exists():
        # timing-only variants, generated on demand (tools/gen_line_loop.py --ab)
        subprocess.run([sys.executable, str(ROOT / "tools" / "gen_line_loop.py"), "--ab"], check=True)
    if rev and not (ROOT / ".git").exists():      # the GPU box: no history, use the prebuilt library
        if not out.exists():
            raise FileNotFoundError(f"{out} (revision {rev}) must be built before the GPU run")
        return out
    if rev:
        tree = BUILD / f"rev_{name}"
        (tree / "csrc").mkdir(parents=True, exist_ok=True)
        (tree / "include").mkdir(parents=True, exist_ok=True)
        for rel, dst in (("zsummerx_amd/csrc/zrc4.hip", tree / "csrc" / "zrc4.hip"),
                         ("zsummerx_amd/csrc/zrc4_kernels.hpp", tree / "csrc" / "zrc4_kernels.hpp"),
                         ("zsummerx_amd/csrc/zrc4_win.hpp", tree / "csrc" / "zrc4_win.hpp"),
                         ("zsummerx_amd/csrc/zrc4_line_loop.inc", tree / "csrc" / "zrc4_line_loop.inc"),
                         ("zsummerx_amd/csrc/zrc4_ks.inc", tree / "csrc" / "zrc4_ks.inc"),
                         ("include/zrc4.h", tree / "include" / "zrc4.h")):
            got = subprocess.run(["git", "show", f"{rev}:{rel}"], cwd=ROOT, capture_output=True)
            if got.returncode != 0:
                if rel.endswith((".inc", "zrc4_win.hpp")):   # older revisions lack these
                    continue
                got.check_returncode()
            blob = got.stdout
            if not dst.exists() or dst.read_bytes() != blob:
                dst.write_bytes(blob)
        srcs, inc = [tree / "csrc" / "zrc4.hip"], tree / "include"
        deps = [tree / "csrc" / "zrc4.hip", tree / "csrc" / "zrc4_kernels.hpp", inc / "zrc4.h"]
    if _stale(out, deps):
        BUILD.mkdir(exist_ok=True)
        cmd = [_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
               f"-I{inc}", *[f"-D{k}={v}" for k, v in defines.items()],
               "-o", str(out), *map(str, srcs)]
        subprocess.run(cmd, check=True, cwd=BUILD)
    return out


def build_synth(force: bool = False) -> Path:
    src = CSRC / "synth.cpp"
    if force or _stale(SYNTH, [src]):
        cmd = ["g++", "-O3", "-std=c++17", "-fPIC", "-shared", "-pthread", "-o", str(SYNTH), str(src)]
        subprocess.run(cmd, check=True)
    return SYNTH


def build_frame(force: bool = False) -> Path:
    """The session engine: host C++ (g++) against the HIP runtime API and the
    C-ABI of libzrc4.so; the stress driver links it (rpath $ORIGIN)."""
    lib = build_lib(force)
    if force or _stale(FRAME, FRAME_DEPS + [lib]):
        cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-Wextra", "-Wno-unused-parameter",
               "-D__HIP_PLATFORM_AMD__", f"-I{ROOT / 'include'}", f"-I{ROCM / 'include'}",
               "-o", str(FRAME), *map(str, FRAME_SOURCES),
               f"-L{PKG}", "-lzrc4", f"-L{ROCM / 'lib'}", "-lamdhip64",
               "-Wl,-rpath,$ORIGIN", f"-Wl,-rpath,{ROCM / 'lib'}"]
        subprocess.run(cmd, check=True)
    src = ROOT / "tools" / "frame_stress.cpp"
    if force or _stale(STRESS, [src, FRAME] + FRAME_DEPS):
        STRESS.parent.mkdir(exist_ok=True)
        cmd = ["g++", "-O2", "-std=c++17", "-Wall", "-Wextra", "-Wno-unused-parameter",
               f"-I{ROOT / 'include'}", "-o", str(STRESS), str(src),
               f"-L{PKG}", "-lzsx_frame", "-lzrc4", "-ldl",
               "-Wl,-rpath,$ORIGIN/..", f"-Wl,-rpath,{ROCM / 'lib'}"]
        subprocess.run(cmd, check=True)
    return FRAME


SANITIZE = ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=undefined", "-g"]
TSAN = ["-fsanitize=thread", "-g"]


def build_test_tools(force: bool = False, sanitize: bool | str = False) -> Path:
    """Test infrastructure (links the oracle; never part of the product):
      tools/bin/hooks_check      the device Rc4Hooks driven like the engine,
                                 every byte checked against the oracle (GPU)
      tools/bin/hooks_check_emu  the same host logic over a CPU emulation of
                                 the zrc4 C-ABI (tests/cpp/emu_zrc4_hip.cpp)
      tools/bin/frame_stress_emu the engine + device hooks over that emulation
      tools/bin/emu_declared_check  the emulation's declared-group refusals
                                 against the GPU's rules
    sanitize=True builds only the two emulated binaries, with ASan + UBSan,
    into tools/bin/san/ (scripts/sanitize.sh runs the CPU suites on them);
    sanitize="thread" the same with ThreadSanitizer into tools/bin/tsan/ (the
    reservoir's XOR worker threads)."""
    frame = build_frame(force)
    sub = {False: "", True: "san", "thread": "tsan"}[sanitize]
    out = ROOT / "tools" / "bin" / sub
    out.mkdir(parents=True, exist_ok=True)
    orc = ROOT / "oracle" / "liboracle.so"
    chk = ROOT / "tests" / "cpp" / "hooks_check.cpp"
    emu = ROOT / "tests" / "cpp" / "emu_zrc4_hip.cpp"
    dev = ENGINE / "rc4_hooks_device.cpp"
    common = ["-std=c++17", f"-I{ROOT / 'include'}", f"-I{ROOT / 'oracle'}"]
    emu_flags = ["-D__HIP_PLATFORM_AMD__", f"-I{ROCM / 'include'}"]
    oracle_link = [f"-L{ROOT / 'oracle'}", "-loracle", "-Wl,-rpath,$ORIGIN/../../oracle"]
    jobs = [
        (out / "hooks_check", [chk, orc, frame] + FRAME_DEPS,
         ["g++", "-O2", *common, "-o", str(out / "hooks_check"), str(chk), *oracle_link,
          f"-L{PKG}", "-lzsx_frame", "-lzrc4", "-lpthread", "-Wl,-rpath,$ORIGIN/../../zsummerx_amd",
          f"-Wl,-rpath,{ROCM / 'lib'}"]),
        (out / "hooks_check_emu", [chk, orc, emu] + FRAME_DEPS,
         ["g++", "-O2", *common, *emu_flags, "-o", str(out / "hooks_check_emu"), str(chk), str(dev), str(emu),
          *oracle_link, "-lpthread"]),
        (out / "emu_declared_check", [orc, emu, ROOT / "tests" / "cpp" / "emu_declared_check.cpp", ROOT / "include" / "zrc4.h"],
         ["g++", "-O2", *common, *emu_flags, "-o", str(out / "emu_declared_check"),
          str(ROOT / "tests" / "cpp" / "emu_declared_check.cpp"), str(emu), *oracle_link, "-lpthread"]),
        (out / "frame_stress_emu", [orc, emu, ROOT / "tools" / "frame_stress.cpp"] + FRAME_DEPS,
         ["g++", "-O2", *common, *emu_flags, "-o", str(out / "frame_stress_emu"), str(ROOT / "tools" / "frame_stress.cpp"),
          *map(str, FRAME_SOURCES), str(emu), *oracle_link, "-ldl", "-lpthread"]),
    ]
    if sanitize:
        flags = TSAN if sanitize == "thread" else SANITIZE
        jobs = [(t, d, [c[0], *flags, *c[1:], "-Wl,-rpath,$ORIGIN/../../../oracle"])
                for t, d, c in jobs if t.name.endswith("_emu")]
    for target, deps, cmd in jobs:
        if force or _stale(target, deps):
            subprocess.run(cmd, check=True)
    return out


def build_mirror_bench(force: bool = False) -> Path:
    """tools/bin/mirror_bench: per-call cost of the drop-in RC4Encryption mirror
    (tools/mirror_bench.cpp)."""
    src = ROOT / "tools" / "mirror_bench.cpp"
    out = ROOT / "tools" / "bin" / "mirror_bench"
    out.parent.mkdir(parents=True, exist_ok=True)
    deps = [src, LIB, ROOT / "include" / "zsummerx_amd" / "rc4_encryption.h", ROOT / "include" / "zrc4.h"]
    if force or _stale(out, deps):
        subprocess.run(["g++", "-O2", "-std=c++17", f"-I{ROOT / 'include'}", str(src), f"-L{PKG}", "-lzrc4",
                        "-Wl,-rpath,$ORIGIN/../../zsummerx_amd", "-o", str(out)], check=True)
    return out


def build_ubench(force: bool = False) -> None:
    """tools/ubench/traffic_calib: the known-byte-count kernels the PMC
    traffic passes calibrate FETCH_SIZE against (scripts/pmc_traffic.sh)."""
    src = ROOT / "tools" / "ubench" / "traffic_calib.hip"
    out = src.with_suffix("")
    if force or _stale(out, [src]):
        subprocess.run([_hipcc(), f"--offload-arch={ARCH}", "-O2", "-o", str(out), str(src)], check=True)


def build_oracle() -> None:
    subprocess.run(["make", "-s", "-C", str(ROOT / "oracle")], check=True)


# A/B builds the GPU tests load (tests/test_gpu_parity.py): built with the
# product so that no test compiles on the GPU box.
TEST_VARIANTS = {"wintag4": {"ZRC4_WIN_TAG_LIMIT": 4},
                 "testhooks": {"ZRC4_TEST_HOOKS": 1},      # fault injection (zrc4_ks.inc), never the product
                 "preclaim1": {"ZRC4_GR_PRECLAIM_MAX": 1}}  # grouped claims in the loop from the 2nd bucket on


def build_all(force: bool = False) -> None:
    build_lib(force)
    for name, defs in TEST_VARIANTS.items():
        build_variant(name, defs)
    build_synth(force)
    build_frame(force)
    build_oracle()
    build_test_tools(force)
    build_ubench(force)
    build_mirror_bench(force)


if __name__ == "__main__":
    import sys
    build_all(force="--force" in sys.argv)
    print("built", LIB, SYNTH)
