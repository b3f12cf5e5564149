"""The device Rc4Hooks (zsummerx_amd/engine/rc4_hooks_device.cpp) driven with
the session engine's call pattern -- seeding both streams per session, rounds
of crypt() over ragged spans inside pooled SessionBlocks, reconnect reseeds --
every byte checked against the oracle RC4 (rc4_encryption.h:46-93) by
tests/cpp/hooks_check.cpp.

CPU: the hooks' host logic (keystream-reservoir levels, ring wrap, two-piece
top-ups, refill commits, reseed drains) over a CPU emulation of the zrc4
C-ABI (tests/cpp/emu_zrc4_hip.cpp).  GPU: the real gfx950 path, reservoir and
direct modes."""
import json
import subprocess

import pytest

from conftest import ROOT

BIN = ROOT / "tools" / "bin"


@pytest.fixture(scope="module")
def tools(built):
    import os
    from pathlib import Path
    from zsummerx_amd import build
    if os.environ.get("ZSX_TOOLS_BIN"):            # scripts/sanitize.sh: ASan/UBSan builds
        return Path(os.environ["ZSX_TOOLS_BIN"])
    build.build_test_tools()
    return BIN


def run(exe, *args, env=None):
    p = subprocess.run([str(exe), *map(str, args)], capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0, (p.stdout, p.stderr)
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert out["ok"], out
    return out


def test_emulated_declared_refusals_match_the_gpu_rules(tools):
    """the CPU emulation the engine tests run on refuses declared
    buckets as the GPU does -- at most 256 buckets only the bucket whose ids
    leave its declared group; above 256 also the bucket that legitimately
    declares a group those ids name (the declared-check kernel's blocking,
    include/zrc4.h).  GPU side: test_gpu_declared.py."""
    exe = tools / "emu_declared_check"
    if not exe.exists():                               # sanitizer tool dirs build only the engine binaries
        pytest.skip("emu_declared_check not in this tools dir")
    p = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    assert p.stdout.count("-> ok") == 5, p.stdout


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_reservoir_host_logic_emulated(tools, seed):
    run(tools / "hooks_check_emu", "device", 48, 150, seed)


@pytest.mark.parametrize("ring", [256, 1000, 4096])
def test_reservoir_small_rings_emulated(tools, ring):
    # rings far below the span sizes: wrap-around, partial coverage + tail crypts
    out = run(tools / "hooks_check_emu", "device", 40, 120, 5, ring)
    assert out["hooks"]["tail_bytes"] > 0 and out["hooks"]["ring_bytes"] > 0


@pytest.mark.parametrize("threads", [2, 4])
def test_reservoir_parallel_xor_emulated(tools, threads):
    """The host XOR spread over worker threads (XorPool) for every batch
    (threshold 0): same bytes as the oracle, ring wrap included."""
    import os
    env = dict(os.environ, ZSX_XOR_THREADS=str(threads), ZSX_XOR_MIN_BYTES="0")
    out = run(tools / "hooks_check_emu", "device", 64, 120, 13, 4096, env=env)
    assert out["hooks"]["xor_threads"] == threads and out["hooks"]["ring_bytes"] > 0


@pytest.mark.parametrize("seed", [1, 3])
def test_adaptive_mode_switches_emulated(tools, seed):
    """Adaptive hooks (r03): with the switch point near this run's ~166 KB per
    call the moving average crosses it both ways -- refills stop (spans drain
    their rings, then go to the device as tails) and resume -- and every byte
    still matches the oracle."""
    import os
    env = dict(os.environ, ZSX_RC4_DIRECT_BYTES="170000")
    out = run(tools / "hooks_check_emu", "device", 48, 150, seed, env=env)
    h = out["hooks"]
    assert 0 < h["direct_calls"] < 150, h
    assert h["refill_launches"] > 0 and h["ring_bytes"] > 0 and h["tail_bytes"] > 0, h


def test_adaptive_mode_all_direct_emulated(tools):
    import os
    env = dict(os.environ, ZSX_RC4_DIRECT_BYTES="1")
    out = run(tools / "hooks_check_emu", "device", 48, 150, 2, env=env)
    assert out["hooks"]["direct_calls"] == 150 and out["hooks"]["ring_bytes"] == 0, out["hooks"]


def test_adaptive_mode_off_emulated(tools):
    import os
    env = dict(os.environ, ZSX_RC4_DIRECT_BYTES="0")
    out = run(tools / "hooks_check_emu", "device", 48, 150, 2, env=env)
    assert out["hooks"]["direct_calls"] == 0 and out["hooks"]["direct_bytes"] == 0, out["hooks"]


def test_direct_host_logic_emulated(tools):
    run(tools / "hooks_check_emu", "direct", 16, 40, 9)


@pytest.mark.gpu
@pytest.mark.parametrize("mode,sessions,rounds,seed", [("device", 64, 300, 1), ("device", 300, 100, 7),
                                                        ("device", 2048, 50, 3), ("direct", 64, 80, 2),
                                                        ("direct", 1024, 30, 4)])
def test_device_hooks_vs_oracle(tools, mode, sessions, rounds, seed):
    run(tools / "hooks_check", mode, sessions, rounds, seed)


@pytest.mark.gpu
def test_device_hooks_reservoir_at_scale(tools):
    """2 048 sessions with the adaptive switch off: the reservoir path itself
    at a size where the default hooks would run direct launches."""
    import os
    out = run(tools / "hooks_check", "device", 2048, 50, 3, env=dict(os.environ, ZSX_RC4_DIRECT_BYTES="0"))
    assert out["hooks"]["ring_bytes"] > 0 and out["hooks"]["direct_calls"] == 0, out["hooks"]


@pytest.mark.gpu
def test_device_hooks_parallel_xor(tools):
    import os
    # 512 sessions a call is past the adaptive switch point: the reservoir alone here
    env = dict(os.environ, ZSX_XOR_THREADS="4", ZSX_XOR_MIN_BYTES="0", ZSX_RC4_DIRECT_BYTES="0")
    out = run(tools / "hooks_check", "device", 512, 60, 17, env=env)
    assert out["hooks"]["xor_threads"] == 4 and out["hooks"]["ring_bytes"] > 0


@pytest.mark.gpu
def test_device_hooks_small_ring(tools):
    out = run(tools / "hooks_check", "device", 96, 150, 11, 1000)
    assert out["hooks"]["tail_bytes"] > 0 and out["hooks"]["ring_bytes"] > 0


@pytest.mark.gpu
def test_device_hooks_adaptive_mode_switches(tools):
    import os
    env = dict(os.environ, ZSX_RC4_DIRECT_BYTES="170000")
    out = run(tools / "hooks_check", "device", 48, 150, 3, env=env)
    h = out["hooks"]
    assert 0 < h["direct_calls"] < 150 and h["refill_launches"] > 0 and h["tail_bytes"] > 0, h


@pytest.mark.gpu
def test_device_hooks_synchronous_refill(tools):
    import os
    env = dict(os.environ, ZSX_RESERVOIR_SYNC_REFILL="1")
    run(tools / "hooks_check", "device", 64, 120, 4, env=env)
