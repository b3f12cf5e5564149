"""Batched session engine (include/zsummerx_amd/frame.h): the RC4 hook sites
of TcpSession (src/frame/session.cpp:110-111 seeding, :313-323 recv decrypt,
:496-499 / :535-538 / :603-606 send encrypt) driven over real TCP sockets.

Wire parity: an independent Python peer speaks the reference protocol with
the oracle RC4 (one RC4Encryption per direction, both seeded from the same
key, rc4_encryption.h:46-93) and proto4z framing (proto4z.h:704-748); the
engine, running the hooks batched per event-loop iteration, must produce and
accept exactly the reference's bytes.

CPU tests run the engine with the oracle loaded as its hooks (host logic:
batching, keystream order, framing, send-queue merging).  GPU tests run the
product hooks (--rc4 device: one gfx950 launch per iteration over pinned
SessionBlocks) against the same oracle peer."""
import json
import random
import socket
import struct
import subprocess
import threading

import pytest

from conftest import ROOT, soak_seeds

STRESS = __import__('pathlib').Path(__import__('os').environ.get('ZSX_STRESS', str(ROOT / 'zsummerx_amd' / 'bin' / 'frame_stress')))
ORACLE_HOOKS = "host:" + str(ROOT / "oracle" / "liboracle.so")
KEY = b"frame-parity-key\x00with-nul"   # NUL bytes count (makeSBox takes std::string)
POLICY_REQ = b"<policy-file-request/>\x00"
POLICY_RESP = (b'<cross-domain-policy><allow-access-from domain="*" to-ports="*"/>'
               b"</cross-domain-policy>\x00")


@pytest.fixture(scope="module")
def stress(built):
    from zsummerx_amd import build
    build.build_frame()
    assert STRESS.exists()
    return STRESS


def rc4(key=KEY):
    import pyoracle
    return pyoracle.Rc4(key)


def packet(rng, size, tag):
    body = bytes(rng.getrandbits(8) for _ in range(size - 8))
    return struct.pack("<IHH", size, 0, tag & 0xFFFF) + body


def recv_exact(s, n):
    out = bytearray()
    while len(out) < n:
        b = s.recv(n - len(out))
        if not b:
            raise EOFError(f"peer closed after {len(out)} of {n} bytes")
        out += b
    return bytes(out)


class Server:
    """frame_stress --mode server; yields its port, returns its JSON stats."""

    def __init__(self, stress, hooks, exit_after, *extra):
        self.p = subprocess.Popen([str(stress), "--mode", "server", "--rc4", hooks, "--key-hex", KEY.hex(),
                                   "--seconds", "60", "--warmup", "0", "--exit-after", str(exit_after), *extra],
                                  stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
        line = self.p.stdout.readline()
        if not line.startswith("PORT "):
            self.p.kill()
            raise RuntimeError(f"server did not start: {line!r} {self.p.stderr.read()}")
        self.port = int(line.split()[1])
        self.port2 = None
        if "--plain-accepter" in extra:
            line = self.p.stdout.readline()
            if not line.startswith("PORT2 "):
                self.p.kill()
                raise RuntimeError(f"server did not open the plain accepter: {line!r}")
            self.port2 = int(line.split()[1])

    def finish(self, timeout=60):
        out, err = self.p.communicate(timeout=timeout)
        assert self.p.returncode == 0, err
        return json.loads(out.strip().splitlines()[-1])


class _Plain:
    """RC4 off (_rc4TcpEncryption empty): the wire carries the plaintext."""

    def encryption(self, b):
        return bytes(b)


def echo_client(port, seed, npk, results, idx, keyed=True):
    """Send npk proto4z packets, RC4-encrypted with the oracle (or in clear
    when keyed is False), in random chunkings (splits inside headers and
    bodies, several packets per write); read the echoes back and decrypt them
    with the oracle."""
    rng = random.Random(seed)
    wr, rd = (rc4(), rc4()) if keyed else (_Plain(), _Plain())   # session.cpp:110-111: same key both ways
    plain = b"".join(packet(rng, rng.choice([8, 9, 64, 1000, 1024, 4096, 20000, rng.randint(8, 3000)]), i)
                     for i in range(npk))
    wire = wr.encryption(plain)
    with socket.create_connection(("127.0.0.1", port), timeout=30) as s:
        s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        got = bytearray()
        pos = 0
        while pos < len(wire):
            n = rng.choice([1, 3, 7, 100, 1500, 9000, 40000])
            s.sendall(wire[pos:pos + n])
            pos += n
            s.setblocking(False)
            try:
                while True:
                    b = s.recv(1 << 16)
                    if not b:
                        break
                    got += b
            except BlockingIOError:
                pass
            s.setblocking(True)
        s.settimeout(30)
        got += recv_exact(s, len(wire) - len(got))
    results[idx] = (plain, bytes(got), rd.encryption(bytes(got)))


def run_echo_parity(stress, hooks, nclients=6, npk=40, extra=(), seed0=1000):
    srv = Server(stress, hooks, nclients, *extra)
    results = [None] * nclients
    th = [threading.Thread(target=echo_client, args=(srv.port, seed0 + i, npk, results, i)) for i in range(nclients)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    if any(r is None for r in results):
        srv.p.kill()
        _, err = srv.p.communicate(timeout=30)
        raise AssertionError(f"clients {[i for i, r in enumerate(results) if r is None]} did not finish; "
                             f"server stderr: {err[-3000:]}")
    stats = srv.finish()
    for i, r in enumerate(results):
        plain, cipher, decrypted = r
        assert len(cipher) == len(plain)
        # the server's ciphertext is exactly RC4Encryption(key) over the echoed bytes
        assert cipher == rc4().encryption(plain), f"client {i}: server wire bytes differ from the reference RC4"
        assert decrypted == plain
    assert stats["recv_packs"] == nclients * npk
    assert stats["linked"] == nclients
    return stats


def run_mixed_keyed_plain(stress, hooks, nclients=4, npk=30):
    """Row a6 (config.h:196, session.cpp:313-316): ONE engine, ONE hooks
    object, keyed and keyless sessions in the same event-loop iterations.
    Keyed sessions must echo reference RC4 on the wire, keyless ones the
    plaintext itself, and neither may disturb the other's keystream."""
    srv = Server(stress, hooks, 2 * nclients, "--plain-accepter")
    results = [None] * (2 * nclients)
    th = [threading.Thread(target=echo_client, args=(srv.port if i % 2 == 0 else srv.port2, 2000 + i, npk,
                                                      results, i, i % 2 == 0))
          for i in range(2 * nclients)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    if any(r is None for r in results):
        srv.p.kill()
        _, err = srv.p.communicate(timeout=30)
        raise AssertionError(f"clients {[i for i, r in enumerate(results) if r is None]} did not finish; "
                             f"server stderr: {err[-3000:]}")
    stats = srv.finish()
    for i, (plain, wire, decrypted) in enumerate(results):
        if i % 2 == 0:
            assert wire == rc4().encryption(plain), f"keyed client {i}: wire is not the reference RC4"
            assert wire != plain
        else:
            assert wire == plain, f"keyless client {i}: wire must be the plaintext (RC4 off)"
        assert decrypted == plain
    assert stats["recv_packs"] == 2 * nclients * npk
    assert stats["linked"] == 2 * nclients
    return stats


def run_engine_client(stress, hooks, nsess=4, echoes=25, block=1024, depth=2):
    """The engine as the connecting side against a Python oracle server."""
    lst = socket.socket()
    lst.bind(("127.0.0.1", 0))
    lst.listen(64)
    port = lst.getsockname()[1]
    errors = []

    def serve_one(conn):
        rd, wr = rc4(), rc4()
        buf = b""
        try:
            with conn:
                while True:
                    b = conn.recv(1 << 16)
                    if not b:
                        return
                    buf += rd.encryption(b)
                    out = b""
                    while len(buf) >= 6:                     # proto4z.h:704-748
                        ln = struct.unpack_from("<I", buf)[0]
                        if ln < 6 or ln > 20480:
                            errors.append(f"bad length {ln}")
                            return
                        if len(buf) < ln:
                            break
                        out += buf[:ln]
                        buf = buf[ln:]
                    if out:
                        conn.sendall(wr.encryption(out))
        except (ConnectionResetError, BrokenPipeError):
            return      # the engine closes after its last echo with packets still in flight (depth > 1)
        except Exception as e:                                # noqa: BLE001
            errors.append(repr(e))

    def acceptor():
        for _ in range(nsess):
            c, _ = lst.accept()
            threading.Thread(target=serve_one, args=(c,), daemon=True).start()

    threading.Thread(target=acceptor, daemon=True).start()
    p = subprocess.run([str(stress), "--mode", "client", "--port", str(port), "--rc4", hooks,
                        "--key-hex", KEY.hex(), "--sessions", str(nsess), "--echoes", str(echoes),
                        "--block", str(block), "--depth", str(depth), "--seconds", "60", "--warmup", "0"],
                       capture_output=True, text=True, timeout=120)
    lst.close()
    assert p.returncode == 0, p.stderr
    st = json.loads(p.stdout.strip().splitlines()[-1])
    assert not errors, errors
    assert st["mismatches"] == 0
    assert st["echoes"] == nsess * echoes
    return st


def run_flash_policy(stress, hooks):
    """session.cpp:290-311: the probe is matched on the raw bytes (not
    decrypted), the answer goes out through send() -- i.e. encrypted -- and the
    read stream is untouched, so the next packet decrypts from offset 0."""
    srv = Server(stress, hooks, 1, "--flash-policy")
    wr, rd = rc4(), rc4()
    with socket.create_connection(("127.0.0.1", srv.port), timeout=30) as s:
        s.sendall(POLICY_REQ)
        resp = recv_exact(s, len(POLICY_RESP))
        assert rd.encryption(resp) == POLICY_RESP
        pk = packet(random.Random(5), 300, 1)
        s.sendall(wr.encryption(pk))
        assert rd.encryption(recv_exact(s, len(pk))) == pk
    srv.finish()


def run_corrupt_closes(stress, hooks, extra=()):
    """A length field below the 6-byte header is BCT_CORRUPTION: the session is
    closed (session.cpp:355-361), the peer sees EOF."""
    srv = Server(stress, hooks, 1, *extra)
    wr = rc4()
    with socket.create_connection(("127.0.0.1", srv.port), timeout=30) as s:
        s.sendall(wr.encryption(struct.pack("<IHH", 3, 0, 0)))
        assert s.recv(100) == b""
    st = srv.finish()
    assert st["closed"] == 1


# ------------------------------------------------------------------ CPU
@pytest.fixture(scope="module")
def stress_emu(built):
    """The engine with the DEVICE hooks' host logic (keystream reservoirs) over a
    CPU emulation of the zrc4 C-ABI (tests/cpp/emu_zrc4_hip.cpp)."""
    import os
    from zsummerx_amd import build
    if os.environ.get("ZSX_TOOLS_BIN"):            # scripts/sanitize.sh: ASan/UBSan builds
        return __import__('pathlib').Path(os.environ["ZSX_TOOLS_BIN"]) / "frame_stress_emu"
    build.build_test_tools()
    return ROOT / "tools" / "bin" / "frame_stress_emu"


def test_engine_echo_parity_emulated_device_hooks(stress_emu):
    st = run_echo_parity(stress_emu, "device")
    assert st["rc4"] == "zrc4-gfx950"


def test_engine_as_client_emulated_device_hooks(stress_emu):
    run_engine_client(stress_emu, "device", nsess=6, echoes=30, block=3000, depth=3)


def test_engine_echo_parity_cpu_hooks(stress):
    run_echo_parity(stress, ORACLE_HOOKS)


def test_mixed_keyed_and_keyless_emulated_device_hooks(stress_emu):
    st = run_mixed_keyed_plain(stress_emu, "device")
    assert st["rc4"] == "zrc4-gfx950"


def test_device_framing_emulated(stress_emu):
    """Receive blocks framed in the decrypt launch (setDeviceFraming, direct
    hooks): same wire bytes and packet stream as host framing."""
    st = run_echo_parity(stress_emu, "device-direct", extra=("--device-framing",))
    assert st["device_framed"] > 0


def test_device_framing_corrupt_closes_emulated(stress_emu):
    run_corrupt_closes(stress_emu, "device-direct", extra=("--device-framing",))


def test_mixed_keyed_and_keyless_cpu_hooks(stress):
    run_mixed_keyed_plain(stress, ORACLE_HOOKS)


def test_engine_as_client_cpu_hooks(stress):
    run_engine_client(stress, ORACLE_HOOKS)


def test_flash_policy_cpu_hooks(stress):
    run_flash_policy(stress, ORACLE_HOOKS)


def test_corrupt_packet_closes_cpu_hooks(stress):
    run_corrupt_closes(stress, ORACLE_HOOKS)


def test_loopback_cpu_hooks(stress):
    p = subprocess.run([str(stress), "--rc4", ORACLE_HOOKS, "--sessions", "16", "--depth", "3",
                        "--seconds", "0.5", "--warmup", "0.1"], capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, p.stderr
    st = json.loads(p.stdout)
    assert st["mismatches"] == 0 and st["echoes"] > 0 and st["linked"] == 32
    assert st["spans_per_call"] > 1.0          # hooks really are batched


def test_no_device_is_loud(stress):
    import torch  # noqa: F401  (only to know whether a GPU exists here)
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    if stress.name.endswith("_emu"):
        pytest.skip("ZSX_STRESS is the CPU emulation of the C-ABI (scripts/sanitize.sh)")
    p = subprocess.run([str(stress), "--rc4", "device", "--seconds", "0.1"], capture_output=True, text=True,
                       timeout=60)
    assert p.returncode == 1 and "gfx950" in p.stderr


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
def test_engine_echo_parity_device(stress):
    st = run_echo_parity(stress, "device")
    assert st["rc4"] == "zrc4-gfx950"


@pytest.mark.gpu
@pytest.mark.parametrize("seed", soak_seeds())
def test_engine_echo_parity_device_soak(stress, seed):
    """Echo parity from other seeds (one by default; scripts/r06_soak.sh runs
    many through $ZRC4_SOAK_SEEDS): reservoir, direct or direct with device
    framing, 2-16 clients, 10-60 packets each, random chunkings."""
    rng = random.Random(9000 + seed)
    hooks, extra = rng.choice([("device", ()), ("device-direct", ()), ("device-direct", ("--device-framing",))])
    st = run_echo_parity(stress, hooks, nclients=rng.randint(2, 16), npk=rng.randint(10, 60), extra=extra,
                         seed0=100_000 * seed)
    assert st["rc4"].startswith("zrc4-gfx950")


@pytest.mark.gpu
def test_mixed_keyed_and_keyless_device(stress):
    st = run_mixed_keyed_plain(stress, "device")
    assert st["rc4"] == "zrc4-gfx950"


@pytest.mark.gpu
def test_mixed_keyed_and_keyless_device_direct(stress):
    st = run_mixed_keyed_plain(stress, "device-direct")
    assert st["rc4"] == "zrc4-gfx950-direct"


@pytest.mark.gpu
def test_device_framing_echo_parity_device(stress):
    st = run_echo_parity(stress, "device-direct", extra=("--device-framing",))
    assert st["rc4"] == "zrc4-gfx950-direct" and st["device_framed"] > 0


@pytest.mark.gpu
def test_device_framing_corrupt_closes_device(stress):
    run_corrupt_closes(stress, "device-direct", extra=("--device-framing",))


@pytest.mark.gpu
def test_engine_as_client_device(stress):
    st = run_engine_client(stress, "device", nsess=8, echoes=40, block=2000, depth=3)
    assert st["rc4"] == "zrc4-gfx950"


@pytest.mark.gpu
def test_flash_policy_device(stress):
    run_flash_policy(stress, "device")


@pytest.mark.gpu
def test_corrupt_packet_closes_device(stress):
    run_corrupt_closes(stress, "device")


@pytest.mark.gpu
def test_loopback_device(stress):
    p = subprocess.run([str(stress), "--rc4", "device", "--sessions", "64", "--depth", "4",
                        "--seconds", "1", "--warmup", "0.2"], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    st = json.loads(p.stdout)
    assert st["rc4"] == "zrc4-gfx950"
    assert st["mismatches"] == 0 and st["echoes"] > 0 and st["linked"] == 128
