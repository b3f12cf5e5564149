"""The reference's OWN frame code, run end to end over the mirror.

oracle/_ref/ref_frame_client is /root/reference/src/frame (session.cpp,
manager.cpp), src/epoll, src/timer and src/common compiled unchanged with
include/compat first (oracle/Makefile, target ref-frame), plus a small client
main (tools/ref_frame_client.cpp): N connecters with _rc4TcpEncryption set
(include/zsummerX/frame/config.h:196), each echoing proto4z packets.  Every
RC4 hook of the reference's TcpSession -- seeding on connect
(src/frame/session.cpp:110-111), the recv decrypt (:313-323), the send
encrypts (:496-499, :535-538, :603-606) -- runs zsummerx_amd::RC4Encryption.

Peers:
  * an independent Python server speaking the reference protocol with the
    ORACLE RC4 (one stream per direction, seeded from the key): it decrypts
    what the client put on the wire, checks the framing, and echoes; the
    client checks every echoed byte.  So the wire bytes the reference's
    session produced through the mirror are the reference RC4's;
  * the batched session engine as the server (frame_stress --mode server),
    with the device hooks on the GPU.
CPU tests use ref_frame_client_emu: the same objects over the CPU emulation
of the C-ABI (tests/cpp/emu_zrc4_hip.cpp).  The binaries are built where
/root/reference exists and travel prebuilt to the GPU box."""
import json
import socket
import struct
import subprocess
import threading

import pytest

from conftest import ROOT

REF = ROOT / "oracle" / "_ref"
CLIENT = REF / "ref_frame_client"
CLIENT_EMU = REF / "ref_frame_client_emu"
KEY = b"ref-frame-key\x00\x01\xfe"          # NUL and high bytes count (makeSBox takes std::string)


def rc4(key=KEY):
    import pyoracle
    return pyoracle.Rc4(key)


def oracle_server(nsess, errors):
    """A listening socket whose accepted connections run the reference
    protocol with the oracle RC4 and echo every complete proto4z packet."""
    lst = socket.socket()
    lst.bind(("127.0.0.1", 0))
    lst.listen(128)
    stats = {"packets": 0, "bytes": 0}
    lock = threading.Lock()

    def serve_one(conn):
        rd, wr = rc4(), rc4()          # session.cpp:110-111: both directions from the same key
        buf = b""
        try:
            with conn:
                while True:
                    b = conn.recv(1 << 16)
                    if not b:
                        return
                    buf += rd.encryption(b)
                    out = b""
                    while len(buf) >= 6:                          # HasRawPacket, proto4z.h:704-748
                        ln = struct.unpack_from("<I", buf)[0]
                        if ln < 6 or ln > 20480:
                            errors.append(f"bad length {ln}")
                            return
                        if len(buf) < ln:
                            break
                        out += buf[:ln]
                        buf = buf[ln:]
                        with lock:
                            stats["packets"] += 1
                            stats["bytes"] += ln
                    if out:
                        conn.sendall(wr.encryption(out))
        except (ConnectionResetError, BrokenPipeError):
            return
        except Exception as e:                                    # noqa: BLE001
            errors.append(repr(e))

    def acceptor():
        for _ in range(nsess):
            try:
                c, _ = lst.accept()
            except OSError:
                return
            threading.Thread(target=serve_one, args=(c,), daemon=True).start()

    threading.Thread(target=acceptor, daemon=True).start()
    return lst, stats


def run_client(binary, port, nsess, echoes, block, depth, seed=1):
    p = subprocess.run([str(binary), "--port", str(port), "--key-hex", KEY.hex(), "--sessions", str(nsess),
                        "--echoes", str(echoes), "--block", str(block), "--depth", str(depth), "--seed", str(seed),
                        "--seconds", "90"], capture_output=True, text=True, timeout=150)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert lines, (p.returncode, p.stdout[-2000:], p.stderr[-2000:])
    st = json.loads(lines[-1])
    assert p.returncode == 0, (st, p.stderr[-2000:])
    assert st["mismatches"] == 0 and st["closed_early"] == 0
    assert st["echoes"] == nsess * echoes and st["linked"] == nsess
    return st


def against_oracle(binary, nsess, echoes, block, depth):
    errors = []
    lst, stats = oracle_server(nsess, errors)
    try:
        st = run_client(binary, lst.getsockname()[1], nsess, echoes, block, depth)
    finally:
        lst.close()
    assert not errors, errors
    # every packet the reference session put on the wire decrypted, with the
    # oracle, to a well-formed packet the client then got back unchanged
    assert stats["packets"] == nsess * echoes
    return st


def against_engine(binary, stress, hooks, nsess, echoes, block, depth, extra=()):
    srv = subprocess.Popen([str(stress), "--mode", "server", "--rc4", hooks, "--key-hex", KEY.hex(),
                            "--seconds", "90", "--warmup", "0", "--exit-after", str(nsess), *extra],
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        line = srv.stdout.readline()
        assert line.startswith("PORT "), (line, srv.stderr.read() if srv.poll() is not None else "")
        st = run_client(binary, int(line.split()[1]), nsess, echoes, block, depth)
        out, err = srv.communicate(timeout=90)
        assert srv.returncode == 0, err[-2000:]
        sst = json.loads(out.strip().splitlines()[-1])
        assert sst["recv_packs"] == nsess * echoes, sst
    finally:
        if srv.poll() is None:
            srv.kill()
            srv.wait()
    return st, sst


def _need(path):
    if not path.exists():
        pytest.skip(f"{path.name} not built (oracle/Makefile ref-frame needs /root/reference)")


# ------------------------------------------------------------------ CPU
def test_reference_client_emulated_vs_oracle_server(built):
    _need(CLIENT_EMU)
    against_oracle(CLIENT_EMU, nsess=6, echoes=30, block=1024, depth=2)
    against_oracle(CLIENT_EMU, nsess=3, echoes=10, block=20480, depth=1)    # SESSION_BLOCK_SIZE packets


def test_reference_client_emulated_vs_engine_cpu_hooks(built):
    _need(CLIENT_EMU)
    from zsummerx_amd import build
    build.build_frame()
    stress = ROOT / "zsummerx_amd" / "bin" / "frame_stress"
    against_engine(CLIENT_EMU, stress, "host:" + str(ROOT / "oracle" / "liboracle.so"), nsess=4, echoes=25,
                   block=1024, depth=2)


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
def test_reference_client_on_gpu_mirror_vs_oracle_server(built):
    """The reference's TcpSession with the gfx950 mirror as its RC4: its wire
    bytes decrypt with the oracle, and the oracle's replies decrypt back."""
    _need(CLIENT)
    against_oracle(CLIENT, nsess=8, echoes=40, block=1024, depth=2)
    against_oracle(CLIENT, nsess=4, echoes=8, block=20480, depth=2)


@pytest.mark.gpu
def test_reference_client_on_gpu_mirror_vs_engine_device_hooks(built):
    """Both ends on the GPU path: the reference's session code (mirror) as
    the client, the batched engine with device hooks as the server."""
    _need(CLIENT)
    from zsummerx_amd import build
    build.build_frame()
    stress = ROOT / "zsummerx_amd" / "bin" / "frame_stress"
    st, sst = against_engine(CLIENT, stress, "device", nsess=8, echoes=40, block=1024, depth=2)
    assert "gfx950" in sst["rc4"], sst                # the engine ran the device hooks
