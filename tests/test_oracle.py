"""CPU tests: the oracle (C restatement) pinned against the golden fixtures
produced by the real reference header, and against the reference itself when
oracle/_ref is present.  No GPU needed."""
import hashlib

import numpy as np
import pytest

import pyoracle
from zsummerx_amd import synth


def test_wikipedia_kats(kat):
    for v in kat["wikipedia"]:
        r = pyoracle.Rc4(bytes.fromhex(v["key"]))
        assert r.encryption(bytes.fromhex(v["plaintext"])).hex() == v["ciphertext"]


def test_rfc6229_offsets(kat):
    for v in kat["rfc6229"]:
        ks = pyoracle.Rc4(bytes.fromhex(v["key"])).encryption(bytes(4112))
        for o, want in v["offsets"].items():
            assert ks[int(o):int(o) + 16].hex() == want, (v["key"], o)
    for v in kat["rfc6229_published"]:
        ks = pyoracle.Rc4(bytes.fromhex(v["key"])).encryption(bytes(v["offset"] + 16))
        assert ks[v["offset"]:].hex() == v["keystream"]


def test_edge_cases(edge):
    for c in edge:
        r = pyoracle.Rc4(bytes.fromhex(c["key"]))
        data = bytearray.fromhex(c["data"])
        if "length" in c:
            r.encryption(data, c["length"])
            out = bytes(data)
        elif c["splits"]:
            out, pos = b"", 0
            for s in c["splits"]:
                out += r.encryption(bytes(data[pos:pos + s]))
                pos += s
        else:
            out = r.encryption(bytes(data))
        assert out.hex() == c["out"], c["name"]
        sb, x, y = r.state()
        assert (sb.hex(), x, y) == (c["state"]["sbox"], c["state"]["x"], c["state"]["y"]), c["name"]


def test_key_semantics(edge):
    by = {c["name"]: c for c in edge}
    assert by["key_300"]["out"] == by["key_300_prefix256"]["out"]
    assert by["nul_key"]["out"] != by["nul_key_truncation"]["out"]
    assert by["split_3_7"]["out"] == by["split_whole_10"]["out"]
    # empty key -> identity box (rc4_encryption.h:50-56)
    assert by["empty_key"]["state"]["sbox"][:8] != ""


def test_batch_small(batch_small):
    b = batch_small
    n = b["key_len"].size
    ob = pyoracle.Batch(n)
    ob.make_sbox(b["keys"], b["key_off"], b["key_len"])
    scratch = np.zeros(1000, dtype=np.uint8)
    ob.crypt(scratch, np.zeros(n, dtype=np.uint64), b["adv"])
    pay = b["payload_in"].copy()
    ob.crypt(pay, b["off"], b["length"], threads=3)
    assert np.array_equal(pay, b["payload_out"])
    for i in range(n):
        sb, x, y = ob.state(i)
        assert sb == b["states"][i, :256].tobytes() and (x, y) == tuple(b["states"][i, 256:])


def test_pure_python_matches_oracle():
    rng = np.random.default_rng(5)
    for _ in range(20):
        key = rng.integers(0, 256, size=int(rng.integers(0, 40)), dtype=np.uint8).tobytes()
        data = rng.integers(0, 256, size=int(rng.integers(0, 300)), dtype=np.uint8).tobytes()
        assert pyoracle.py_rc4(key, data) == pyoracle.Rc4(key).encryption(data)


@pytest.mark.skipif(pyoracle.ref_lib() is None, reason="oracle/_ref not built (no /root/reference)")
def test_oracle_vs_reference_random():
    rng = np.random.default_rng(11)
    for _ in range(200):
        key = rng.integers(0, 256, size=int(rng.integers(0, 400)), dtype=np.uint8).tobytes()
        a, b = pyoracle.Rc4(key), pyoracle.RefRc4(key)
        for _ in range(3):
            data = rng.integers(0, 256, size=int(rng.integers(0, 2000)), dtype=np.uint8).tobytes()
            assert a.encryption(data) == b.encryption(data)
        assert a.state() == b.state()


def _oracle_run(w):
    ob = pyoracle.Batch(w.n)
    ob.make_sbox(w.keys, w.key_off, w.key_len)
    ob.crypt(np.zeros(1000, dtype=np.uint8), np.zeros(w.n, dtype=np.uint64), w.adv, threads=8)
    out = w.payload.copy()
    ob.crypt(out, w.off, w.length, threads=8)
    states = np.empty((w.n, 258), dtype=np.uint8)
    for i in range(w.n):
        sb, x, y = ob.state(i)
        states[i, :256] = np.frombuffer(sb, dtype=np.uint8)
        states[i, 256:] = (x, y)
    return out, states


@pytest.mark.parametrize("cfg", ["cfg2", "cfg3", "cfg4"])
def test_synth_digests(cfg, synth_digests):
    S, L = synth.CONFIGS[cfg]
    d = synth_digests[cfg]
    w = synth.make(0, S, L, threads=8)
    assert hashlib.sha256(w.payload.tobytes()).hexdigest() == d["payload_in_sha256"]
    out, states = _oracle_run(w)
    assert hashlib.sha256(out.tobytes()).hexdigest() == d["ciphertext_sha256"]
    assert hashlib.sha256(states.tobytes()).hexdigest() == d["states_sha256"]


def test_synth_shard_consistency():
    """A shard [first, first+n) of a workload equals the same slice of the whole."""
    whole = synth.make(0, 64, 256)
    part = synth.make(24, 16, 256)
    assert np.array_equal(whole.keys.reshape(64, 16)[24:40], part.keys.reshape(16, 16))
    assert np.array_equal(whole.payload[24 * 256:40 * 256], part.payload)
    assert np.array_equal(whole.adv[24:40], part.adv)


def test_window_rules_match_serial_prga():
    """The speculative-window rules crypt_win_kernel runs (tools/window_sim.py,
    DESIGN.md §3.8) reproduce the serial PRGA byte for byte and state for
    state, from fresh and resumed streams, at the window widths 8 and 16; and
    the committed prefix is never empty."""
    import random
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tools"))
    import window_sim as ws
    rng = random.Random(7)
    for w in (8, 16):
        for _ in range(6):
            key = bytes(rng.randrange(256) for _ in range(rng.randrange(0, 33)))
            S = ws.ksa(key)
            _, S, x, y = ws.prga_serial(S, 0, 0, rng.randrange(0, 400))
            n = 700
            want, Sw, xw, yw = ws.prga_serial(S, x, y, n)
            got, Sg, xg, yg, windows = ws.prga_window(S, x, y, n, w)
            assert got == want and (Sg, xg, yg) == (Sw, xw, yw)
            assert windows <= n
        # oracle agreement on the same key
        r = pyoracle.Rc4(b"window")
        S = ws.ksa(b"window")
        got, *_ = ws.prga_window(S, 0, 0, 300, w)
        assert bytes(got) == r.encryption(bytes(300))
