"""The reference's C# client cipher against the server side (CPU, no GPU).

zsummerX ships a second RC4 for its C# clients: Proto4z.RC4Encryption
(depends/proto4z/Proto4z.cs:43-98), restated here line for line in Python.
Its PRGA is the C++ one (rc4_encryption.h:74-93); its KSA takes the key as a
C# string and uses the low byte of each UTF-16 code unit, where the C++ KSA
(rc4_encryption.h:46-72) uses the bytes of a std::string.  So a C# peer and
the server agree exactly when the server's key bytes are those low bytes:
any ASCII key does.  The oracle (pinned to the compiled C++ header, and the
device path pinned to the oracle) is checked against the restatement on that
contract, and the one divergence is pinned so that it stays documented
("C# clients")."""
import random
import struct

import pyoracle


class CsRc4:
    """Proto4z.cs:43-98, restated (ints for the box, byte casts as written)."""

    def make_sbox(self, obscure: str):
        self.box = list(range(256))
        self.x = self.y = 0
        if len(obscure) > 0:
            j = k = 0
            raw = obscure.encode("utf-16-le")                 # char[] obs = obscure.ToCharArray()
            units = list(struct.unpack(f"<{len(raw) // 2}H", raw))
            for i in range(256):
                tmp = self.box[i]
                j = (j + tmp + (units[k] & 0xFF)) & 0xFF
                self.box[i] = self.box[j]
                self.box[j] = tmp
                k += 1
                if k >= len(units):
                    k = 0

    def encryption(self, data: bytearray, offset: int, length: int):
        x, y = self.x, self.y
        for i in range(offset, offset + length):
            x = (x + 1) & 0xFF
            a = self.box[x]
            y = (y + a) & 0xFF
            b = self.box[x] = self.box[y]
            self.box[y] = a
            data[i] ^= self.box[(a + b) & 0xFF]
        self.x, self.y = x, y


def _cs_stream(key: str, chunks):
    c = CsRc4()
    c.make_sbox(key)
    out = b""
    for ch in chunks:
        buf = bytearray(ch)
        c.encryption(buf, 0, len(buf))
        out += bytes(buf)
    return out


def test_ascii_keys_interoperate_with_the_server_cipher():
    rng = random.Random(43)
    for _ in range(40):
        key = "".join(chr(rng.randint(0x20, 0x7E)) for _ in range(rng.randint(1, 40)))
        msg = bytes(rng.randrange(256) for _ in range(rng.randint(1, 3000)))
        cuts = sorted(rng.sample(range(1, len(msg)), min(4, len(msg) - 1))) if len(msg) > 1 else []
        chunks = [msg[a:b] for a, b in zip([0] + cuts, cuts + [len(msg)])]
        server = pyoracle.Rc4(key.encode("ascii"))
        want = b"".join(server.encryption(ch) for ch in chunks)
        assert _cs_stream(key, chunks) == want, key


def test_empty_key_is_the_identity_box_on_both_sides():
    msg = bytes(range(200))
    assert _cs_stream("", [msg]) == pyoracle.Rc4(b"").encryption(msg)


def test_non_ascii_keys_follow_the_utf16_low_bytes():
    """'clé' is 63 6c e9 to the C# KSA (low bytes of its UTF-16 units) and
    63 6c c3 a9 as UTF-8: the C# peer matches a server keyed with the former,
    not the latter; an astral character contributes its two surrogates' low
    bytes."""
    msg = bytes(range(256)) * 4
    for key, low in (("clé", b"cl\xe9"), ("k中", b"k\x2d"), ("a\U0001F600", b"a\x3d\x00")):
        got = _cs_stream(key, [msg])
        assert got == pyoracle.Rc4(low).encryption(msg), key
        assert got != pyoracle.Rc4(key.encode("utf-8")).encryption(msg), key
