// C++ test of include/zsummerx_amd/rc4_encryption.h (the reference-shaped
// class over libzrc4.so).  Exit code 0 = pass.  Needs a gfx950 GPU.
//
// Vectors: the published Wikipedia RC4 KATs (also pinned against the real
// reference header in tests/golden/kat.json).
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "zsummerx_amd/rc4_encryption.h"

using zsummerx_amd::RC4Encryption;
using zsummerx_amd::Rc4Arena;
using zsummerx_amd::Rc4Batch;

static int fails = 0;
#define CHECK(c)                                                        \
    do {                                                                \
        if (!(c)) {                                                     \
            std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c);     \
            ++fails;                                                    \
        }                                                               \
    } while (0)

static std::string hex(const unsigned char *p, size_t n)
{
    static const char *d = "0123456789ABCDEF";
    std::string s;
    for (size_t i = 0; i < n; ++i) { s += d[p[i] >> 4]; s += d[p[i] & 15]; }
    return s;
}

int main()
{
    const char *kat[][3] = {{"Key", "Plaintext", "BBF316E8D940AF0AD3"},
                            {"Wiki", "pedia", "1021BF0420"},
                            {"Secret", "Attack at dawn", "45A01F645FC35B383552544B9BF5"}};
    for (auto &k : kat) {
        RC4Encryption r;
        r.makeSBox(k[0]);
        std::vector<unsigned char> b(k[1], k[1] + std::strlen(k[1]));
        r.encryption(b.data(), (int)b.size());
        CHECK(hex(b.data(), b.size()) == k[2]);
    }
    // split invariance + length <= 0 no-op (rc4_encryption.h:81)
    {
        RC4Encryption a, b;
        a.makeSBox("Key");
        b.makeSBox("Key");
        unsigned char x[10] = {0}, y[10] = {0};
        a.encryption(x, 10);
        b.encryption(y, 3);
        b.encryption(y + 3, 0);
        b.encryption(y + 3, -4);
        b.encryption(y + 3, 7);
        CHECK(std::memcmp(x, y, 10) == 0);
    }
    // NUL inside the key counts (std::string length, not strlen)
    {
        RC4Encryption a, b;
        a.makeSBox(std::string("a\0b", 3));
        b.makeSBox(std::string("a"));
        unsigned char x[8] = {0}, y[8] = {0};
        a.encryption(x, 8);
        b.encryption(y, 8);
        CHECK(std::memcmp(x, y, 8) != 0);
    }
    // Two peers as TcpSession hooks: client write stream -> server read
    // stream, both seeded from the same key (session.cpp:110-111; the build
    // also seeds on accept), through the batched per-iteration path.
    {
        const int kPeers = 300;
        std::vector<RC4Encryption> cw(kPeers), sr(kPeers);
        for (int i = 0; i < kPeers; ++i) {
            std::string key = "session-key-" + std::to_string(i);
            cw[i].makeSBox(key);
            sr[i].makeSBox(key);
        }
        std::vector<std::vector<unsigned char>> plain(kPeers), wire(kPeers);
        for (int i = 0; i < kPeers; ++i) {
            plain[i].resize(1 + (i * 37) % 3000);
            for (size_t j = 0; j < plain[i].size(); ++j) plain[i][j] = (unsigned char)(i * 131 + j * 7);
            wire[i] = plain[i];
        }
        zrc4_ctx *ctx = Rc4Arena::instance().ctx(cw[0].slot());
        for (int i = 0; i < kPeers; ++i) CHECK(cw[i].slot() / Rc4Arena::kChunk == 0 && sr[i].slot() / Rc4Arena::kChunk == 0);
        Rc4Batch send_batch(ctx), recv_batch(ctx);
        for (int i = 0; i < kPeers; ++i)
            send_batch.add(Rc4Arena::local(cw[i].slot()), wire[i].data(), (unsigned)wire[i].size());
        CHECK(send_batch.flush() == ZRC4_OK);
        int differs = 0;
        for (int i = 0; i < kPeers; ++i) differs += wire[i] != plain[i];
        CHECK(differs == kPeers);
        for (int i = 0; i < kPeers; ++i)
            recv_batch.add(Rc4Arena::local(sr[i].slot()), wire[i].data(), (unsigned)wire[i].size());
        CHECK(recv_batch.flush() == ZRC4_OK);
        for (int i = 0; i < kPeers; ++i) CHECK(wire[i] == plain[i]);
    }
    // value semantics: a copy continues the same stream from the same point
    {
        RC4Encryption a;
        a.makeSBox("Key");
        unsigned char x[9] = {0};
        a.encryption(x, 4);
        RC4Encryption b(a), c;
        c = a;
        unsigned char p[5] = {0}, q[5] = {0}, r[5] = {0};
        a.encryption(p, 5);
        b.encryption(q, 5);
        c.encryption(r, 5);
        CHECK(std::memcmp(p, q, 5) == 0 && std::memcmp(p, r, 5) == 0);
        unsigned char whole[9] = {0};
        RC4Encryption d;
        d.makeSBox("Key");
        d.encryption(whole, 9);
        CHECK(std::memcmp(whole + 4, q, 5) == 0);
        RC4Encryption m(std::move(b));                 // move keeps the slot and its state
        unsigned char t[3] = {0}, u[3] = {0};
        m.encryption(t, 3);
        c.encryption(u, 3);
        CHECK(std::memcmp(t, u, 3) == 0);
    }
    // slots recycle with the empty-key state; more than one 65 536-stream chunk
    {
        uint32_t first;
        {
            RC4Encryption a;
            a.makeSBox("something");
            first = a.slot();
        }
        RC4Encryption b;                               // reuses a's slot, identity state
        CHECK(b.slot() == first);
        unsigned char x[8] = {0}, y[8] = {0};
        b.encryption(x, 8);
        RC4Encryption e;
        e.makeSBox("");
        e.encryption(y, 8);
        CHECK(std::memcmp(x, y, 8) == 0);
        std::vector<RC4Encryption> many(Rc4Arena::kChunk + 100);
        CHECK(many.back().slot() >= Rc4Arena::kChunk);
        many.back().makeSBox("Key");
        std::vector<unsigned char> z(9, 0);
        many.back().encryption(z.data(), 9);
        CHECK(hex(z.data(), 9) != "000000000000000000");
        unsigned char kp[9];
        std::memcpy(kp, "Plaintext", 9);
        for (int i = 0; i < 9; ++i) kp[i] ^= z[i];
        CHECK(hex(kp, 9) == "BBF316E8D940AF0AD3");
    }
    std::printf(fails ? "FAILED %d\n" : "ok\n", fails);
    return fails ? 1 : 0;
}
