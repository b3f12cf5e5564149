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
#include "rc4_oracle.h"   // test infrastructure: the CPU restatement (oracle/)

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
        zrc4_ks *ks = Rc4Arena::instance().ks(cw[0].slot());
        for (int i = 0; i < kPeers; ++i) CHECK(cw[i].slot() / Rc4Arena::kChunk == 0 && sr[i].slot() / Rc4Arena::kChunk == 0);
        Rc4Batch send_batch(ks), recv_batch(ks);
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
    // The reservoir under a session's call pattern: many streams, calls of
    // 0..3000 bytes (bursts larger than the ring), reseeds, copies taken
    // mid-stream, batched and per-call paths mixed, every byte against the
    // oracle; then the reservoir statistics show both host-XOR and device-tail
    // bytes were exercised.
    {
        const int kStreams = 200, kRounds = 60;
        std::vector<RC4Encryption> r(kStreams);
        std::vector<oracle_rc4_state> o(kStreams);
        uint64_t rng = 12345;
        auto next = [&rng]() { rng = rng * 6364136223846793005ull + 1442695040888963407ull; return (uint32_t)(rng >> 33); };
        for (int i = 0; i < kStreams; ++i) {
            std::string key = "reservoir-" + std::to_string(i * 7919);
            r[i].makeSBox(key);
            oracle_make_sbox(&o[i], reinterpret_cast<const uint8_t *>(key.data()), key.size());
        }
        int bad = 0;
        for (int round = 0; round < kRounds; ++round) {
            zrc4_ks *ks = Rc4Arena::instance().ks(r[0].slot());
            Rc4Batch batch(ks);
            std::vector<std::vector<unsigned char>> bufs(kStreams), want(kStreams);
            for (int i = 0; i < kStreams; ++i) {
                const uint32_t n = (next() % 7 == 0) ? 1000 + next() % 2000 : next() % 600;
                bufs[i].resize(n);
                for (auto &b : bufs[i]) b = (unsigned char)next();
                want[i] = bufs[i];
                oracle_encryption(&o[i], want[i].data(), (long)n);
                if (round % 2 == 0 && Rc4Arena::instance().ks(r[i].slot()) == ks)
                    batch.add(Rc4Arena::local(r[i].slot()), bufs[i].data(), n);
                else
                    r[i].encryption(bufs[i].data(), (int)n);
            }
            CHECK(batch.flush() == ZRC4_OK);
            for (int i = 0; i < kStreams; ++i) bad += bufs[i] != want[i];
            if (round % 10 == 5) {              // reseed some, copy some
                for (int i = 0; i < kStreams; i += 17) {
                    std::string key = "re-" + std::to_string(round * 1000 + i);
                    r[i].makeSBox(key);
                    oracle_make_sbox(&o[i], reinterpret_cast<const uint8_t *>(key.data()), key.size());
                }
                for (int i = 3; i + 1 < kStreams; i += 29) {
                    r[i + 1] = r[i];            // value copy mid-stream, keystream buffered or not
                    o[i + 1] = o[i];
                }
            }
        }
        CHECK(bad == 0);
        uint64_t st[6] = {0};
        CHECK(zrc4_ks_stats(Rc4Arena::instance().ks(r[0].slot()), st) == ZRC4_OK);
        std::printf("reservoir: ring %llu B, tail %llu B in %llu launches, refill %llu B in %llu launches, %llu waits\n",
                    (unsigned long long)st[0], (unsigned long long)st[1], (unsigned long long)st[2],
                    (unsigned long long)st[3], (unsigned long long)st[4], (unsigned long long)st[5]);
        CHECK(st[0] > 0 && st[1] > 0 && st[4] > 0);
    }
    std::printf(fails ? "FAILED %d\n" : "ok\n", fails);
    return fails ? 1 : 0;
}
