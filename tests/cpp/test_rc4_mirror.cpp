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
        Rc4Batch send_batch, recv_batch;
        for (int i = 0; i < kPeers; ++i) send_batch.add(cw[i].slot(), wire[i].data(), (unsigned)wire[i].size());
        CHECK(send_batch.flush() == ZRC4_OK);
        int differs = 0;
        for (int i = 0; i < kPeers; ++i) differs += wire[i] != plain[i];
        CHECK(differs == kPeers);
        for (int i = 0; i < kPeers; ++i) recv_batch.add(sr[i].slot(), wire[i].data(), (unsigned)wire[i].size());
        CHECK(recv_batch.flush() == ZRC4_OK);
        for (int i = 0; i < kPeers; ++i) CHECK(wire[i] == plain[i]);
    }
    std::printf(fails ? "FAILED %d\n" : "ok\n", fails);
    return fails ? 1 : 0;
}
