// hooks_check.cpp -- TEST INFRASTRUCTURE ONLY.
// Drives an Rc4Hooks (the device hooks of libzsx_frame.so, or any other) with
// the engine's call pattern -- seed both streams of S sessions, then rounds of
// crypt() over random spans inside pooled blocks, reseeding some sessions on
// the way -- and checks every byte against the oracle RC4
// (oracle/rc4_oracle.c, pinned to rc4_encryption.h:46-93).
//   usage: hooks_check [device|direct] [sessions] [rounds] [seed] [ring bytes]
// (a small ring forces ring wrap-around, partial ring coverage and tail
// crypts on most calls).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "zrc4.h"
#include "zsummerx_amd/rc4_hooks.h"
extern "C" {
#include "rc4_oracle.h"
}

using namespace zsummerx_amd;

int main(int argc, char **argv)
{
    const std::string mode = argc > 1 ? argv[1] : "device";
    const uint32_t S = argc > 2 ? (uint32_t)std::atoi(argv[2]) : 64;
    const int rounds = argc > 3 ? std::atoi(argv[3]) : 200;
    std::mt19937 rng(argc > 4 ? std::atoi(argv[4]) : 1);
    const uint32_t slots = 2 * S;
    const uint32_t ring = argc > 5 ? (uint32_t)std::atoi(argv[5]) : 32768u;
    std::unique_ptr<Rc4Hooks> h = makeDeviceRc4Hooks(0, slots, mode == "direct" ? 0u : ring);
    const size_t blk = 20544;
    uint8_t *pool = static_cast<uint8_t *>(h->allocBlocks(slots * blk + 64));
    std::vector<oracle_rc4_state> ref(slots);
    std::vector<std::string> keys(S);
    auto seedSession = [&](uint32_t s) {
        std::string k;
        const int kl = 1 + (int)(rng() % 30);
        for (int i = 0; i < kl; ++i) k.push_back((char)(rng() & 255));
        keys[s] = k;
        const uint32_t two[2] = {2 * s, 2 * s + 1};
        h->seed(two, 2, k);
        oracle_make_sbox(&ref[2 * s], reinterpret_cast<const uint8_t *>(k.data()), k.size());
        oracle_make_sbox(&ref[2 * s + 1], reinterpret_cast<const uint8_t *>(k.data()), k.size());
    };
    for (uint32_t s = 0; s < S; ++s) seedSession(s);
    std::vector<uint8_t> want(slots * blk);
    unsigned long long bytes = 0;
    for (int r = 0; r < rounds; ++r) {
        if (r && r % 37 == 0) seedSession(rng() % S);            // reconnect
        std::vector<Rc4Span> spans;
        for (uint32_t sl = 0; sl < slots; ++sl) {
            if (rng() % 3 == 0) continue;                         // idle this round
            const uint32_t pick = rng() % 10;
            const uint32_t len = pick < 3 ? 1 + rng() % 16 : pick < 8 ? 1 + rng() % 2048 : 1 + rng() % 20480;
            const uint32_t start = (uint32_t)(rng() % (20480 - len + 1));
            uint8_t *d = pool + 64 + sl * blk + start;
            for (uint32_t i = 0; i < len; ++i) d[i] = (uint8_t)rng();
            std::memcpy(&want[sl * blk + start], d, len);
            oracle_encryption(&ref[sl], &want[sl * blk + start], len);
            spans.push_back({sl, len, d});
            bytes += len;
        }
        const int rc = h->crypt(spans.data(), (uint32_t)spans.size());
        if (rc) {
            std::printf("{\"ok\": false, \"round\": %d, \"rc\": %d}\n", r, rc);
            return 1;
        }
        for (const Rc4Span &sp : spans) {
            const uint8_t *w = &want[sp.slot * blk + (sp.data - (pool + 64 + sp.slot * blk))];
            for (uint32_t i = 0; i < sp.len; ++i)
                if (sp.data[i] != w[i]) {
                    std::printf("{\"ok\": false, \"mode\": \"%s\", \"round\": %d, \"slot\": %u, \"len\": %u, "
                                "\"byte\": %u, \"got\": %u, \"want\": %u}\n",
                                mode.c_str(), r, sp.slot, sp.len, i, sp.data[i], w[i]);
                    return 2;
                }
        }
    }
    // a slot twice in one call is refused (rc4_hooks.h contract), state untouched
    {
        uint8_t *d = pool + 64;
        const Rc4Span dup[2] = {{0, 16, d}, {0, 16, d + 32}};
        const int rc = h->crypt(dup, 2);
        if (rc != ZRC4_ERR_INVALID_ARG) {
            std::printf("{\"ok\": false, \"duplicate_rc\": %d}\n", rc);
            return 4;
        }
    }
    std::printf("{\"ok\": true, \"mode\": \"%s\", \"sessions\": %u, \"rounds\": %d, \"bytes\": %llu, "
                "\"hooks\": %s}\n", mode.c_str(), S, rounds, bytes, h->stats().c_str());
    h->freeBlocks(pool);
    return 0;
}
