// synth.cpp -- synthetic workload generator for the RC4 bench and tests
// (SURVEY.md §8d).  Not part of the C-ABI product library; built into
// zsummerx_amd/libzrc4_synth.so.
//
//   keys:    session s gets 16 bytes = two std::mt19937_64(seed=1) outputs,
//            little-endian, in session order (global session id).
//   payload: bytes of std::mt19937_64(seed=42) outputs, little-endian,
//            filling the contiguous [S][L] buffer in order.
//   advance: session s's stream is pre-advanced by (s*37) % 1000 bytes.
#include <cstdint>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

namespace {
inline void put64(uint8_t *d, uint64_t v)
{
    for (int i = 0; i < 8; ++i) d[i] = (uint8_t)(v >> (8 * i));
}
}  // namespace

extern "C" {

// keys for global sessions [first, first+n): 16 bytes each into out[n*16].
void zrc4_synth_keys(uint64_t first, uint64_t n, uint8_t *out)
{
    std::mt19937_64 g(1);
    g.discard(2 * first);
    for (uint64_t i = 0; i < n; ++i) {
        put64(out + 16 * i, g());
        put64(out + 16 * i + 8, g());
    }
}

// payload bytes [byte_first, byte_first + nbytes) of the seed-42 stream.
// byte_first must be a multiple of 8.  Chunks are generated in parallel with
// independent discard() offsets (the result does not depend on `threads`).
int zrc4_synth_payload(uint64_t byte_first, uint64_t nbytes, uint8_t *out, int threads)
{
    if (byte_first % 8) return -1;
    if (threads < 1) threads = 1;
    const uint64_t words = (nbytes + 7) / 8;
    const uint64_t per = (words + threads - 1) / threads;
    auto work = [&](int t) {
        const uint64_t w0 = per * t, w1 = w0 + per < words ? w0 + per : words;
        if (w0 >= w1) return;
        std::mt19937_64 g(42);
        g.discard(byte_first / 8 + w0);
        for (uint64_t w = w0; w < w1; ++w) {
            const uint64_t v = g();
            const uint64_t b = 8 * w;
            if (b + 8 <= nbytes) put64(out + b, v);
            else for (uint64_t i = 0; b + i < nbytes; ++i) out[b + i] = (uint8_t)(v >> (8 * i));
        }
    };
    if (threads == 1) { work(0); return 0; }
    std::vector<std::thread> ts;
    for (int t = 0; t < threads; ++t) ts.emplace_back(work, t);
    for (auto &t : ts) t.join();
    return 0;
}

// pre-advance lengths (s*37) % 1000 for global sessions [first, first+n).
void zrc4_synth_advance(uint64_t first, uint64_t n, uint32_t *out)
{
    for (uint64_t i = 0; i < n; ++i) out[i] = (uint32_t)(((first + i) * 37u) % 1000u);
}

}  // extern "C"
