// oracle/ref_shim.cpp -- TEST INFRASTRUCTURE ONLY.
//
// Compiles the REAL reference RC4 (/root/reference/depends/rc4/rc4_encryption.h,
// included where it lies, never copied) behind a tiny extern "C" surface so the
// golden-fixture generator (tests/golden/make_golden.py) and the CPU-only tests
// can run the reference itself, and so that bench.py's cpu_baseline leg can
// time it (zrc4_ref_crypt_rate).  Built by oracle/Makefile into
// oracle/_ref/libzrc4_ref.so, only when /root/reference is present.
//
// The reference header includes nothing itself; its includers provide <string>
// first (include/zsummerX/common/common.h:78 comes after the std headers).
#include <string>
#include <cstring>
#include <cstdint>
#include <chrono>
#include <atomic>
#include <thread>
#include <vector>
#include <rc4/rc4_encryption.h>
#include <proto4z/proto4z.h>   // HasRawPacket (depends/proto4z/proto4z.h:704-748), header-only

static_assert(sizeof(RC4Encryption) == 2 * sizeof(int) + 256 * sizeof(int),
              "reference state is int _x, _y, _box[256] (rc4_encryption.h:96-98)");

extern "C" {

int zrc4_ref_state_size(void) { return (int)sizeof(RC4Encryption); }

// RC4Encryption::makeSBox(std::string) -- rc4_encryption.h:46-72.  The key is
// built with an explicit length so embedded NULs survive, as std::string does.
void zrc4_ref_make_sbox(void *st, const uint8_t *key, size_t keylen)
{
    std::string k(reinterpret_cast<const char *>(key), keylen);
    static_cast<RC4Encryption *>(st)->makeSBox(k);
}

// RC4Encryption::encryption(unsigned char*, int) -- rc4_encryption.h:74-93.
void zrc4_ref_encryption(void *st, uint8_t *data, int length)
{
    static_cast<RC4Encryption *>(st)->encryption(data, length);
}

// Read the private state out of the standard-layout object: int _x, _y,
// _box[256] in declaration order (rc4_encryption.h:96-98).
void zrc4_ref_get_state(const void *st, uint8_t sbox[256], uint8_t *x, uint8_t *y)
{
    int raw[258];
    std::memcpy(raw, st, sizeof(raw));
    *x = (uint8_t)raw[0];
    *y = (uint8_t)raw[1];
    for (int i = 0; i < 256; ++i) sbox[i] = (uint8_t)raw[2 + i];
}

// Cross-timing helper: crypt n sessions (state array of n objects), return
// seconds spent in encryption() calls only (KSA excluded), single thread.
double zrc4_ref_crypt_batch(void *states, uint8_t *payload, const uint64_t *off,
                            const uint32_t *len, uint32_t n)
{
    RC4Encryption *s = static_cast<RC4Encryption *>(states);
    auto t0 = std::chrono::steady_clock::now();
    for (uint32_t i = 0; i < n; ++i) s[i].encryption(payload + off[i], (int)len[i]);
    auto t1 = std::chrono::steady_clock::now();
    return std::chrono::duration<double>(t1 - t0).count();
}

// CPU baseline (bench.py cpu_baseline, kind "reference"): `threads` workers,
// worker t re-crypting its contiguous share of the n sessions through the
// reference's encryption() until `seconds` have passed, all released at once;
// returns payload bytes per second over the common window.
double zrc4_ref_crypt_rate(void *states, uint8_t *payload, const uint64_t *off, const uint32_t *len,
                           uint32_t n, int threads, double seconds)
{
    if (threads < 1) threads = 1;
    if ((uint32_t)threads > n) threads = (int)n;
    RC4Encryption *s = static_cast<RC4Encryption *>(states);
    std::atomic<int> ready(0);
    std::atomic<bool> go(false);
    std::vector<unsigned long long> bytes((size_t)threads, 0ull);
    std::vector<std::thread> pool;
    typedef std::chrono::steady_clock clk;
    clk::time_point deadline = clk::now();   // workers read it only after `go`
    bool failed = false;
    for (int t = 0; t < threads && !failed; ++t) {
        try {
        pool.emplace_back([&, t]() {
            const uint32_t b = (uint32_t)((uint64_t)n * t / threads), e = (uint32_t)((uint64_t)n * (t + 1) / threads);
            unsigned long long done = 0;
            ready.fetch_add(1);
            while (!go.load(std::memory_order_acquire)) {}
            while (clk::now() < deadline) {
                for (uint32_t i = b; i < e; ++i) {
                    s[i].encryption(payload + off[i], (int)len[i]);
                    done += len[i];
                }
            }
            bytes[(size_t)t] = done;
        });
        } catch (...) {          // no thread: release the started ones at once and report failure
            failed = true;
        }
    }
    if (failed) {
        go.store(true, std::memory_order_release);
        for (auto &th : pool) th.join();
        return -1.0;
    }
    while (ready.load() != threads) {}
    const clk::time_point t0 = clk::now();
    deadline = t0 + std::chrono::duration_cast<clk::duration>(std::chrono::duration<double>(seconds));
    go.store(true, std::memory_order_release);
    for (auto &th : pool) th.join();
    const double dt = std::chrono::duration<double>(clk::now() - t0).count();
    unsigned long long total = 0;
    for (unsigned long long v : bytes) total += v;
    return (double)total / dt;
}

// zsummer::proto4z::HasRawPacket -- the reference's framing check, as
// TcpSession::onRecv calls it through DefaultRawPacketCheck
// (include/zsummerX/frame/manager.h:53-57).  Returns the IntegrityType
// (0 intact, 1 shortage, 2 corrupted) and its length result in *second.
int zrc4_ref_has_raw_packet(const uint8_t *buff, uint32_t cur, uint32_t bound_len, uint32_t max_len,
                            uint32_t *second)
{
    auto r = zsummer::proto4z::HasRawPacket(reinterpret_cast<const char *>(buff), cur, bound_len, max_len);
    *second = r.second;
    return (int)r.first;
}

}  // extern "C"
