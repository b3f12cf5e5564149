// emu_zrc4_hip.cpp -- TEST INFRASTRUCTURE ONLY.
//
// A CPU emulation of exactly the surface zsummerx_amd/engine/rc4_hooks_device.cpp
// uses -- the zrc4 C-ABI (include/zrc4.h) and a handful of HIP runtime calls --
// so the device hooks' HOST logic (reservoir levels, ring positions, top-up
// pieces, refill commits, reseeding) can be exercised on a machine without a
// GPU.  Every "launch" runs synchronously on the CPU; RC4 is the oracle
// restatement (oracle/rc4_oracle.c, pinned to rc4_encryption.h:46-93).  It is
// linked only into tests' emulated frame_stress binary (tests/test_frame.py),
// never into the product library.
#include <hip/hip_runtime_api.h>

#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <vector>

#include "zrc4.h"
extern "C" {
#include "rc4_oracle.h"
}

struct zrc4_ctx {
    std::vector<oracle_rc4_state> st;
};

extern "C" {

int zrc4_create(zrc4_ctx **out, int, uint32_t capacity)
{
    auto *c = new zrc4_ctx();
    c->st.resize((capacity + 255u) & ~255u);
    for (auto &s : c->st) oracle_make_sbox(&s, nullptr, 0);
    *out = c;
    return ZRC4_OK;
}
int zrc4_destroy(zrc4_ctx *c)
{
    delete c;
    return ZRC4_OK;
}
uint32_t zrc4_capacity(const zrc4_ctx *c) { return (uint32_t)c->st.size(); }
int zrc4_ksa(zrc4_ctx *c, const uint32_t *ids, const uint8_t *keys, const uint64_t *ko, const uint32_t *kl,
             uint32_t n, void *)
{
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t s = ids ? ids[i] : i;
        if (s >= c->st.size()) return ZRC4_ERR_SLOT_RANGE;
        oracle_make_sbox(&c->st[s], keys + ko[i], kl[i]);
    }
    return ZRC4_OK;
}
int zrc4_crypt(zrc4_ctx *c, const uint32_t *ids, uint8_t *payload, const uint64_t *off, const uint32_t *len,
               uint32_t n, void *)
{
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t s = ids ? ids[i] : i;
        if (s >= c->st.size()) return ZRC4_ERR_SLOT_RANGE;
        oracle_encryption(&c->st[s], payload + off[i], (long)len[i]);
    }
    return ZRC4_OK;
}
// Same contract checks as crypt_kernel<kGrouped>: a bucket's busy entries
// must share one group, and no other bucket of the call may name that group
// (else the bucket is skipped and ZRC4_ERR_GROUP reported; here the first
// bucket to name a group keeps it).
int zrc4_crypt_grouped(zrc4_ctx *c, const uint32_t *ids, uint8_t *payload, const uint64_t *off,
                       const uint32_t *len, uint32_t n, void *)
{
    int rc = ZRC4_OK;
    std::vector<uint32_t> held;
    for (uint32_t b = 0; b < n; b += 256) {
        const uint32_t e = b + 256 < n ? b + 256 : n;
        uint32_t gmin = 0xFFFFFFFFu, gmax = 0;
        for (uint32_t i = b; i < e; ++i) {
            if (!len[i] || ids[i] == ZRC4_IDLE_SLOT) continue;
            if (ids[i] >= c->st.size()) return ZRC4_ERR_SLOT_RANGE;
            gmin = ids[i] / 256 < gmin ? ids[i] / 256 : gmin;
            gmax = ids[i] / 256 > gmax ? ids[i] / 256 : gmax;
        }
        if (gmin != 0xFFFFFFFFu && gmin != gmax) {
            rc = ZRC4_ERR_GROUP;
            continue;
        }
        if (gmin != 0xFFFFFFFFu) {
            if (std::find(held.begin(), held.end(), gmin) != held.end()) {
                rc = ZRC4_ERR_GROUP;
                continue;
            }
            held.push_back(gmin);
        }
        for (uint32_t i = b; i < e; ++i)
            if (len[i] && ids[i] != ZRC4_IDLE_SLOT) oracle_encryption(&c->st[ids[i]], payload + off[i], (long)len[i]);
    }
    return rc;
}
int zrc4_crypt_grouped_frame(zrc4_ctx *c, const uint32_t *ids, uint8_t *payload, const uint64_t *off,
                             const uint32_t *len, uint32_t n, const zrc4_frame_args *f, void *s)
{
    const int rc = zrc4_crypt_grouped(c, ids, payload, off, len, n, s);
    oracle_frame_scan(payload, f->off, f->len, f->bound, n, f->max_packets, f->npk, f->used, f->status, f->pkt_len);
    return rc;
}
// zrc4_crypt_grouped_declared: a bucket with a busy entry outside its
// declared group is skipped (ZRC4_ERR_GROUP), then zrc4_crypt_grouped.
int zrc4_crypt_grouped_declared(zrc4_ctx *c, const uint32_t *ids, const uint32_t *bg, uint8_t *payload,
                                const uint64_t *off, const uint32_t *len, uint32_t n,
                                const struct zrc4_frame_args *f, void *s)
{
    if (n && (!ids || !bg)) return ZRC4_ERR_INVALID_ARG;
    const uint32_t groups = (uint32_t)((c->st.size() + 255) / 256);
    for (uint32_t b = 0; b < (n + 255) / 256; ++b)
        if (bg[b] >= groups && bg[b] != ZRC4_IDLE_SLOT) return ZRC4_ERR_INVALID_ARG;
    std::vector<uint32_t> kept(ids, ids + n);
    std::vector<uint32_t> lost;           // groups a disagreeing bucket's ids name
    int rc = ZRC4_OK;
    for (uint32_t b = 0; b < n; b += 256) {
        const uint32_t e = b + 256 < n ? b + 256 : n;
        bool bad = false;
        for (uint32_t i = b; i < e; ++i)
            if (len[i] && ids[i] != ZRC4_IDLE_SLOT && ids[i] < c->st.size() && ids[i] / 256 != bg[b / 256]) bad = true;
        if (bad) {
            rc = ZRC4_ERR_GROUP;
            for (uint32_t i = b; i < e; ++i) {
                if (len[i] && ids[i] != ZRC4_IDLE_SLOT && ids[i] < c->st.size()) lost.push_back(ids[i] / 256);
                kept[i] = ZRC4_IDLE_SLOT;
            }
        }
    }
    // Above 256 buckets the GPU checks the declarations in a kernel before the
    // crypt launch (include/zrc4.h): a disagreeing bucket's ids also block the
    // groups they name, so every other bucket declaring one of them is refused
    // too.  At most 256 buckets the groups travel in the kernel arguments and
    // only the disagreeing bucket is refused.
    if ((n + 255) / 256 > 256 && !lost.empty()) {
        for (uint32_t b = 0; b < n; b += 256) {
            if (std::find(lost.begin(), lost.end(), bg[b / 256]) == lost.end()) continue;
            const uint32_t e = b + 256 < n ? b + 256 : n;
            for (uint32_t i = b; i < e; ++i) kept[i] = ZRC4_IDLE_SLOT;
        }
    }
    const int r2 = f ? zrc4_crypt_grouped_frame(c, kept.data(), payload, off, len, n, f, s)
                     : zrc4_crypt_grouped(c, kept.data(), payload, off, len, n, s);
    return r2 ? r2 : rc;
}
int zrc4_xor_ring(zrc4_ctx *, uint8_t *ring, uint32_t cap, const uint32_t *rid, const uint32_t *pos,
                  uint8_t *payload, const uint64_t *off, const uint32_t *len, uint32_t n, void *)
{
    for (uint32_t i = 0; i < n; ++i) {
        uint8_t *r = ring + (size_t)rid[i] * cap;
        uint8_t *d = payload + off[i];
        for (uint32_t k = 0; k < len[i]; ++k) {
            uint32_t q = pos[i] + k;
            if (q >= cap) q -= cap;
            d[k] ^= r[q];
            r[q] = 0;
        }
    }
    return ZRC4_OK;
}
// Keystream reservoirs (zrc4_ks_*) as their observable semantics: the C++
// mirror (include/zsummerx_amd/rc4_encryption.h) over this emulation crypts
// every call straight on the oracle state (no rings to emulate: a reservoir
// changes when keystream is made, never which bytes come out).
struct zrc4_ks {
    zrc4_ctx *c;
};
int zrc4_ks_create(zrc4_ctx *c, uint32_t, zrc4_ks **out)
{
    *out = new zrc4_ks{c};
    return ZRC4_OK;
}
int zrc4_ks_destroy(zrc4_ks *k)
{
    delete k;
    return ZRC4_OK;
}
int zrc4_ks_crypt(zrc4_ks *k, const uint32_t *ids, uint8_t *const *data, const uint32_t *len, uint32_t n)
{
    for (uint32_t i = 0; i < n; ++i) {
        if (ids[i] >= k->c->st.size()) return ZRC4_ERR_SLOT_RANGE;
        oracle_encryption(&k->c->st[ids[i]], data[i], (long)len[i]);
    }
    return ZRC4_OK;
}
int zrc4_ks_make_sbox(zrc4_ks *k, uint32_t id, const uint8_t *key, size_t keylen)
{
    if (id >= k->c->st.size()) return ZRC4_ERR_SLOT_RANGE;
    oracle_make_sbox(&k->c->st[id], key, keylen);
    return ZRC4_OK;
}
int zrc4_ks_copy(zrc4_ks *dk, uint32_t dst, zrc4_ks *sk, uint32_t src)
{
    if (dst >= dk->c->st.size() || src >= sk->c->st.size()) return ZRC4_ERR_SLOT_RANGE;
    dk->c->st[dst] = sk->c->st[src];
    return ZRC4_OK;
}
int zrc4_sync(zrc4_ctx *, void *) { return ZRC4_OK; }
int zrc4_poll_faults(zrc4_ctx *) { return ZRC4_OK; }
const char *zrc4_strerror(int) { return "emulated zrc4"; }

}  // extern "C"

// HIP runtime calls used by the hooks (C++ linkage, as hip_runtime_api.h declares them).
hipError_t hipSetDevice(int) { return hipSuccess; }
hipError_t hipHostMalloc(void **p, size_t n, unsigned int)
{
    *p = std::aligned_alloc(64, (n + 63) / 64 * 64);
    return *p ? hipSuccess : hipErrorOutOfMemory;
}
hipError_t hipHostFree(void *p)
{
    std::free(p);
    return hipSuccess;
}
hipError_t hipMalloc(void **p, size_t n)
{
    *p = std::aligned_alloc(64, (n + 63) / 64 * 64);
    return *p ? hipSuccess : hipErrorOutOfMemory;
}
hipError_t hipFree(void *p)
{
    std::free(p);
    return hipSuccess;
}
hipError_t hipMemsetAsync(void *p, int v, size_t n, hipStream_t)
{
    std::memset(p, v, n);
    return hipSuccess;
}
static int g_stream_tag;
hipError_t hipStreamCreateWithFlags(hipStream_t *s, unsigned int)
{
    *s = reinterpret_cast<hipStream_t>(&g_stream_tag);
    return hipSuccess;
}
hipError_t hipStreamSynchronize(hipStream_t) { return hipSuccess; }
hipError_t hipStreamDestroy(hipStream_t) { return hipSuccess; }
static int g_event_tag;
hipError_t hipEventCreateWithFlags(hipEvent_t *e, unsigned)
{
    *e = reinterpret_cast<hipEvent_t>(&g_event_tag);
    return hipSuccess;
}
hipError_t hipEventRecord(hipEvent_t, hipStream_t) { return hipSuccess; }
// Alternate "not ready" / "done" so both commit paths (poll and wait) run.
hipError_t hipEventQuery(hipEvent_t)
{
    static unsigned k;
    return (++k % 3) ? hipErrorNotReady : hipSuccess;
}
hipError_t hipEventSynchronize(hipEvent_t) { return hipSuccess; }
hipError_t hipEventDestroy(hipEvent_t) { return hipSuccess; }
