// zrc4.hip -- C-ABI implementation (include/zrc4.h) over the gfx950 kernels.
//
// Host side of the drop-in for RC4Encryption (depends/rc4/rc4_encryption.h:43-99).
// The device arena replaces the by-value RC4Encryption members of TcpSession
// (include/zsummerX/frame/session.h:115-116); see INTEGRATION.md.
#include "zrc4.h"
#include "zrc4_kernels.hpp"
#include "zrc4_win.hpp"

#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <vector>
#include <new>
#include <thread>

#ifndef ZRC4_HALF
#define ZRC4_HALF 1   // A/B knob: 0 runs few-group range batches on whole-group workgroups too
#endif
#ifndef ZRC4_WIN_MAX_GROUPS
#define ZRC4_WIN_MAX_GROUPS 32   // aligned range and grouped batches of at most this many groups run
                                 // 16 lanes per stream (crypt_win_kernel, zrc4_win.hpp); 0 = never
#endif
static_assert(ZRC4_WIN_MAX_GROUPS <= zrc4::kWinMaxBuckets, "declared window groups travel in WinGroups");

struct zrc4_ctx {
    int device;
    int num_cus;
    uint32_t capacity;      // multiple of 256
    uint8_t *arena;         // capacity/256 groups x 64 KiB S-box images
    uint16_t *xy;           // per slot: x | y << 8
    uint8_t *sink;          // crypt_kernel's per-thread sink slots (loads/stores past a
                            // session's last block in the DPP line loop)
    uint32_t *err;          // latched device-side faults (zrc4::kErrWords words, one per
                            // kind) in pinned host memory: kernels latch with a plain
                            // store, the host reads them after the stream wait (no
                            // read-back copy).  Per context, not per stream.
    // staging for the *_host entry points (grown on demand)
    uint8_t *d_stage;
    size_t d_stage_bytes;
    uint8_t *h_stage;       // pinned
    size_t h_stage_bytes;
    hipStream_t stream;     // private stream for the host entry points
    unsigned long long *claim;   // grouped launches' (group, part) claim words (zrc4::Claim), zeroed
    uint32_t epoch;              // the last grouped launch's claim tag
    // Declared bucket groups of large declared launches (decl_check_kernel
    // reads them zero-copy): a ring of coherent pinned buffers, each reused
    // once the check kernel that read it has run (its event).  A pageable
    // hipMemcpyAsync here blocked the host until the stream drained: +4.7 us
    // per cfg3 call back to back (profiles/r05/ab_ids_modes.log).
    static constexpr int kDeclRing = 4;
    uint32_t *h_decl[kDeclRing];
    uint32_t h_decl_cap[kDeclRing];
    hipEvent_t decl_ev[kDeclRing];
    bool decl_ev_live[kDeclRing];
    uint32_t decl_next;
};

namespace {

int hip_err(hipError_t e) { return e == hipSuccess ? ZRC4_OK : ZRC4_ERR_HIP; }

#define ZRC4_TRY(expr)                          \
    do {                                        \
        hipError_t e_ = (expr);                 \
        if (e_ != hipSuccess) return ZRC4_ERR_HIP; \
    } while (0)

int set_device(const zrc4_ctx *c)
{
    return hip_err(hipSetDevice(c->device));
}

int grow_stage(zrc4_ctx *c, size_t bytes)
{
    if (bytes <= c->d_stage_bytes && bytes <= c->h_stage_bytes) return ZRC4_OK;
    size_t want = 1u << 20;
    while (want < bytes) want <<= 1;
    if (c->d_stage) (void)hipFree(c->d_stage);
    if (c->h_stage) (void)hipHostFree(c->h_stage);
    c->d_stage = nullptr;
    c->h_stage = nullptr;
    c->d_stage_bytes = c->h_stage_bytes = 0;
    if (hipMalloc(&c->d_stage, want) != hipSuccess) return ZRC4_ERR_OUT_OF_MEMORY;
    // coherent: small batches run on it in place, and kernels are dispatched
    // with agent-scope acquire (a non-coherent line could be stale in L2)
    if (hipHostMalloc(&c->h_stage, want, hipHostMallocCoherent) != hipSuccess)
        return ZRC4_ERR_OUT_OF_MEMORY;
    c->d_stage_bytes = c->h_stage_bytes = want;
    return ZRC4_OK;
}

size_t align16(size_t v) { return (v + 15u) & ~(size_t)15u; }

constexpr size_t kZeroCopyMax = 256u << 10;   // *_host batches up to this size run on pinned staging in place

// Kernel choice per launch: more 256-slot groups than CUs -> the persistent
// throughput kernel (2 workgroups per CU, whole-line stores through the DPP
// transpose); otherwise one group per workgroup (crypt_kernel: chain-bound,
// per-lane stores).  A/B: the DPP path is 5-7 us slower at one group per CU
// (cfg2 56.1 vs 48.8 us, cfg3 28.1 vs 22.7 us; profiles/r02_ab_dpp_direct.log).
// With `fr`, the framing walk of every entry runs in the same launch: in the
// direct kernels' epilogue, or in the persistent kernel's tail.
//
// `decl` (kGrouped only): the caller's declared group per 256-entry bucket, in
// host memory (zrc4_crypt_grouped_declared).  Window launches take it in the
// kernel arguments (the image leaves at kernel entry); larger launches check
// it first in decl_check_kernel, which blocks the groups of a disagreeing
// bucket through the claims.  `decl_trusted`: the groups were computed here
// from host ids (zrc4_crypt_host), so larger launches skip the check.
int launch_crypt(zrc4_ctx *c, int mode, const uint32_t *ids, uint32_t first_slot, uint8_t *payload,
                 const uint64_t *off, const uint32_t *len, uint32_t n, hipStream_t s,
                 const zrc4::FrameArgs *fr = nullptr, const uint32_t *decl = nullptr, bool decl_trusted = false)
{
    if (n == 0) return ZRC4_OK;
    if (mode == zrc4::kRange && (uint64_t)first_slot + n > c->capacity) return ZRC4_ERR_SLOT_RANGE;
    zrc4::Claim cl{nullptr, 0u, nullptr};
    if (mode == zrc4::kGrouped) {
        // a fresh tag per grouped launch; on the 32-bit wrap the words are
        // zeroed first (stream-ordered before this launch)
        if (++c->epoch == 0u) {
            ZRC4_TRY(hipMemsetAsync(c->claim, 0, (size_t)(c->capacity / zrc4::kGroup) * zrc4::kClaimParts * 8u, s));
            c->epoch = 1u;
        }
        cl = zrc4::Claim{c->claim, c->epoch,
                         reinterpret_cast<const uint32_t *>(c->claim + (size_t)(c->capacity / zrc4::kGroup) * zrc4::kClaimParts)};
    }
    const uint32_t grid = (n + zrc4::kGroup - 1) / zrc4::kGroup;
    const dim3 blk(zrc4::kGroup);
    const bool stream_kernel = grid > (uint32_t)c->num_cus;
    // (the grouped stream kernel computes entry indexes of the bucket after
    // next in 32 bits)
    if (mode == zrc4::kGrouped && stream_kernel && n > 0xFFF00000u) return ZRC4_ERR_INVALID_ARG;
    // Few aligned groups: 16 lanes per stream (speculative windows), one wave
    // per 4 streams, 64 workgroups per group.
    if (grid <= (uint32_t)ZRC4_WIN_MAX_GROUPS &&
        ((mode == zrc4::kRange && (first_slot & 255u) == 0u) || mode == zrc4::kGrouped)) {
        const dim3 wgrid(64u * grid), wblk(64);
        const zrc4::FrameArgs fa = fr ? *fr : zrc4::FrameArgs{};
        zrc4::WinGroups dg{};
        if (decl && mode == zrc4::kGrouped)
            for (uint32_t b = 0; b < grid; ++b) dg.g[b] = decl[b];
#define ZRC4_WIN(MODE_, FRAME_, DECL_)                                                                          \
    hipLaunchKernelGGL((zrc4::crypt_win_kernel<MODE_, FRAME_, DECL_>), wgrid, wblk, 0, s, c->arena, c->xy, ids, \
                       first_slot, payload, off, len, n, c->capacity, c->err, c->sink, fa, cl, dg)
        if (mode == zrc4::kRange && fr)
            ZRC4_WIN(zrc4::kRange, true, false);
        else if (mode == zrc4::kRange)
            ZRC4_WIN(zrc4::kRange, false, false);
        else if (decl && fr)
            ZRC4_WIN(zrc4::kGrouped, true, true);
        else if (decl)
            ZRC4_WIN(zrc4::kGrouped, false, true);
        else if (fr)
            ZRC4_WIN(zrc4::kGrouped, true, false);
        else
            ZRC4_WIN(zrc4::kGrouped, false, false);
#undef ZRC4_WIN
        return hipGetLastError() == hipSuccess ? ZRC4_OK : ZRC4_ERR_LAUNCH;
    }
    // Declared groups on the half-group / whole-group kernels (at most 256
    // buckets, one bucket per CU): in the kernel arguments, checked there.
    if (decl && mode == zrc4::kGrouped && !stream_kernel && grid <= zrc4::kBodyMaxBuckets) {
        zrc4::BucketGroups dg{};
        for (uint32_t b = 0; b < grid; ++b) dg.g[b] = decl[b];
        const zrc4::FrameArgs fa = fr ? *fr : zrc4::FrameArgs{};
        const bool half = ZRC4_HALF && 2u * grid <= (uint32_t)c->num_cus;
#define ZRC4_DECL(FRAME_, HALF_, GRID_, BLK_)                                                                  \
    hipLaunchKernelGGL((zrc4::crypt_decl_kernel<FRAME_, HALF_>), GRID_, BLK_, 0, s, c->arena, c->xy, ids, payload, \
                       off, len, n, c->capacity, c->err, c->sink, fa, cl, dg)
        if (half && fr)
            ZRC4_DECL(true, true, dim3(2u * grid), dim3(zrc4::kHalfBlock));
        else if (half)
            ZRC4_DECL(false, true, dim3(2u * grid), dim3(zrc4::kHalfBlock));
        else if (fr)
            ZRC4_DECL(true, false, dim3(grid), blk);
        else
            ZRC4_DECL(false, false, dim3(grid), blk);
#undef ZRC4_DECL
        return hipGetLastError() == hipSuccess ? ZRC4_OK : ZRC4_ERR_LAUNCH;
    }
    if (decl && mode == zrc4::kGrouped && !decl_trusted) {
        // check the declared groups before the crypt launch (stream-ordered):
        // a disagreeing bucket's groups are claimed under this launch's epoch
        const int k = (int)(c->decl_next++ % (uint32_t)zrc4_ctx::kDeclRing);
        if (c->decl_ev_live[k]) ZRC4_TRY(hipEventSynchronize(c->decl_ev[k]));    // its last reader has run
        if (!c->decl_ev[k] && hipEventCreateWithFlags(&c->decl_ev[k], hipEventDisableTiming) != hipSuccess)
            return ZRC4_ERR_HIP;
        if (grid > c->h_decl_cap[k]) {
            if (c->h_decl[k]) (void)hipHostFree(c->h_decl[k]);
            c->h_decl[k] = nullptr;
            c->h_decl_cap[k] = 0;
            uint32_t want = 1024u;
            while (want < grid) want <<= 1;
            void *p = nullptr;
            if (hipHostMalloc(&p, (size_t)want * 4u, hipHostMallocCoherent) != hipSuccess) return ZRC4_ERR_OUT_OF_MEMORY;
            c->h_decl[k] = static_cast<uint32_t *>(p);
            c->h_decl_cap[k] = want;
        }
        memcpy(c->h_decl[k], decl, (size_t)grid * 4u);
        hipLaunchKernelGGL(zrc4::decl_check_kernel, dim3(grid), blk, 0, s, ids, len, n, c->h_decl[k], c->capacity,
                           cl, c->err);
        if (hipGetLastError() != hipSuccess) return ZRC4_ERR_LAUNCH;
        ZRC4_TRY(hipEventRecord(c->decl_ev[k], s));
        c->decl_ev_live[k] = true;
    }
    // Few whole groups: half-group workgroups, one per CU (2 waves per CU).
    // A grouped bucket's slots may sit in either half whatever its entry
    // count, so it always gets both halves.
    const bool half = ZRC4_HALF && 2u * grid <= (uint32_t)c->num_cus &&
                      ((mode == zrc4::kRange && (first_slot & 255u) == 0u) || mode == zrc4::kGrouped);
    if (half) {
        const dim3 hblk(zrc4::kHalfBlock);
        const dim3 hgrid(mode == zrc4::kGrouped ? 2u * grid : (n + zrc4::kGroup / 2 - 1) / (zrc4::kGroup / 2));
        const zrc4::FrameArgs fa = fr ? *fr : zrc4::FrameArgs{};
        if (mode == zrc4::kRange) {
            if (fr)
                hipLaunchKernelGGL((zrc4::crypt_half_kernel<zrc4::kRange, true>), hgrid, hblk, 0, s, c->arena, c->xy,
                                   ids, first_slot, payload, off, len, n, c->capacity, c->err, c->sink, fa);
            else
                hipLaunchKernelGGL((zrc4::crypt_half_kernel<zrc4::kRange, false>), hgrid, hblk, 0, s, c->arena, c->xy,
                                   ids, first_slot, payload, off, len, n, c->capacity, c->err, c->sink, fa);
        } else {
            if (fr)
                hipLaunchKernelGGL((zrc4::crypt_half_kernel<zrc4::kGrouped, true>), hgrid, hblk, 0, s, c->arena,
                                   c->xy, ids, first_slot, payload, off, len, n, c->capacity, c->err, c->sink, fa, cl);
            else
                hipLaunchKernelGGL((zrc4::crypt_half_kernel<zrc4::kGrouped, false>), hgrid, hblk, 0, s, c->arena,
                                   c->xy, ids, first_slot, payload, off, len, n, c->capacity, c->err, c->sink, fa, cl);
        }
        return hipGetLastError() == hipSuccess ? ZRC4_OK : ZRC4_ERR_LAUNCH;
    }
    if (fr && !stream_kernel) {
        if (mode == zrc4::kRange)
            hipLaunchKernelGGL((zrc4::crypt_kernel<zrc4::kRange, true>), dim3(grid), blk, 0, s, c->arena, c->xy,
                               ids, first_slot, payload, off, len, n, c->capacity, c->err, c->sink, *fr);
        else if (mode == zrc4::kGrouped)
            hipLaunchKernelGGL((zrc4::crypt_kernel<zrc4::kGrouped, true>), dim3(grid), blk, 0, s, c->arena, c->xy,
                               ids, first_slot, payload, off, len, n, c->capacity, c->err, c->sink, *fr, cl);
        else
            return ZRC4_ERR_INVALID_ARG;
        return hipGetLastError() == hipSuccess ? ZRC4_OK : ZRC4_ERR_LAUNCH;
    }
    if (stream_kernel) {
        // with `fr`, the framing walk runs in the same launch, in each
        // workgroup's tail over the chunks it decrypted (frame_walk_chunks)
        const uint32_t wgs = std::min(grid, 2u * (uint32_t)c->num_cus);
        const zrc4::FrameArgs fa = fr ? *fr : zrc4::FrameArgs{};
#define ZRC4_STREAM(PF_, GR_)                                                                                   \
    do {                                                                                                       \
        if (fr)                                                                                                \
            hipLaunchKernelGGL((zrc4::crypt_stream_kernel<PF_, GR_, true>), dim3(wgs), blk, 0, s, c->arena,    \
                               c->xy, ids, first_slot, payload, off, len, n, c->capacity, c->err, c->sink, cl, \
                               fa);                                                                            \
        else                                                                                                   \
            hipLaunchKernelGGL((zrc4::crypt_stream_kernel<PF_, GR_, false>), dim3(wgs), blk, 0, s, c->arena,   \
                               c->xy, ids, first_slot, payload, off, len, n, c->capacity, c->err, c->sink, cl, \
                               fa);                                                                            \
    } while (0)
        if (mode == zrc4::kGrouped)
            ZRC4_STREAM(true, true);
        else if (mode == zrc4::kRange && (first_slot & 255u) == 0u)
            ZRC4_STREAM(true, false);
        else
            ZRC4_STREAM(false, false);
#undef ZRC4_STREAM
    } else if (mode == zrc4::kRange) {
        hipLaunchKernelGGL(zrc4::crypt_kernel<zrc4::kRange>, dim3(grid), blk, 0, s, c->arena, c->xy, ids,
                           first_slot, payload, off, len, n, c->capacity, c->err, c->sink);
    } else if (mode == zrc4::kGrouped) {
        hipLaunchKernelGGL(zrc4::crypt_kernel<zrc4::kGrouped>, dim3(grid), blk, 0, s, c->arena, c->xy, ids,
                           first_slot, payload, off, len, n, c->capacity, c->err, c->sink, zrc4::FrameArgs{}, cl);
    } else {
        hipLaunchKernelGGL(zrc4::crypt_kernel<zrc4::kIds>, dim3(grid), blk, 0, s, c->arena, c->xy, ids,
                           first_slot, payload, off, len, n, c->capacity, c->err, c->sink);
    }
    return hipGetLastError() == hipSuccess ? ZRC4_OK : ZRC4_ERR_LAUNCH;
}

int launch_ksa(zrc4_ctx *c, const uint32_t *ids, uint32_t first_slot, const uint8_t *keys,
               const uint64_t *key_off, const uint32_t *key_len, uint32_t n, hipStream_t s)
{
    if (n == 0) return ZRC4_OK;
    if (!ids && (uint64_t)first_slot + n > c->capacity) return ZRC4_ERR_SLOT_RANGE;
    const uint32_t grid = (n + zrc4::kGroup - 1) / zrc4::kGroup;
    hipLaunchKernelGGL(zrc4::ksa_kernel, dim3(grid), dim3(zrc4::kGroup), 0, s, c->arena, c->xy,
                       ids, first_slot, keys, key_off, key_len, n, c->capacity, c->err);
    return hipGetLastError() == hipSuccess ? ZRC4_OK : ZRC4_ERR_LAUNCH;
}

// The per-iteration completion point of the session engine's hooks: ONE
// stream wait, then the latch word is read straight from pinned memory (a
// device-to-host copy of it used to cost another ~11 us per call).
int read_faults(zrc4_ctx *c)
{
    volatile uint32_t *e = c->err;
    int rc = ZRC4_OK;
    if (e[zrc4::kErrLdsLayout]) rc = ZRC4_ERR_INTERNAL;
    else if (e[zrc4::kErrGroup]) rc = ZRC4_ERR_GROUP;
    else if (e[zrc4::kErrSlotRange]) rc = ZRC4_ERR_SLOT_RANGE;
    for (uint32_t i = 0; i < zrc4::kErrWords; ++i) e[i] = 0u;
    return rc;
}

int check_err(zrc4_ctx *c, hipStream_t s)
{
    ZRC4_TRY(hipStreamSynchronize(s));
    return read_faults(c);
}

}  // namespace

extern "C" {

int zrc4_create(zrc4_ctx **out, int device, uint32_t capacity)
{
    if (!out || capacity == 0) return ZRC4_ERR_INVALID_ARG;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return ZRC4_ERR_NO_DEVICE;
    if (device < 0 || device >= ndev) return ZRC4_ERR_NO_DEVICE;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return ZRC4_ERR_NO_DEVICE;
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return ZRC4_ERR_NO_DEVICE;
    if (hipSetDevice(device) != hipSuccess) return ZRC4_ERR_NO_DEVICE;

    zrc4_ctx *c = new (std::nothrow) zrc4_ctx();
    if (!c) return ZRC4_ERR_OUT_OF_MEMORY;
    c->device = device;
    c->num_cus = prop.multiProcessorCount;
    const uint64_t cap = ((uint64_t)capacity + 255u) & ~(uint64_t)255u;
    if (cap > 0xFFFFFF00ull) { delete c; return ZRC4_ERR_INVALID_ARG; }
    c->capacity = (uint32_t)cap;
    const size_t groups = c->capacity / zrc4::kGroup;
    bool ok = hipMalloc(&c->arena, groups * (size_t)zrc4::kGroupBytes) == hipSuccess &&
              hipMalloc(&c->xy, (size_t)c->capacity * sizeof(uint16_t)) == hipSuccess &&
              hipMalloc(&c->sink, zrc4::kSinkBytes) == hipSuccess &&
              hipHostMalloc(&c->err, zrc4::kErrWords * sizeof(uint32_t), hipHostMallocCoherent) == hipSuccess &&
              // + 16 zero bytes after the claim words (Claim::zero; the epoch-wrap memset stops before them)
              hipMalloc(&c->claim, (groups * zrc4::kClaimParts + 2) * sizeof(unsigned long long)) == hipSuccess &&
              hipMemset(c->claim, 0, (groups * zrc4::kClaimParts + 2) * sizeof(unsigned long long)) == hipSuccess &&
              hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) == hipSuccess;
    if (!ok) { zrc4_destroy(c); return ZRC4_ERR_OUT_OF_MEMORY; }
    // Fresh slots hold the reference's empty-key state: identity box, x = y = 0
    // (what makeSBox("") produces, rc4_encryption.h:48-53).
    for (uint32_t i = 0; i < zrc4::kErrWords; ++i) c->err[i] = 0u;
    hipLaunchKernelGGL(zrc4::identity_kernel, dim3((unsigned)groups), dim3(zrc4::kGroup), 0,
                       c->stream, c->arena);
    if (hipGetLastError() != hipSuccess ||
        hipMemsetAsync(c->xy, 0, (size_t)c->capacity * sizeof(uint16_t), c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess) {
        zrc4_destroy(c);
        return ZRC4_ERR_HIP;
    }
    *out = c;
    return ZRC4_OK;
}

int zrc4_destroy(zrc4_ctx *c)
{
    if (!c) return ZRC4_ERR_INVALID_ARG;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->arena) (void)hipFree(c->arena);
    if (c->xy) (void)hipFree(c->xy);
    if (c->sink) (void)hipFree(c->sink);
    if (c->claim) (void)hipFree(c->claim);
    for (int k = 0; k < zrc4_ctx::kDeclRing; ++k) {
        if (c->decl_ev_live[k]) (void)hipEventSynchronize(c->decl_ev[k]);   // a check kernel may still read h_decl
        if (c->decl_ev[k]) (void)hipEventDestroy(c->decl_ev[k]);
        if (c->h_decl[k]) (void)hipHostFree(c->h_decl[k]);
    }
    if (c->err) (void)hipHostFree(c->err);
    if (c->d_stage) (void)hipFree(c->d_stage);
    if (c->h_stage) (void)hipHostFree(c->h_stage);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return ZRC4_OK;
}

uint32_t zrc4_capacity(const zrc4_ctx *c) { return c ? c->capacity : 0u; }

int zrc4_ksa(zrc4_ctx *c, const uint32_t *ids, const uint8_t *keys, const uint64_t *key_off,
             const uint32_t *key_len, uint32_t n, void *stream)
{
    if (!c) return ZRC4_ERR_INVALID_ARG;
    if (n && (!key_len || !key_off)) return ZRC4_ERR_INVALID_ARG;
    int rc = set_device(c);
    if (rc) return rc;
    return launch_ksa(c, ids, 0, keys, key_off, key_len, n, (hipStream_t)stream);
}

int zrc4_crypt(zrc4_ctx *c, const uint32_t *ids, uint8_t *payload, const uint64_t *off,
               const uint32_t *len, uint32_t n, void *stream)
{
    if (!c) return ZRC4_ERR_INVALID_ARG;
    if (n && (!payload || !off || !len)) return ZRC4_ERR_INVALID_ARG;
    int rc = set_device(c);
    if (rc) return rc;
    return launch_crypt(c, ids ? zrc4::kIds : zrc4::kRange, ids, 0, payload, off, len, n, (hipStream_t)stream);
}

int zrc4_ksa_range(zrc4_ctx *c, uint32_t first_slot, const uint8_t *keys,
                   const uint64_t *key_off, const uint32_t *key_len, uint32_t n, void *stream)
{
    if (!c) return ZRC4_ERR_INVALID_ARG;
    if (n && (!key_len || !key_off)) return ZRC4_ERR_INVALID_ARG;
    int rc = set_device(c);
    if (rc) return rc;
    return launch_ksa(c, nullptr, first_slot, keys, key_off, key_len, n, (hipStream_t)stream);
}

int zrc4_crypt_range(zrc4_ctx *c, uint32_t first_slot, uint8_t *payload, const uint64_t *off,
                     const uint32_t *len, uint32_t n, void *stream)
{
    if (!c) return ZRC4_ERR_INVALID_ARG;
    if (n && (!payload || !off || !len)) return ZRC4_ERR_INVALID_ARG;
    int rc = set_device(c);
    if (rc) return rc;
    return launch_crypt(c, zrc4::kRange, nullptr, first_slot, payload, off, len, n, (hipStream_t)stream);
}

int zrc4_crypt_grouped(zrc4_ctx *c, const uint32_t *ids, uint8_t *payload, const uint64_t *off,
                       const uint32_t *len, uint32_t n, void *stream)
{
    if (!c) return ZRC4_ERR_INVALID_ARG;
    if (n && (!ids || !payload || !off || !len)) return ZRC4_ERR_INVALID_ARG;
    int rc = set_device(c);
    if (rc) return rc;
    return launch_crypt(c, zrc4::kGrouped, ids, 0, payload, off, len, n, (hipStream_t)stream);
}

namespace {
int frame_args(const zrc4_frame_args *f, uint32_t n, zrc4::FrameArgs &out)
{
    if (!f) return ZRC4_ERR_INVALID_ARG;
    if (n && (!f->off || !f->len || !f->npk || !f->used || !f->status || (f->max_packets && !f->pkt_len)))
        return ZRC4_ERR_INVALID_ARG;
    out.off = f->off;
    out.len = f->len;
    out.bound = f->bound;
    out.maxp = f->max_packets;
    out.npk = f->npk;
    out.used = f->used;
    out.status = f->status;
    out.pkt_len = f->max_packets ? f->pkt_len : nullptr;
    return ZRC4_OK;
}
}  // namespace

int zrc4_crypt_range_frame(zrc4_ctx *c, uint32_t first_slot, uint8_t *payload, const uint64_t *off,
                           const uint32_t *len, uint32_t n, const zrc4_frame_args *frame, void *stream)
{
    if (!c) return ZRC4_ERR_INVALID_ARG;
    if (n && (!payload || !off || !len)) return ZRC4_ERR_INVALID_ARG;
    zrc4::FrameArgs fr;
    int rc = frame_args(frame, n, fr);
    if (rc) return rc;
    if ((rc = set_device(c))) return rc;
    return launch_crypt(c, zrc4::kRange, nullptr, first_slot, payload, off, len, n, (hipStream_t)stream, &fr);
}

int zrc4_crypt_grouped_frame(zrc4_ctx *c, const uint32_t *ids, uint8_t *payload, const uint64_t *off,
                             const uint32_t *len, uint32_t n, const zrc4_frame_args *frame, void *stream)
{
    if (!c) return ZRC4_ERR_INVALID_ARG;
    if (n && (!ids || !payload || !off || !len)) return ZRC4_ERR_INVALID_ARG;
    zrc4::FrameArgs fr;
    int rc = frame_args(frame, n, fr);
    if (rc) return rc;
    if ((rc = set_device(c))) return rc;
    return launch_crypt(c, zrc4::kGrouped, ids, 0, payload, off, len, n, (hipStream_t)stream, &fr);
}

int zrc4_crypt_grouped_declared(zrc4_ctx *c, const uint32_t *ids, const uint32_t *bucket_group, uint8_t *payload,
                                const uint64_t *off, const uint32_t *len, uint32_t n,
                                const struct zrc4_frame_args *frame, void *stream)
{
    if (!c) return ZRC4_ERR_INVALID_ARG;
    if (n && (!ids || !bucket_group || !payload || !off || !len)) return ZRC4_ERR_INVALID_ARG;
    const uint32_t nb = (uint32_t)(((uint64_t)n + zrc4::kGroup - 1) / zrc4::kGroup);
    const uint32_t groups = c->capacity / zrc4::kGroup;
    for (uint32_t b = 0; b < nb; ++b)
        if (bucket_group[b] >= groups && bucket_group[b] != ZRC4_IDLE_SLOT) return ZRC4_ERR_INVALID_ARG;
    zrc4::FrameArgs fr;
    int rc = frame ? frame_args(frame, n, fr) : ZRC4_OK;
    if (rc) return rc;
    if ((rc = set_device(c))) return rc;
    return launch_crypt(c, zrc4::kGrouped, ids, 0, payload, off, len, n, (hipStream_t)stream, frame ? &fr : nullptr,
                        bucket_group);
}

int zrc4_xor_ring(zrc4_ctx *c, uint8_t *ring, uint32_t ring_cap, const uint32_t *rid,
                  const uint32_t *pos, uint8_t *payload, const uint64_t *off, const uint32_t *len,
                  uint32_t n, void *stream)
{
    if (!c) return ZRC4_ERR_INVALID_ARG;
    if (n == 0) return ZRC4_OK;
    if (!ring || ring_cap == 0 || !rid || !pos || !payload || !off || !len) return ZRC4_ERR_INVALID_ARG;
    int rc = set_device(c);
    if (rc) return rc;
    hipLaunchKernelGGL(zrc4::xor_ring_kernel, dim3(n), dim3(256), 0, (hipStream_t)stream, ring, ring_cap,
                       rid, pos, payload, off, len, n);
    return hipGetLastError() == hipSuccess ? ZRC4_OK : ZRC4_ERR_LAUNCH;
}

int zrc4_frame_scan(zrc4_ctx *c, const uint8_t *buf, const uint64_t *off, const uint32_t *len,
                    uint32_t bound, uint32_t n, uint32_t max_packets, uint32_t *npk, uint32_t *used,
                    uint32_t *status, uint32_t *pkt_len, void *stream)
{
    if (!c) return ZRC4_ERR_INVALID_ARG;
    if (n == 0) return ZRC4_OK;
    if (!buf || !off || !len || !npk || !used || !status || (max_packets && !pkt_len))
        return ZRC4_ERR_INVALID_ARG;
    int rc = set_device(c);
    if (rc) return rc;
    hipLaunchKernelGGL(zrc4::frame_scan_kernel, dim3((n + 255u) / 256u), dim3(256), 0, (hipStream_t)stream,
                       buf, off, len, bound, n, max_packets, npk, used, status, max_packets ? pkt_len : nullptr);
    return hipGetLastError() == hipSuccess ? ZRC4_OK : ZRC4_ERR_LAUNCH;
}

int zrc4_poll_faults(zrc4_ctx *c)
{
    if (!c) return ZRC4_ERR_INVALID_ARG;
    return read_faults(c);
}

int zrc4_sync(zrc4_ctx *c, void *stream)
{
    if (!c) return ZRC4_ERR_INVALID_ARG;
    int rc = set_device(c);
    if (rc) return rc;
    return check_err(c, (hipStream_t)stream);
}

int zrc4_ksa_host(zrc4_ctx *c, const uint32_t *ids, const uint8_t *keys, size_t keys_bytes,
                  const uint64_t *key_off, const uint32_t *key_len, uint32_t n)
{
    if (!c) return ZRC4_ERR_INVALID_ARG;
    if (n == 0) return ZRC4_OK;
    if (!key_off || !key_len || (keys_bytes && !keys)) return ZRC4_ERR_INVALID_ARG;
    for (uint32_t i = 0; i < n; ++i)
        if (key_len[i] && (key_off[i] > keys_bytes || key_len[i] > keys_bytes - key_off[i]))
            return ZRC4_ERR_INVALID_ARG;
    int rc = set_device(c);
    if (rc) return rc;
    const size_t o_ids = 0, s_ids = ids ? align16((size_t)n * 4) : 0;
    const size_t o_off = o_ids + s_ids, s_off = align16((size_t)n * 8);
    const size_t o_len = o_off + s_off, s_len = align16((size_t)n * 4);
    const size_t o_key = o_len + s_len, total = o_key + align16(keys_bytes ? keys_bytes : 1);
    if ((rc = grow_stage(c, total))) return rc;
    if (ids) memcpy(c->h_stage + o_ids, ids, (size_t)n * 4);
    memcpy(c->h_stage + o_off, key_off, (size_t)n * 8);
    memcpy(c->h_stage + o_len, key_len, (size_t)n * 4);
    if (keys_bytes) memcpy(c->h_stage + o_key, keys, keys_bytes);
    // Small batches run on the pinned staging copy in place (zero-copy over
    // PCIe: one launch and one wait instead of copy + launch + wait).
    uint8_t *st = c->h_stage;
    if (total > kZeroCopyMax) {
        ZRC4_TRY(hipMemcpyAsync(c->d_stage, c->h_stage, total, hipMemcpyHostToDevice, c->stream));
        st = c->d_stage;
    }
    rc = launch_ksa(c, ids ? (const uint32_t *)(st + o_ids) : nullptr, 0,
                    st + o_key, (const uint64_t *)(st + o_off), (const uint32_t *)(st + o_len), n, c->stream);
    if (rc) {
        (void)hipStreamSynchronize(c->stream);     // a queued H2D still reads the staging buffer
        return rc;
    }
    return check_err(c, c->stream);
}

// Payload staging copies of the *_host calls (caller memory <-> pinned
// staging): one host thread moves ~8 GB/s, so copies of 2 MiB and more are
// split over up to 8 threads (r06: 512 MiB took ~67 ms on one thread).  If
// a thread cannot be started, its share is copied on the calling thread.
static void par_memcpy(uint8_t *dst, const uint8_t *src, size_t n)
{
    constexpr size_t kPerThreadMin = 1u << 20;
    size_t nt = n / kPerThreadMin;
    const unsigned hw = std::thread::hardware_concurrency();
    if (nt > 8) nt = 8;
    if (hw && nt > hw) nt = hw;
    if (nt <= 1) {
        memcpy(dst, src, n);
        return;
    }
    const size_t per = ((n + nt - 1) / nt + 4095) & ~(size_t)4095;
    std::vector<std::thread> th;
    size_t started = 1;                     // chunk 0 is this thread's
    try {
        th.reserve(nt - 1);
        for (; started < nt && started * per < n; ++started) {
            const size_t a = started * per, len = std::min(per, n - a);
            th.emplace_back([=] { memcpy(dst + a, src + a, len); });
        }
    } catch (...) {
    }
    memcpy(dst, src, std::min(per, n));
    for (size_t t = started; t * per < n; ++t) memcpy(dst + t * per, src + t * per, std::min(per, n - t * per));
    for (auto &t : th) t.join();
}

// The chunked D2H of a piped zrc4_crypt_host: chunk k's copy is recorded
// with an event and copied out to the caller once it has landed, while the
// later chunks are still in flight.  The kernel ran before the first chunk's
// copy, so the fault latch is final once that chunk has landed: on a fault
// nothing is copied out (as on the unpiped path).  Without events (creation
// failed) it waits for the stream and copies everything at once.
static constexpr size_t kPipeChunk = 16u << 20;

static int copy_back_piped(zrc4_ctx *c, uint8_t *payload, size_t o_pay, size_t payload_bytes)
{
    std::vector<hipEvent_t> ev;
    ev.reserve(payload_bytes / kPipeChunk + 1);
    bool evs = true, copies = true;
    for (size_t a = 0; a < payload_bytes; a += kPipeChunk) {
        const size_t l = std::min(kPipeChunk, payload_bytes - a);
        hipError_t e = hipMemcpyAsync(c->h_stage + o_pay + a, c->d_stage + o_pay + a, l, hipMemcpyDeviceToHost,
                                      c->stream);
        if (e != hipSuccess) copies = evs = false;
        hipEvent_t x = nullptr;
        if (evs && hipEventCreateWithFlags(&x, hipEventDisableTiming) == hipSuccess) {
            if (hipEventRecord(x, c->stream) == hipSuccess) {
                ev.push_back(x);
                continue;
            }
            (void)hipEventDestroy(x);
        }
        evs = false;
    }
    int rc = ZRC4_OK;
    if (!copies) {                         // a chunk never left the device: copy nothing out
        rc = check_err(c, c->stream);
        if (rc == ZRC4_OK) rc = ZRC4_ERR_HIP;
    } else if (!evs || ev.empty() || hipEventSynchronize(ev[0]) != hipSuccess) {
        rc = check_err(c, c->stream);
        if (rc == ZRC4_OK) par_memcpy(payload, c->h_stage + o_pay, payload_bytes);
    } else if ((rc = read_faults(c)) == ZRC4_OK) {
        for (size_t k = 0, a = 0; a < payload_bytes; ++k, a += kPipeChunk) {
            if (hipEventSynchronize(ev[k]) != hipSuccess) {
                rc = ZRC4_ERR_HIP;
                break;
            }
            par_memcpy(payload + a, c->h_stage + o_pay + a, std::min(kPipeChunk, payload_bytes - a));
        }
    }
    (void)hipStreamSynchronize(c->stream);
    for (hipEvent_t x : ev) (void)hipEventDestroy(x);
    return rc;
}

int zrc4_crypt_host(zrc4_ctx *c, const uint32_t *ids, uint8_t *payload, size_t payload_bytes,
                    const uint64_t *off, const uint32_t *len, uint32_t n)
{
    if (!c) return ZRC4_ERR_INVALID_ARG;
    if (n == 0) return ZRC4_OK;
    if (!off || !len || (payload_bytes && !payload)) return ZRC4_ERR_INVALID_ARG;
    for (uint32_t i = 0; i < n; ++i) {
        if (len[i] && (off[i] > payload_bytes || len[i] > payload_bytes - off[i]))
            return ZRC4_ERR_INVALID_ARG;
        // (ZRC4_IDLE_SLOT included: the kernels would skip it as padding)
        if (ids && ids[i] >= c->capacity) return ZRC4_ERR_SLOT_RANGE;
    }
    int rc = set_device(c);
    if (rc) return rc;
    // Several arbitrary ids: bucket them by 256-slot group here (the
    // zrc4_crypt_grouped contract), so every group's S-boxes move as one
    // coalesced image instead of 256 strided byte accesses per slot.  A slot
    // may appear once per call (as for every batched entry point).
    // Bucketing is one counting pass over the groups (r06; a comparison sort
    // of the ids cost 91 ms at 524 288 entries, more than the copies): bucket
    // b = the b-th group with entries, in ascending group order, its entries in
    // call order; a 256-bit mask per group finds a repeated slot.
    const bool grouped = ids && n > 1;
    std::vector<uint32_t> bgroup, bstart;     // bgroup: each bucket's group, declared to the kernel
    uint32_t buckets = 0;
    if (grouped) {
        const uint32_t ngroups = c->capacity / zrc4::kGroup;
        std::vector<uint64_t> seen((size_t)ngroups * 4, 0);
        bstart.assign(ngroups, ZRC4_IDLE_SLOT);
        for (uint32_t i = 0; i < n; ++i) {
            const uint32_t g = ids[i] >> 8, k = ids[i] & 255u;
            uint64_t &w = seen[(size_t)g * 4 + (k >> 6)];
            if (w >> (k & 63u) & 1u) return ZRC4_ERR_INVALID_ARG;
            w |= 1ull << (k & 63u);
            bstart[g] = 0;
        }
        for (uint32_t g = 0; g < ngroups; ++g)
            if (bstart[g] != ZRC4_IDLE_SLOT) {
                bstart[g] = buckets++ * zrc4::kGroup;
                bgroup.push_back(g);
            }
    }
    const uint32_t m = grouped ? buckets * zrc4::kGroup : n;      // entries the kernel sees
    const size_t o_ids = 0, s_ids = ids ? align16((size_t)m * 4) : 0;
    const size_t o_off = o_ids + s_ids, s_off = align16((size_t)m * 8);
    const size_t o_len = o_off + s_off, s_len = align16((size_t)m * 4);
    const size_t o_pay = o_len + s_len, total = o_pay + align16(payload_bytes ? payload_bytes : 1);
    if ((rc = grow_stage(c, total))) return rc;
    if (grouped) {
        uint32_t *bi = reinterpret_cast<uint32_t *>(c->h_stage + o_ids);
        uint64_t *bo = reinterpret_cast<uint64_t *>(c->h_stage + o_off);
        uint32_t *bl = reinterpret_cast<uint32_t *>(c->h_stage + o_len);
        for (uint32_t e = 0; e < m; ++e) {
            bi[e] = ZRC4_IDLE_SLOT;
            bo[e] = 0;
            bl[e] = 0;
        }
        for (uint32_t i = 0; i < n; ++i) {
            const uint32_t e = bstart[ids[i] >> 8]++;     // (at most 256 per group: no slot twice)
            bi[e] = ids[i];
            bo[e] = off[i];
            bl[e] = len[i];
        }
    } else {
        if (ids) memcpy(c->h_stage + o_ids, ids, (size_t)n * 4);
        memcpy(c->h_stage + o_off, off, (size_t)n * 8);
        memcpy(c->h_stage + o_len, len, (size_t)n * 4);
    }
    // Small batches (the per-call RC4Encryption::encryption drop-in) run on
    // the pinned staging copy in place: no H2D / D2H copies on the latency
    // path.  Large ones are copied so the kernel streams HBM, not PCIe; from
    // 2 chunks of kPipeChunk on, the payload moves chunk by chunk so each
    // chunk's host copy overlaps the previous chunk's DMA (and, on the way
    // back, the next chunk's DMA overlaps this chunk's host copy).
    const bool zero_copy = total <= kZeroCopyMax;
    const bool piped = !zero_copy && payload_bytes >= 2 * kPipeChunk;
    uint8_t *st = c->h_stage;
    if (piped) {
        // (a failed enqueue returns only once the chunks already queued have
        // left the staging buffer, which the next call rewrites)
        bool ok = hipMemcpyAsync(c->d_stage, c->h_stage, o_pay, hipMemcpyHostToDevice, c->stream) == hipSuccess;
        for (size_t a = 0; ok && a < payload_bytes; a += kPipeChunk) {
            const size_t l = std::min(kPipeChunk, payload_bytes - a);
            par_memcpy(c->h_stage + o_pay + a, payload + a, l);
            ok = hipMemcpyAsync(c->d_stage + o_pay + a, c->h_stage + o_pay + a, l, hipMemcpyHostToDevice,
                                c->stream) == hipSuccess;
        }
        if (!ok) {
            (void)hipStreamSynchronize(c->stream);
            return ZRC4_ERR_HIP;
        }
        st = c->d_stage;
    } else {
        if (payload_bytes) par_memcpy(c->h_stage + o_pay, payload, payload_bytes);
        if (!zero_copy) {
            ZRC4_TRY(hipMemcpyAsync(c->d_stage, c->h_stage, total, hipMemcpyHostToDevice, c->stream));
            st = c->d_stage;
        }
    }
    rc = launch_crypt(c, grouped ? zrc4::kGrouped : ids ? zrc4::kIds : zrc4::kRange,
                      ids ? (const uint32_t *)(st + o_ids) : nullptr, 0, st + o_pay, (const uint64_t *)(st + o_off),
                      (const uint32_t *)(st + o_len), m, c->stream, nullptr, grouped ? bgroup.data() : nullptr,
                      true);
    if (rc) {
        // whatever was queued before the failure (the H2D copies, a check
        // kernel reading the zero-copy tables) still reads the staging
        // buffer, which the next call rewrites: drain it first
        (void)hipStreamSynchronize(c->stream);
        return rc;
    }
    if (piped) return copy_back_piped(c, payload, o_pay, payload_bytes);
    if (payload_bytes && !zero_copy &&
        hipMemcpyAsync(c->h_stage + o_pay, c->d_stage + o_pay, payload_bytes, hipMemcpyDeviceToHost,
                       c->stream) != hipSuccess) {
        (void)hipStreamSynchronize(c->stream);
        return ZRC4_ERR_HIP;
    }
    rc = check_err(c, c->stream);
    if (rc) return rc;
    if (payload_bytes) par_memcpy(payload, c->h_stage + o_pay, payload_bytes);
    return ZRC4_OK;
}

int zrc4_make_sbox(zrc4_ctx *c, uint32_t id, const uint8_t *key, size_t keylen)
{
    if (!c || (keylen && !key)) return ZRC4_ERR_INVALID_ARG;
    if (id >= c->capacity) return ZRC4_ERR_SLOT_RANGE;
    // Only the first 256 key bytes can reach the S-box (the KSA runs i = 0..255
    // and reads key[i % len], rc4_encryption.h:60-70).
    const size_t kl = keylen > 256 ? 256 : keylen;
    const uint64_t ko = 0;
    const uint32_t kl32 = (uint32_t)kl;
    return zrc4_ksa_host(c, &id, key, kl, &ko, &kl32, 1);
}

int zrc4_encryption(zrc4_ctx *c, uint32_t id, uint8_t *data, int length)
{
    if (!c) return ZRC4_ERR_INVALID_ARG;
    if (id >= c->capacity) return ZRC4_ERR_SLOT_RANGE;
    if (length <= 0) return ZRC4_OK;  // for (i = 0; i < length; ...) never runs (:81)
    if (!data) return ZRC4_ERR_INVALID_ARG;
    const uint64_t o = 0;
    const uint32_t l = (uint32_t)length;
    return zrc4_crypt_host(c, &id, data, (size_t)length, &o, &l, 1);
}

int zrc4_get_state(zrc4_ctx *c, uint32_t id, uint8_t sbox[256], uint8_t *x, uint8_t *y)
{
    if (!c || !sbox || !x || !y) return ZRC4_ERR_INVALID_ARG;
    if (id >= c->capacity) return ZRC4_ERR_SLOT_RANGE;
    int rc = set_device(c);
    if (rc) return rc;
    const uint8_t *img = c->arena + (size_t)(id >> 8) * zrc4::kGroupBytes;
    const uint32_t j = id & 255u, w = j >> 6, l = j & 63u;
    const uint32_t col = ((l & 31u) << 2) | (l >> 5) | ((w & 1u) << 1) | ((w >> 1) << 7);
    ZRC4_TRY(hipMemcpy2DAsync(sbox, 1, img + col, 256, 1, 256, hipMemcpyDeviceToHost, c->stream));
    uint16_t v = 0;
    ZRC4_TRY(hipMemcpyAsync(&v, c->xy + id, 2, hipMemcpyDeviceToHost, c->stream));
    ZRC4_TRY(hipStreamSynchronize(c->stream));
    *x = (uint8_t)(v & 255u);
    *y = (uint8_t)(v >> 8);
    return ZRC4_OK;
}

int zrc4_set_state(zrc4_ctx *c, uint32_t id, const uint8_t sbox[256], uint8_t x, uint8_t y)
{
    if (!c || !sbox) return ZRC4_ERR_INVALID_ARG;
    if (id >= c->capacity) return ZRC4_ERR_SLOT_RANGE;
    int rc = set_device(c);
    if (rc) return rc;
    uint8_t *img = c->arena + (size_t)(id >> 8) * zrc4::kGroupBytes;
    const uint32_t j = id & 255u, w = j >> 6, l = j & 63u;
    const uint32_t col = ((l & 31u) << 2) | (l >> 5) | ((w & 1u) << 1) | ((w >> 1) << 7);
    uint8_t tmp[258];
    memcpy(tmp, sbox, 256);
    const uint16_t v = (uint16_t)(x | (y << 8));
    ZRC4_TRY(hipMemcpy2DAsync(img + col, 256, tmp, 1, 1, 256, hipMemcpyHostToDevice, c->stream));
    ZRC4_TRY(hipMemcpyAsync(c->xy + id, &v, 2, hipMemcpyHostToDevice, c->stream));
    ZRC4_TRY(hipStreamSynchronize(c->stream));
    return ZRC4_OK;
}

int zrc4_get_states(zrc4_ctx *c, uint32_t first_slot, uint32_t n, uint8_t *sbox, uint8_t *x, uint8_t *y)
{
    if (!c) return ZRC4_ERR_INVALID_ARG;
    if (n == 0) return ZRC4_OK;
    if (!sbox || !x || !y) return ZRC4_ERR_INVALID_ARG;
    if ((uint64_t)first_slot + n > c->capacity) return ZRC4_ERR_SLOT_RANGE;
    int rc = set_device(c);
    if (rc) return rc;
    const uint32_t g0 = first_slot / zrc4::kGroup, g1 = (first_slot + n - 1) / zrc4::kGroup;
    std::vector<uint8_t> img;
    std::vector<uint16_t> v(n);
    try {
        img.resize((size_t)(g1 - g0 + 1) * zrc4::kGroupBytes);
    } catch (const std::bad_alloc &) {
        return ZRC4_ERR_OUT_OF_MEMORY;
    }
    ZRC4_TRY(hipMemcpyAsync(img.data(), c->arena + (size_t)g0 * zrc4::kGroupBytes, img.size(), hipMemcpyDeviceToHost,
                            c->stream));
    ZRC4_TRY(hipMemcpyAsync(v.data(), c->xy + first_slot, (size_t)n * 2u, hipMemcpyDeviceToHost, c->stream));
    ZRC4_TRY(hipStreamSynchronize(c->stream));
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t id = first_slot + i, j = id & 255u;
        const uint8_t *g = img.data() + (size_t)(id / zrc4::kGroup - g0) * zrc4::kGroupBytes + zrc4::col_of(j);
        uint8_t *o = sbox + (size_t)i * 256u;
        for (uint32_t k = 0; k < 256u; ++k) o[k] = g[k << 8];
        x[i] = (uint8_t)(v[i] & 255u);
        y[i] = (uint8_t)(v[i] >> 8);
    }
    return ZRC4_OK;
}

const char *zrc4_strerror(int code)
{
    switch (code) {
    case ZRC4_OK: return "ok";
    case ZRC4_ERR_INVALID_ARG: return "invalid argument";
    case ZRC4_ERR_NO_DEVICE: return "no usable gfx950 (MI355X) HIP device";
    case ZRC4_ERR_OUT_OF_MEMORY: return "device or pinned memory allocation failed";
    case ZRC4_ERR_LAUNCH: return "kernel launch failed";
    case ZRC4_ERR_SLOT_RANGE: return "slot id out of range (>= capacity)";
    case ZRC4_ERR_HIP: return "HIP runtime error";
    case ZRC4_ERR_GROUP: return "zrc4_crypt_grouped: a 256-entry bucket mixes slot groups";
    case ZRC4_ERR_INTERNAL: return "internal error: S-box image not at LDS offset 0";
    case ZRC4_ERR_STATE: return "slot state lost (a failed reservoir crypt): reseed it with zrc4_ks_make_sbox or zrc4_ks_copy";
    default: return "unknown zrc4 error";
    }
}

const char *zrc4_version(void) { return "zrc4-mi355x 0.2 (gfx950)"; }

#if ZRC4_TIMING
// Diagnostic builds only: the per-wave timestamp records (zrc4_kernels.hpp,
// Stamps) live in the context's sink buffer.
int zrc4_debug_sink(zrc4_ctx *c, void **out)
{
    if (!c || !out) return ZRC4_ERR_INVALID_ARG;
    *out = c->sink;
    return ZRC4_OK;
}
#endif

}  // extern "C"

#include "zrc4_ks.inc"   // keystream reservoirs (zrc4_ks_*)
