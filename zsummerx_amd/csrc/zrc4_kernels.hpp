// zrc4_kernels.hpp -- gfx950 (CDNA4) kernels for the zsummerX RC4 path.
//
// Reference algorithm: /root/reference/depends/rc4/rc4_encryption.h
//   makeSBox   :46-72  -> ksa_kernel
//   encryption :74-93  -> crypt_kernel
//
// Work decomposition
//   One lane = one RC4 stream (slot).  RC4 is serial inside a stream (each
//   byte's swap feeds the next read, rc4_encryption.h:83-88), so the only
//   parallelism is across streams.  A 256-thread workgroup (4 waves) owns one
//   256-slot GROUP and keeps the group's 256 S-boxes in LDS (64 KiB), so a CU
//   holds 2 groups = 512 live streams; no MFMA (byte work).
//
// LDS image of a group (also the HBM arena image, so state load/store is a
// straight coalesced 64 KiB copy):
//   byte address of entry k of group-lane j = (k << 8) | col(j)
//   col(j) = (lane&31)<<2 | lane>>5 | (wave&1)<<1 | (wave>>1)<<7
//   -> dword bank = lane&31: the 32 lanes of a ds_read/ds_write lane group hit
//      32 distinct banks for ANY indices k (conflict-free), and every address
//      is a 16-bit value whose top byte is the S-box index, so x/y/t updates
//      are single 16-bit adds (wrap mod 256 for free).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace zrc4 {

constexpr int kGroup = 256;            // slots per workgroup / arena group
constexpr int kGroupBytes = 256 * 256; // 64 KiB S-box image per group

enum : uint32_t { kErrSlotRange = 1u };

__device__ __forceinline__ uint32_t col_of(uint32_t j)
{
    const uint32_t w = j >> 6, l = j & 63u;
    return ((l & 31u) << 2) | (l >> 5) | ((w & 1u) << 1) | ((w >> 1) << 7);
}

// ---------------------------------------------------------------------------
// Group state load / store.
//   fast: the workgroup's 256 entries are exactly slots g*256 .. g*256+255
//         (or ids == NULL): copy the 64 KiB image as 16 B per lane, coalesced.
//   slow: arbitrary slot ids: each lane gathers its own 256 bytes (strided).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void image_to_lds(uint8_t *lds, const uint8_t *img)
{
    const uint4 *src = reinterpret_cast<const uint4 *>(img);
    uint4 *dst = reinterpret_cast<uint4 *>(lds);
#pragma unroll
    for (int i = 0; i < 16; ++i) dst[i * 256 + threadIdx.x] = src[i * 256 + threadIdx.x];
}

__device__ __forceinline__ void lds_to_image(uint8_t *img, const uint8_t *lds)
{
    const uint4 *src = reinterpret_cast<const uint4 *>(lds);
    uint4 *dst = reinterpret_cast<uint4 *>(img);
#pragma unroll
    for (int i = 0; i < 16; ++i) dst[i * 256 + threadIdx.x] = src[i * 256 + threadIdx.x];
}

__device__ __forceinline__ void gather_column(uint8_t *lds, uint32_t col,
                                              const uint8_t *arena, uint32_t slot)
{
    const uint8_t *img = arena + (size_t)(slot >> 8) * kGroupBytes + col_of(slot & 255u);
    for (int k = 0; k < 256; ++k) lds[(k << 8) | col] = img[k << 8];
}

__device__ __forceinline__ void scatter_column(uint8_t *arena, uint32_t slot,
                                               const uint8_t *lds, uint32_t col)
{
    uint8_t *img = arena + (size_t)(slot >> 8) * kGroupBytes + col_of(slot & 255u);
    for (int k = 0; k < 256; ++k) img[k << 8] = lds[(k << 8) | col];
}

// ---------------------------------------------------------------------------
// One PRGA step (rc4_encryption.h:83-88) on 16-bit LDS addresses.
// Loop state between steps:
//   xa = address of S[x]        (x = the last index used)
//   ya = address of S[y]
//   an = S[x+1] as it will be seen by the next step (prefetched one step
//        early, forwarded from this step's S[y] = a write when y == x+1)
// The next-x read is issued before this step's two writes, so the only
// LDS round trip on the byte-to-byte chain is the S[y] read.
// ---------------------------------------------------------------------------
struct Rc4Lane {
    uint32_t xa, ya, an, col;
};

__device__ __forceinline__ uint32_t prga_step(uint8_t *S, Rc4Lane &st)
{
    const uint32_t xa = (st.xa + 256u) & 0xFFFFu;     // x = (u8)(x+1)
    const uint32_t a = st.an;                          // a = S[x]
    const uint32_t ya = (st.ya + (a << 8)) & 0xFFFFu;  // y = (u8)(y+a)
    const uint32_t b = S[ya];                          // b = S[y]
    const uint32_t xn = (xa + 256u) & 0xFFFFu;
    const uint32_t p = S[xn];                          // prefetch S[x+1]
    S[xa] = (uint8_t)b;                                // S[x] = b
    S[ya] = (uint8_t)a;                                // S[y] = a
    const uint32_t ta = (((a + b) << 8) | st.col) & 0xFFFFu;
    const uint32_t k = S[ta];                          // S[(u8)(a+b)]
    st.an = (xn == ya) ? a : p;
    st.xa = xa;
    st.ya = ya;
    return k;
}

// 4 keystream bytes packed little-endian into one dword.
__device__ __forceinline__ uint32_t prga_word(uint8_t *S, Rc4Lane &st)
{
    const uint32_t k0 = prga_step(S, st);
    const uint32_t k1 = prga_step(S, st);
    const uint32_t k2 = prga_step(S, st);
    const uint32_t k3 = prga_step(S, st);
    return k0 | (k1 << 8) | (k2 << 16) | (k3 << 24);
}

__device__ __forceinline__ uint4 xor16(uint8_t *S, Rc4Lane &st, uint4 v)
{
    v.x ^= prga_word(S, st);
    v.y ^= prga_word(S, st);
    v.z ^= prga_word(S, st);
    v.w ^= prga_word(S, st);
    return v;
}

// Crypt one lane's message in place: unaligned head bytes, 64-byte blocks
// with the next block's loads issued before the current block's keystream,
// 16-byte chunks, tail bytes.
__device__ __forceinline__ void crypt_message(uint8_t *S, Rc4Lane &st,
                                              uint8_t *msg, uint32_t len)
{
    uint32_t head = (16u - ((uint32_t)(uintptr_t)msg & 15u)) & 15u;
    if (head > len) head = len;
    for (uint32_t i = 0; i < head; ++i) msg[i] ^= (uint8_t)prga_step(S, st);
    msg += head;
    len -= head;

    uint4 *p = reinterpret_cast<uint4 *>(msg);
    uint32_t nblk = len >> 6;
    if (nblk) {
        uint4 c0 = p[0], c1 = p[1], c2 = p[2], c3 = p[3];
        for (uint32_t b = 0; b < nblk; ++b) {
            uint4 n0, n1, n2, n3;
            const bool more = (b + 1) < nblk;
            if (more) { n0 = p[4]; n1 = p[5]; n2 = p[6]; n3 = p[7]; }
            p[0] = xor16(S, st, c0);
            p[1] = xor16(S, st, c1);
            p[2] = xor16(S, st, c2);
            p[3] = xor16(S, st, c3);
            p += 4;
            if (more) { c0 = n0; c1 = n1; c2 = n2; c3 = n3; }
        }
    }
    uint32_t rem = len & 63u;
    while (rem >= 16u) {
        *p = xor16(S, st, *p);
        ++p;
        rem -= 16u;
    }
    uint8_t *t = reinterpret_cast<uint8_t *>(p);
    for (uint32_t i = 0; i < rem; ++i) t[i] ^= (uint8_t)prga_step(S, st);
}

// ---------------------------------------------------------------------------
// crypt_kernel: batched RC4Encryption::encryption.
// grid = ceil(n / 256) workgroups of 256 threads; workgroup w handles batch
// entries [w*256, w*256+256).
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256, 2)
crypt_kernel(uint8_t *__restrict__ arena, uint16_t *__restrict__ xy,
             const uint32_t *__restrict__ ids, uint8_t *__restrict__ payload,
             const uint64_t *__restrict__ off, const uint32_t *__restrict__ len,
             uint32_t n, uint32_t capacity, uint32_t *__restrict__ err)
{
    __shared__ __attribute__((aligned(16))) uint8_t S[kGroupBytes];

    const uint32_t j = threadIdx.x;
    const uint32_t e = blockIdx.x * kGroup + j;
    const bool valid = e < n;
    uint32_t slot = valid ? (ids ? ids[e] : e) : 0xFFFFFFFFu;
    if (valid && slot >= capacity) {
        atomicOr(err, kErrSlotRange);
        slot = 0xFFFFFFFFu;
    }
    const bool active = slot != 0xFFFFFFFFu;
    const uint32_t mylen = active ? len[e] : 0u;

    // Fast path: this workgroup covers one whole aligned group.  With
    // ids == NULL group w is exactly slots [w*256, w*256+256) (entries >= n
    // belong to no other workgroup, and their state is copied back unchanged).
    bool whole;
    uint32_t g;
    if (!ids) {
        whole = true;
        g = blockIdx.x;
    } else {
        const uint32_t first = (blockIdx.x * kGroup < n) ? ids[blockIdx.x * kGroup] : 0u;
        g = first >> 8;
        whole = __syncthreads_and(active && slot == ((first & ~255u) + j) && (first & 255u) == 0u);
    }

    const uint32_t col = col_of(j);
    if (whole) {
        image_to_lds(S, arena + (size_t)g * kGroupBytes);
        __syncthreads();
    } else if (active && mylen) {
        gather_column(S, col, arena, slot);
    }

    if (active && mylen) {
        const uint16_t sxy = xy[slot];
        const uint32_t x = sxy & 255u, y = sxy >> 8;
        Rc4Lane st;
        st.col = col;
        st.xa = (x << 8) | col;
        st.ya = (y << 8) | col;
        st.an = S[(((x + 1u) & 255u) << 8) | col];
        crypt_message(S, st, payload + off[e], mylen);
        xy[slot] = (uint16_t)((st.xa >> 8) | (st.ya & 0xFF00u));
    }

    if (whole) {
        __syncthreads();
        lds_to_image(arena + (size_t)g * kGroupBytes, S);
    } else if (active && mylen) {
        scatter_column(arena, slot, S, col);
    }
}

// ---------------------------------------------------------------------------
// ksa_kernel: batched RC4Encryption::makeSBox (rc4_encryption.h:46-72).
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256, 2)
ksa_kernel(uint8_t *__restrict__ arena, uint16_t *__restrict__ xy,
           const uint32_t *__restrict__ ids, const uint8_t *__restrict__ keys,
           const uint64_t *__restrict__ key_off, const uint32_t *__restrict__ key_len,
           uint32_t n, uint32_t capacity, uint32_t *__restrict__ err)
{
    __shared__ __attribute__((aligned(16))) uint8_t S[kGroupBytes];

    const uint32_t j = threadIdx.x;
    const uint32_t e = blockIdx.x * kGroup + j;
    const bool valid = e < n;
    uint32_t slot = valid ? (ids ? ids[e] : e) : 0xFFFFFFFFu;
    if (valid && slot >= capacity) {
        atomicOr(err, kErrSlotRange);
        slot = 0xFFFFFFFFu;
    }
    const bool active = slot != 0xFFFFFFFFu;

    bool whole;
    uint32_t g;
    if (!ids) {
        // Entries >= n of the last group are not re-seeded: load the image so
        // their state is written back unchanged.
        whole = true;
        g = blockIdx.x;
    } else {
        const uint32_t first = (blockIdx.x * kGroup < n) ? ids[blockIdx.x * kGroup] : 0u;
        g = first >> 8;
        whole = __syncthreads_and(active && slot == ((first & ~255u) + j) && (first & 255u) == 0u);
    }
    const bool partial = !ids && (blockIdx.x + 1u) * kGroup > n;
    const uint32_t col = col_of(j);

    if (whole && partial) {
        image_to_lds(S, arena + (size_t)g * kGroupBytes);
        __syncthreads();
    }
    if (active) {
        // identity box (:50-53)
        for (int k = 0; k < 256; ++k) S[(k << 8) | col] = (uint8_t)k;
        const uint32_t kl = key_len[e];
        if (kl) {
            const uint8_t *key = keys + key_off[e];
            uint32_t jj = 0, kk = 0;
            for (int i0 = 0; i0 < 256; i0 += 16) {
                uint32_t kb[16];
#pragma unroll
                for (int u = 0; u < 16; ++u) {      // key[k], k cycles mod len (:67-70)
                    kb[u] = key[kk];
                    if (++kk >= kl) kk = 0;
                }
#pragma unroll
                for (int u = 0; u < 16; ++u) {
                    const uint32_t ia = ((uint32_t)(i0 + u) << 8) | col;
                    const uint32_t v = S[ia];
                    jj = (jj + v + kb[u]) & 255u;   // j = (u8)(j + tmp + obs[k])
                    const uint32_t ja = (jj << 8) | col;
                    S[ia] = S[ja];
                    S[ja] = (uint8_t)v;
                }
            }
        }
        xy[slot] = 0;                                // _x = _y = 0 (:48-49)
    }
    if (whole) {
        __syncthreads();
        lds_to_image(arena + (size_t)g * kGroupBytes, S);
    } else if (active) {
        scatter_column(arena, slot, S, col);
    }
}

// identity_kernel: every slot of every group gets the identity S-box (row k of
// a group image is 256 copies of k).  One workgroup per group.
__global__ void __launch_bounds__(256)
identity_kernel(uint8_t *__restrict__ arena)
{
    uint4 *img = reinterpret_cast<uint4 *>(arena + (size_t)blockIdx.x * kGroupBytes);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const uint32_t q = i * 256 + threadIdx.x;     // uint4 index; row = q / 16
        const uint32_t v = (q >> 4) * 0x01010101u;
        img[q] = make_uint4(v, v, v, v);
    }
}

}  // namespace zrc4
