// win_ubench.hip -- lane-parallel speculative RC4 windows (tools/window_sim.py)
// as a keystream-only kernel: 8 lanes per stream, one window of up to 8 PRGA
// steps per iteration.  Checks every keystream byte and final state against a
// serial CPU PRGA and reports cycles per byte per stream.
//   build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/ubench/win_ubench.hip -o tools/ubench/win_ubench
//   run:   tools/ubench/win_ubench [streams] [bytes] [W=8|16] [waves_per_block]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <random>
#include <algorithm>
#include "../../zsummerx_amd/csrc/zrc4_win.hpp"
#include "win64_loop.hpp"
#include "win12_loop.hpp"
#include "win_var.hpp"
#include "win_repair.hpp"
#include "win_var2.hpp"
#include "win_var3.hpp"
#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int MAXN = (int)zrc4::kWinRing;   // keystream ring per stream (bytes)

// Lean variant, W = 8 or 16 lanes per stream: one-hot cut bits from
// med3(d, l, W), min-lane markers (ds_max of (tag << 8) | (255 - l)) for the
// duplicate-j rule and for K's "written by a committed step <= l" test, y'
// summed in-lane from the window bytes (no cross-lane gather).
template <int W>
__device__ __forceinline__ uint32_t orW(uint32_t v)
{
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);
    if (W == 16) v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false);
    return v;
}

__device__ __forceinline__ uint32_t mask_lt(uint32_t c, uint32_t q)   // bytes k < c of dword q
{
    return c <= 4 * q ? 0u : (c >= 4 * q + 4 ? 0xFFFFFFFFu : (0xFFFFFFFFu >> (32 - 8 * (c - 4 * q))));
}

template <int W, int WPB>
__global__ void __launch_bounds__(64 * WPB)
win_kernel(const uint8_t *sbox_in, const uint16_t *xy_in, uint8_t *ks_out, uint8_t *sbox_out,
           uint16_t *xy_out, uint64_t *cyc, uint32_t *wins, int nstreams, int N)
{
    constexpr int SPW = 64 / W;                 // streams per wave
    constexpr int ND = W / 4;                   // window dwords
    __shared__ __attribute__((aligned(16))) uint8_t Sb[WPB * SPW * 256];
    __shared__ uint32_t Mk[WPB * SPW * 256];
    __shared__ __attribute__((aligned(16))) uint8_t Ring[WPB * SPW * MAXN];

    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t l = lane % W, g = wv * SPW + lane / W;
    const int s = blockIdx.x * (WPB * SPW) + (int)g;
    const bool live = s < nstreams;
    uint8_t *S = Sb + g * 256;
    uint32_t *M = Mk + g * 256;
    uint8_t *R = Ring + g * MAXN;
    for (int k = 0; k < 256 / W; ++k) S[l * (256 / W) + k] = live ? sbox_in[(size_t)s * 256 + l * (256 / W) + k] : 0;
    for (int k = 0; k < 256 / W; ++k) M[l * (256 / W) + k] = 0;
    uint32_t xa = live ? ((xy_in[s] + 1) & 0xFF) : 1, y = live ? (xy_in[s] >> 8) : 0;
    __syncthreads();

    uint32_t m[ND];
#pragma unroll
    for (int q = 0; q < ND; ++q) m[q] = mask_lt(l + 1, q);
    const uint32_t sel_l = 0x0C0C0C00u | (l & 3);
    uint32_t V = (1u << 8) | (255 - l);         // marker value of this lane, tag in bits 8+
    uint32_t rem = live ? (uint32_t)N : 0u, p = 0, nw = 0;
    const uint32_t *S32 = reinterpret_cast<const uint32_t *>(S);
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    while (__builtin_amdgcn_ballot_w64(rem != 0)) {
        nw += rem != 0;
        uint32_t D[ND + 1], A[ND];
        const uint32_t w0 = xa >> 2;
#pragma unroll
        for (int q = 0; q <= ND; ++q) D[q] = S32[(w0 + q) & 63];
#pragma unroll
        for (int q = 0; q < ND; ++q) A[q] = __builtin_amdgcn_alignbyte(D[q + 1], D[q], xa);
        uint32_t J = y;
#pragma unroll
        for (int q = 0; q < ND; ++q) J = __builtin_amdgcn_sad_u8(A[q] & m[q], 0, J);
        J &= 255;
        uint32_t aw = A[0];
#pragma unroll
        for (int q = 1; q < ND; ++q) aw = (l >> 2) == (uint32_t)q ? A[q] : aw;
        const uint32_t a = __builtin_amdgcn_perm(0, aw, sel_l);
        const uint32_t b = S[J];
        atomicMax(&M[J], V);
        const uint32_t mr = __hip_atomic_load(&M[J], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const uint32_t d = (J - xa) & 255;
        const uint32_t c = d < l ? l : (d < (uint32_t)W ? d : (uint32_t)W);  // med3(d, l, W)
        uint32_t oh = ((1u << c) | (mr != V ? (1u << l) : 0u)) & ~1u;
        oh = orW<W>(oh | (1u << W));
        uint32_t cut = __builtin_ctz(oh);
        cut = cut < rem ? cut : rem;
        const uint32_t t = (a + b) & 255;
        const uint32_t k0 = S[t];
        if (l < cut) {
            S[(xa + l) & 255] = (uint8_t)b;
            S[J] = (uint8_t)a;
        }
        const uint32_t k1 = S[t];
        const uint32_t mt = M[t];
        const bool own = ((t - xa) & 255) <= l || mt >= V;
        if (l < cut) R[(p + l) & (MAXN - 1)] = (uint8_t)(own ? k1 : k0);
#pragma unroll
        for (int q = 0; q < ND; ++q) y = __builtin_amdgcn_sad_u8(A[q] & mask_lt(cut, q), 0, y);
        y &= 255;
        xa = (xa + cut) & 255;
        p += cut;
        rem -= cut;
        V += 256;
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    __syncthreads();
    if (live) {
        for (int k = 0; k < N / W; ++k) ks_out[(size_t)s * N + l * (N / W) + k] = R[l * (N / W) + k];
        for (int k = 0; k < 256 / W; ++k) sbox_out[(size_t)s * 256 + l * (256 / W) + k] = S[l * (256 / W) + k];
        if (l == 0) {
            xy_out[s] = (uint16_t)(((xa - 1) & 255) | (y << 8));
            cyc[s] = t1 - t0;
            wins[s] = nw;
        }
    }
}


// v3: S-box stored twice (S[p] and S[p + 256] written together, so a window
// never wraps and reads as 5 aligned dwords), a_l read directly, y' from a
// DPP max over lanes (l < cut ? l << 8 | J : 0) computed under the next
// window's read round trip.
template <int W>
__device__ __forceinline__ uint32_t maxW(uint32_t v)
{
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false));
    if (W == 16) v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false));
    return v;
}

template <int W, int WPB>
__global__ void __launch_bounds__(64 * WPB)
win3_kernel(const uint8_t *sbox_in, const uint16_t *xy_in, uint8_t *ks_out, uint8_t *sbox_out,
            uint16_t *xy_out, uint64_t *cyc, uint32_t *wins, int nstreams, int N)
{
    constexpr int SPW = 64 / W;
    constexpr int ND = W / 4;
    __shared__ __attribute__((aligned(16))) uint8_t Sb[WPB * SPW * 512];
    __shared__ uint32_t Mk[WPB * SPW * 256];
    __shared__ __attribute__((aligned(16))) uint8_t Ring[WPB * SPW * MAXN];

    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t l = lane % W, g = wv * SPW + lane / W;
    const int s = blockIdx.x * (WPB * SPW) + (int)g;
    const bool live = s < nstreams;
    uint8_t *S = Sb + g * 512;
    uint32_t *M = Mk + g * 256;
    uint8_t *R = Ring + g * MAXN;
    for (int k = 0; k < 256 / W; ++k) {
        const uint8_t v = live ? sbox_in[(size_t)s * 256 + l * (256 / W) + k] : 0;
        S[l * (256 / W) + k] = v;
        S[256 + l * (256 / W) + k] = v;
        M[l * (256 / W) + k] = 0;
    }
    uint32_t xa = live ? ((xy_in[s] + 1) & 0xFF) : 1, y = live ? (xy_in[s] >> 8) : 0;
    __syncthreads();

    uint32_t m[ND];
#pragma unroll
    for (int q = 0; q < ND; ++q) m[q] = mask_lt(l + 1, q);
    uint32_t V = (1u << 8) | (255 - l);
    uint32_t rem = live ? (uint32_t)N : 0u, p = 0, nw = 0;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    while (__builtin_amdgcn_ballot_w64(rem != 0)) {
        nw += rem != 0;
        const uint32_t *Wp = reinterpret_cast<const uint32_t *>(S + (xa & 0xFCu));
        uint32_t D[ND + 1], A[ND];
#pragma unroll
        for (int q = 0; q <= ND; ++q) D[q] = Wp[q];
        const uint32_t a = S[xa + l];
#pragma unroll
        for (int q = 0; q < ND; ++q) A[q] = __builtin_amdgcn_alignbyte(D[q + 1], D[q], xa);
        uint32_t J = y;
#pragma unroll
        for (int q = 0; q < ND; ++q) J = __builtin_amdgcn_sad_u8(A[q] & m[q], 0, J);
        J &= 255;
        const uint32_t b = S[J];
        atomicMax(&M[J], V);
        const uint32_t mr = __hip_atomic_load(&M[J], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const uint32_t d = (J - xa) & 255;
        const uint32_t c = min(max(d, l), (uint32_t)W);   // med3(d, l, W)
        uint32_t oh = ((1u << c) | (mr != V ? (1u << l) : 0u)) & ~1u;
        oh = orW<W>(oh | (1u << W));
        uint32_t cut = __builtin_ctz(oh);
        cut = cut < rem ? cut : rem;
        const uint32_t t = (a + b) & 255;
        const uint32_t k0 = S[t];
        if (l < cut) {
            const uint32_t i = (xa + l) & 255;
            S[i] = (uint8_t)b;
            S[i + 256] = (uint8_t)b;
            S[J] = (uint8_t)a;
            S[J + 256] = (uint8_t)a;
        }
        const uint32_t k1 = S[t];
        const uint32_t mt = M[t];
        const bool own = ((t - xa) & 255) <= l || mt >= V;
        if (l < cut) R[(p + l) & (MAXN - 1)] = (uint8_t)(own ? k1 : k0);
        const uint32_t yl = maxW<W>(l < cut ? ((l + 1) << 8) | J : 0u);
        y = cut ? (yl & 255) : y;
        xa = (xa + cut) & 255;
        p += cut;
        rem -= cut;
        V += 256;
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    __syncthreads();
    if (live) {
        for (int k = 0; k < N / W; ++k) ks_out[(size_t)s * N + l * (N / W) + k] = R[l * (N / W) + k];
        for (int k = 0; k < 256 / W; ++k) sbox_out[(size_t)s * 256 + l * (256 / W) + k] = S[l * (256 / W) + k];
        if (l == 0) {
            xy_out[s] = (uint16_t)(((xa - 1) & 255) | (y << 8));
            cyc[s] = t1 - t0;
            wins[s] = nw;
        }
    }
}


// v4: the W = 16 window loop as one asm statement (hand-scheduled):
//   reads of window n issue first; the tail of window n-1 (y' max over lanes,
//   keystream select, ring write) runs under their round trip; the prefix
//   (alignbyte, and, sad tree) -> b / marker reads -> rules under that round
//   trip -> marker rule -> DPP OR -> cut -> k0 read -> commit (4 writes, both
//   S copies) -> k1 / marker(t) reads -> state updates.
// Pinned temporaries: v100-v104 window dwords, v105-v135 scratch; s[40:47].
#define WIN_TAIL                                                                                  \
    "s_nop 1\n\t"                                                                                 \
    "v_max_u32_dpp v120, v120, v120 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"           \
    "s_nop 1\n\t"                                                                                 \
    "v_max_u32_dpp v120, v120, v120 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"           \
    "s_nop 1\n\t"                                                                                 \
    "v_max_u32_dpp v120, v120, v120 row_half_mirror row_mask:0xf bank_mask:0xf\n\t"               \
    "s_nop 1\n\t"                                                                                 \
    "v_max_u32_dpp v120, v120, v120 row_mirror row_mask:0xf bank_mask:0xf\n\t"                    \
    "s_waitcnt lgkmcnt(%[tailcnt])\n\t"                                                           \
    "v_cmp_ge_u32_e64 s[42:43], v123, %[v]\n\t"                                                   \
    "s_or_b64 s[42:43], s[42:43], s[44:45]\n\t"                                                   \
    "v_cndmask_b32_e64 v124, v121, v122, s[42:43]\n\t"                                            \
    "s_mov_b64 s[40:41], exec\n\t"                                                                \
    "s_mov_b64 exec, s[46:47]\n\t"                                                                \
    "ds_write_b8 v125, v124\n\t"                                                                  \
    "s_mov_b64 exec, s[40:41]\n\t"                                                                \
    "v_and_b32 %[y], 0xff, v120\n\t"                                                              \
    "v_add_u32 %[v], 0x100, %[v]\n\t"

template <int WPB>
__global__ void __launch_bounds__(64 * WPB)
win4_kernel(const uint8_t *sbox_in, const uint16_t *xy_in, uint8_t *ks_out, uint8_t *sbox_out,
            uint16_t *xy_out, uint64_t *cyc, uint32_t *wins, int nstreams, int N)
{
    constexpr int W = 16, SPW = 4;
    __shared__ __attribute__((aligned(1024))) uint32_t Mk[WPB * SPW * 256];
    __shared__ __attribute__((aligned(1024))) uint8_t Ring[WPB * SPW * MAXN];
    __shared__ __attribute__((aligned(512))) uint8_t Sb[WPB * SPW * 512];

    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t l = lane % W, g = wv * SPW + lane / W;
    const int s = blockIdx.x * (WPB * SPW) + (int)g;
    const bool live = s < nstreams;
    uint8_t *S = Sb + g * 512;
    uint32_t *M = Mk + g * 256;
    uint8_t *R = Ring + g * MAXN;
    for (int k = 0; k < 256 / W; ++k) {
        const uint8_t v = live ? sbox_in[(size_t)s * 256 + l * (256 / W) + k] : 0;
        S[l * (256 / W) + k] = v;
        S[256 + l * (256 / W) + k] = v;
        M[l * (256 / W) + k] = 0;
    }
    uint32_t xa = live ? ((xy_in[s] + 1) & 0xFF) : 1, y = live ? (xy_in[s] >> 8) : 0;
    __syncthreads();

    const uint32_t m0 = mask_lt(l + 1, 0), m1 = mask_lt(l + 1, 1), m2 = mask_lt(l + 1, 2), m3 = mask_lt(l + 1, 3);
    const uint32_t bitl16 = (1u << l) | 0x10000u, l1 = (l + 1) << 8;
    const uint32_t sb = (uint32_t)(uintptr_t)S, mb = (uint32_t)(uintptr_t)M, rb = (uint32_t)(uintptr_t)R;
    uint32_t V = (1u << 8) | (255 - l);
    uint32_t rem = live ? (uint32_t)N : 0u, rp = l;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    asm volatile(
        // prologue: no previous window (empty commit mask, y' = y)
        "s_mov_b64 s[46:47], 0\n\t"
        "v_mov_b32 v120, %[y]\n\t"
        "s_mov_b64 s[44:45], 0\n\t"
        "WIN_LOOP_%=:\n\t"
        // window n reads
        "v_and_b32 v105, 0xfc, %[xa]\n\t"
        "v_add_u32 v105, %[sb], v105\n\t"
        "v_add3_u32 v106, %[sb], %[xa], %[l]\n\t"
        "ds_read2_b32 v[100:101], v105 offset1:1\n\t"
        "ds_read2_b32 v[102:103], v105 offset0:2 offset1:3\n\t"
        "ds_read_b32 v104, v105 offset:16\n\t"
        "ds_read_u8 v107, v106\n\t"
        // window n-1 tail
        WIN_TAIL
        "s_waitcnt lgkmcnt(0)\n\t"
        // prefix: J = y + a_0 + ... + a_l
        "v_alignbyte_b32 v108, v101, v100, %[xa]\n\t"
        "v_alignbyte_b32 v109, v102, v101, %[xa]\n\t"
        "v_alignbyte_b32 v110, v103, v102, %[xa]\n\t"
        "v_alignbyte_b32 v111, v104, v103, %[xa]\n\t"
        "v_and_b32 v108, v108, %[m0]\n\t"
        "v_and_b32 v110, v110, %[m2]\n\t"
        "v_and_b32 v109, v109, %[m1]\n\t"
        "v_and_b32 v111, v111, %[m3]\n\t"
        "v_sad_u8 v112, v108, 0, %[y]\n\t"
        "v_sad_u8 v113, v110, 0, 0\n\t"
        "v_sad_u8 v112, v109, 0, v112\n\t"
        "v_sad_u8 v113, v111, 0, v113\n\t"
        "v_add_u32 v112, v112, v113\n\t"
        "v_and_b32 v112, 0xff, v112\n\t"                       // J (byte)
        "v_add_u32 v114, %[sb], v112\n\t"                       // &S[J]
        "v_lshl_add_u32 v115, v112, 2, %[mb]\n\t"               // &M[J]
        "ds_read_u8 v116, v114\n\t"                             // b
        "ds_max_u32 v115, %[v]\n\t"
        "ds_read_b32 v117, v115\n\t"                            // marker winner
        // rule on d = J - x - 1 (under the round trip)
        "v_sub_u32 v118, v112, %[xa]\n\t"
        "v_and_b32 v118, 0xff, v118\n\t"
        "v_med3_u32 v118, v118, %[l], 16\n\t"
        "v_lshlrev_b32 v118, v118, 1\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "v_cmp_ne_u32 vcc, v117, %[v]\n\t"
        "v_cndmask_b32 v119, %[c16], %[bitl16], vcc\n\t"
        "v_and_or_b32 v118, v118, -2, v119\n\t"
        "s_nop 1\n\t"
        "v_or_b32_dpp v118, v118, v118 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_or_b32_dpp v118, v118, v118 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_or_b32_dpp v118, v118, v118 row_half_mirror row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_or_b32_dpp v118, v118, v118 row_mirror row_mask:0xf bank_mask:0xf\n\t"
        "v_add3_u32 v126, %[sb], v107, v116\n\t"                // &S[a + b] (doubled S: no wrap)
        "ds_read_u8 v121, v126\n\t"                             // k0 = S0[t]
        "v_ffbl_b32 v118, v118\n\t"
        "v_min_u32 v118, v118, %[rem]\n\t"                      // cut
        "v_cmp_lt_u32 vcc, %[l], v118\n\t"
        "s_and_saveexec_b64 s[40:41], vcc\n\t"
        "s_mov_b64 s[46:47], exec\n\t"
        "v_xor_b32 v127, 0x100, v106\n\t"
        "ds_write_b8 v106, v116\n\t"                            // S[i] = b, both copies
        "ds_write_b8 v127, v116\n\t"
        "ds_write_b8 v114, v107\n\t"                            // S[J] = a, both copies
        "ds_write_b8 v114, v107 offset:256\n\t"
        "s_mov_b64 exec, s[40:41]\n\t"
        "ds_read_u8 v122, v126\n\t"                             // k1 = S_final[t]
        "v_add_u32 v128, v107, v116\n\t"
        "v_and_b32 v128, 0xff, v128\n\t"                        // t
        "v_lshl_add_u32 v129, v128, 2, %[mb]\n\t"
        "ds_read_b32 v123, v129\n\t"                            // marker of t
        "v_sub_u32 v128, v128, %[xa]\n\t"
        "v_and_b32 v128, 0xff, v128\n\t"
        "v_cmp_le_u32_e64 s[44:45], v128, %[l]\n\t"             // t is an i of a step <= l
        "v_bfi_b32 v125, %[rmask], %[rp], %[rb]\n\t"            // ring slot of this lane
        "v_or_b32 v130, %[l1], v112\n\t"
        "v_cndmask_b32 v120, %[y], v130, vcc\n\t"               // y' candidate
        "v_add_u32 %[xa], %[xa], v118\n\t"
        "v_and_b32 %[xa], 0xff, %[xa]\n\t"
        "v_add_u32 %[rp], %[rp], v118\n\t"
        "v_sub_u32 %[rem], %[rem], v118\n\t"
        "v_cmp_ne_u32 vcc, 0, %[rem]\n\t"
        "s_cbranch_vccnz WIN_LOOP_%=\n\t"
        WIN_TAIL
        "s_waitcnt lgkmcnt(0)\n\t"
        : [xa] "+v"(xa), [y] "+v"(y), [v] "+v"(V), [rem] "+v"(rem), [rp] "+v"(rp)
        : [l] "v"(l), [sb] "v"(sb), [mb] "v"(mb), [rb] "v"(rb), [m0] "v"(m0), [m1] "v"(m1), [m2] "v"(m2),
          [m3] "v"(m3), [bitl16] "v"(bitl16), [l1] "v"(l1), [rmask] "s"((uint32_t)(MAXN - 1)), [tailcnt] "n"(4), [c16] "v"(0x10000u)
        : "memory", "vcc", "scc", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109",
          "v110", "v111", "v112", "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122",
          "v123", "v124", "v125", "v126", "v127", "v128", "v129", "v130", "s40", "s41", "s42", "s43", "s44",
          "s45", "s46", "s47");
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    __syncthreads();
    if (live) {
        for (int k = 0; k < N / W; ++k) ks_out[(size_t)s * N + l * (N / W) + k] = R[l * (N / W) + k];
        for (int k = 0; k < 256 / W; ++k) sbox_out[(size_t)s * 256 + l * (256 / W) + k] = S[l * (256 / W) + k];
        if (l == 0) {
            xy_out[s] = (uint16_t)(((xa - 1) & 255) | ((y & 255) << 8));
            cyc[s] = t1 - t0;
            wins[s] = (V >> 8) - 2;
        }
    }
}


// v6: the product loop (zrc4::win_windows, zsummerx_amd/csrc/zrc4_win.hpp)
// on a linear S-box layout: the tuning harness for the library kernel (the
// loop uses only the first 256 bytes of each stream's 512-byte S area).
__global__ void __launch_bounds__(64)
win6_kernel(const uint8_t *sbox_in, const uint16_t *xy_in, uint8_t *ks_out, uint8_t *sbox_out,
            uint16_t *xy_out, uint64_t *cyc, uint32_t *wins, int nstreams, int N)
{
    constexpr int W = 16, SPW = 4;
    __shared__ __attribute__((aligned(1024))) uint32_t Mk[SPW * 256];
    __shared__ __attribute__((aligned(MAXN))) uint8_t Ring[SPW * MAXN];
    __shared__ __attribute__((aligned(512))) uint8_t Sb[SPW * 512];
    const uint32_t lane = threadIdx.x, l = lane % W, g = lane / W;
    const int s = blockIdx.x * SPW + (int)g;
    const bool live = s < nstreams;
    uint8_t *S = Sb + g * 512;
    uint32_t *M = Mk + g * 256;
    uint8_t *R = Ring + g * MAXN;
    for (int k = 0; k < 256 / W; ++k) {
        const uint8_t v = live ? sbox_in[(size_t)s * 256 + l * (256 / W) + k] : 0;
        S[l * (256 / W) + k] = v;
        S[256 + l * (256 / W) + k] = v;
        M[l * (256 / W) + k] = 0;
    }
    const uint32_t sxy = live ? xy_in[s] : 0;
    __syncthreads();
    zrc4::WinLane w{((sxy & 0xFFu) + 1u) & 0xFFu, sxy >> 8, (1u << 8) | (255u - l), l};
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    zrc4::win_windows(w, live ? (uint32_t)N : 0u, l, (uint32_t)(uintptr_t)S, (uint32_t)(uintptr_t)M,
                      (uint32_t)(uintptr_t)R);
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    __syncthreads();
    if (live) {
        for (int k = 0; k < N / W; ++k) ks_out[(size_t)s * N + l * (N / W) + k] = R[l * (N / W) + k];
        for (int k = 0; k < 256 / W; ++k) sbox_out[(size_t)s * 256 + l * (256 / W) + k] = S[l * (256 / W) + k];
        if (l == 0) {
            xy_out[s] = (uint16_t)(((w.xa - 1) & 255) | ((w.y & 255) << 8));
            cyc[s] = t1 - t0;
            wins[s] = (w.v >> 8) - 1;
        }
    }
}

// v17 (mode 17): variant S (tools/ubench/win_var3.hpp): J, d and x + 1 masked by SDWA byte writes
// on a linear S-box layout: the tuning harness for the library kernel (the
// loop uses only the first 256 bytes of each stream's 512-byte S area).
__global__ void __launch_bounds__(64)
win17_kernel(const uint8_t *sbox_in, const uint16_t *xy_in, uint8_t *ks_out, uint8_t *sbox_out,
            uint16_t *xy_out, uint64_t *cyc, uint32_t *wins, int nstreams, int N)
{
    constexpr int W = 16, SPW = 4;
    __shared__ __attribute__((aligned(1024))) uint32_t Mk[SPW * 256];
    __shared__ __attribute__((aligned(MAXN))) uint8_t Ring[SPW * MAXN];
    __shared__ __attribute__((aligned(512))) uint8_t Sb[SPW * 512];
    const uint32_t lane = threadIdx.x, l = lane % W, g = lane / W;
    const int s = blockIdx.x * SPW + (int)g;
    const bool live = s < nstreams;
    uint8_t *S = Sb + g * 512;
    uint32_t *M = Mk + g * 256;
    uint8_t *R = Ring + g * MAXN;
    for (int k = 0; k < 256 / W; ++k) {
        const uint8_t v = live ? sbox_in[(size_t)s * 256 + l * (256 / W) + k] : 0;
        S[l * (256 / W) + k] = v;
        S[256 + l * (256 / W) + k] = v;
        M[l * (256 / W) + k] = 0;
    }
    const uint32_t sxy = live ? xy_in[s] : 0;
    __syncthreads();
    zrc4::WinLane w{((sxy & 0xFFu) + 1u) & 0xFFu, sxy >> 8, (1u << 8) | (255u - l), l};
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    zrc4::win_windows_S(w, live ? (uint32_t)N : 0u, l, (uint32_t)(uintptr_t)S, (uint32_t)(uintptr_t)M,
                      (uint32_t)(uintptr_t)R);
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    __syncthreads();
    if (live) {
        for (int k = 0; k < N / W; ++k) ks_out[(size_t)s * N + l * (N / W) + k] = R[l * (N / W) + k];
        for (int k = 0; k < 256 / W; ++k) sbox_out[(size_t)s * 256 + l * (256 / W) + k] = S[l * (256 / W) + k];
        if (l == 0) {
            xy_out[s] = (uint16_t)(((w.xa - 1) & 255) | ((w.y & 255) << 8));
            cyc[s] = t1 - t0;
            wins[s] = (w.v >> 8) - 1;
        }
    }
}

// mode 18: variant Sae (tools/ubench/win_var3.hpp): J, d and x + 1 masked by SDWA byte writes
// on a linear S-box layout: the tuning harness for the library kernel (the
// loop uses only the first 256 bytes of each stream's 512-byte S area).
__global__ void __launch_bounds__(64)
win18_kernel(const uint8_t *sbox_in, const uint16_t *xy_in, uint8_t *ks_out, uint8_t *sbox_out,
            uint16_t *xy_out, uint64_t *cyc, uint32_t *wins, int nstreams, int N)
{
    constexpr int W = 16, SPW = 4;
    __shared__ __attribute__((aligned(1024))) uint32_t Mk[SPW * 256];
    __shared__ __attribute__((aligned(MAXN))) uint8_t Ring[SPW * MAXN];
    __shared__ __attribute__((aligned(512))) uint8_t Sb[SPW * 512];
    const uint32_t lane = threadIdx.x, l = lane % W, g = lane / W;
    const int s = blockIdx.x * SPW + (int)g;
    const bool live = s < nstreams;
    uint8_t *S = Sb + g * 512;
    uint32_t *M = Mk + g * 256;
    uint8_t *R = Ring + g * MAXN;
    for (int k = 0; k < 256 / W; ++k) {
        const uint8_t v = live ? sbox_in[(size_t)s * 256 + l * (256 / W) + k] : 0;
        S[l * (256 / W) + k] = v;
        S[256 + l * (256 / W) + k] = v;
        M[l * (256 / W) + k] = 0;
    }
    const uint32_t sxy = live ? xy_in[s] : 0;
    __syncthreads();
    zrc4::WinLane w{((sxy & 0xFFu) + 1u) & 0xFFu, sxy >> 8, (1u << 8) | (255u - l), l};
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    zrc4::win_windows_Sae(w, live ? (uint32_t)N : 0u, l, (uint32_t)(uintptr_t)S, (uint32_t)(uintptr_t)M,
                      (uint32_t)(uintptr_t)R);
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    __syncthreads();
    if (live) {
        for (int k = 0; k < N / W; ++k) ks_out[(size_t)s * N + l * (N / W) + k] = R[l * (N / W) + k];
        for (int k = 0; k < 256 / W; ++k) sbox_out[(size_t)s * 256 + l * (256 / W) + k] = S[l * (256 / W) + k];
        if (l == 0) {
            xy_out[s] = (uint16_t)(((w.xa - 1) & 255) | ((w.y & 255) << 8));
            cyc[s] = t1 - t0;
            wins[s] = (w.v >> 8) - 1;
        }
    }
}

// mode 19: variant Sbe (tools/ubench/win_var3.hpp): J, d and x + 1 masked by SDWA byte writes
// on a linear S-box layout: the tuning harness for the library kernel (the
// loop uses only the first 256 bytes of each stream's 512-byte S area).
__global__ void __launch_bounds__(64)
win19_kernel(const uint8_t *sbox_in, const uint16_t *xy_in, uint8_t *ks_out, uint8_t *sbox_out,
            uint16_t *xy_out, uint64_t *cyc, uint32_t *wins, int nstreams, int N)
{
    constexpr int W = 16, SPW = 4;
    __shared__ __attribute__((aligned(1024))) uint32_t Mk[SPW * 256];
    __shared__ __attribute__((aligned(MAXN))) uint8_t Ring[SPW * MAXN];
    __shared__ __attribute__((aligned(512))) uint8_t Sb[SPW * 512];
    const uint32_t lane = threadIdx.x, l = lane % W, g = lane / W;
    const int s = blockIdx.x * SPW + (int)g;
    const bool live = s < nstreams;
    uint8_t *S = Sb + g * 512;
    uint32_t *M = Mk + g * 256;
    uint8_t *R = Ring + g * MAXN;
    for (int k = 0; k < 256 / W; ++k) {
        const uint8_t v = live ? sbox_in[(size_t)s * 256 + l * (256 / W) + k] : 0;
        S[l * (256 / W) + k] = v;
        S[256 + l * (256 / W) + k] = v;
        M[l * (256 / W) + k] = 0;
    }
    const uint32_t sxy = live ? xy_in[s] : 0;
    __syncthreads();
    zrc4::WinLane w{((sxy & 0xFFu) + 1u) & 0xFFu, sxy >> 8, (1u << 8) | (255u - l), l};
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    zrc4::win_windows_Sbe(w, live ? (uint32_t)N : 0u, l, (uint32_t)(uintptr_t)S, (uint32_t)(uintptr_t)M,
                      (uint32_t)(uintptr_t)R);
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    __syncthreads();
    if (live) {
        for (int k = 0; k < N / W; ++k) ks_out[(size_t)s * N + l * (N / W) + k] = R[l * (N / W) + k];
        for (int k = 0; k < 256 / W; ++k) sbox_out[(size_t)s * 256 + l * (256 / W) + k] = S[l * (256 / W) + k];
        if (l == 0) {
            xy_out[s] = (uint16_t)(((w.xa - 1) & 255) | ((w.y & 255) << 8));
            cyc[s] = t1 - t0;
            wins[s] = (w.v >> 8) - 1;
        }
    }
}

// v16: variant R (tools/ubench/win_var2.hpp): the duplicate rule from ds_max_rtn
// on a linear S-box layout: the tuning harness for the library kernel (the
// loop uses only the first 256 bytes of each stream's 512-byte S area).
__global__ void __launch_bounds__(64)
win16_kernel(const uint8_t *sbox_in, const uint16_t *xy_in, uint8_t *ks_out, uint8_t *sbox_out,
            uint16_t *xy_out, uint64_t *cyc, uint32_t *wins, int nstreams, int N)
{
    constexpr int W = 16, SPW = 4;
    __shared__ __attribute__((aligned(1024))) uint32_t Mk[SPW * 256];
    __shared__ __attribute__((aligned(MAXN))) uint8_t Ring[SPW * MAXN];
    __shared__ __attribute__((aligned(512))) uint8_t Sb[SPW * 512];
    const uint32_t lane = threadIdx.x, l = lane % W, g = lane / W;
    const int s = blockIdx.x * SPW + (int)g;
    const bool live = s < nstreams;
    uint8_t *S = Sb + g * 512;
    uint32_t *M = Mk + g * 256;
    uint8_t *R = Ring + g * MAXN;
    for (int k = 0; k < 256 / W; ++k) {
        const uint8_t v = live ? sbox_in[(size_t)s * 256 + l * (256 / W) + k] : 0;
        S[l * (256 / W) + k] = v;
        S[256 + l * (256 / W) + k] = v;
        M[l * (256 / W) + k] = 0;
    }
    const uint32_t sxy = live ? xy_in[s] : 0;
    __syncthreads();
    zrc4::WinLane w{((sxy & 0xFFu) + 1u) & 0xFFu, sxy >> 8, (1u << 8) | (255u - l), l};
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    zrc4::win_windows_R(w, live ? (uint32_t)N : 0u, l, (uint32_t)(uintptr_t)S, (uint32_t)(uintptr_t)M,
                      (uint32_t)(uintptr_t)R);
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    __syncthreads();
    if (live) {
        for (int k = 0; k < N / W; ++k) ks_out[(size_t)s * N + l * (N / W) + k] = R[l * (N / W) + k];
        for (int k = 0; k < 256 / W; ++k) sbox_out[(size_t)s * 256 + l * (256 / W) + k] = S[l * (256 / W) + k];
        if (l == 0) {
            xy_out[s] = (uint16_t)(((w.xa - 1) & 255) | ((w.y & 255) << 8));
            cyc[s] = t1 - t0;
            wins[s] = (w.v >> 8) - 1;
        }
    }
}

// v8: the r02 v12 loop (tools/ubench/win12_loop.hpp), A/B against v6 (zrc4::win_windows, zsummerx_amd/csrc/zrc4_win.hpp)
// on a linear S-box layout: the tuning harness for the library kernel (the
// loop uses only the first 256 bytes of each stream's 512-byte S area).
__global__ void __launch_bounds__(64)
win8_kernel(const uint8_t *sbox_in, const uint16_t *xy_in, uint8_t *ks_out, uint8_t *sbox_out,
            uint16_t *xy_out, uint64_t *cyc, uint32_t *wins, int nstreams, int N)
{
    constexpr int W = 16, SPW = 4;
    __shared__ __attribute__((aligned(1024))) uint32_t Mk[SPW * 256];
    __shared__ __attribute__((aligned(MAXN))) uint8_t Ring[SPW * MAXN];
    __shared__ __attribute__((aligned(512))) uint8_t Sb[SPW * 512];
    const uint32_t lane = threadIdx.x, l = lane % W, g = lane / W;
    const int s = blockIdx.x * SPW + (int)g;
    const bool live = s < nstreams;
    uint8_t *S = Sb + g * 512;
    uint32_t *M = Mk + g * 256;
    uint8_t *R = Ring + g * MAXN;
    for (int k = 0; k < 256 / W; ++k) {
        const uint8_t v = live ? sbox_in[(size_t)s * 256 + l * (256 / W) + k] : 0;
        S[l * (256 / W) + k] = v;
        S[256 + l * (256 / W) + k] = v;
        M[l * (256 / W) + k] = 0;
    }
    const uint32_t sxy = live ? xy_in[s] : 0;
    __syncthreads();
    zrc4::WinLane w{((sxy & 0xFFu) + 1u) & 0xFFu, sxy >> 8, (1u << 8) | (255u - l), l};
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    zrc4::win_windows_v12(w, live ? (uint32_t)N : 0u, l, (uint32_t)(uintptr_t)S, (uint32_t)(uintptr_t)M,
                      (uint32_t)(uintptr_t)R);
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    __syncthreads();
    if (live) {
        for (int k = 0; k < N / W; ++k) ks_out[(size_t)s * N + l * (N / W) + k] = R[l * (N / W) + k];
        for (int k = 0; k < 256 / W; ++k) sbox_out[(size_t)s * 256 + l * (256 / W) + k] = S[l * (256 / W) + k];
        if (l == 0) {
            xy_out[s] = (uint16_t)(((w.xa - 1) & 255) | ((w.y & 255) << 8));
            cyc[s] = t1 - t0;
            wins[s] = (w.v >> 8) - 1;
        }
    }
}

// v9: variant A (tools/ubench/win_var.hpp) (zrc4::win_windows, zsummerx_amd/csrc/zrc4_win.hpp)
// on a linear S-box layout: the tuning harness for the library kernel (the
// loop uses only the first 256 bytes of each stream's 512-byte S area).
__global__ void __launch_bounds__(64)
win9_kernel(const uint8_t *sbox_in, const uint16_t *xy_in, uint8_t *ks_out, uint8_t *sbox_out,
            uint16_t *xy_out, uint64_t *cyc, uint32_t *wins, int nstreams, int N)
{
    constexpr int W = 16, SPW = 4;
    __shared__ __attribute__((aligned(1024))) uint32_t Mk[SPW * 256];
    __shared__ __attribute__((aligned(MAXN))) uint8_t Ring[SPW * MAXN];
    __shared__ __attribute__((aligned(512))) uint8_t Sb[SPW * 512];
    const uint32_t lane = threadIdx.x, l = lane % W, g = lane / W;
    const int s = blockIdx.x * SPW + (int)g;
    const bool live = s < nstreams;
    uint8_t *S = Sb + g * 512;
    uint32_t *M = Mk + g * 256;
    uint8_t *R = Ring + g * MAXN;
    for (int k = 0; k < 256 / W; ++k) {
        const uint8_t v = live ? sbox_in[(size_t)s * 256 + l * (256 / W) + k] : 0;
        S[l * (256 / W) + k] = v;
        S[256 + l * (256 / W) + k] = v;
        M[l * (256 / W) + k] = 0;
    }
    const uint32_t sxy = live ? xy_in[s] : 0;
    __syncthreads();
    zrc4::WinLane w{((sxy & 0xFFu) + 1u) & 0xFFu, sxy >> 8, (1u << 8) | (255u - l), l};
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    zrc4::win_windows_A(w, live ? (uint32_t)N : 0u, l, (uint32_t)(uintptr_t)S, (uint32_t)(uintptr_t)M,
                      (uint32_t)(uintptr_t)R);
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    __syncthreads();
    if (live) {
        for (int k = 0; k < N / W; ++k) ks_out[(size_t)s * N + l * (N / W) + k] = R[l * (N / W) + k];
        for (int k = 0; k < 256 / W; ++k) sbox_out[(size_t)s * 256 + l * (256 / W) + k] = S[l * (256 / W) + k];
        if (l == 0) {
            xy_out[s] = (uint16_t)(((w.xa - 1) & 255) | ((w.y & 255) << 8));
            cyc[s] = t1 - t0;
            wins[s] = (w.v >> 8) - 1;
        }
    }
}

// v10: same as v6 since v17 (variant B shipped) (zrc4::win_windows, zsummerx_amd/csrc/zrc4_win.hpp)
// on a linear S-box layout: the tuning harness for the library kernel (the
// loop uses only the first 256 bytes of each stream's 512-byte S area).
__global__ void __launch_bounds__(64)
win10_kernel(const uint8_t *sbox_in, const uint16_t *xy_in, uint8_t *ks_out, uint8_t *sbox_out,
            uint16_t *xy_out, uint64_t *cyc, uint32_t *wins, int nstreams, int N)
{
    constexpr int W = 16, SPW = 4;
    __shared__ __attribute__((aligned(1024))) uint32_t Mk[SPW * 256];
    __shared__ __attribute__((aligned(MAXN))) uint8_t Ring[SPW * MAXN];
    __shared__ __attribute__((aligned(512))) uint8_t Sb[SPW * 512];
    const uint32_t lane = threadIdx.x, l = lane % W, g = lane / W;
    const int s = blockIdx.x * SPW + (int)g;
    const bool live = s < nstreams;
    uint8_t *S = Sb + g * 512;
    uint32_t *M = Mk + g * 256;
    uint8_t *R = Ring + g * MAXN;
    for (int k = 0; k < 256 / W; ++k) {
        const uint8_t v = live ? sbox_in[(size_t)s * 256 + l * (256 / W) + k] : 0;
        S[l * (256 / W) + k] = v;
        S[256 + l * (256 / W) + k] = v;
        M[l * (256 / W) + k] = 0;
    }
    const uint32_t sxy = live ? xy_in[s] : 0;
    __syncthreads();
    zrc4::WinLane w{((sxy & 0xFFu) + 1u) & 0xFFu, sxy >> 8, (1u << 8) | (255u - l), l};
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    zrc4::win_windows(w, live ? (uint32_t)N : 0u, l, (uint32_t)(uintptr_t)S, (uint32_t)(uintptr_t)M,
                      (uint32_t)(uintptr_t)R);
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    __syncthreads();
    if (live) {
        for (int k = 0; k < N / W; ++k) ks_out[(size_t)s * N + l * (N / W) + k] = R[l * (N / W) + k];
        for (int k = 0; k < 256 / W; ++k) sbox_out[(size_t)s * 256 + l * (256 / W) + k] = S[l * (256 / W) + k];
        if (l == 0) {
            xy_out[s] = (uint16_t)(((w.xa - 1) & 255) | ((w.y & 255) << 8));
            cyc[s] = t1 - t0;
            wins[s] = (w.v >> 8) - 1;
        }
    }
}

// v10: variant C (tools/ubench/win_var.hpp) (zrc4::win_windows, zsummerx_amd/csrc/zrc4_win.hpp)
// on a linear S-box layout: the tuning harness for the library kernel (the
// loop uses only the first 256 bytes of each stream's 512-byte S area).
__global__ void __launch_bounds__(64)
win11_kernel(const uint8_t *sbox_in, const uint16_t *xy_in, uint8_t *ks_out, uint8_t *sbox_out,
            uint16_t *xy_out, uint64_t *cyc, uint32_t *wins, int nstreams, int N)
{
    constexpr int W = 16, SPW = 4;
    __shared__ __attribute__((aligned(1024))) uint32_t Mk[SPW * 256];
    __shared__ __attribute__((aligned(MAXN))) uint8_t Ring[SPW * MAXN];
    __shared__ __attribute__((aligned(512))) uint8_t Sb[SPW * 512];
    const uint32_t lane = threadIdx.x, l = lane % W, g = lane / W;
    const int s = blockIdx.x * SPW + (int)g;
    const bool live = s < nstreams;
    uint8_t *S = Sb + g * 512;
    uint32_t *M = Mk + g * 256;
    uint8_t *R = Ring + g * MAXN;
    for (int k = 0; k < 256 / W; ++k) {
        const uint8_t v = live ? sbox_in[(size_t)s * 256 + l * (256 / W) + k] : 0;
        S[l * (256 / W) + k] = v;
        S[256 + l * (256 / W) + k] = v;
        M[l * (256 / W) + k] = 0;
    }
    const uint32_t sxy = live ? xy_in[s] : 0;
    __syncthreads();
    zrc4::WinLane w{((sxy & 0xFFu) + 1u) & 0xFFu, sxy >> 8, (1u << 8) | (255u - l), l};
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    zrc4::win_windows_C(w, live ? (uint32_t)N : 0u, l, (uint32_t)(uintptr_t)S, (uint32_t)(uintptr_t)M,
                      (uint32_t)(uintptr_t)R);
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    __syncthreads();
    if (live) {
        for (int k = 0; k < N / W; ++k) ks_out[(size_t)s * N + l * (N / W) + k] = R[l * (N / W) + k];
        for (int k = 0; k < 256 / W; ++k) sbox_out[(size_t)s * 256 + l * (256 / W) + k] = S[l * (256 / W) + k];
        if (l == 0) {
            xy_out[s] = (uint16_t)(((w.xa - 1) & 255) | ((w.y & 255) << 8));
            cyc[s] = t1 - t0;
            wins[s] = (w.v >> 8) - 1;
        }
    }
}

// v10: variant D (tools/ubench/win_var.hpp) (zrc4::win_windows, zsummerx_amd/csrc/zrc4_win.hpp)
// on a linear S-box layout: the tuning harness for the library kernel (the
// loop uses only the first 256 bytes of each stream's 512-byte S area).
__global__ void __launch_bounds__(64)
win12_kernel(const uint8_t *sbox_in, const uint16_t *xy_in, uint8_t *ks_out, uint8_t *sbox_out,
            uint16_t *xy_out, uint64_t *cyc, uint32_t *wins, int nstreams, int N)
{
    constexpr int W = 16, SPW = 4;
    __shared__ __attribute__((aligned(1024))) uint32_t Mk[SPW * 256];
    __shared__ __attribute__((aligned(MAXN))) uint8_t Ring[SPW * MAXN];
    __shared__ __attribute__((aligned(512))) uint8_t Sb[SPW * 512];
    const uint32_t lane = threadIdx.x, l = lane % W, g = lane / W;
    const int s = blockIdx.x * SPW + (int)g;
    const bool live = s < nstreams;
    uint8_t *S = Sb + g * 512;
    uint32_t *M = Mk + g * 256;
    uint8_t *R = Ring + g * MAXN;
    for (int k = 0; k < 256 / W; ++k) {
        const uint8_t v = live ? sbox_in[(size_t)s * 256 + l * (256 / W) + k] : 0;
        S[l * (256 / W) + k] = v;
        S[256 + l * (256 / W) + k] = v;
        M[l * (256 / W) + k] = 0;
    }
    const uint32_t sxy = live ? xy_in[s] : 0;
    __syncthreads();
    zrc4::WinLane w{((sxy & 0xFFu) + 1u) & 0xFFu, sxy >> 8, (1u << 8) | (255u - l), l};
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    zrc4::win_windows_D(w, live ? (uint32_t)N : 0u, l, (uint32_t)(uintptr_t)S, (uint32_t)(uintptr_t)M,
                      (uint32_t)(uintptr_t)R);
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    __syncthreads();
    if (live) {
        for (int k = 0; k < N / W; ++k) ks_out[(size_t)s * N + l * (N / W) + k] = R[l * (N / W) + k];
        for (int k = 0; k < 256 / W; ++k) sbox_out[(size_t)s * 256 + l * (256 / W) + k] = S[l * (256 / W) + k];
        if (l == 0) {
            xy_out[s] = (uint16_t)(((w.xa - 1) & 255) | ((w.y & 255) << 8));
            cyc[s] = t1 - t0;
            wins[s] = (w.v >> 8) - 1;
        }
    }
}

// v13: repaired windows (tools/ubench/win_repair.hpp, compiled HIP), W = 16,
// 4 streams per wave; compare with mode 1 (the product rules in compiled HIP)
// and mode 6 (the product asm loop).
__global__ void __launch_bounds__(64)
win13_kernel(const uint8_t *sbox_in, const uint16_t *xy_in, uint8_t *ks_out, uint8_t *sbox_out,
             uint16_t *xy_out, uint64_t *cyc, uint32_t *wins, int nstreams, int N)
{
    constexpr int W = 16, SPW = 4;
    __shared__ __attribute__((aligned(1024))) uint32_t Mlo[SPW * 256];
    __shared__ __attribute__((aligned(1024))) uint32_t Mhi[SPW * 256];
    __shared__ __attribute__((aligned(MAXN))) uint8_t Ring[SPW * MAXN];
    __shared__ __attribute__((aligned(256))) uint8_t Sb[SPW * 256];
    const uint32_t lane = threadIdx.x, l = lane % W, g = lane / W;
    const int s = blockIdx.x * SPW + (int)g;
    const bool live = s < nstreams;
    uint8_t *S = Sb + g * 256;
    uint8_t *R = Ring + g * MAXN;
    for (int k = 0; k < 256 / W; ++k) {
        S[l * (256 / W) + k] = live ? sbox_in[(size_t)s * 256 + l * (256 / W) + k] : 0;
        Mlo[g * 256 + l * (256 / W) + k] = 0;
        Mhi[g * 256 + l * (256 / W) + k] = 0;
    }
    const uint32_t sxy = live ? xy_in[s] : 0;
    __syncthreads();
    uint32_t xa = ((sxy & 0xFFu) + 1u) & 0xFFu, y = sxy >> 8, tag = 1, rp = 0;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    const uint32_t nw = zrc4::win_repair_windows(xa, y, tag, live ? (uint32_t)N : 0u, rp, l, S, Mlo + g * 256,
                                                 Mhi + g * 256, R, MAXN);
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    __syncthreads();
    if (live) {
        for (int k = 0; k < N / W; ++k) ks_out[(size_t)s * N + l * (N / W) + k] = R[l * (N / W) + k];
        for (int k = 0; k < 256 / W; ++k) sbox_out[(size_t)s * 256 + l * (256 / W) + k] = S[l * (256 / W) + k];
        if (l == 0) {
            xy_out[s] = (uint16_t)(((xa - 1) & 255) | ((y & 255) << 8));
            cyc[s] = t1 - t0;
            wins[s] = nw;
        }
    }
}


// v15: the product loop (zrc4::win_windows) with 2 streams per wave (lanes
// 32-63 idle), so 4 096 streams take 2 048 waves: 2 per SIMD instead of 1.
// Does a second wave on each SIMD hide the loop's LDS round trips?
__global__ void __launch_bounds__(64)
win15_kernel(const uint8_t *sbox_in, const uint16_t *xy_in, uint8_t *ks_out, uint8_t *sbox_out,
             uint16_t *xy_out, uint64_t *cyc, uint32_t *wins, int nstreams, int N)
{
    constexpr int W = 16, SPW = 4, LIVE = 2;
    __shared__ __attribute__((aligned(1024))) uint32_t Mk[SPW * 256];
    __shared__ __attribute__((aligned(MAXN))) uint8_t Ring[SPW * MAXN];
    __shared__ __attribute__((aligned(512))) uint8_t Sb[SPW * 512];
    const uint32_t lane = threadIdx.x, l = lane % W, g = lane / W;
    const int s = blockIdx.x * LIVE + (int)g;
    const bool live = g < (uint32_t)LIVE && s < nstreams;
    uint8_t *S = Sb + g * 512;
    uint32_t *M = Mk + g * 256;
    uint8_t *R = Ring + g * MAXN;
    for (int k = 0; k < 256 / W; ++k) {
        const uint8_t v = live ? sbox_in[(size_t)s * 256 + l * (256 / W) + k] : 0;
        S[l * (256 / W) + k] = v;
        S[256 + l * (256 / W) + k] = v;
        M[l * (256 / W) + k] = 0;
    }
    const uint32_t sxy = live ? xy_in[s] : 0;
    __syncthreads();
    zrc4::WinLane w{((sxy & 0xFFu) + 1u) & 0xFFu, sxy >> 8, (1u << 8) | (255u - l), l};
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    zrc4::win_windows(w, live ? (uint32_t)N : 0u, l, (uint32_t)(uintptr_t)S, (uint32_t)(uintptr_t)M,
                      (uint32_t)(uintptr_t)R);
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    __syncthreads();
    if (live) {
        for (int k = 0; k < N / W; ++k) ks_out[(size_t)s * N + l * (N / W) + k] = R[l * (N / W) + k];
        for (int k = 0; k < 256 / W; ++k) sbox_out[(size_t)s * 256 + l * (256 / W) + k] = S[l * (256 / W) + k];
        if (l == 0) {
            xy_out[s] = (uint16_t)(((w.xa - 1) & 255) | ((w.y & 255) << 8));
            cyc[s] = t1 - t0;
            wins[s] = (w.v >> 8) - 1;
        }
    }
}

// v7: one stream per wave, W = 64 (zrc4::win64_windows).
__global__ void __launch_bounds__(64)
win7_kernel(const uint8_t *sbox_in, const uint16_t *xy_in, uint8_t *ks_out, uint8_t *sbox_out,
            uint16_t *xy_out, uint64_t *cyc, uint32_t *wins, int nstreams, int N)
{
    __shared__ __attribute__((aligned(1024))) uint32_t M[256];
    __shared__ __attribute__((aligned(MAXN))) uint8_t R[MAXN];
    __shared__ __attribute__((aligned(256))) uint8_t S[256];
    const uint32_t l = threadIdx.x;
    const int s = blockIdx.x;
    for (int k = 0; k < 4; ++k) {
        S[l * 4 + k] = sbox_in[(size_t)s * 256 + l * 4 + k];
        M[l * 4 + k] = 0;
    }
    const uint32_t sxy = xy_in[s];
    __syncthreads();
    uint32_t xa = __builtin_amdgcn_readfirstlane(((sxy & 0xFFu) + 1u) & 0xFFu);
    uint32_t y = __builtin_amdgcn_readfirstlane(sxy >> 8);
    uint32_t rp = 0, v = (1u << 8) | (255u - l);
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
#ifdef ZW64_DEBUG_CAP
    uint32_t dbg[4];
    zrc4::win64_windows(xa, y, v, (uint32_t)N, rp, l, (uint32_t)(uintptr_t)S, (uint32_t)(uintptr_t)M,
                        (uint32_t)(uintptr_t)R, dbg);
    if (s == 0 && l < 12) printf("lane %u J %u maxM %x maddr %x d %u\n", l, dbg[0], dbg[1], dbg[2], dbg[3]);
#else
    zrc4::win64_windows(xa, y, v, (uint32_t)N, rp, l, (uint32_t)(uintptr_t)S, (uint32_t)(uintptr_t)M,
                        (uint32_t)(uintptr_t)R);
#endif
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    __syncthreads();
    for (int k = 0; k < N / 64; ++k) ks_out[(size_t)s * N + l * (N / 64) + k] = R[l * (N / 64) + k];
    for (int k = 0; k < 4; ++k) sbox_out[(size_t)s * 256 + l * 4 + k] = S[l * 4 + k];
    if (l == 0) {
        xy_out[s] = (uint16_t)(((xa - 1) & 255) | ((y & 255) << 8));
        cyc[s] = t1 - t0;
        wins[s] = (v >> 8) - 1;
#ifdef ZW64_DEBUG_CAP
        printf("dbg stream %d: rp(cut total) %u xa %u y %u v %x R %u %u %u %u %u %u S[188] %u M[188] %x M[76] %x M[235] %x\n", s, rp, xa, y, v,
               R[0], R[1], R[2], R[3], R[4], R[5], S[188], M[188], M[76], M[235]);
#endif
    }
}

static void ksa(uint8_t *S, const uint8_t *key, int kl)
{
    for (int i = 0; i < 256; ++i) S[i] = (uint8_t)i;
    int j = 0;
    for (int i = 0; i < 256; ++i) {
        j = (j + S[i] + (kl ? key[i % kl] : 0)) & 255;
        std::swap(S[i], S[j]);
    }
}

static void prga(uint8_t *S, uint32_t &x, uint32_t &y, uint8_t *out, int n)
{
    for (int k = 0; k < n; ++k) {
        x = (x + 1) & 255;
        const uint8_t a = S[x];
        y = (y + a) & 255;
        const uint8_t b = S[y];
        S[x] = b;
        S[y] = a;
        out[k] = S[(a + b) & 255];
    }
}

template <int W, int WPB, int V3>
static void run(int ns, int N, int reps)
{
    std::mt19937 rng(7);
    std::vector<uint8_t> sb((size_t)ns * 256), sbw((size_t)ns * 256), ksw((size_t)ns * N), tmp(4096);
    std::vector<uint16_t> xy(ns), xyw(ns);
    for (int s = 0; s < ns; ++s) {
        uint8_t key[40];
        const int kl = rng() % 40;
        for (int k = 0; k < kl; ++k) key[k] = (uint8_t)rng();
        ksa(&sb[(size_t)s * 256], key, kl);
        uint32_t x = 0, y = 0;
        prga(&sb[(size_t)s * 256], x, y, tmp.data(), rng() % 600);   // mid-stream state
        xy[s] = (uint16_t)(x | (y << 8));
        memcpy(&sbw[(size_t)s * 256], &sb[(size_t)s * 256], 256);
        prga(&sbw[(size_t)s * 256], x, y, &ksw[(size_t)s * N], N);
        xyw[s] = (uint16_t)(x | (y << 8));
    }
    uint8_t *dsb, *dks, *dsbo;
    uint16_t *dxy, *dxyo;
    uint64_t *dcyc;
    uint32_t *dwin;
    CHECK(hipMalloc(&dsb, sb.size()));
    CHECK(hipMalloc(&dsbo, sb.size()));
    CHECK(hipMalloc(&dks, ksw.size()));
    CHECK(hipMalloc(&dxy, ns * 2));
    CHECK(hipMalloc(&dxyo, ns * 2));
    CHECK(hipMalloc(&dcyc, ns * 8));
    CHECK(hipMalloc(&dwin, ns * 4));
    CHECK(hipMemcpy(dsb, sb.data(), sb.size(), hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dxy, xy.data(), ns * 2, hipMemcpyHostToDevice));
    const int blocks = (ns + WPB * (64 / W) - 1) / (WPB * (64 / W));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    std::vector<float> ms;
    for (int r = 0; r < reps; ++r) {
        CHECK(hipEventRecord(e0));
        if constexpr (V3 == 19) win19_kernel<<<(ns + 3) / 4, 64>>>(dsb, dxy, dks, dsbo, dxyo, dcyc, dwin, ns, N);
        else if constexpr (V3 == 18) win18_kernel<<<(ns + 3) / 4, 64>>>(dsb, dxy, dks, dsbo, dxyo, dcyc, dwin, ns, N);
        else if constexpr (V3 == 17) win17_kernel<<<(ns + 3) / 4, 64>>>(dsb, dxy, dks, dsbo, dxyo, dcyc, dwin, ns, N);
        else if constexpr (V3 == 16) win16_kernel<<<(ns + 3) / 4, 64>>>(dsb, dxy, dks, dsbo, dxyo, dcyc, dwin, ns, N);
        else if constexpr (V3 == 15) win15_kernel<<<(ns + 1) / 2, 64>>>(dsb, dxy, dks, dsbo, dxyo, dcyc, dwin, ns, N);
        else if constexpr (V3 == 13) win13_kernel<<<(ns + 3) / 4, 64>>>(dsb, dxy, dks, dsbo, dxyo, dcyc, dwin, ns, N);
        else if constexpr (V3 == 12) win12_kernel<<<(ns + 3) / 4, 64>>>(dsb, dxy, dks, dsbo, dxyo, dcyc, dwin, ns, N);
        else if constexpr (V3 == 11) win11_kernel<<<(ns + 3) / 4, 64>>>(dsb, dxy, dks, dsbo, dxyo, dcyc, dwin, ns, N);
        else if constexpr (V3 == 10) win10_kernel<<<(ns + 3) / 4, 64>>>(dsb, dxy, dks, dsbo, dxyo, dcyc, dwin, ns, N);
        else if constexpr (V3 == 9) win9_kernel<<<(ns + 3) / 4, 64>>>(dsb, dxy, dks, dsbo, dxyo, dcyc, dwin, ns, N);
        else if constexpr (V3 == 8) win8_kernel<<<(ns + 3) / 4, 64>>>(dsb, dxy, dks, dsbo, dxyo, dcyc, dwin, ns, N);
        else if constexpr (V3 == 7) win7_kernel<<<ns, 64>>>(dsb, dxy, dks, dsbo, dxyo, dcyc, dwin, ns, N);
        else if (V3 == 6) win6_kernel<<<(ns + 3) / 4, 64>>>(dsb, dxy, dks, dsbo, dxyo, dcyc, dwin, ns, N);
        else if (V3 == 2) win4_kernel<WPB><<<blocks, 64 * WPB>>>(dsb, dxy, dks, dsbo, dxyo, dcyc, dwin, ns, N);
        else if (V3) win3_kernel<W, WPB><<<blocks, 64 * WPB>>>(dsb, dxy, dks, dsbo, dxyo, dcyc, dwin, ns, N);
        else win_kernel<W, WPB><<<blocks, 64 * WPB>>>(dsb, dxy, dks, dsbo, dxyo, dcyc, dwin, ns, N);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float t;
        CHECK(hipEventElapsedTime(&t, e0, e1));
        ms.push_back(t);
    }
    std::vector<uint8_t> ks(ksw.size()), sbo(sb.size());
    std::vector<uint16_t> xyo(ns);
    std::vector<uint64_t> cyc(ns);
    std::vector<uint32_t> win(ns);
    CHECK(hipMemcpy(ks.data(), dks, ks.size(), hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(sbo.data(), dsbo, sbo.size(), hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(xyo.data(), dxyo, ns * 2, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(cyc.data(), dcyc, ns * 8, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(win.data(), dwin, ns * 4, hipMemcpyDeviceToHost));
    long bad_ks = 0, bad_st = 0, first = -1;
    for (size_t i = 0; i < ks.size(); ++i)
        if (ks[i] != ksw[i]) { ++bad_ks; if (first < 0) first = (long)i; }
    for (int s = 0; s < ns; ++s)
        if (memcmp(&sbo[(size_t)s * 256], &sbw[(size_t)s * 256], 256) || xyo[s] != xyw[s]) ++bad_st;
    double cs = 0, ws = 0;
    uint64_t cmax = 0;
    for (int s = 0; s < ns; ++s) { cs += (double)cyc[s]; ws += win[s]; if (cyc[s] > cmax) cmax = cyc[s]; }
    std::sort(ms.begin(), ms.end());
    printf("{\"v3\": %d, \"W\": %d, \"wpb\": %d, \"streams\": %d, \"bytes\": %d, \"bad_ks\": %ld, \"first_bad\": %ld, \"bad_state\": %ld, "
           "\"memtime_per_byte_mean\": %.2f, \"memtime_per_byte_max\": %.2f, \"bytes_per_window\": %.3f, "
           "\"kernel_ms_median\": %.4f, \"ns_per_byte\": %.2f}\n",
           V3, W, WPB, ns, N, bad_ks, first, bad_st, cs / ns / N, (double)cmax / N, (double)ns * N / ws,
           ms[ms.size() / 2], ms[ms.size() / 2] * 1e6 / N);
    (void)hipFree(dsb); (void)hipFree(dsbo); (void)hipFree(dks); (void)hipFree(dxy); (void)hipFree(dxyo); (void)hipFree(dcyc); (void)hipFree(dwin);
}

int main(int argc, char **argv)
{
    const int ns = argc > 1 ? atoi(argv[1]) : 4096;
    const int N = argc > 2 ? atoi(argv[2]) : 1024;
    const int w = argc > 3 ? atoi(argv[3]) : 16;
    const int wpb = argc > 4 ? atoi(argv[4]) : 1;
    if (N > MAXN || N % 16) { printf("bytes must be a multiple of 16 and <= %d\n", MAXN); return 1; }
    const int v3 = argc > 5 ? atoi(argv[5]) : 1;
    if (v3 == 19) run<16, 1, 19>(ns, N, 20);
    else if (v3 == 18) run<16, 1, 18>(ns, N, 20);
    else if (v3 == 17) run<16, 1, 17>(ns, N, 20);
    else if (v3 == 16) run<16, 1, 16>(ns, N, 20);
    else if (v3 == 15) run<16, 1, 15>(ns, N, 20);
    else if (v3 == 13) run<16, 1, 13>(ns, N, 20);
    else if (v3 == 12) run<16, 1, 12>(ns, N, 20);
    else if (v3 == 11) run<16, 1, 11>(ns, N, 20);
    else if (v3 == 10) run<16, 1, 10>(ns, N, 20);
    else if (v3 == 9) run<16, 1, 9>(ns, N, 20);
    else if (v3 == 8) run<16, 1, 8>(ns, N, 20);
    else if (v3 == 7) run<64, 1, 7>(ns, N, 20);
    else if (v3 == 6) run<16, 1, 6>(ns, N, 20);
    else if (v3 == 2) { if (wpb == 1) run<16, 1, 2>(ns, N, 20); else run<16, 2, 2>(ns, N, 20); }
    else if (v3) { if (w == 8) run<8, 1, 1>(ns, N, 20); else if (wpb == 1) run<16, 1, 1>(ns, N, 20); else run<16, 2, 1>(ns, N, 20); }
    else if (w == 8) { if (wpb == 1) run<8, 1, 0>(ns, N, 20); else run<8, 2, 0>(ns, N, 20); }
    else { if (wpb == 1) run<16, 1, 0>(ns, N, 20); else run<16, 2, 0>(ns, N, 20); }
    return 0;
}
