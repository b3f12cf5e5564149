// win_repair.hpp -- A/B only (tools/ubench/win_ubench.hip modes 13 / 14):
// speculative RC4 windows that REPAIR stale b reads instead of cutting at
// them (tools/window_repair_sim.py states the rules and checks them against a
// plain PRGA).  Reference PRGA: depends/rc4/rc4_encryption.h:81-89.
//
// W = 16 lanes per stream, 4 streams per wave, compiled HIP (builtins for
// the DPP scans and ds_bpermute), so it is compared against mode 1 (win3,
// the same product rules in compiled HIP) and mode 6 (the product asm loop).
// Per window, lane l of a stream (x = window-start x + 1 + l - 1):
//   i_l = x+1+l, a_l = S0[i_l], J_l = y + a_0 + .. + a_l, b_l = S0[J_l]
//   Mlo / Mhi: ds_max of (tag << 8 | 255 - l) and (tag << 8 | l) at J_l:
//              the lowest / highest lane whose j is J_l
//   dup_l = Mlo[J_l] < l     (an earlier lane's j is my j: b_l = a_lo)
//   dr_l  = d_l < l          (d_l = J_l - x - 1: b_l = the true b of lane d_l)
//   cut at the first lane l with: l >= rem; a stale a (lane k < l with
//   J_k = i_l, posted by lane k as bit d_k when k < d_k < W); the middle of
//   three equal j's (Mlo < l < Mhi); a d-repair whose source lane was itself
//   repaired (bit d_l of the stream's repaired-lane mask).
//   true b: bt_l = dup ? a_lo : dr ? bt1_{d_l} : b_l  (bt1 = after the dup repair)
//   commit: S[i_l] = bt_l, then S[J_l] = a_l by the last committed writer of J_l
//   keystream of lane l (t_l = a_l + bt_l): a of the highest / lowest lane
//   <= l whose j is t_l, else bt of lane t_l - x - 1 if <= l, else S0[t_l]
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace zrc4 {

// inclusive prefix sum over the 16 lanes of a DPP row
__device__ __forceinline__ uint32_t row_scan16(uint32_t v)
{
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);   // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);   // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);   // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);   // row_shr:8
    return v;
}

// OR over the 16 lanes of a row
__device__ __forceinline__ uint32_t row_or16(uint32_t v)
{
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);    // quad_perm [1,0,3,2]
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);    // quad_perm [2,3,0,1]
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);   // row_half_mirror
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false);   // row_mirror
    return v;
}

// value of lane src (0..15) of this lane's row
__device__ __forceinline__ uint32_t row_pull(uint32_t v, uint32_t row_base, uint32_t src)
{
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)((row_base + src) << 2), (int)v);
}

// Windows until `rem` bytes are consumed (rem equal inside a stream's 16
// lanes; 0 = idle).  S: the stream's 256-byte S-box (256-aligned), Mlo / Mhi:
// 256-entry marker tables (zeroed before the first call, tags from w.v >> 8),
// R: keystream ring of `ring` bytes (power of two).  Returns windows run.
__device__ __forceinline__ uint32_t win_repair_windows(uint32_t &xa, uint32_t &y, uint32_t &tag, uint32_t rem,
                                                       uint32_t &rp, uint32_t l, uint8_t *S, uint32_t *Mlo,
                                                       uint32_t *Mhi, uint8_t *R, uint32_t ring)
{
    constexpr uint32_t W = 16;
    const uint32_t row_base = (threadIdx.x & 63u) & ~15u;
    uint32_t nw = 0;
    while (__builtin_amdgcn_ballot_w64(rem != 0u)) {
        nw += rem != 0u;
        const uint32_t vlo = (tag << 8) | (255u - l), vhi = (tag << 8) | l;
        const uint32_t i = (xa + l) & 255u;
        const uint32_t a = S[i];
        const uint32_t J = (y + row_scan16(a)) & 255u;
        const uint32_t b = S[J];
        atomicMax(&Mlo[J], vlo);
        atomicMax(&Mhi[J], vhi);
        const uint32_t mlo = __hip_atomic_load(&Mlo[J], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const uint32_t mhi = __hip_atomic_load(&Mhi[J], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const uint32_t lo = 255u - (mlo & 255u), hi = mhi & 255u;
        const uint32_t d = (J - xa) & 255u;
        const bool dup = lo < l, dr = d < l;
        const uint32_t repm = row_or16((dup || dr) ? (1u << l) : 0u);
        const bool mid3 = lo < l && l < hi;
        const bool chain = dr && !dup && ((repm >> d) & 1u);
        uint32_t oh = (l < d && d < W) ? (1u << d) : 0u;
        if (mid3 || chain) oh |= 1u << l;
        oh = row_or16(oh | (1u << W));
        uint32_t cut = (uint32_t)__builtin_ctz(oh);
        cut = cut < rem ? cut : rem;
        // true b: the dup repair, then the d repair from the source lane
        const uint32_t alo = row_pull(a, row_base, lo);
        const uint32_t bt1 = dup ? alo : b;
        const uint32_t bsrc = row_pull(bt1, row_base, dr ? d & 15u : l);
        const uint32_t bt = (dr && !dup) ? bsrc : bt1;
        // keystream: the last write <= l to t, else S0[t] (read before the commit)
        const uint32_t t = (a + bt) & 255u;
        const uint32_t k0 = S[t];
        const uint32_t tlo_r = Mlo[t], thi_r = Mhi[t];
        const uint32_t tlo = (tlo_r >> 8) == tag ? 255u - (tlo_r & 255u) : W;
        const uint32_t thi = (thi_r >> 8) == tag ? (thi_r & 255u) : W;
        const uint32_t e = (t - xa) & 255u;
        const bool jw = thi <= l || tlo <= l;
        const uint32_t src = thi <= l ? thi : (tlo <= l ? tlo : (e <= l ? e : l));
        const uint32_t pk = row_pull(a | (bt << 8), row_base, src & 15u);
        const uint32_t ks = jw ? (pk & 255u) : (e <= l ? (pk >> 8) & 255u : k0);
        // (one wave: LDS ops retire in program order, so the S0 reads above
        // precede the commit, and the i-writes precede the J-writes)
        if (l < cut) S[i] = (uint8_t)bt;
        if (l < cut && (hi == l || hi >= cut)) S[J] = (uint8_t)a;
        if (l < cut) R[(rp + l) & (ring - 1u)] = (uint8_t)ks;
        // y' = J of the last committed lane, x += cut
        const uint32_t yl = __builtin_amdgcn_ds_bpermute((int)((row_base + (cut ? cut - 1u : 0u)) << 2), (int)J);
        y = cut ? (yl & 255u) : y;
        xa = (xa + cut) & 255u;
        rp += cut;
        rem -= cut;
        tag += 1u;
    }
    return nw;
}

}  // namespace zrc4
