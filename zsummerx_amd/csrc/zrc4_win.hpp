// zrc4_win.hpp -- lane-parallel speculative RC4 windows for chain-bound launches.
//
// Reference: /root/reference/depends/rc4/rc4_encryption.h:81-89 (the PRGA).
//
// The lane-per-stream kernels (zrc4_kernels.hpp) run one PRGA step per lane
// per ~96 cycles: one LDS round trip plus the step's issue.  A launch with few
// sessions (4 096 x 1 KiB = 16 groups, 1 024 x 64 KiB = 4 groups) leaves most
// of the chip idle at that per-stream rate.  Here W = 16 lanes run one stream:
// each lane takes one step of a window of 16 from the window-start state, and
// the window commits the longest prefix that provably equals the serial order
// (tools/window_sim.py states and checks the rules):
//
//   i_l = x+1+l, a_l = S0[i_l], j_l = y + a_0 + .. + a_l, b_l = S0[j_l],
//   d_l = (j_l - x - 1) mod 256
//   d_l < l           -> b_l read a byte an earlier step swapped   -> cut <= l
//   l < d_l < 16      -> step l swaps a later step's i              -> cut <= d_l
//   j_k == j_l, k < l -> b_l read a byte step k swapped             -> cut <= l
//
// Committed steps touch pairwise distinct bytes, so their swaps are written in
// parallel; keystream byte l is S_final[t_l] if a committed step <= l wrote
// t_l = a_l + b_l, else S0[t_l].  About 10 bytes commit per window.
//
// One 64-thread workgroup = one wave = 4 streams x 16 lanes.  Per stream in
// LDS: the S-box (256-aligned, so S[(x + 1 + l) mod 256] and S[(a + b) mod
// 256] are one SDWA byte add into a register holding the base), a 256-entry
// marker table
// (ds_max of (window tag << 8) | (255 - l): the read-back names the lowest lane
// whose j hit that byte this window -> the duplicate-j rule and the keystream
// rule), and a keystream ring of kWinRing bytes.  Payload is XORed from the
// ring per chunk of kWinRing bytes, loads issued a chunk ahead.
//
// Arena access: the 4 streams of a workgroup are the 4 slots whose S-box
// bytes share one dword of every image row (col bits 0-1 = lane >> 5,
// wave & 1, see col_of), so the state moves as 256 aligned dword loads and
// stores per workgroup: group-lanes 128h + L + 32b, b = 0..3, for dword
// column q = 32h + L.
#pragma once
#include "zrc4_kernels.hpp"

namespace zrc4 {

constexpr uint32_t kWinLanes = 16;           // W: lanes (steps) per stream window
constexpr uint32_t kWinStreams = 4;          // streams per wave / workgroup
constexpr uint32_t kWinRing = 2048;          // keystream chunk per stream (bytes)
constexpr uint32_t kWinUnits = kWinRing / 16 / kWinLanes;   // 16-byte payload units per lane per chunk
#ifndef ZRC4_WIN_TAG_LIMIT
#define ZRC4_WIN_TAG_LIMIT (1u << 23)
#endif
constexpr uint32_t kWinTagLimit = ZRC4_WIN_TAG_LIMIT;      // marker tags restart past this (24-bit field)

struct WinLane {
    uint32_t xa;     // x + 1 (byte)
    uint32_t y;      // y (byte)
    uint32_t v;      // marker value: window tag << 8 | (255 - l)
    uint32_t rp;     // stream position + l (ring slot before masking)
};

// Windows until every stream of the wave has consumed `rem` bytes (rem is per
// lane, equal inside a stream's 16 lanes; 0 = idle).  One asm statement; the
// loop is rotated so that window n+1's read leaves right behind window n's
// commit writes.  Per iteration n (a_l of window n already in flight):
//   1. two DPP chains interleaved step for step, so neither needs an s_nop:
//      the inclusive scan of a over the stream's 16 lanes (row_shr 1, 2, 4,
//      8: J_l = y + a_0 + .. + a_l; step 1 reads the a_l load directly, zero
//      at row starts) and window n-1's y' = J of its last committed lane (max
//      over the 16 lanes of (l + 1) << 8 | J, else the old y); window n-1's
//      keystream select (S_final if a committed step <= l wrote t, else S0)
//      in the last slots;
//   2. b_l = S0[J_l] and the marker max / read-back issue, window n-1's ring
//      store behind them (not waited for); under that round trip the d rule (one-hot of med3(d, l, 16), none when d == l), the
//      rem cap (bit min(rem, 16)) and the same one-hot plus bit l for a
//      duplicate j;
//   3. the duplicate-j rule (a select), DPP OR over the 16 lanes with the
//      keystream address work and S0[t] read in the DPP wait slots, cut =
//      lowest bit, window n+1's a_l address = this one's plus cut (SDWA byte
//      add into the base register);
//   4. commit (2 byte writes) under exec = lanes < cut, window n+1's a_l
//      read, S_final[t] and marker(t) reads, then x, rem, the ring position
//      and the commit mask under that round trip.
// Every DPP read of a VGPR sits at least two VALU ops (or an s_nop) after the
// VALU write of it.  Pinned temporaries v106-v131, s[40:47].
// (v_dot4_u32_u8 prefix sums over the window bytes were tried: the dot4
// accumulator chain read stale values on MI355X -- bit-exact only because the
// wrong j always tripped the duplicate rule -- and the DPP scan needs no
// window bytes at all.)
// ZRC4_WIN_SDWA (A/B only): the masks of J, d and x + 1 folded into SDWA
// byte writes (3 instructions less per window; tools/ubench win_var3.hpp).
#ifndef ZRC4_WIN_SDWA
#define ZRC4_WIN_SDWA 0
#endif
// ZRC4_WIN_ALIGN (A/B only): the loop head aligned to 2^N bytes (s_nop padding
// before it, run once); 0 = no directive (the default ISA).
#ifndef ZRC4_WIN_ALIGN
#define ZRC4_WIN_ALIGN 0
#endif
#define ZW_STR2(x) #x
#define ZW_STR(x) ZW_STR2(x)
#if ZRC4_WIN_ALIGN
#define ZW_LOOP_ALIGN ".p2align " ZW_STR(ZRC4_WIN_ALIGN) "\n\t"
#else
#define ZW_LOOP_ALIGN ""
#endif
#define ZW_ADDR(XA)                                                                               \
    "v_add_u32_sdwa v106, " XA ", %[l] dst_sel:BYTE_0 dst_unused:UNUSED_PRESERVE src0_sel:DWORD "  \
    "src1_sel:DWORD\n\t"
__device__ __forceinline__ void win_windows(WinLane &w, uint32_t rem, uint32_t l, uint32_t sb, uint32_t mb,
                                            uint32_t rb)
{
    const uint32_t bitl = 1u << l, l1 = (l + 1) << 8;
    asm volatile(
        "s_mov_b64 s[46:47], 0\n\t"                             // no window n-1 yet: empty commit mask
        "v_and_b32 v120, 0xff, %[y]\n\t"
        "s_mov_b64 s[44:45], 0\n\t"
        "v_mov_b32 v123, 0\n\t"
        "v_mov_b32 v106, %[sb]\n\t"                              // S base (256-aligned) in bytes 1-3
        "v_mov_b32 v126, %[sb]\n\t"
        ZW_ADDR("%[xa]")
        "ds_read_u8 v107, v106\n\t"                             // a_l of window 0
        ZW_LOOP_ALIGN
        "ZW_LOOP_%=:\n\t"
        // 1. scan of a, tail of window n-1
        "s_waitcnt lgkmcnt(0)\n\t"
        "v_add_u32_dpp v112, v107, v107 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_max_u32_dpp v120, v120, v120 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_cmp_ge_u32_e64 s[42:43], v123, %[v]\n\t"
        "v_add_u32_dpp v112, v112, v112 row_shr:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_max_u32_dpp v120, v120, v120 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "v_add_u32 %[v], 0x100, %[v]\n\t"
        "v_add_u32_dpp v112, v112, v112 row_shr:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_max_u32_dpp v120, v120, v120 row_half_mirror row_mask:0xf bank_mask:0xf\n\t"
        "s_or_b64 s[42:43], s[42:43], s[44:45]\n\t"
        "v_cndmask_b32_e64 v124, v121, v122, s[42:43]\n\t"
        "v_add_u32_dpp v112, v112, v112 row_shr:8 row_mask:0xf bank_mask:0xf\n\t"
        "v_max_u32_dpp v120, v120, v120 row_mirror row_mask:0xf bank_mask:0xf\n\t"
#if ZRC4_WIN_SDWA
        "v_add_u32_sdwa v112, v112, v120 dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0\n\t"   // J = scan + y' (mod 256)
        // 2. b / marker round trip, d rule and rem cap under it
        "v_and_b32 %[y], 0xff, v120\n\t"                      // (one op between the SDWA byte write and its readers)
        "v_add_u32 v114, %[sb], v112\n\t"
#else
        "v_add_u32 v112, v112, v120\n\t"                       // + y' (byte 0 of v120; J is masked below)
        // 2. b / marker round trip, d rule and rem cap under it
        "v_add_u32_sdwa v114, %[sb], v112 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0\n\t"
        "v_and_b32 v112, 0xff, v112\n\t"                       // J
#endif
        "v_lshl_add_u32 v115, v112, 2, %[mb]\n\t"
        "ds_read_u8 v116, v114\n\t"                             // b_l = S0[J]
        "ds_max_u32 v115, %[v]\n\t"
        "ds_read_b32 v117, v115\n\t"                            // lowest lane with this J
        "s_mov_b64 s[40:41], exec\n\t"
        "s_mov_b64 exec, s[46:47]\n\t"
        "ds_write_b8 v125, v124\n\t"                            // window n-1's ring store, behind the round trip
        "s_mov_b64 exec, s[40:41]\n\t"
#if ZRC4_WIN_SDWA
        "v_sub_u32_sdwa v118, v112, %[xa] dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:DWORD\n\t"   // d
        "v_or_b32 v130, %[l1], v112\n\t"                        // y' candidate of this lane (between)
#else
        "v_and_b32 %[y], 0xff, v120\n\t"
        "v_sub_u32 v118, v112, %[xa]\n\t"
        "v_and_b32 v118, 0xff, v118\n\t"                       // d
#endif
        "v_med3_u32 v119, v118, %[l], 16\n\t"
        "v_cmp_ne_u32 vcc, v118, %[l]\n\t"
        "v_cndmask_b32 v119, 16, v119, vcc\n\t"
        "v_lshlrev_b32 v118, v119, 1\n\t"                       // bit 16 = no d conflict
        "v_min_u32 v119, 16, %[rem]\n\t"
        "v_lshlrev_b32 v119, v119, 1\n\t"
        "v_or_b32 v118, v118, v119\n\t"                        // + bit min(rem, 16): cut <= rem
        "v_or_b32 v119, v118, %[bitl]\n\t"                     // the same if this lane's J repeats
#if !ZRC4_WIN_SDWA
        "v_or_b32 v130, %[l1], v112\n\t"                        // y' candidate of this lane
#endif
        "v_bfi_b32 v125, %[rmask], %[rp], %[rb]\n\t"            // ring slot of this lane
        "s_waitcnt lgkmcnt(1)\n\t"
        // 3. duplicate-J rule, OR over the stream's 16 lanes, cut
        "v_cmp_ne_u32 vcc, v117, %[v]\n\t"
        "v_cndmask_b32 v118, v118, v119, vcc\n\t"
        "v_add_u32_sdwa v126, v107, v116 dst_sel:BYTE_0 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n\t"   // &S[t]
        "v_add_u32 v128, v107, v116\n\t"
        "ds_read_u8 v121, v126\n\t"                             // S0[t]
        "v_or_b32_dpp v118, v118, v118 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_sub_u32 v131, v128, %[xa]\n\t"
        "v_and_b32 v128, 0xff, v128\n\t"                       // t
        "v_or_b32_dpp v118, v118, v118 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "v_and_b32 v131, 0xff, v131\n\t"                       // e = t - x - 1
        "v_lshl_add_u32 v129, v128, 2, %[mb]\n\t"
        "v_or_b32_dpp v118, v118, v118 row_half_mirror row_mask:0xf bank_mask:0xf\n\t"
        "v_cmp_le_u32_e64 s[44:45], v131, %[l]\n\t"             // t is the i of a step <= l
        "v_mov_b32 v131, v106\n\t"                              // &S[i_l] of window n
        "v_or_b32_dpp v118, v118, v118 row_mirror row_mask:0xf bank_mask:0xf\n\t"
        "v_ffbl_b32 v118, v118\n\t"                             // cut
        "v_cmp_lt_u32 vcc, %[l], v118\n\t"
        "v_add_u32_sdwa v106, v106, v118 dst_sel:BYTE_0 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0 src1_sel:DWORD\n\t"   // window n+1's a_l address
        // 4. commit, then window n+1's read right behind it
        "s_and_saveexec_b64 s[40:41], vcc\n\t"
        "ds_write_b8 v131, v116\n\t"                            // S[i_l] = b_l
        "ds_write_b8 v114, v107\n\t"                            // S[J_l] = a_l
        "s_mov_b64 exec, s[40:41]\n\t"
        "ds_read_u8 v107, v106\n\t"                             // a_l of window n+1
        "ds_read_u8 v122, v126\n\t"                             // S_final[t]
        "ds_read_b32 v123, v129\n\t"                            // lowest lane whose J == t
        "s_and_b64 s[46:47], vcc, s[40:41]\n\t"                 // commit mask (ring store next iteration)
        "v_cndmask_b32 v120, %[y], v130, vcc\n\t"
#if ZRC4_WIN_SDWA
        "v_add_u32_sdwa %[xa], %[xa], v118 dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:DWORD\n\t"
#else
        "v_add_u32 %[xa], %[xa], v118\n\t"
        "v_and_b32 %[xa], 0xff, %[xa]\n\t"
#endif
        "v_sub_u32 %[rem], %[rem], v118\n\t"
        "v_add_u32 %[rp], %[rp], v118\n\t"
        "v_cmp_ne_u32 vcc, 0, %[rem]\n\t"
        "s_cbranch_vccnz ZW_LOOP_%=\n\t"
        // drain: tail of the last window (window n's read is harmless)
        "s_waitcnt lgkmcnt(0)\n\t"
        "v_max_u32_dpp v120, v120, v120 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_cmp_ge_u32_e64 s[42:43], v123, %[v]\n\t"
        "s_or_b64 s[42:43], s[42:43], s[44:45]\n\t"
        "v_cndmask_b32_e64 v124, v121, v122, s[42:43]\n\t"
        "v_max_u32_dpp v120, v120, v120 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_max_u32_dpp v120, v120, v120 row_half_mirror row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_max_u32_dpp v120, v120, v120 row_mirror row_mask:0xf bank_mask:0xf\n\t"
        "s_mov_b64 s[40:41], exec\n\t"
        "s_mov_b64 exec, s[46:47]\n\t"
        "ds_write_b8 v125, v124\n\t"
        "s_mov_b64 exec, s[40:41]\n\t"
        "v_and_b32 %[y], 0xff, v120\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        : [xa] "+v"(w.xa), [y] "+v"(w.y), [v] "+v"(w.v), [rem] "+v"(rem), [rp] "+v"(w.rp)
        : [l] "v"(l), [sb] "v"(sb), [mb] "v"(mb), [rb] "v"(rb), [bitl] "v"(bitl), [l1] "v"(l1),
          [rmask] "s"(kWinRing - 1)
        : "memory", "vcc", "scc", "v106", "v107", "v112", "v114", "v115", "v116", "v117", "v118", "v119", "v120",
          "v121", "v122", "v123", "v124", "v125", "v126", "v128", "v129", "v130", "v131", "s40", "s41",
          "s42", "s43", "s44", "s45", "s46", "s47");
}

// Declared bucket groups of a grouped window launch (zrc4_crypt_grouped_declared):
// bucket b's group, or ZRC4_INVALID for a bucket with no busy entry.  Passed
// by value, so it sits in the kernel-argument segment and is read with the
// launch's other arguments: no dependent memory round trip before the image.
constexpr uint32_t kWinMaxBuckets = 32;      // == ZRC4_WIN_MAX_GROUPS
struct WinGroups {
    uint32_t g[kWinMaxBuckets];
};

// Chain-bound launches with few groups: grid = 64 x groups (range batches
// with first_slot % 256 == 0) or 64 x buckets (grouped batches) workgroups of
// one wave.
//   kRange:   stream b of dword column q is entry g*256 + 128h + L + 32b.
//   kGrouped: every workgroup reads its bucket's 256 entries, checks the
//             bucket contract as crypt_kernel<kGrouped> does (one group, no
//             slot twice; else kErrGroup and the bucket is skipped whole) and
//             builds slot -> entry, length, offset tables in LDS (in the ring,
//             before the ring is used); the image load is issued from the
//             first busy id's group ahead of the table build.
//   DECL:     (kGrouped) the bucket's group comes from the caller (WinGroups):
//             the image, x/y and claim are issued at entry, beside the
//             bucket's entries, and a busy entry outside the declared group
//             refuses the bucket (kErrGroup) exactly as a mixed bucket is.
//   FRAME:    onRecv's framing walk (frame_walk, §8f row 4) of every entry in
//             the same launch: a stream's entry by its lane 0 once the
//             stream's bytes are decrypted; grouped entries that decrypt
//             nothing (idle ids, length 0, idle buckets) by lane q of the
//             bucket's workgroup q (entries q + 64r), on the raw bytes.
template <int MODE, bool FRAME, bool DECL = false>
__global__ void __launch_bounds__(64)
crypt_win_kernel(uint8_t *__restrict__ arena, uint16_t *__restrict__ xy, const uint32_t *__restrict__ ids,
                 uint32_t first_slot, uint8_t *__restrict__ payload, const uint64_t *__restrict__ off,
                 const uint32_t *__restrict__ len, uint32_t n, uint32_t capacity, uint32_t *__restrict__ err,
                 uint8_t *__restrict__ sink, FrameArgs fr, Claim cl, WinGroups dg = WinGroups{})
{
    Stamps ts;                                   // ZRC4_TIMING builds only (zrc4_kernels.hpp)
    stamp(ts, 0);
    __shared__ __attribute__((aligned(1024))) uint32_t Mk[kWinStreams * 256];
    __shared__ __attribute__((aligned(kWinRing))) uint8_t Ring[kWinStreams * kWinRing];
    __shared__ __attribute__((aligned(256))) uint8_t Sb[kWinStreams * 256];

    // workgroup k runs on XCD k mod 8.  With a multiple of 8 groups, all 64
    // columns of a group sit on one XCD (its image lines fill one L2);
    // otherwise the 8 columns an XCD takes from each group are adjacent.
    const uint32_t k = blockIdx.x, xcd = k & 7u, idx = k >> 3;
    const bool local = ((gridDim.x >> 6) & 7u) == 0u;
    const uint32_t q = local ? (idx & 63u) : ((idx & 7u) | (xcd << 3));
    const uint32_t wg = local ? (((idx >> 6) << 3) | xcd) : (idx >> 3);   // group (kRange) or bucket (kGrouped)
    const uint32_t lane = threadIdx.x, l = lane & 15u, b = lane >> 4;
    const uint32_t kb = ((q >> 5) << 7) + (q & 31u) + 32u * b;             // group-lane of this lane's stream
    uint32_t slot, L = 0, ent = 0;                                         // ent: this stream's batch entry
    uint64_t O = 0;
    bool valid;
    uint32_t rows[4];
    uint32_t sxy, sxy_g;                                                   // sxy_g: kGrouped's x/y on the guess
    unsigned long long cold = 0;                                           // kGrouped: the claim of column q (Claim)
    uint32_t gclaim = 0;                                                   // kGrouped: the group claimed
    bool bad = false;                                                      // kGrouped: the bucket breaks the contract
    if constexpr (MODE == kRange) {
        const uint32_t e = wg * kGroup + kb;
        ent = e;
        slot = first_slot + e;
        valid = e < n;
        if (!__builtin_amdgcn_ballot_w64(valid)) return;                      // whole dword column idle
        const uint8_t *img = arena + (size_t)(slot >> 8) * kGroupBytes + 4u * q;
#pragma unroll
        for (int r = 0; r < 4; ++r)
            rows[r] = *reinterpret_cast<const uint32_t *>(img + (size_t)(lane + 64u * r) * 256u);
        if (valid) {
            L = len[e];
            O = off[e];
        }
        sxy = valid ? xy[slot] : 0u;
    } else {
        uint32_t *te = reinterpret_cast<uint32_t *>(Ring);                    // slot & 255 -> entry
        uint32_t *tl = te + 256;                                              // length
        uint64_t *to = reinterpret_cast<uint64_t *>(Ring + 2048);             // offset
        uint32_t *fl = reinterpret_cast<uint32_t *>(Ring + 4096);             // 256-bit seen map, bad flag
        uint32_t idq[4], lq[4];
        uint64_t oq[4];
        bool bq[4];
        uint32_t gw = ZRC4_INVALID;
        // all twelve entry loads first, the checks after (a check inside the
        // load loop would wait for every load issued before it)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t e = wg * kGroup + lane + 64u * r;
            const bool v = e < n;
            idq[r] = v ? ids[e] : ZRC4_INVALID;
            lq[r] = v ? len[e] : 0u;
            oq[r] = v ? off[e] : 0u;
        }
        if constexpr (DECL) {
            // the declared group: image, x/y and claim leave right behind the
            // entries, in the same round trip (without it they wait for the
            // entries' ids); the entry checks wait for the entries only, and
            // the claim (asm, uncounted by the compiler) for nothing before
            // the first XOR pass
            // (an idle bucket reads group 0's image and drops it: loads on
            // every path keep the compiler's counted waits exact)
            gw = dg.g[wg];
            const uint32_t gl = gw != ZRC4_INVALID ? gw : 0u;
            const uint8_t *img = arena + (size_t)gl * kGroupBytes + 4u * q;
#pragma unroll
            for (int r = 0; r < 4; ++r)
                rows[r] = *reinterpret_cast<const uint32_t *>(img + (size_t)(lane + 64u * r) * 256u);
            sxy_g = xy[gl * 256u + kb];
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) te[lane + 64u * r] = ZRC4_INVALID;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            if (idq[r] >= capacity && idq[r] != ZRC4_INVALID) {             // ZRC4_IDLE_SLOT pads buckets
                latch_fault(err, kErrSlotRange);
                idq[r] = ZRC4_INVALID;
            }
            bq[r] = idq[r] != ZRC4_INVALID && lq[r] != 0u;
        }
        if (lane < 9) fl[lane] = 0u;
        if constexpr (!DECL) {
#pragma unroll
            for (int r = 3; r >= 0; --r) {
                const uint64_t bm = __builtin_amdgcn_ballot_w64(bq[r]);
                if (bm) gw = __builtin_amdgcn_readlane(idq[r], (int)__builtin_ctzll(bm)) >> 8;
            }
        }
        if constexpr (FRAME) {                        // entries that decrypt nothing: raw framing
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const uint32_t e = wg * kGroup + lane + 64u * r;
                if (lane == q && e < n && !bq[r])
                    frame_walk(payload + fr.off[e], fr.len[e], fr.bound, fr.maxp, e, fr.npk, fr.used, fr.status,
                               fr.pkt_len);
            }
        }
        if (gw == ZRC4_INVALID) {                                             // idle bucket
            if constexpr (DECL) {                                             // declared idle, yet a busy entry: refused
                const bool busy = __builtin_amdgcn_ballot_w64(bq[0] | bq[1] | bq[2] | bq[3]) != 0ull;
                if (busy && q == 0u && lane == 0) latch_fault(err, kErrGroup);
            }
            return;
        }
        if constexpr (!DECL) {
            gw = __builtin_amdgcn_readfirstlane(gw);
            const uint8_t *img = arena + (size_t)gw * kGroupBytes + 4u * q;  // speculative: the first busy id's group
#pragma unroll
            for (int r = 0; r < 4; ++r)
                rows[r] = *reinterpret_cast<const uint32_t *>(img + (size_t)(lane + 64u * r) * 256u);
            // x/y of the stream on the same guess (no round trip after the table build)
            sxy_g = xy[gw * 256u + kb];
        }
        gclaim = gw;
        __syncthreads();
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            if (bq[r]) {
                const uint32_t kk = idq[r] & 255u;
                if ((idq[r] >> 8) != gw) fl[8] = 1u;                                     // another group
                if (atomicOr(&fl[kk >> 5], 1u << (kk & 31u)) & (1u << (kk & 31u))) fl[8] = 1u;   // a slot twice
                te[kk] = wg * kGroup + lane + 64u * r;
                tl[kk] = lq[r];
                to[kk] = oq[r];
            }
        }
        __syncthreads();
        slot = gw * 256u + kb;
        ent = te[kb];
        valid = ent != ZRC4_INVALID;
        if (valid) {
            L = tl[kb];
            O = to[kb];
        }
        bad = fl[8] != 0u;
    }
    uint8_t *img = arena + (size_t)(slot >> 8) * kGroupBytes + 4u * q;
    uint8_t *msg = payload + O;
    const bool aligned = ((uintptr_t)msg & 15u) == 0u;

    // The S-boxes into LDS (the wave's 4 streams share every dword of the
    // image column) and the markers cleared.  kGrouped: before the payload
    // prefetch, whose addresses come from the slot table (a second round
    // trip): with the prefetch issued first, the compiler's wait for the
    // image column (older, on a path the per-lane prefetch branches join)
    // drained the prefetch too, a round trip on the way to the first window
    // (r05 timeline: prologue 3.84 vs 2.24 us range, profiles/r05/tl1/).
#define ZRC4_WIN_FILL                                                                       \
    do {                                                                                    \
        _Pragma("unroll") for (int r = 0; r < 4; ++r) {                                     \
            const uint32_t kk = lane + 64u * r;                                             \
            _Pragma("unroll") for (uint32_t s4 = 0; s4 < 4; ++s4) {                         \
                const uint8_t v = (uint8_t)(rows[r] >> (8 * s4));                           \
                Sb[s4 * 256u + kk] = v;                                                     \
            }                                                                               \
        }                                                                                   \
        _Pragma("unroll") for (int i = 0; i < 4; ++i)                                       \
            reinterpret_cast<uint4 *>(Mk)[lane + 64 * i] = make_uint4(0, 0, 0, 0);         \
    } while (0)
    if constexpr (MODE == kGrouped) {
        if (bad) {
            claim_wait(cold);                                                 // (no load left in flight at exit)
            if (lane == 0) latch_fault(err, kErrGroup);
            return;
        }
        sxy = valid ? sxy_g : 0u;
        if (!__builtin_amdgcn_ballot_w64(valid)) {
            claim_wait(cold);
            return;
        }
        ZRC4_WIN_FILL;
    }

    // payload prefetch of chunk 0 (aligned messages: whole 16-byte units).
    // kGrouped: issued before the claim's answer is waited for (reads of the
    // caller's entries only; a refused bucket drops them), on every lane
    // (units past the message read the lane's sink bytes) so that the
    // compiler's wait for x/y below counts exactly and leaves the claim --
    // issued right after, from asm -- in flight until the first XOR pass.
    uint4 pre[kWinUnits];
#pragma unroll
    for (uint32_t u = 0; u < kWinUnits; ++u) {
        const uint32_t pos = 16u * (l + kWinLanes * u);
        if constexpr (MODE == kGrouped)
            pre[u] = *reinterpret_cast<const uint4 *>(aligned && pos + 16u <= L ? msg + pos : sink + 16u * lane);
        else if (aligned && pos + 16u <= L)
            pre[u] = *reinterpret_cast<const uint4 *>(msg + pos);
    }
    if constexpr (MODE == kGrouped) cold = claim_part_async(cl, gclaim, q, wg);

    uint8_t *S = Sb + b * 256u;
    uint32_t *M = Mk + b * 256u;
    uint8_t *R = Ring + b * kWinRing;
    if constexpr (MODE != kGrouped) ZRC4_WIN_FILL;
#undef ZRC4_WIN_FILL
    __syncthreads();                                 // (grouped: also the tables read before the ring is used)
    stamp(ts, 1);

    const uint32_t sb = (uint32_t)(uintptr_t)S, mb = (uint32_t)(uintptr_t)M, rb = (uint32_t)(uintptr_t)R;
    WinLane w{((sxy & 0xFFu) + 1u) & 0xFFu, sxy >> 8, (1u << 8) | (255u - l), l};

    for (uint32_t c0 = 0; __builtin_amdgcn_ballot_w64(c0 < L); c0 += kWinRing) {
        const uint32_t c1 = L < c0 + kWinRing ? L : c0 + kWinRing;
        const uint32_t rem = c0 < L ? c1 - c0 : 0u;
        // window tags are 24 bits: long before they wrap (a 2 KiB chunk takes
        // < 2 048 windows), the markers are cleared and the tags restart
        if (w.v >= (kWinTagLimit << 8)) {
#pragma unroll
            for (int i = 0; i < 4; ++i) reinterpret_cast<uint4 *>(Mk)[lane + 64 * i] = make_uint4(0, 0, 0, 0);
            w.v = (1u << 8) | (255u - l);
        }
        win_windows(w, rem, l, sb, mb, rb);
        if constexpr (MODE == kGrouped) {
            // The claim's answer is first needed here: nothing has been
            // written yet (the windows run in LDS), so its round trip hides
            // under the first chunk's keystream.  lost: another bucket of
            // this launch holds column q; store nothing.
            if (c0 == 0u) {
                claim_wait(cold);        // (the XOR pass below waits for the payload prefetch anyway)
                if (claim_lost(cl, ((unsigned long long)__builtin_amdgcn_readfirstlane((uint32_t)(cold >> 32))) << 32)) {
                    if (lane == 0) latch_fault(err, kErrGroup);
                    return;
                }
            }
        }
        // XOR pass of [c0, c1): whole 16-byte units from the prefetch, bytes
        // otherwise (streams already past their end skip it: c1 - c0 would wrap)
        if (c0 >= L) {
        } else if (aligned) {
#pragma unroll
            for (uint32_t u = 0; u < kWinUnits; ++u) {
                const uint32_t pos = c0 + 16u * (l + kWinLanes * u);
                if (pos + 16u <= c1) {
                    const uint4 ks = *reinterpret_cast<const uint4 *>(R + (pos & (kWinRing - 1u)));
                    uint4 v = pre[u];
                    v.x ^= ks.x; v.y ^= ks.y; v.z ^= ks.z; v.w ^= ks.w;
                    *reinterpret_cast<uint4 *>(msg + pos) = v;
                }
            }
            const uint32_t tpos = c0 + ((c1 - c0) & ~15u) + l;                  // ragged tail: < 16 bytes
            if (tpos < c1) msg[tpos] ^= R[tpos & (kWinRing - 1u)];
        } else {
            for (uint32_t pos = c0 + l; pos < c1; pos += kWinLanes) msg[pos] ^= R[pos & (kWinRing - 1u)];
        }
        // prefetch of the next chunk
        const uint32_t n0 = c0 + kWinRing;
#pragma unroll
        for (uint32_t u = 0; u < kWinUnits; ++u) {
            const uint32_t pos = n0 + 16u * (l + kWinLanes * u);
            if (aligned && pos + 16u <= L) pre[u] = *reinterpret_cast<const uint4 *>(msg + pos);
        }
    }

    stamp(ts, 2);
    if (valid && l == 0) xy[slot] = (uint16_t)(((w.xa - 1u) & 0xFFu) | ((w.y & 0xFFu) << 8));
    if constexpr (FRAME) {
        // the stream's 16 lanes stored its bytes: they must have landed
        // before lane 0 reads the headers back
        __builtin_amdgcn_s_waitcnt(0);
        if (valid && l == 0)
            frame_walk(payload + fr.off[ent], fr.len[ent], fr.bound, fr.maxp, ent, fr.npk, fr.used, fr.status,
                       fr.pkt_len);
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const uint32_t kk = lane + 64u * r;
        const uint32_t v = (uint32_t)Sb[kk] | ((uint32_t)Sb[256u + kk] << 8) | ((uint32_t)Sb[512u + kk] << 16) |
                           ((uint32_t)Sb[768u + kk] << 24);
        *reinterpret_cast<uint32_t *>(img + (size_t)kk * 256u) = v;
    }
#if ZRC4_TIMING
    __builtin_amdgcn_s_waitcnt(0);
    stamp(ts, 3);
    stamps_out(ts, sink, wg * 64u + q);          // record of the workgroup's column
#else
    (void)sink;
#endif
}

}  // namespace zrc4
