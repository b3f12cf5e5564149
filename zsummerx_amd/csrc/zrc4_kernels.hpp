// zrc4_kernels.hpp -- gfx950 (CDNA4) kernels for the zsummerX RC4 path.
//
// Reference algorithm: /root/reference/depends/rc4/rc4_encryption.h
//   makeSBox   :46-72  -> ksa_kernel
//   encryption :74-93  -> crypt_kernel (<= 1 group per CU), crypt_stream_kernel
//
// Only the instantiated product paths live here.  The round-1 A/B variants
// (LDS-staged quad / line stores, whole-line loads, step-order, stagger,
// ablation and cache-policy knobs) are reproducible from git revision 849e847
// with tools/ab_bench.py --variant name@849e847:KNOB=v.
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
//   The hand-written steps use these addresses as ABSOLUTE LDS addresses, so
//   the S-box image must sit at LDS offset 0 of the workgroup; every kernel
//   checks that at entry (lds_base_ok) and latches kErrLdsLayout otherwise.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace zrc4 {

constexpr int kGroup = 256;            // slots per workgroup / arena group
constexpr int kGroupBytes = 256 * 256; // 64 KiB S-box image per group

// Fault latch: words in pinned host memory, one per fault kind; every
// faulting lane stores 1 with a plain system-scope store (no read-modify-
// write), the host reads and clears them after its stream wait (zrc4_sync).
enum : uint32_t {
    kErrSlotRange = 0,   // a slot id >= capacity (entry skipped)
    kErrLdsLayout = 1,   // the S-box image is not at LDS offset 0 (launch skipped)
    kErrGroup = 2,       // zrc4_crypt_grouped: a bucket mixes slot groups (bucket skipped)
    kErrWords = 4,
};

__device__ __forceinline__ void latch_fault(uint32_t *err, uint32_t kind)
{
    __hip_atomic_store(err + kind, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Cross-bucket half of the zrc4_crypt_grouped contract ("no other bucket of
// the call touches that group", include/zrc4.h): every workgroup of a grouped
// launch claims the part of its bucket's group it moves -- whole group: part
// 0; half-group workgroups: the half h; the window kernel: its dword column q
// -- by one agent-scope 64-bit exchange of (launch epoch << 32 | bucket) into
// a per-context word per (group, part).  Reading back this launch's epoch
// means another bucket of the same launch holds that part: the workgroup
// latches kErrGroup and writes nothing, so no S-box byte, x/y or payload byte
// is ever raced.  The host gives every grouped launch a fresh non-zero epoch
// (words are zeroed whenever the 32-bit epoch wraps).  The exchange is issued
// with the speculative image loads (the first busy id's group), so its round
// trip hides under theirs; a bucket that breaks the one-group rule may
// therefore also block the bucket of the group its first busy id names.
constexpr uint32_t kClaimParts = 64;
struct Claim {
    unsigned long long *word;   // [groups][kClaimParts]
    uint32_t epoch;
    const uint32_t *zero;       // 16 zero bytes (crypt_stream_kernel<true, true>: the entry of an idle lane)
};

__device__ __forceinline__ unsigned long long claim_part(const Claim &cl, uint32_t g, uint32_t part,
                                                         uint32_t bucket)
{
    return __hip_atomic_exchange(cl.word + (size_t)g * kClaimParts + part,
                                 ((unsigned long long)cl.epoch << 32) | bucket, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
}

// The same exchange issued from asm by lane 0 with the rest of the wave
// masked off: the compiler neither sees nor counts it, so its waits for older
// loads do not also wait for the atomic's round trip (a lane-0-only atomic in
// compiler code sits on a divergent path, and the waitcnt pass then drains
// with vmcnt(0) at the next wait).  The caller retires it explicitly
// (claim_wait) before reading the answer; lane 0 must be active here.
__device__ __forceinline__ unsigned long long claim_part_async(const Claim &cl, uint32_t g, uint32_t part,
                                                               uint32_t bucket)
{
    unsigned long long old;
    uint64_t sv;
    const unsigned long long v = ((unsigned long long)cl.epoch << 32) | bucket;
    unsigned long long *addr = cl.word + (size_t)g * kClaimParts + part;
    asm volatile("s_mov_b64 %[sv], exec\n\t"
                 "s_mov_b64 exec, 1\n\t"
                 "global_atomic_swap_x2 %[old], %[a], %[v], off sc0\n\t"
                 "s_mov_b64 exec, %[sv]"
                 : [old] "=&v"(old), [sv] "=&s"(sv)
                 : [a] "v"(addr), [v] "v"(v)
                 : "memory");
    return old;
}

// claim_part_async under a wave-uniform predicate tested INSIDE the asm
// (ADVICE r05): the statement runs on every path and defines its result on
// every path (0 when the predicate is false), so the compiler has no phi to
// merge it through -- a merge copy of a register whose atomic is still in
// flight would read it before claim_wait.
__device__ __forceinline__ unsigned long long claim_part_async_if(const Claim &cl, uint32_t g, uint32_t part,
                                                                  uint32_t bucket, uint32_t pred)
{
    unsigned long long old;
    uint64_t sv;
    const unsigned long long v = ((unsigned long long)cl.epoch << 32) | bucket;
    unsigned long long *addr = cl.word + (size_t)g * kClaimParts + part;
    asm volatile("v_mov_b64 %[old], 0\n\t"
                 "s_cmp_eq_u32 %[p], 0\n\t"
                 "s_cbranch_scc1 CLAIM_SKIP_%=\n\t"
                 "s_mov_b64 %[sv], exec\n\t"
                 "s_mov_b64 exec, 1\n\t"
                 "global_atomic_swap_x2 %[old], %[a], %[v], off sc0\n\t"
                 "s_mov_b64 exec, %[sv]\n\t"
                 "CLAIM_SKIP_%=:"
                 : [old] "=&v"(old), [sv] "=&s"(sv)
                 : [a] "v"(addr), [v] "v"(v), [p] "s"(__builtin_amdgcn_readfirstlane(pred))
                 : "memory", "scc");
    return old;
}

// Retire every VMEM op in flight, claim_part_async's answer included.
__device__ __forceinline__ void claim_wait(unsigned long long &old)
{
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(old) :: "memory");
}

__device__ __forceinline__ bool claim_lost(const Claim &cl, unsigned long long old)
{
    return (uint32_t)(old >> 32) == cl.epoch;
}

// The asm addresses S-box bytes absolutely (no base register): S must be the
// workgroup's first LDS byte.  (uint32_t) of a generic LDS pointer is its
// offset inside the LDS aperture.
__device__ __forceinline__ bool lds_base_ok(const uint8_t *S, uint32_t *err)
{
    if ((uint32_t)(uintptr_t)S == 0u) return true;
    if (threadIdx.x == 0) latch_fault(err, kErrLdsLayout);
    return false;
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__host__ __device__ __forceinline__ uint32_t col_of(uint32_t j)
{
    const uint32_t w = j >> 6, l = j & 63u;
    return ((l & 31u) << 2) | (l >> 5) | ((w & 1u) << 1) | ((w >> 1) << 7);
}

// The persistent kernel's image moves (prefetch, LDS fill, copy-out): thread
// j takes the 16-byte chunks at img_vo(j) + 4096 i, i < 16.  Waves 2p and
// 2p+1 (the two waves whose columns have bit 7 = p, col_of) move exactly
// bytes [128p, 128p + 128) of every 256-byte row -- their own half of the
// image, one whole 128-byte line per 8 lanes -- so a wave pair can fill and
// copy out its half without the other pair.
__device__ __forceinline__ uint32_t img_vo(uint32_t j)
{
    return (((j & 127u) >> 3) << 8) | (j & 128u) | ((j & 7u) << 4);
}

// ---------------------------------------------------------------------------
// Diagnostic timing build (ZRC4_TIMING=1, never the product): lane 0 of each
// wave stamps s_memrealtime (100 MHz) and s_memtime (shader clock) at kernel
// entry, S-boxes in LDS, keystream done, and state stored; the 64-byte record
// of global wave w (thread index / 64) goes to sink + (w & 1023) * 64
// (zrc4_debug_sink exports the sink in such builds; tools/kernel_timeline.py).
// ---------------------------------------------------------------------------
#ifndef ZRC4_TIMING
#define ZRC4_TIMING 0
#endif
struct Stamps {
    uint64_t r[4], c[4];
};
__device__ __forceinline__ void stamp(Stamps &s, int i)
{
#if ZRC4_TIMING
    s.r[i] = __builtin_amdgcn_s_memrealtime();
    s.c[i] = __builtin_amdgcn_s_memtime();
#endif
}
// crypt_stream_kernel (ZRC4_TIMING): lane 0 of the first wave of each wave
// pair (waves 0 and 2) of workgroup wg stamps event i (0 entry, 1 + 2k / 2 +
// 2k group k's keystream start / end, 15 exit; 9-13 inside boundary 0) as
// s_memrealtime into record r = 2 wg + pair (512 workgroups, 1 024 pairs) of
// the stamp area after the crypt_kernel records: rt[r][16] at kStampBase,
// entry / exit shader clocks at + 128 KiB, HW_ID / XCC_ID at + 144 KiB.
constexpr uint32_t kStampBase = 65536u + 16384u;
constexpr uint32_t kStampBytes = 131072u + 16384u + 8192u;
__device__ __forceinline__ void stream_stamp(uint8_t *sink, uint32_t i)
{
#if ZRC4_TIMING
    if ((threadIdx.x & 127u) == 0u && blockIdx.x < 512u && i < 16u) {
        const uint32_t r = blockIdx.x * 2u + (threadIdx.x >> 7);
        uint8_t *b = sink + kStampBase;
        reinterpret_cast<uint64_t *>(b)[r * 16u + i] = __builtin_amdgcn_s_memrealtime();
        if (i == 0u || i == 15u)
            reinterpret_cast<uint64_t *>(b + 131072u)[r * 2u + (i ? 1u : 0u)] = __builtin_amdgcn_s_memtime();
        if (i == 0u) {
            uint32_t hw, xcc;
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)\n\ts_getreg_b32 %1, hwreg(HW_REG_XCC_ID)"
                         : "=s"(hw), "=s"(xcc));
            uint32_t *o = reinterpret_cast<uint32_t *>(b + 131072u + 16384u) + r * 2u;
            o[0] = hw;
            o[1] = xcc;
        }
    }
#endif
}

// `wave`: the wave's index in batch-entry order (entry >> 6).
__device__ __forceinline__ void stamps_out(const Stamps &s, uint8_t *sink, uint32_t wave)
{
#if ZRC4_TIMING
    if ((threadIdx.x & 63u) == 0u) {
        uint64_t *o = reinterpret_cast<uint64_t *>(sink + ((wave & 1023u) * 64u));
        for (int i = 0; i < 4; ++i) {
            o[i] = s.r[i];
            o[4 + i] = s.c[i];
        }
        // where the wave ran: HW_ID (wave/simd/cu/sh/se fields) and XCC_ID,
        // after the 64 KiB of stamps (the timing build's sink is larger)
        uint32_t hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)\n\ts_getreg_b32 %1, hwreg(HW_REG_XCC_ID)"
                     : "=s"(hw), "=s"(xcc));
        uint32_t *w = reinterpret_cast<uint32_t *>(sink + 65536u + (wave & 1023u) * 8u);
        w[0] = hw;
        w[1] = xcc;
    }
#endif
}

// ---------------------------------------------------------------------------
// Group state load / store.
//   fast: the workgroup owns one whole 256-slot group: copy the 64 KiB image
//         as 16 B per lane, coalesced.
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
// PRGA (rc4_encryption.h:81-89) on 16-bit LDS addresses.
//
// Lane state (all addresses are (index << 8) | col, bytes 2-3 zero):
//   x0 = address of S[x]  where x is the NEXT index to use (stored x + 1)
//   a0 = S[x]             (already read)
//   ya = address of S[y]
//   ta = col in byte 0, scratch index in byte 1 (hand-written path only)
//
// Per byte the LDS ops are issued in the order
//     b = S[y+a] ; S[y] = a ; p = S[x+1] ; S[x] = b ; k = S[a+b]
// Reading S[x+1] after the S[y] = a write needs no forwarding (the S[x] = b
// write goes to x != x+1), and the b -> S[x] = b wait no longer gates the
// next byte, so the byte-to-byte chain holds one LDS round trip (b and p are
// in flight together).  Swapping the reference's write order (S[x] = b then
// S[y] = a, :86-87) is exact: the two only collide when x == y, and then
// b == a.
// ---------------------------------------------------------------------------
struct Rc4Lane {
    uint32_t x0, a0, ya, ta, x1, col;
};

__device__ __forceinline__ void lane_init(Rc4Lane &st, const uint8_t *S, uint32_t col, uint32_t sxy)
{
    const uint32_t x = sxy & 255u, y = (sxy >> 8) & 255u;
    st.col = col;
    st.x0 = (((x + 1u) & 255u) << 8) | col;
    st.a0 = S[st.x0];
    st.ya = (y << 8) | col;
    st.ta = col;
    st.x1 = col;
}

__device__ __forceinline__ uint16_t lane_xy(const Rc4Lane &st)
{
    return (uint16_t)((((st.x0 >> 8) - 1u) & 255u) | (st.ya & 0xFF00u));
}

// Portable C step with the same state layout (head/tail bytes, 16-B chunks).
__device__ __forceinline__ uint32_t prga_step(uint8_t *S, Rc4Lane &st)
{
    const uint32_t a = st.a0;
    const uint32_t ya = (st.ya & 0xFFu) | ((st.ya + (a << 8)) & 0xFF00u);  // y = (u8)(y+a)
    const uint32_t b = S[ya];                                                // b = S[y]
    S[ya] = (uint8_t)a;                                                      // S[y] = a
    const uint32_t xn = (st.x0 & 0xFFu) | ((st.x0 + 256u) & 0xFF00u);
    const uint32_t p = S[xn];                                                // next a
    S[st.x0] = (uint8_t)b;                                                   // S[x] = b
    const uint32_t k = S[(((a + b) << 8) & 0xFF00u) | st.col];               // S[(u8)(a+b)]
    st.a0 = p;
    st.x0 = xn;
    st.ya = ya;
    return k;
}

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

// Hand-written gfx950 step.  Each index update is ONE SDWA add that rewrites
// byte 1 of an address register in place (dst_sel:BYTE_1, UNUSED_PRESERVE):
// the mod-256 wrap is free and col (byte 0) is untouched.  The keystream byte
// of step s is XORed into its payload byte at the end of step s+1 (its read
// is retired by step s+1's waits) with one SDWA xor on that byte lane.
// (ds_read_u8_d16_hi does NOT preserve the low half on gfx950 -- measured --
// so keystream bytes are not packed through d16 loads.)
//
// XC = address of S[x] for this step; XN = address of S[x+1], derived from XC
// inside the step right before its read.  XC is free after the S[x] = b write.
// Per byte: 4 VALU + 5 LDS + 2 waits.
// x + 1: ZRC4_XADD16 (default) adds 0x100 (SGPR operand c100) with a 16-bit
// add, whose wrap at 65 536 is the mod-256 wrap of byte 1 (XN and XC hold
// the same col in byte 0, bits 16-31 stay zero): a 4-byte VOP2 encoding
// instead of the 8-byte SDWA add.
#ifndef ZRC4_XADD16
#define ZRC4_XADD16 1
#endif
#if ZRC4_XADD16
#define ZRC4_XINC(XC, XN) "v_add_u16_e32 %[" #XN "], %[c100], %[" #XC "]\n\t"
#else
#define ZRC4_XINC(XC, XN)                                                                        \
    "v_add_u32_sdwa %[" #XN "], 1, %[" #XC "] dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE "        \
    "src0_sel:DWORD src1_sel:BYTE_1\n\t"
#endif
// ZRC4_AB_LDS (timing-only ablations, outputs wrong): 1 drops the S[x] = b
// write, 2 drops the keystream read S[t] -- how much the LDS pipe bounds the
// step at 8 waves per CU.
#ifndef ZRC4_AB_LDS
#define ZRC4_AB_LDS 0
#endif
#if ZRC4_AB_LDS == 1
#define ZRC4_CORE_XW(XC)
#define ZRC4_CORE_KR(K) "s_waitcnt lgkmcnt(1)\n\t"
#elif ZRC4_AB_LDS == 2
#define ZRC4_CORE_XW(XC) "ds_write_b8 %[" #XC "], %[b]\n\t"
#define ZRC4_CORE_KR(K) "s_waitcnt lgkmcnt(1)\n\t"
#else
#define ZRC4_CORE_XW(XC) "ds_write_b8 %[" #XC "], %[b]\n\t"
#define ZRC4_CORE_KR(K) "ds_read_u8 %[" #K "], %[ta]\n\t" "s_waitcnt lgkmcnt(2)\n\t"
#endif
#define ZRC4_CORE(XC, XN, A, P, K)                                                               \
    "v_add_u32_sdwa %[ya], %[ya], %[" #A "] dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE "          \
    "src0_sel:BYTE_1 src1_sel:BYTE_0\n\t"                                                        \
    "ds_read_u8 %[b], %[ya]\n\t"                                                                 \
    "ds_write_b8 %[ya], %[" #A "]\n\t"                                                           \
    ZRC4_XINC(XC, XN)                                                                            \
    "ds_read_u8 %[" #P "], %[" #XN "]\n\t"                                                       \
    "s_waitcnt lgkmcnt(2)\n\t"                                                                   \
    ZRC4_CORE_XW(XC)                                                                             \
    "v_add_u32_sdwa %[ta], %[" #A "], %[b] dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE "           \
    "src0_sel:BYTE_0 src1_sel:BYTE_0\n\t"                                                        \
    ZRC4_CORE_KR(K)

#define ZRC4_E ZRC4_CORE(x0, x1, a0, a1, k0)   // even step: keystream -> k0
#define ZRC4_O ZRC4_CORE(x1, x0, a1, a0, k1)   // odd step:  keystream -> k1

// 64-byte blocks are kept as uint4[4] so every 16 bytes sits in an aligned
// 4-register tuple (one dwordx4 each).
__device__ __forceinline__ void load64(uint4 (&q)[4], const uint4 *p)
{
#pragma unroll
    for (int i = 0; i < 4; ++i) q[i] = p[i];
}

// Bytes before the first 16-byte boundary of a message (<= len).
__device__ __forceinline__ uint32_t head_bytes(const uint8_t *msg, uint32_t len)
{
    const uint32_t h = (16u - ((uint32_t)(uintptr_t)msg & 15u)) & 15u;
    return h < len ? h : len;
}

// ---------------------------------------------------------------------------
// The whole 64-byte block loop as ONE asm statement (direct-store path).
// hipcc's code between per-block asm statements (register copies, exec
// bookkeeping, address math: ~40 instructions per block) cost ~6 % of the
// loop; here a block costs 4 loads + 4 stores + 9 scalar/vector ops.
//   * payload blocks ping-pong between two PINNED register tuples,
//     A = v40..v55 and B = v56..v71, so the dwordx4 loads/stores and the
//     per-byte SDWA xors name the same registers;
//   * the next block's four loads go out under the loop's full exec (a lane
//     with no next block re-reads its current block), so every vmcnt wait is
//     a static count; one s_waitcnt vmcnt(8) per block (in-order VMEM
//     completion: the 8 younger ops are the previous block's stores and this
//     prefetch);
//   * exec shrinks as lanes run out of blocks (ragged batches), and is
//     restored on exit.  Lanes keep their own pointer and RC4 state;
//   * block 0 runs its keystream AHEAD of its payload (ZL_FIRST): the 64
//     keystream bytes go into K = v72..v87 (cleared) and only then does the
//     wave wait for block 0's loads -- vmcnt(4): block 1's four prefetch
//     loads are the only younger VMEM ops -- and XOR K into A.  The caller
//     issues block 0 from asm (issue_block_asm) before the LDS fill, so its
//     HBM round trip overlaps the fill and 64 PRGA steps.
// On entry A holds (or is loading) block 0, nblk >= 1 for every active lane.
// Cache policy: plain loads and stores (nt stores cost cfg3 +2.7 %, r01).
// ---------------------------------------------------------------------------
#define ZL_XOR(R, SEL, K)                                                                        \
    "v_xor_b32_sdwa " #R ", " #R ", %[" #K "] dst_sel:" #SEL                                     \
    " dst_unused:UNUSED_PRESERVE src0_sel:" #SEL " src1_sel:BYTE_0\n\t"
#define ZL_W0(D)                                                                                 \
    ZRC4_E ZRC4_O ZL_XOR(D, BYTE_0, k0) ZRC4_E ZL_XOR(D, BYTE_1, k1)                            \
    ZRC4_O ZL_XOR(D, BYTE_2, k0)
#define ZL_W(DP, D)                                                                              \
    ZRC4_E ZL_XOR(DP, BYTE_3, k1) ZRC4_O ZL_XOR(D, BYTE_0, k0)                                  \
    ZRC4_E ZL_XOR(D, BYTE_1, k1) ZRC4_O ZL_XOR(D, BYTE_2, k0)
#define ZL_BLOCK(d0, d1, d2, d3, d4, d5, d6, d7, d8, d9, d10, d11, d12, d13, d14, d15)            \
    ZL_W0(d0) ZL_W(d0, d1) ZL_W(d1, d2) ZL_W(d2, d3) ZL_W(d3, d4) ZL_W(d4, d5)                  \
    ZL_W(d5, d6) ZL_W(d6, d7) ZL_W(d7, d8) ZL_W(d8, d9) ZL_W(d9, d10) ZL_W(d10, d11)            \
    ZL_W(d11, d12) ZL_W(d12, d13) ZL_W(d13, d14) ZL_W(d14, d15)                                 \
    "s_waitcnt lgkmcnt(0)\n\t" ZL_XOR(d15, BYTE_3, k1)
// payload tuples: A = v40..v55, B = v56..v71
#define ZL_A0 "v[40:43]"
#define ZL_A1 "v[44:47]"
#define ZL_A2 "v[48:51]"
#define ZL_A3 "v[52:55]"
#define ZL_B0 "v[56:59]"
#define ZL_B1 "v[60:63]"
#define ZL_B2 "v[64:67]"
#define ZL_B3 "v[68:71]"
// Next block's four loads into R: from pa + 64, or -- for lanes with no next
// block -- a harmless re-read of the current block (pa).  pa = v[88:89],
// pn = v[90:91].
#define ZL_PREFETCH(R0, R1, R2, R3)                                                              \
    "s_add_u32 %[i1], %[i], 1\n\t"                                                               \
    "v_cmp_lt_u32_e32 vcc, %[i1], %[nblk]\n\t"                                                   \
    "v_lshl_add_u64 v[90:91], v[88:89], 0, 64\n\t"                                               \
    "v_cndmask_b32_e32 v90, v88, v90, vcc\n\t"                                                   \
    "v_cndmask_b32_e32 v91, v89, v91, vcc\n\t"                                                   \
    "global_load_dwordx4 " R0 ", v[90:91], off\n\t"                                              \
    "global_load_dwordx4 " R1 ", v[90:91], off offset:16\n\t"                                    \
    "global_load_dwordx4 " R2 ", v[90:91], off offset:32\n\t"                                    \
    "global_load_dwordx4 " R3 ", v[90:91], off offset:48\n\t"
#define ZL_STORE(R0, R1, R2, R3)                                                                 \
    "global_store_dwordx4 v[88:89], " R0 ", off\n\t"                                             \
    "global_store_dwordx4 v[88:89], " R1 ", off offset:16\n\t"                                   \
    "global_store_dwordx4 v[88:89], " R2 ", off offset:32\n\t"                                   \
    "global_store_dwordx4 v[88:89], " R3 ", off offset:48\n\t"                                   \
    "v_lshl_add_u64 v[88:89], v[88:89], 0, 64\n\t"                                               \
    "s_add_u32 %[i], %[i], 1\n\t"
#define ZL_ACTIVE                                                                                \
    "v_cmp_lt_u32_e32 vcc, %[i], %[nblk]\n\t"                                                    \
    "s_and_b64 exec, exec, vcc\n\t"                                                              \
    "s_cbranch_execz ZL_DONE_%=\n\t"
#define ZL_HALF_A                                                                                \
    ZL_ACTIVE                                                                                    \
    ZL_PREFETCH(ZL_B0, ZL_B1, ZL_B2, ZL_B3)                                                      \
    "s_waitcnt vmcnt(8)\n\t"                                                                     \
    ZL_BLOCK(v40, v41, v42, v43, v44, v45, v46, v47, v48, v49, v50, v51, v52, v53, v54, v55)    \
    ZL_STORE(ZL_A0, ZL_A1, ZL_A2, ZL_A3)
#define ZL_HALF_B                                                                                \
    ZL_ACTIVE                                                                                    \
    ZL_PREFETCH(ZL_A0, ZL_A1, ZL_A2, ZL_A3)                                                      \
    "s_waitcnt vmcnt(8)\n\t"                                                                     \
    ZL_BLOCK(v56, v57, v58, v59, v60, v61, v62, v63, v64, v65, v66, v67, v68, v69, v70, v71)    \
    ZL_STORE(ZL_B0, ZL_B1, ZL_B2, ZL_B3)
// ZRC4_BLK_DEFER (A/B, default 0 = the ISA above): each block's keystream
// goes into K first (byte moves, as block 0's does) and the wait for the
// block's payload comes after it, so a block's loads have two blocks of
// keystream time to land instead of one (+16 VALU per block for the XOR).
#ifndef ZRC4_BLK_DEFER
#define ZRC4_BLK_DEFER 0
#endif
#define ZL_MOVK(R, SEL, K)                                                                       \
    "v_mov_b32_sdwa " #R ", %[" #K "] dst_sel:" #SEL " dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0\n\t"
#define ZL_W0K(D)                                                                                \
    ZRC4_E ZRC4_O ZL_MOVK(D, BYTE_0, k0) ZRC4_E ZL_MOVK(D, BYTE_1, k1)                          \
    ZRC4_O ZL_MOVK(D, BYTE_2, k0)
#define ZL_WK(DP, D)                                                                             \
    ZRC4_E ZL_MOVK(DP, BYTE_3, k1) ZRC4_O ZL_MOVK(D, BYTE_0, k0)                                \
    ZRC4_E ZL_MOVK(D, BYTE_1, k1) ZRC4_O ZL_MOVK(D, BYTE_2, k0)
#define ZL_BLOCKK                                                                                \
    ZL_W0K(v72) ZL_WK(v72, v73) ZL_WK(v73, v74) ZL_WK(v74, v75) ZL_WK(v75, v76) ZL_WK(v76, v77)   \
    ZL_WK(v77, v78) ZL_WK(v78, v79) ZL_WK(v79, v80) ZL_WK(v80, v81) ZL_WK(v81, v82)               \
    ZL_WK(v82, v83) ZL_WK(v83, v84) ZL_WK(v84, v85) ZL_WK(v85, v86) ZL_WK(v86, v87)               \
    "s_waitcnt lgkmcnt(0)\n\t" ZL_MOVK(v87, BYTE_3, k1)
#define ZL_KXOR(d0, d1, d2, d3, d4, d5, d6, d7, d8, d9, d10, d11, d12, d13, d14, d15)            \
    "v_xor_b32_e32 " #d0 ", " #d0 ", v72\n\tv_xor_b32_e32 " #d1 ", " #d1 ", v73\n\t"                 \
    "v_xor_b32_e32 " #d2 ", " #d2 ", v74\n\tv_xor_b32_e32 " #d3 ", " #d3 ", v75\n\t"                 \
    "v_xor_b32_e32 " #d4 ", " #d4 ", v76\n\tv_xor_b32_e32 " #d5 ", " #d5 ", v77\n\t"                 \
    "v_xor_b32_e32 " #d6 ", " #d6 ", v78\n\tv_xor_b32_e32 " #d7 ", " #d7 ", v79\n\t"                 \
    "v_xor_b32_e32 " #d8 ", " #d8 ", v80\n\tv_xor_b32_e32 " #d9 ", " #d9 ", v81\n\t"                 \
    "v_xor_b32_e32 " #d10 ", " #d10 ", v82\n\tv_xor_b32_e32 " #d11 ", " #d11 ", v83\n\t"             \
    "v_xor_b32_e32 " #d12 ", " #d12 ", v84\n\tv_xor_b32_e32 " #d13 ", " #d13 ", v85\n\t"             \
    "v_xor_b32_e32 " #d14 ", " #d14 ", v86\n\tv_xor_b32_e32 " #d15 ", " #d15 ", v87\n\t"
#if ZRC4_BLK_DEFER
#undef ZL_HALF_A
#undef ZL_HALF_B
#define ZL_HALF_A                                                                                \
    ZL_ACTIVE                                                                                    \
    ZL_PREFETCH(ZL_B0, ZL_B1, ZL_B2, ZL_B3)                                                      \
    ZL_BLOCKK                                                                                    \
    "s_waitcnt vmcnt(8)\n\t"                                                                     \
    ZL_KXOR(v40, v41, v42, v43, v44, v45, v46, v47, v48, v49, v50, v51, v52, v53, v54, v55)     \
    ZL_STORE(ZL_A0, ZL_A1, ZL_A2, ZL_A3)
#define ZL_HALF_B                                                                                \
    ZL_ACTIVE                                                                                    \
    ZL_PREFETCH(ZL_A0, ZL_A1, ZL_A2, ZL_A3)                                                      \
    ZL_BLOCKK                                                                                    \
    "s_waitcnt vmcnt(8)\n\t"                                                                     \
    ZL_KXOR(v56, v57, v58, v59, v60, v61, v62, v63, v64, v65, v66, v67, v68, v69, v70, v71)     \
    ZL_STORE(ZL_B0, ZL_B1, ZL_B2, ZL_B3)
#endif
#define ZL_FIRST                                                                                 \
    "s_mov_b32 %[i], 0\n\t"                                                                      \
    ZL_PREFETCH(ZL_B0, ZL_B1, ZL_B2, ZL_B3)                                                      \
    "v_mov_b32 v72, 0\n\tv_mov_b32 v73, 0\n\tv_mov_b32 v74, 0\n\tv_mov_b32 v75, 0\n\t"             \
    "v_mov_b32 v76, 0\n\tv_mov_b32 v77, 0\n\tv_mov_b32 v78, 0\n\tv_mov_b32 v79, 0\n\t"             \
    "v_mov_b32 v80, 0\n\tv_mov_b32 v81, 0\n\tv_mov_b32 v82, 0\n\tv_mov_b32 v83, 0\n\t"             \
    "v_mov_b32 v84, 0\n\tv_mov_b32 v85, 0\n\tv_mov_b32 v86, 0\n\tv_mov_b32 v87, 0\n\t"             \
    ZL_BLOCK(v72, v73, v74, v75, v76, v77, v78, v79, v80, v81, v82, v83, v84, v85, v86, v87)    \
    "s_waitcnt vmcnt(4)\n\t"                                                                     \
    "v_xor_b32_e32 v40, v40, v72\n\tv_xor_b32_e32 v41, v41, v73\n\t"                               \
    "v_xor_b32_e32 v42, v42, v74\n\tv_xor_b32_e32 v43, v43, v75\n\t"                               \
    "v_xor_b32_e32 v44, v44, v76\n\tv_xor_b32_e32 v45, v45, v77\n\t"                               \
    "v_xor_b32_e32 v46, v46, v78\n\tv_xor_b32_e32 v47, v47, v79\n\t"                               \
    "v_xor_b32_e32 v48, v48, v80\n\tv_xor_b32_e32 v49, v49, v81\n\t"                               \
    "v_xor_b32_e32 v50, v50, v82\n\tv_xor_b32_e32 v51, v51, v83\n\t"                               \
    "v_xor_b32_e32 v52, v52, v84\n\tv_xor_b32_e32 v53, v53, v85\n\t"                               \
    "v_xor_b32_e32 v54, v54, v86\n\tv_xor_b32_e32 v55, v55, v87\n\t"                               \
    ZL_STORE(ZL_A0, ZL_A1, ZL_A2, ZL_A3)                                                         \
    "s_branch ZL_MID_%=\n\t"

__device__ __forceinline__ void crypt_blocks_asm(Rc4Lane &st, uint4 *&p, uint32_t nblk,
                                                 const uint4 (&A)[4])
{
    u32x4 a0 = {A[0].x, A[0].y, A[0].z, A[0].w}, a1 = {A[1].x, A[1].y, A[1].z, A[1].w};
    u32x4 a2 = {A[2].x, A[2].y, A[2].z, A[2].w}, a3 = {A[3].x, A[3].y, A[3].z, A[3].w};
    u32x4 b0, b1, b2, b3, q0, q1, q2, q3;
    uint64_t pa = (uint64_t)(uintptr_t)p, pn, save;
    uint32_t i, i1, b, k0, k1, a1s;
    asm volatile(
        "s_mov_b64 %[save], exec\n\t"
        ZL_FIRST
        "ZL_LOOP_%=:\n\t"
        ZL_HALF_A
        "ZL_MID_%=:\n\t"
        ZL_HALF_B
        "s_branch ZL_LOOP_%=\n\t"
        "ZL_DONE_%=:\n\t"
        "s_mov_b64 exec, %[save]\n\t"
        : [ya] "+v"(st.ya), [ta] "+v"(st.ta), [x0] "+v"(st.x0), [x1] "+v"(st.x1),
          [a0] "+v"(st.a0), [a1] "=&v"(a1s), [b] "=&v"(b), [k0] "=&v"(k0), [k1] "=&v"(k1),
          "+{v[88:89]}"(pa), "=&{v[90:91]}"(pn), [i] "=&s"(i), [i1] "=&s"(i1), [save] "=&s"(save),
          "+{v[40:43]}"(a0), "+{v[44:47]}"(a1), "+{v[48:51]}"(a2), "+{v[52:55]}"(a3),
          "=&{v[56:59]}"(b0), "=&{v[60:63]}"(b1), "=&{v[64:67]}"(b2), "=&{v[68:71]}"(b3),
          "=&{v[72:75]}"(q0), "=&{v[76:79]}"(q1), "=&{v[80:83]}"(q2), "=&{v[84:87]}"(q3)
        : [nblk] "v"(nblk), [c100] "s"(0x100u)
        : "memory", "vcc", "scc");
    p = reinterpret_cast<uint4 *>((uintptr_t)pa);
}

// Block 0 of a message issued from asm into the pinned A tuples, so hipcc
// neither counts nor waits for it (crypt_blocks_asm's lead block does).
__device__ __forceinline__ void issue_block_asm(uint4 (&A)[4], const uint8_t *msg)
{
    u32x4 a0, a1, a2, a3;
    asm volatile(
        "global_load_dwordx4 v[40:43], %[p], off\n\t"
        "global_load_dwordx4 v[44:47], %[p], off offset:16\n\t"
        "global_load_dwordx4 v[48:51], %[p], off offset:32\n\t"
        "global_load_dwordx4 v[52:55], %[p], off offset:48\n\t"
        : "=&{v[40:43]}"(a0), "=&{v[44:47]}"(a1), "=&{v[48:51]}"(a2), "=&{v[52:55]}"(a3)
        : [p] "v"(msg)
        : "memory");
    A[0] = make_uint4(a0[0], a0[1], a0[2], a0[3]);
    A[1] = make_uint4(a1[0], a1[1], a1[2], a1[3]);
    A[2] = make_uint4(a2[0], a2[1], a2[2], a2[3]);
    A[3] = make_uint4(a3[0], a3[1], a3[2], a3[3]);
}

// Crypt one lane's message in place: unaligned head bytes, 64-byte blocks
// (crypt_blocks_asm), 16-byte chunks, tail bytes.  If `pre` is set, A already
// holds the first 64-byte block (issued by the caller ahead of the LDS fill).
__device__ __forceinline__ void crypt_message(uint8_t *S, Rc4Lane &st, uint8_t *msg,
                                              uint32_t len, uint4 (&A)[4], bool pre)
{
    const uint32_t head = head_bytes(msg, len);
    for (uint32_t i = 0; i < head; ++i) msg[i] ^= (uint8_t)prga_step(S, st);
    msg += head;
    len -= head;

    uint4 *p = reinterpret_cast<uint4 *>(msg);
    const uint32_t nblk = len >> 6;
    if (nblk) {
        if (!pre) issue_block_asm(A, reinterpret_cast<const uint8_t *>(p));
        crypt_blocks_asm(st, p, nblk, A);
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

__device__ __forceinline__ uint32_t wave_max(uint32_t v)
{
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        const uint32_t o = __shfl_xor(v, m, 64);
        v = o > v ? o : v;
    }
    return v;
}

// ---------------------------------------------------------------------------
// Throughput-regime message loop with an in-register transpose (two
// workgroups per CU, crypt_stream_kernel).
//
// Why: whole 128-byte lines are the only fast store shape at 8 waves/CU
// (8 lanes per line: 5.65 TB/s vs 0.96 TB/s for per-lane 16-B pieces,
// tools/ubench/lds_ubench.hip), but a lane owns its own session's bytes.
// The 8x8 transpose of 16-byte chunks inside each group of 8 consecutive
// lanes runs on VALU with v_cndmask_b32_dpp butterflies (96 VALU per line per
// lane, no LDS: LDS staging cost ~11 % extra LDS cycles in this LDS-bound
// regime, r01 ablation), and the whole block loop is one asm statement
// generated by tools/gen_line_loop.py (zrc4_line_loop.inc) so every VMEM op
// is issued with the full exec mask and the vmcnt waits are exact counts:
//   * loads: per lane, the line two iterations ahead (blocks b+4, b+5),
//     clamped to the lane's sink slot past its session's end (whole-line
//     loads plus a second transpose were 4 % slower, r01);
//   * stores (nt): chunk i of the line of session 8g+q from lane 8g+i, or the
//     sink past that session's last block (ragged batches);
//   * exec is narrowed only around the keystream of each 64-byte block.
// The caller loads line 0 (P) before the S-box image fill and issues line 1
// (Q) after it (issue_line1_asm); the loop's first half skips its wait.
// ---------------------------------------------------------------------------
typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x32 __attribute__((ext_vector_type(32)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// ZRC4_PRIO (crypt_stream_kernel): the two workgroups of a CU share its SIMDs
// (one wave of each per SIMD) and the older wave wins the issue arbitration,
// so one workgroup runs ahead (a CU's two workgroups differ by up to 7 us per
// group, profiles/r02/stream_tl_pairs.log) and the other finishes alone at the
// 4-wave rate.  1: alternate which of a SIMD's two waves (wave slot parity,
// HW_ID) has the higher priority from one group to the next (cfg5 288.4 ->
// 284.2 us; alternating every line-loop half: 286.3, profiles/r02/ab_prio.log).
#ifndef ZRC4_PRIO
#define ZRC4_PRIO 1
#endif

#if defined(ZRC4_LL_AB) && ZRC4_LL_AB
#include "ab/zrc4_line_loop_ab.inc"   // timing-only A/B builds (tools/ab_bench.py --no-check)
#else
#include "zrc4_line_loop.inc"
#endif

constexpr uint32_t kSinkSlot = 256;                 // bytes of sink per thread (128-B line + offsets)
constexpr uint32_t kSinkBytes = kGroup * kSinkSlot  // one 64 KiB sink per context, shared by all workgroups
                                + (ZRC4_TIMING ? 16384u + kStampBytes : 0u);  // + where each timed wave ran, stream stamps

// line = blocks at b0 (16 B x 4) and b1 (16 B x 4)
__device__ __forceinline__ void preload_line(u32x32 &v, const uint8_t *b0, const uint8_t *b1)
{
    const u32x4 *p0 = reinterpret_cast<const u32x4 *>(b0);
    const u32x4 *p1 = reinterpret_cast<const u32x4 *>(b1);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const u32x4 t0 = p0[i], t1 = p1[i];
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            v[4 * i + d] = t0[d];
            v[16 + 4 * i + d] = t1[d];
        }
    }
}

// Everything about a group's messages the line loop needs that does not
// depend on the S-boxes, so it can be computed (and the first two lines
// loaded) before the group's S-box image is in LDS.
//   p      the message after its unaligned head bytes, nblk its 64-byte blocks
// The line roles (line_roles) are derived from these right where they are
// needed: holding 24 more VGPRs across a group boundary spilled the
// persistent kernel.
struct LineSetup {
    uint64_t p;
    uint32_t nblk, wmax;
};

__device__ __forceinline__ void line_setup(LineSetup &ls, const uint8_t *msg, uint32_t len)
{
    const uint32_t h = head_bytes(msg, len);
    ls.p = (uint64_t)(uintptr_t)(msg + h);
    ls.nblk = (len - h) >> 6;
    ls.wmax = __builtin_amdgcn_readfirstlane(wave_max(ls.nblk));
}

// Store role: lane 8g+i moves chunk i of the line of session 8g+q at addr_q;
// lim_q = blocks of that session minus (i >= 4), so chunk i of the line at
// block b exists iff b < lim_q.
__device__ __forceinline__ void line_roles(u32x16 &addr, u32x8 &lim, const LineSetup &ls)
{
    const uint32_t lane = threadIdx.x & 63u, i = lane & 7u;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const int src = (int)(lane & ~7u) | q;
        const uint64_t a = __shfl(ls.p, src, 64) + 16u * i;
        const uint32_t nb = __shfl(ls.nblk, src, 64);
        addr[2 * q] = (uint32_t)a;
        addr[2 * q + 1] = (uint32_t)(a >> 32);
        lim[q] = nb > (i >> 2) ? nb - (i >> 2) : 0u;
    }
}

// Line 0 (the lane's own blocks 0, 1; the sink past the session's end): the
// compiler's loads, retired before the S-box fill.
__device__ __forceinline__ void preload_line0(u32x32 &P, const LineSetup &ls, const uint8_t *sk)
{
    const uint8_t *p = reinterpret_cast<const uint8_t *>((uintptr_t)ls.p);
    const uint32_t nb = ls.nblk;
    preload_line(P, nb > 0 ? p : sk, nb > 1 ? p + 64 : sk + 64);
}

// Line 0 of the next group from asm (ZRC4_LINE0_ASM, r04 A/B knob, off):
// issued after the keystream, before the image copy-out, and waited for
// after the next fill with a counted vmcnt(16) (the 16 image stores are the
// only younger VMEM ops); as compiler loads the compiler drains everything
// there (vmcnt(0)), the image stores included.  Same-process medians
// (profiles/r04/grp/ab_range.log, ab_grouped.log): cfg5 287.2 vs 286.2 us,
// grouped cfg5 298.0 vs 296.4 -- the drain costs nothing measurable (most
// 1 KiB groups load line 0 inside the last half, p_async), so the simpler
// compiler form stays.
#ifndef ZRC4_LINE0_ASM
#define ZRC4_LINE0_ASM 0
#endif
__device__ __forceinline__ void issue_line0_asm(u32x32 &P, const LineSetup &ls, const uint8_t *sk)
{
    const uint8_t *p = reinterpret_cast<const uint8_t *>((uintptr_t)ls.p);
    const uint32_t nb = ls.nblk;
    const uint8_t *b0 = nb > 0 ? p : sk, *b1 = nb > 1 ? p + 64 : sk + 64;
    asm volatile(
        "global_load_dwordx4 v[40:43], %[a0], off\n\t"
        "global_load_dwordx4 v[44:47], %[a0], off offset:16\n\t"
        "global_load_dwordx4 v[48:51], %[a0], off offset:32\n\t"
        "global_load_dwordx4 v[52:55], %[a0], off offset:48\n\t"
        "global_load_dwordx4 v[56:59], %[a1], off\n\t"
        "global_load_dwordx4 v[60:63], %[a1], off offset:16\n\t"
        "global_load_dwordx4 v[64:67], %[a1], off offset:32\n\t"
        "global_load_dwordx4 v[68:71], %[a1], off offset:48\n\t"
        : "=&{v[40:71]}"(P)
        : [a0] "v"(b0), [a1] "v"(b1)
        : "memory");
}

// Line 1 (blocks 2, 3), issued from asm after the S-box fill, so it is in
// flight while line 0's keystream runs (the loop's first half is entered past
// its wait; the second half's counted wait retires it).  Only when the wave
// has a second line (wmax > 2): otherwise no half would wait for these
// registers before the compiler reuses them.
__device__ __forceinline__ void issue_line1_asm(u32x32 &Q, const LineSetup &ls, const uint8_t *sk)
{
    const uint8_t *p = reinterpret_cast<const uint8_t *>((uintptr_t)ls.p);
    const uint32_t nb = ls.nblk;
    const uint8_t *b0 = nb > 2 ? p + 128 : sk, *b1 = nb > 3 ? p + 192 : sk + 64;
    asm volatile(
        "global_load_dwordx4 v[72:75], %[a0], off\n\t"
        "global_load_dwordx4 v[76:79], %[a0], off offset:16\n\t"
        "global_load_dwordx4 v[80:83], %[a0], off offset:32\n\t"
        "global_load_dwordx4 v[84:87], %[a0], off offset:48\n\t"
        "global_load_dwordx4 v[88:91], %[a1], off\n\t"
        "global_load_dwordx4 v[92:95], %[a1], off offset:16\n\t"
        "global_load_dwordx4 v[96:99], %[a1], off offset:32\n\t"
        "global_load_dwordx4 v[100:103], %[a1], off offset:48\n\t"
        : "=&{v[72:103]}"(Q)
        : [a0] "v"(b0), [a1] "v"(b1)
        : "memory");
}

__device__ __forceinline__ uint32_t hw_id()
{
    uint32_t hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    return hw;
}

// The line loop, halves sb = 0, 2, ... until sb >= wend (wend = wmax: the
// whole message; wmax rounded down to a multiple of 4, minus 2: all but a
// final Q half, crypt_last_half_asm).  Returns sb.
__device__ __forceinline__ uint32_t crypt_lines_asm(Rc4Lane &st, u32x32 &P, u32x32 &Q, const LineSetup &ls,
                                                    u32x16 &addr, const u32x8 &lim, u32x2 sink, uint32_t &palo,
                                                    uint32_t &pahi, uint32_t wend)
{
    u32x16 X;
    u32x8 T;
    uint32_t b, k0, k1, a1s, sb, s1;
    uint64_t full, msk;
    asm volatile(
        "s_mov_b64 %[full], exec\n\t"
        "s_mov_b32 %[sb], 0\n\t"
        "s_branch LL_PSTART_%=\n\t"
        "LL_LOOP_%=:\n\t"
        ZRC4_LL_HALF_P
        ZRC4_LL_HALF_Q
        "s_branch LL_LOOP_%=\n\t"
        "LL_DONE_%=:\n\t"
        "s_mov_b64 exec, %[full]\n\t"
        "s_nop 1\n\t"                          // store-data VGPRs: VMEM store -> VALU write hazard
        : [ya] "+v"(st.ya), [ta] "+v"(st.ta), [x0] "+v"(st.x0), [x1] "+v"(st.x1), [a0] "+v"(st.a0),
          [a1] "=&v"(a1s), [b] "=&v"(b), [k0] "=&v"(k0), [k1] "=&v"(k1),
          [palo] "+v"(palo), [pahi] "+v"(pahi), [sb] "=&s"(sb), [s1] "=&s"(s1),
          [full] "=&s"(full), [msk] "=&s"(msk),
          "+{v[40:71]}"(P), "+{v[72:103]}"(Q), "=&{v[104:119]}"(X), "+{v[120:135]}"(addr),
          "=&{v[144:151]}"(T)
        : [nblk] "v"(ls.nblk), [wmax] "s"(ls.wmax), [wend] "s"(wend), "{v[136:143]}"(lim), "{v[152:153]}"(sink),
          [c100] "s"(0x100u)
        : "memory", "vcc", "scc");
    return sb;
}

// The next group's line 0 into P (v40..v71), in asm (ZRC4_NEXT_LINE0):
//   wait for the next group's entries (vmcnt(24): the youngest 24 VMEM ops
//   are the line loop's last loads and stores, or -- two halves -- this
//   group's second image), then per lane, as line_setup / preload_line0 do:
//   m = payload + off, L = valid ? len : 0, h = head bytes, nb = (L - h) / 64,
//   block 0 = nb > 0 ? m + h : sink, block 1 = nb > 1 ? m + h + 64 : sink + 64
//   (v144..v149 are the line loop's temporaries; the sink slot is v152:153).
#define ZRC4_NEXT_LINE0                                                                          \
    "s_waitcnt vmcnt(24)\n\t"                                                                    \
    "v_cmp_ne_u32_e32 vcc, 0, %[nv]\n\t"                                                         \
    "v_cndmask_b32_e32 %[nb], 0, %[nlen], vcc\n\t"                                               \
    "v_lshl_add_u64 v[144:145], %[noff], 0, %[pay]\n\t"                                          \
    "v_sub_u32_e32 %[h], 0, v144\n\t"                                                            \
    "v_and_b32_e32 %[h], 15, %[h]\n\t"                                                           \
    "v_min_u32_e32 %[h], %[h], %[nb]\n\t"                                                        \
    "v_sub_u32_e32 %[nb], %[nb], %[h]\n\t"                                                       \
    "v_lshrrev_b32_e32 %[nb], 6, %[nb]\n\t"                                                      \
    "v_add_co_u32_e32 v144, vcc, v144, %[h]\n\t"                                                 \
    "v_addc_co_u32_e32 v145, vcc, 0, v145, vcc\n\t"                                              \
    "v_lshl_add_u64 v[146:147], v[144:145], 0, 64\n\t"                                           \
    "v_lshl_add_u64 v[148:149], v[152:153], 0, 64\n\t"                                           \
    "v_cmp_lt_u32_e32 vcc, 0, %[nb]\n\t"                                                         \
    "v_cndmask_b32_e32 v144, v152, v144, vcc\n\t"                                                \
    "v_cndmask_b32_e32 v145, v153, v145, vcc\n\t"                                                \
    "v_cmp_lt_u32_e32 vcc, 1, %[nb]\n\t"                                                         \
    "v_cndmask_b32_e32 v146, v148, v146, vcc\n\t"                                                \
    "v_cndmask_b32_e32 v147, v149, v147, vcc\n\t"                                                \
    "global_load_dwordx4 v[40:43], v[144:145], off\n\t"                                          \
    "global_load_dwordx4 v[44:47], v[144:145], off offset:16\n\t"                                \
    "global_load_dwordx4 v[48:51], v[144:145], off offset:32\n\t"                                \
    "global_load_dwordx4 v[52:55], v[144:145], off offset:48\n\t"                                \
    "global_load_dwordx4 v[56:59], v[146:147], off\n\t"                                          \
    "global_load_dwordx4 v[60:63], v[146:147], off offset:16\n\t"                                \
    "global_load_dwordx4 v[64:67], v[146:147], off offset:32\n\t"                                \
    "global_load_dwordx4 v[68:71], v[146:147], off offset:48\n\t"

// The final Q half of a message with an even number of halves, preceded by
// the next group's line-0 loads -- in ONE asm statement: compiler code between
// the line loop and those loads could move the registers of a line still in
// flight.  The loads are younger than this half's line, so its counted waits
// never wait for them, and they have a whole half to land: the statement ends
// waiting for them, so P leaves it as an ordinary value (the compiler moves
// registers freely across the group boundary).
// nlen / noff: the next group's prefetched entry registers themselves (in
// flight until the wait; "+v" so the compiler takes them back from here and
// never copies them before it).
__device__ __forceinline__ void crypt_last_half_next_asm(Rc4Lane &st, u32x32 &P, u32x32 &Q, const LineSetup &ls,
                                                         u32x16 &addr, const u32x8 &lim, u32x2 sink, uint32_t &palo,
                                                         uint32_t &pahi, uint32_t sb, uint32_t &nlen, uint64_t &noff,
                                                         uint32_t nvalid, const uint8_t *payload)
{
    u32x16 X;
    u32x8 T;
    uint32_t b, k0, k1, a1s, s1, h, nb;
    uint64_t full, msk;
    asm volatile(
        "s_mov_b64 %[full], exec\n\t"
        ZRC4_NEXT_LINE0
        ZRC4_LL_HALF_QF
        "LL_DONE_%=:\n\t"
        "s_mov_b64 exec, %[full]\n\t"
        "s_waitcnt vmcnt(8)\n\t"             // the next line 0 (only this half's 8 stores are younger)
        "s_nop 1\n\t"
        : [ya] "+v"(st.ya), [ta] "+v"(st.ta), [x0] "+v"(st.x0), [x1] "+v"(st.x1), [a0] "+v"(st.a0),
          [a1] "=&v"(a1s), [b] "=&v"(b), [k0] "=&v"(k0), [k1] "=&v"(k1),
          [palo] "+v"(palo), [pahi] "+v"(pahi), [sb] "+s"(sb), [s1] "=&s"(s1),
          [full] "=&s"(full), [msk] "=&s"(msk), [h] "=&v"(h), [nb] "=&v"(nb), [nlen] "+v"(nlen), [noff] "+v"(noff),
          "+{v[40:71]}"(P), "+{v[72:103]}"(Q), "=&{v[104:119]}"(X), "+{v[120:135]}"(addr),
          "=&{v[144:151]}"(T)
        : [nblk] "v"(ls.nblk), [wmax] "s"(ls.wmax), [wend] "s"(ls.wmax), "{v[136:143]}"(lim),
          "{v[152:153]}"(sink), [nv] "v"(nvalid), [pay] "s"(payload), [c100] "s"(0x100u)
        : "memory", "vcc", "scc");
}

// One group's messages: head bytes, the line loop (line 0 in P, line 1 in
// flight into Q), then 16-byte chunks and tail bytes.  With `want_next`, a
// wave whose message has an even number of halves (>= 2) also fetches the
// next group's line 0 into P before its final half (nlen / noff / nvalid:
// that group's prefetched entry, crypt_last_half_next_asm); returns true when
// it did.
__device__ __forceinline__ bool crypt_message_dpp(uint8_t *S, Rc4Lane &st, uint8_t *msg, uint32_t len,
                                                  u32x32 &P, u32x32 &Q, const LineSetup &ls, uint8_t *sinkp,
                                                  bool want_next, uint32_t &nlen, uint64_t &noff, uint32_t nvalid,
                                                  const uint8_t *payload)
{
    const uint32_t head = head_bytes(msg, len);
    for (uint32_t i = 0; i < head; ++i) msg[i] ^= (uint8_t)prga_step(S, st);
    msg += head;
    len -= head;
    bool got = false;
    if (ls.wmax) {
        u32x16 addr;
        u32x8 lim;
        line_roles(addr, lim, ls);
        const uint64_t s = (uint64_t)(uintptr_t)sinkp;
        const u32x2 sk2 = u32x2{(uint32_t)s, (uint32_t)(s >> 32)};
        const uint64_t pa = ls.p + 256u;                 // per-lane loads: blocks 4, 5 next
        uint32_t palo = (uint32_t)pa, pahi = (uint32_t)(pa >> 32);
        const uint32_t halves = (ls.wmax + 1u) >> 1;
        got = want_next && halves >= 2u && !(halves & 1u);      // wave-uniform
        const uint32_t sb = crypt_lines_asm(st, P, Q, ls, addr, lim, sk2, palo, pahi,
                                            got ? 2u * (halves - 1u) : ls.wmax);
        if (got)
            crypt_last_half_next_asm(st, P, Q, ls, addr, lim, sk2, palo, pahi, sb, nlen, noff, nvalid, payload);
    }
    uint4 *p = reinterpret_cast<uint4 *>(msg + 64u * ls.nblk);
    uint32_t rem = len & 63u;
    while (rem >= 16u) {
        *p = xor16(S, st, *p);
        ++p;
        rem -= 16u;
    }
    uint8_t *t = reinterpret_cast<uint8_t *>(p);
    for (uint32_t k = 0; k < rem; ++k) t[k] ^= (uint8_t)prga_step(S, st);
    return got;
}

#define ZRC4_INVALID 0xFFFFFFFFu

// zrc4_crypt_grouped_declared with more buckets than the window kernel takes:
// the caller's declared groups (decl[b], ZRC4_INVALID = an idle bucket) are
// checked here, one workgroup per bucket, just before the crypt launch on the
// same stream.  A bucket with a busy entry (id < capacity, len > 0) outside
// its declared group latches kErrGroup and writes the crypt launch's epoch
// into every claim part of each group its busy entries name: the crypt
// kernel's workgroups that claim those groups then read back this launch's
// epoch and store nothing (the rule for two buckets naming one group).
__global__ void __launch_bounds__(256)
decl_check_kernel(const uint32_t *__restrict__ ids, const uint32_t *__restrict__ len, uint32_t n,
                  const uint32_t *__restrict__ decl, uint32_t capacity, Claim cl, uint32_t *__restrict__ err)
{
    __shared__ uint32_t bad;
    const uint32_t b = blockIdx.x, e = b * kGroup + threadIdx.x;
    if (threadIdx.x == 0) bad = 0u;
    __syncthreads();
    const uint32_t id = e < n ? ids[e] : ZRC4_INVALID;
    const bool busy = id < capacity && len[e] != 0u;
    if (busy && (id >> 8) != decl[b]) bad = 1u;
    __syncthreads();
    if (!bad) return;
    if (threadIdx.x == 0) latch_fault(err, kErrGroup);
    if (busy) {
        unsigned long long *w = cl.word + (size_t)(id >> 8) * kClaimParts;
        for (uint32_t p = 0; p < kClaimParts; ++p) w[p] = ((unsigned long long)cl.epoch << 32) | 0xFFFFFFFFull;
    }
}

// One group's 64 KiB S-box image, 16 x 16 B per lane into v160..v223, issued
// from asm and NOT waited for (the caller waits with a counted vmcnt).
// vo0 = the lane's byte offset in the first 4 KiB of the image; load i reads
// vo0 + i * 4 KiB (whole group: 16 * tid; half group h: rows of 16 lanes x
// 16 B starting at byte 128 * h of every 256-B row, image_lane_offset).
__device__ __forceinline__ uint32_t image_lane_offset(uint32_t tid, bool half, uint32_t h)
{
    return half ? ((tid >> 3) << 8) | (h << 7) | ((tid & 7u) << 4) : tid << 4;
}

// A declared grouped bucket's prologue loads in one asm statement
// (crypt_body<kGrouped, DECL>): the thread's K entries (id, length, offset),
// its x/y, then the group's image; the entries and x/y are waited for before
// the statement ends (vmcnt(16): only the image is younger), the image stays
// in flight as issue_image_asm leaves it.  As compiler loads the entries and
// x/y would be waited for with vmcnt(0) -- draining the 64 KiB image, issued
// after them, before the bucket's table could be built.
#define ZRC4_DECL_IMAGE                                                                          \
    "global_load_dwordx4 v[160:163], %[vo], %[ib]\n\t"                                           \
    "v_add_u32 %[vo], 0x1000, %[vo]\n\t"                                                         \
    "global_load_dwordx4 v[164:167], %[vo], %[ib]\n\t"                                           \
    "v_add_u32 %[vo], 0x1000, %[vo]\n\t"                                                         \
    "global_load_dwordx4 v[168:171], %[vo], %[ib]\n\t"                                           \
    "v_add_u32 %[vo], 0x1000, %[vo]\n\t"                                                         \
    "global_load_dwordx4 v[172:175], %[vo], %[ib]\n\t"                                           \
    "v_add_u32 %[vo], 0x1000, %[vo]\n\t"                                                         \
    "global_load_dwordx4 v[176:179], %[vo], %[ib]\n\t"                                           \
    "v_add_u32 %[vo], 0x1000, %[vo]\n\t"                                                         \
    "global_load_dwordx4 v[180:183], %[vo], %[ib]\n\t"                                           \
    "v_add_u32 %[vo], 0x1000, %[vo]\n\t"                                                         \
    "global_load_dwordx4 v[184:187], %[vo], %[ib]\n\t"                                           \
    "v_add_u32 %[vo], 0x1000, %[vo]\n\t"                                                         \
    "global_load_dwordx4 v[188:191], %[vo], %[ib]\n\t"                                           \
    "v_add_u32 %[vo], 0x1000, %[vo]\n\t"                                                         \
    "global_load_dwordx4 v[192:195], %[vo], %[ib]\n\t"                                           \
    "v_add_u32 %[vo], 0x1000, %[vo]\n\t"                                                         \
    "global_load_dwordx4 v[196:199], %[vo], %[ib]\n\t"                                           \
    "v_add_u32 %[vo], 0x1000, %[vo]\n\t"                                                         \
    "global_load_dwordx4 v[200:203], %[vo], %[ib]\n\t"                                           \
    "v_add_u32 %[vo], 0x1000, %[vo]\n\t"                                                         \
    "global_load_dwordx4 v[204:207], %[vo], %[ib]\n\t"                                           \
    "v_add_u32 %[vo], 0x1000, %[vo]\n\t"                                                         \
    "global_load_dwordx4 v[208:211], %[vo], %[ib]\n\t"                                           \
    "v_add_u32 %[vo], 0x1000, %[vo]\n\t"                                                         \
    "global_load_dwordx4 v[212:215], %[vo], %[ib]\n\t"                                           \
    "v_add_u32 %[vo], 0x1000, %[vo]\n\t"                                                         \
    "global_load_dwordx4 v[216:219], %[vo], %[ib]\n\t"                                           \
    "v_add_u32 %[vo], 0x1000, %[vo]\n\t"                                                         \
    "global_load_dwordx4 v[220:223], %[vo], %[ib]\n\t"                                           \
    "s_waitcnt vmcnt(16)\n\t"
__device__ __forceinline__ void decl_prologue_asm1(uint32_t &id0, uint32_t &ln0, uint64_t &of0, uint32_t &xyv,
                                                   u32x32 &ilo, u32x32 &ihi, const uint32_t *aid0,
                                                   const uint32_t *aln0, const uint64_t *aof0, const uint16_t *axy,
                                                   const uint8_t *ibase, uint32_t vo0)
{
    uint32_t vo = vo0;
    asm volatile(
        "global_load_dword %[id0], %[aid0], off\n\t"
        "global_load_dword %[ln0], %[aln0], off\n\t"
        "global_load_dwordx2 %[of0], %[aof0], off\n\t"
        "global_load_ushort %[xyv], %[axy], off\n\t"
        ZRC4_DECL_IMAGE
        : [id0] "=&v"(id0), [ln0] "=&v"(ln0), [of0] "=&v"(of0), [xyv] "=&v"(xyv),
          "=&{v[160:191]}"(ilo), "=&{v[192:223]}"(ihi), [vo] "+v"(vo)
        : [aid0] "v"(aid0), [aln0] "v"(aln0), [aof0] "v"(aof0), [axy] "v"(axy), [ib] "s"(ibase)
        : "memory");
}
__device__ __forceinline__ void decl_prologue_asm2(uint32_t &id0, uint32_t &ln0, uint64_t &of0, uint32_t &id1,
                                                   uint32_t &ln1, uint64_t &of1, uint32_t &xyv, u32x32 &ilo,
                                                   u32x32 &ihi, const uint32_t *aid0, const uint32_t *aln0,
                                                   const uint64_t *aof0, const uint32_t *aid1, const uint32_t *aln1,
                                                   const uint64_t *aof1, const uint16_t *axy, const uint8_t *ibase,
                                                   uint32_t vo0)
{
    uint32_t vo = vo0;
    asm volatile(
        "global_load_dword %[id0], %[aid0], off\n\t"
        "global_load_dword %[ln0], %[aln0], off\n\t"
        "global_load_dwordx2 %[of0], %[aof0], off\n\t"
        "global_load_dword %[id1], %[aid1], off\n\t"
        "global_load_dword %[ln1], %[aln1], off\n\t"
        "global_load_dwordx2 %[of1], %[aof1], off\n\t"
        "global_load_ushort %[xyv], %[axy], off\n\t"
        ZRC4_DECL_IMAGE
        : [id0] "=&v"(id0), [ln0] "=&v"(ln0), [of0] "=&v"(of0), [id1] "=&v"(id1), [ln1] "=&v"(ln1),
          [of1] "=&v"(of1), [xyv] "=&v"(xyv), "=&{v[160:191]}"(ilo), "=&{v[192:223]}"(ihi), [vo] "+v"(vo)
        : [aid0] "v"(aid0), [aln0] "v"(aln0), [aof0] "v"(aof0), [aid1] "v"(aid1), [aln1] "v"(aln1),
          [aof1] "v"(aof1), [axy] "v"(axy), [ib] "s"(ibase)
        : "memory");
}
#undef ZRC4_DECL_IMAGE

__device__ __forceinline__ void issue_image_asm(u32x32 &ilo, u32x32 &ihi, const uint8_t *ibase, uint32_t vo0)
{
    uint32_t vo;
    asm volatile(
        "v_mov_b32 %[vo], %[j]\n\t"
        "global_load_dwordx4 v[160:163], %[vo], %[ib]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_load_dwordx4 v[164:167], %[vo], %[ib]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_load_dwordx4 v[168:171], %[vo], %[ib]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_load_dwordx4 v[172:175], %[vo], %[ib]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_load_dwordx4 v[176:179], %[vo], %[ib]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_load_dwordx4 v[180:183], %[vo], %[ib]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_load_dwordx4 v[184:187], %[vo], %[ib]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_load_dwordx4 v[188:191], %[vo], %[ib]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_load_dwordx4 v[192:195], %[vo], %[ib]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_load_dwordx4 v[196:199], %[vo], %[ib]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_load_dwordx4 v[200:203], %[vo], %[ib]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_load_dwordx4 v[204:207], %[vo], %[ib]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_load_dwordx4 v[208:211], %[vo], %[ib]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_load_dwordx4 v[212:215], %[vo], %[ib]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_load_dwordx4 v[216:219], %[vo], %[ib]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_load_dwordx4 v[220:223], %[vo], %[ib]\n\t"
        : "=&{v[160:191]}"(ilo), "=&{v[192:223]}"(ihi), [vo] "=&v"(vo)
        : [ib] "s"(ibase), [j] "v"(vo0)
        : "memory");
}


// ---------------------------------------------------------------------------
// crypt_kernel: batched RC4Encryption::encryption, one group (or, HALF, one
// half group) per workgroup: launches with at most one group per CU, the
// chain-bound regime.  How batch entry e maps to a slot (MODE):
//   kRange    slot = first_slot + e (ids == NULL; the bench's and the
//             engine's contiguous batches).  The slot is arithmetic and the
//             host has checked first_slot + n <= capacity, so the group image
//             is issued from asm first, then len/off/x-y (no load waits on
//             another: one HBM round trip); the first payload block is
//             issued after a counted wait, so its round trip overlaps the LDS
//             fill.  Whole (coalesced image) iff first_slot % 256 == 0.
//   kGrouped  slot = ids[e]; the caller promises bucket w's busy entries all
//             lie in ONE 256-slot group that no other bucket of the call
//             touches (zrc4_crypt_grouped).  The entries are permuted through
//             LDS so that lane j runs slot g*256 + j (its own, bank-conflict
//             free column; running entries in their given order put lanes of
//             one half-wave on the same LDS banks: cfg2 73.6 vs 48.9 us), and
//             the group image moves as one coalesced copy, so any subset of a
//             group in any order costs what a whole group costs.  A bucket
//             that mixes groups (or repeats a slot) latches kErrGroup and is
//             skipped.
//   kIds      slot = ids[e], arbitrary: whole iff the 256 ids are exactly
//             g*256 .. g*256+255 in order, otherwise each lane gathers and
//             scatters its own 256-byte column (correct, strided).
// HALF (kRange with first_slot % 256 == 0, or kGrouped; few groups): 128-thread workgroups,
// each owning the two waves of a group whose S-boxes share the dwords of one
// 128-byte half of every image row (col_of: (wave >> 1) picks the half), so
// each moves a 32 KiB half image.  The workgroup reserves more LDS than it
// uses so that no two share a CU: at 2 waves per CU a chain step takes
// 41.2 us per KiB against 43.1 at 4 (profiles/r02/tl_waves.log).
// ---------------------------------------------------------------------------
enum CryptMode : int { kIds = 0, kRange = 1, kGrouped = 2 };

// ---------------------------------------------------------------------------
// proto4z framing of decrypted session buffers:
// TcpSession::onRecv's loop (src/frame/session.cpp:329-371) over HasRawPacket
// (depends/proto4z/proto4z.h:704-748): walk from the buffer start, one packet
// per check, until shortage (status 1) or corruption (status 2).  One lane per
// session: a chain of dependent header reads (4 byte loads each, headers sit
// at any alignment).  Bytes past the last header read are never touched.
// Used standalone (frame_scan_kernel) and fused into crypt_kernel's epilogue
// (FRAME = true: each lane frames its own session right after decrypting it,
// no second launch).
// ---------------------------------------------------------------------------
struct FrameArgs {
    const uint64_t *off;   // buffer of entry e = payload + off[e] ...
    const uint32_t *len;   // ... len[e] bytes (the whole receive block, not just the decrypted tail)
    uint32_t bound, maxp;
    uint32_t *npk, *used, *status, *pkt_len;
};

__device__ __forceinline__ uint32_t load_le32(const uint8_t *p)
{
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// HasRawPacket's checks (proto4z.h:704-748) around one header read at u:
// frame_pre before it (0 = read the header), frame_post after it (0 = a
// complete packet of pl bytes); otherwise the stop status.
__device__ __forceinline__ uint32_t frame_pre(uint32_t L, uint32_t u, uint32_t bound)
{
    const uint32_t cur = L - u, bl = bound - u;
    if (bl < cur || bound < bl) return 2u;                        // :708-711
    if (cur < 6u) return 1u;                                      // :715-718 (headLen = 4 + 2, :714)
    return 0u;
}

__device__ __forceinline__ uint32_t frame_post(uint32_t pl, uint32_t L, uint32_t u, uint32_t bound)
{
    const uint32_t cur = L - u, bl = bound - u;
    if (pl < 6u) return 2u;                                       // :718-721
    if (pl > bl) return pl > bound ? 2u : 1u;                     // :722-732
    if (pl > bound) return 2u;                                    // :735-738
    if (pl > cur) return 1u;                                      // :747
    return 0u;
}

__device__ __forceinline__ void frame_walk(const uint8_t *b, uint32_t L, uint32_t bound, uint32_t maxp, uint32_t e,
                                           uint32_t *npk, uint32_t *used, uint32_t *status, uint32_t *pkt_len)
{
    uint32_t u = 0, k = 0, st;
    for (;;) {
        st = frame_pre(L, u, bound);
        if (st) break;
        const uint32_t pl = load_le32(b + u);                     // ReadPodData, :717
        st = frame_post(pl, L, u, bound);
        if (st) break;
        if (pkt_len && k < maxp) pkt_len[(size_t)e * maxp + k] = pl;
        ++k;
        u += pl;
    }
    npk[e] = k;
    used[e] = u;
    status[e] = st;
}

// The framing of every entry of the 256-entry chunks c0, c0 + step, ... <
// nchunks (entry c * 256 + lane): the persistent kernel's tail, after its own
// stores have landed.  Four chunks' walks advance in lockstep, so a lane's
// four header reads per round are in flight together (each walk is a chain
// of dependent round trips).
__device__ __forceinline__ void frame_walk_chunks(const uint8_t *payload, const FrameArgs &fr, uint32_t c0,
                                                  uint32_t step, uint32_t nchunks, uint32_t n, uint32_t lane)
{
    constexpr int kW = 4;
    for (uint32_t c = c0; c < nchunks; c += kW * step) {
        const uint8_t *b[kW];
        uint32_t L[kW], u[kW], k[kW], st[kW], e[kW];
        bool live[kW], valid[kW];
#pragma unroll
        for (int i = 0; i < kW; ++i) {
            const uint32_t ci = c + (uint32_t)i * step;
            e[i] = ci * kGroup + lane;
            valid[i] = ci < nchunks && e[i] < n;
            live[i] = valid[i];
            b[i] = payload + (valid[i] ? fr.off[e[i]] : 0u);
            L[i] = valid[i] ? fr.len[e[i]] : 0u;
            u[i] = k[i] = st[i] = 0u;
        }
        while (live[0] || live[1] || live[2] || live[3]) {
            uint32_t pl[kW];
#pragma unroll
            for (int i = 0; i < kW; ++i) {
                if (live[i]) {
                    st[i] = frame_pre(L[i], u[i], fr.bound);
                    live[i] = st[i] == 0u;
                    if (live[i]) pl[i] = load_le32(b[i] + u[i]);
                }
            }
#pragma unroll
            for (int i = 0; i < kW; ++i) {
                if (live[i]) {
                    st[i] = frame_post(pl[i], L[i], u[i], fr.bound);
                    live[i] = st[i] == 0u;
                    if (live[i]) {
                        if (fr.pkt_len && k[i] < fr.maxp) fr.pkt_len[(size_t)e[i] * fr.maxp + k[i]] = pl[i];
                        ++k[i];
                        u[i] += pl[i];
                    }
                }
            }
        }
#pragma unroll
        for (int i = 0; i < kW; ++i) {
            if (valid[i]) {
                fr.npk[e[i]] = k[i];
                fr.used[e[i]] = u[i];
                fr.status[e[i]] = st[i];
            }
        }
    }
}

// LDS of crypt_kernel: the 64 KiB S-box image at offset 0 (the asm's absolute
// addresses), then 16 B of flags, then the kGrouped entry table (slot -> entry
// index / length / offset).  HALF pads the allocation past 80 KiB so that a
// CU holds one workgroup.
#ifndef ZRC4_HALF_PAD
#define ZRC4_HALF_PAD 1
#endif
#ifndef ZRC4_WPERM
#define ZRC4_WPERM 97
#endif
#ifndef ZRC4_WMAP
#define ZRC4_WMAP 1
#endif
constexpr uint32_t kTabOff = kGroupBytes + 16;
constexpr uint32_t kSidOff = kTabOff + 256 * 16;              // 16 B: the half-group workgroup's SIMD ids
constexpr uint32_t kSmemDirect = kSidOff + 16;                // 69 664 B: two workgroups per CU
constexpr uint32_t kSmemHalf = 96 * 1024;                     // one workgroup per CU

// Workgroup k runs on XCD k mod 8.  xcd_run_map deals the groups so that
// each XCD takes runs of R = ZRC4_XCD_RUN consecutive groups per 8R: k =
// 8R s + 8 r + x -> 8R s + R x + r (bijective; a tail of grid mod 8R groups
// keeps its order; R = 1 is the identity).
#ifndef ZRC4_XCD_RUN
#define ZRC4_XCD_RUN 8
#endif
static_assert(ZRC4_XCD_RUN >= 1 && ZRC4_XCD_RUN <= 32 && (ZRC4_XCD_RUN & (ZRC4_XCD_RUN - 1)) == 0,
              "XCD run length: a power of two");
__device__ __forceinline__ uint32_t xcd_run_map(uint32_t k, uint32_t grid)
{
    constexpr uint32_t R = ZRC4_XCD_RUN, B = 8u * R;
    if (k >= (grid & ~(B - 1u))) return k;
    return (k & ~(B - 1u)) | ((k & 7u) * R) | ((k >> 3) & (R - 1u));
}

// ZRC4_PAIR_DIRECT: whole-group range launches (crypt_kernel<kRange>) by
// wave pairs as the persistent kernel (pair_meet, img_vo): each pair fills,
// runs and copies out its half image without waiting for the other.
// Measured, not kept: with one group per workgroup there is no boundary to
// decouple, only the fill and the end (same process,
// profiles/r04/pdirect/ab_direct.log: cfg3 25.50 vs 25.32 us with the
// barriers, 65 536 x 1 KiB 58.44 vs 58.24, x 512 B 36.60 vs 36.32).
#ifndef ZRC4_PAIR_DIRECT
#define ZRC4_PAIR_DIRECT 0
#endif
__device__ __forceinline__ void pair_meet_d(uint32_t *ctr, uint32_t &gen)
{
    ++gen;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if ((threadIdx.x & 63u) == 0u) __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    while (__builtin_amdgcn_readfirstlane(__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) <
           2u * gen)
        __builtin_amdgcn_s_sleep(1);
    asm volatile("" ::: "memory");
}

// Declared bucket groups of a grouped launch of at most 256 buckets on the
// half-group and whole-group kernels (zrc4_crypt_grouped_declared): bucket
// b's group, ZRC4_INVALID for a bucket with no busy entry.  By value, so it
// sits in the kernel-argument segment (1 KiB).
constexpr uint32_t kBodyMaxBuckets = 256;
struct BucketGroups {
    uint32_t g[kBodyMaxBuckets];
};

template <int MODE, bool FRAME, bool HALF, bool DECL = false>
__device__ __forceinline__ void
crypt_body(uint8_t *__restrict__ arena, uint16_t *__restrict__ xy,
           const uint32_t *__restrict__ ids, uint32_t first_slot,
           uint8_t *__restrict__ payload, const uint64_t *__restrict__ off,
           const uint32_t *__restrict__ len, uint32_t n, uint32_t capacity,
           uint32_t *__restrict__ err, uint8_t *__restrict__ sink, const FrameArgs &fr, const Claim &cl,
           const BucketGroups *dg = nullptr)
{
    static_assert(!HALF || MODE != kIds, "half-group workgroups run range and grouped batches");
    static_assert(!DECL || MODE == kGrouped, "declared groups are a grouped-batch form");
    __shared__ __attribute__((aligned(16))) uint8_t smem[HALF ? kSmemHalf : kSmemDirect];
    uint8_t *S = smem;
    if (!lds_base_ok(S, err)) return;
    Stamps ts;
    stamp(ts, 0);

    constexpr uint32_t kLanes = HALF ? 128u : 256u;
    uint32_t tid = threadIdx.x;
    if constexpr (HALF && ZRC4_HALF_PAD) {
        // The workgroup has 4 waves; the two that work are the ones on SIMDs
        // 1 and 2 (else 1 and 3).  Measured per wave (in-kernel clocks,
        // tools/kernel_timeline.py --placement, profiles/r02/placement_*.log):
        // a lone wave runs the step at 96 cycles/byte on SIMDs 1-3 and 100 on
        // SIMD 0; a pair runs at 96 only when one of them is on SIMD 1
        // ({2,3}, {0,2}, {0,3} pairs: 100).  The other two waves end here.
        uint32_t hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        uint32_t *sid = reinterpret_cast<uint32_t *>(smem + kSidOff);
        const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        if ((threadIdx.x & 63u) == 0u) sid[w] = (hw >> 4) & 3u;
        __syncthreads();
        uint32_t ss[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) ss[i] = __builtin_amdgcn_readfirstlane(sid[i]);
        uint32_t a = 4u, b = 4u, c = 4u;
#pragma unroll
        for (uint32_t i = 0; i < 4u; ++i) {
            if (a == 4u && ss[i] == 1u) a = i;
            if (b == 4u && ss[i] == 2u) b = i;
            if (c == 4u && ss[i] == 3u) c = i;
        }
        if (b == 4u) b = c;
        if (a == 4u || b == 4u) { a = 0u; b = 1u; }      // waves not one per SIMD: the first two
        if (w != a && w != b) return;                    // uniform (SGPR) branch: the wave ends
        tid = (w == a ? 0u : 64u) + (threadIdx.x & 63u);
    }
    // Which group (bucket) this workgroup runs.  Whole-group launches deal
    // the groups to the XCDs in runs of 8 consecutive groups (xcd_run_map,
    // ZRC4_WMAP, r03): with workgroup k -> group k (or r02's 97k mod grid,
    // ZRC4_WMAP=0) XCD x ran only the groups = x mod 8, whose payload and
    // images sit at one offset modulo 8 groups, and the XCD's L2 evicted the
    // lanes' partly written 128-byte lines early: 1.25x the algorithmic write
    // bytes at 256-byte messages, 1.00x with the runs; 65 536 x 1 KiB 60.5 ->
    // 57.2 us, x 2 KiB 110.7 -> 100.3; cfg3 22.9 -> 23.5 (same-process
    // medians, profiles/r03/wmap/).  Half-group launches keep k -> (k/2, k%2)
    // (their A/B was neutral to +2.5 %).
    uint32_t wg = blockIdx.x;
#if ZRC4_WMAP
    if constexpr (!HALF) wg = xcd_run_map(blockIdx.x, gridDim.x);
#else
    if constexpr (!HALF && ZRC4_WPERM != 0) {
        constexpr uint32_t kMul = ZRC4_WPERM + 0u;
        if (gridDim.x % kMul != 0u) wg = (blockIdx.x * kMul) % gridDim.x;
    }
#endif
#if defined(ZRC4_STAGGER) && ZRC4_STAGGER
    // A/B diagnostic (cfg3 write traffic): workgroup start spread over
    // 0..7 x ZRC4_STAGGER x 64 cycles, as a grouped launch's longer prologue spreads it
    if constexpr (MODE == kRange && !HALF)
        for (uint32_t i = 0; i < (blockIdx.x & 7u); ++i) __builtin_amdgcn_s_sleep(ZRC4_STAGGER);
#endif
    const uint32_t e = wg * kLanes + tid;                // batch entry of this thread
    const bool valid = e < n;
    const uint32_t h = HALF ? (wg & 1u) : 0u;            // half of the group (HALF)
    const uint32_t j = h * 128u + tid;                   // group lane
    // (range whole groups by pairs: thread j's chunks sit in its pair's half rows)
    constexpr bool PD = MODE == kRange && !HALF && ZRC4_PAIR_DIRECT;
    const uint32_t vo0 = PD ? image_lane_offset(tid & 127u, true, tid >> 7) : image_lane_offset(tid, HALF, h);
    uint32_t *pdc = reinterpret_cast<uint32_t *>(smem + kGroupBytes) + 4u + __builtin_amdgcn_readfirstlane(tid >> 7);
    uint32_t pdg = 0;
    if constexpr (PD) {
        if (tid < 2u) reinterpret_cast<uint32_t *>(smem + kGroupBytes)[4u + tid] = 0u;
        __syncthreads();
    }
    const uint32_t col = col_of(j);
    // (plain LDS words, ordered by the barriers: as `volatile` they compiled
    // to flat stores with a vmcnt(0) after each, which drained the grouped
    // prologue's image loads before the bucket's table was even built)
    uint32_t *flag = reinterpret_cast<uint32_t *>(smem + kGroupBytes);
    uint4 img[16];
    u32x32 ilo, ihi;

    bool whole;
    uint32_t g, slot, mylen, ent;   // ent: the batch entry this lane runs (kGrouped permutes)
    uint64_t myoff;
    uint16_t sxy;
    if constexpr (MODE == kRange) {
        // Issued from asm, first: hipcc otherwise sinks these loads below its
        // wait for len/off.  Group (first_slot >> 8) + w lies inside the arena
        // even when first_slot is unaligned and the image goes unused.
        g = (first_slot >> 8) + (HALF ? wg >> 1 : wg);
        issue_image_asm(ilo, ihi, arena + (size_t)g * kGroupBytes, vo0);
        whole = (first_slot & 255u) == 0u;
        ent = e;
        mylen = valid ? len[e] : 0u;
        myoff = valid ? off[e] : 0u;
        slot = valid ? first_slot + e : ZRC4_INVALID;
        sxy = valid ? xy[slot] : (uint16_t)0;
    } else if constexpr (MODE == kGrouped) {
        // 1. the bucket's entries (HALF: both halves read all 256, each
        //    thread kPer of them); 2. its group (every busy entry must name
        //    the same one: checked per wave against the wave's guess, then
        //    across waves by one atomic min/max per wave) and the slot ->
        //    entry table; 3. lane j takes the entry of slot g*256 + j.
        constexpr uint32_t kPer = kGroup / kLanes;
        const uint32_t w = HALF ? wg >> 1 : wg;
        uint32_t *te = reinterpret_cast<uint32_t *>(smem + kTabOff);          // entry index
        uint32_t *tl = te + 256;                                              // length
        uint64_t *to = reinterpret_cast<uint64_t *>(smem + kTabOff + 2048);   // offset
        uint32_t idq[kPer], lq[kPer];
        uint64_t oq[kPer];
        bool bq[kPer];
        // DECL: the caller's group for this bucket; its image (asm), x/y and
        // claim leave before the entries, so the entries' round trip covers
        // them (the entry checks below wait for the younger entries, hence
        // for the image too: one round trip, not two)
        uint32_t gdecl = ZRC4_INVALID;
        uint16_t xyd = 0;
        unsigned long long coldd = 0;
        uint32_t rid[kPer], rln[kPer];
        uint64_t rof[kPer];
        if constexpr (DECL) {
            // The entries, x/y and image in one asm statement (decl_prologue_asm*),
            // the entries and x/y waited for inside it; an idle bucket reads
            // group 0's image and drops it (the image registers are loaded on
            // every path: merged with an undefined value, the compiler copied
            // them while in flight).  The claim: thread 0, asm, waited for
            // with the image before the fill.
            gdecl = dg->g[w];
            const uint32_t gl = gdecl != ZRC4_INVALID ? gdecl : 0u;
            const uint32_t e0 = w * kGroup + tid, c0 = e0 < n ? e0 : n - 1u;
            uint32_t xv;
            if constexpr (kPer == 1) {
                decl_prologue_asm1(rid[0], rln[0], rof[0], xv, ilo, ihi, ids + c0, len + c0, off + c0,
                                   xy + gl * 256u + j, arena + (size_t)gl * kGroupBytes, vo0);
            } else {
                const uint32_t e1 = e0 + kLanes, c1 = e1 < n ? e1 : n - 1u;
                decl_prologue_asm2(rid[0], rln[0], rof[0], rid[kPer - 1], rln[kPer - 1], rof[kPer - 1], xv, ilo,
                                   ihi, ids + c0, len + c0, off + c0, ids + c1, len + c1, off + c1,
                                   xy + gl * 256u + j, arena + (size_t)gl * kGroupBytes, vo0);
            }
            xyd = (uint16_t)xv;
            // thread 0 (lane 0 of wave 0) claims; the predicate is wave-uniform
            // and tested inside the asm, which every wave runs (no merge)
            coldd = claim_part_async_if(cl, gl, HALF ? h : 0u, w,
                                        (gdecl != ZRC4_INVALID && __builtin_amdgcn_readfirstlane(tid >> 6) == 0u)
                                            ? 1u : 0u);
        }
#pragma unroll
        for (uint32_t q = 0; q < kPer; ++q) {
            const uint32_t eq = w * kGroup + q * kLanes + tid;
            const bool vq = eq < n;
            uint32_t id = vq ? (DECL ? rid[q] : ids[eq]) : ZRC4_INVALID;
            lq[q] = vq ? (DECL ? rln[q] : len[eq]) : 0u;
            oq[q] = vq ? (DECL ? rof[q] : off[eq]) : 0u;
            if (vq && id >= capacity && id != ZRC4_INVALID) {   // ZRC4_IDLE_SLOT pads buckets
                latch_fault(err, kErrSlotRange);
                id = ZRC4_INVALID;
            }
            idq[q] = id;
            bq[q] = id != ZRC4_INVALID && lq[q] != 0u;
        }
        // Speculative image (and x/y) issue: the wave's first busy id names
        // the bucket's group, so the image load overlaps the table build.  A
        // wave with no busy entry (or a wrong guess: a contract violation,
        // refused below) loads again once the group is known.
        bool have = false;
        uint32_t gw = 0;
        uint16_t xyw = 0;
        unsigned long long cold = 0;
        if constexpr (DECL) {
            have = gdecl != ZRC4_INVALID;
            gw = have ? gdecl : 0u;
            xyw = xyd;
            cold = coldd;
        } else {
#pragma unroll
            for (uint32_t q = 0; q < kPer; ++q) {
                const uint64_t bm = __ballot(bq[q]);
                if (!have && bm) {
                    gw = __builtin_amdgcn_readlane(idq[q], (int)__builtin_ctzll(bm)) >> 8;
                    have = true;
                }
            }
            issue_image_asm(ilo, ihi, arena + (size_t)gw * kGroupBytes, vo0);
            xyw = xy[gw * 256u + j];
            // the claim of this workgroup's part of the group (Claim), by
            // thread 0 on its wave's guess; re-issued below if that wave had
            // no busy entry
            if (tid == 0 && have) cold = claim_part(cl, gw, HALF ? h : 0u, w);
        }
#pragma unroll
        for (uint32_t q = 0; q < kPer; ++q) te[q * kLanes + tid] = ZRC4_INVALID;
        if (tid == 0) {
            flag[0] = 0xFFFFFFFFu;
            flag[1] = 0u;
            flag[2] = 0u;
            flag[3] = 0u;
        }
        __syncthreads();
        if (have && (tid & 63u) == 0u) {
            atomicMin(flag, gw);
            atomicMax(flag + 1, gw);
        }
#pragma unroll
        for (uint32_t q = 0; q < kPer; ++q) {
            if (bq[q]) {
                const uint32_t k = idq[q] & 255u;
                if (DECL && !have) flag[2] = 1u;                                          // declared idle, yet busy
                if ((idq[q] >> 8) != gw) flag[2] = 1u;                                  // another group
                if (atomicExch(&te[k], w * kGroup + q * kLanes + tid) != ZRC4_INVALID) flag[2] = 1u;   // a slot twice
                tl[k] = lq[q];
                to[k] = oq[q];
            }
        }
        const bool busy = bq[HALF ? h : 0u];             // this thread's own entry e
        __syncthreads();
        const uint32_t gmin = flag[0], gmax = flag[1], dup = flag[2];
        if (gmin == 0xFFFFFFFFu || gmin != gmax || dup) {
            if ((gmin != 0xFFFFFFFFu || dup) && tid == 0) latch_fault(err, kErrGroup);
            if constexpr (DECL)                          // (no load left in flight at exit)
                asm volatile("s_waitcnt vmcnt(0)" : "+{v[160:191]}"(ilo), "+{v[192:223]}"(ihi) :: "memory");
            if constexpr (FRAME) {                       // an idle bucket still reports its framing
                // (a refused one writes nothing: a bucket declared idle that
                // holds a busy entry has gmin == INVALID and dup set)
                if (valid && gmin == 0xFFFFFFFFu && !dup)
                    frame_walk(payload + fr.off[e], fr.len[e], fr.bound, fr.maxp, e, fr.npk, fr.used, fr.status,
                               fr.pkt_len);
            }
            return;
        }
        g = __builtin_amdgcn_readfirstlane(gmin);       // uniform (an SGPR base for the asm loads)
        whole = true;
        ent = te[j];
        mylen = ent != ZRC4_INVALID ? tl[j] : 0u;
        myoff = ent != ZRC4_INVALID ? to[j] : 0u;
        slot = g * 256u + j;
        sxy = xyw;
        if (!DECL && (!have || gw != g)) {               // wave-uniform: the guess missed
            asm volatile("s_waitcnt vmcnt(0)" : "+{v[160:191]}"(ilo), "+{v[192:223]}"(ihi) :: "memory");
            issue_image_asm(ilo, ihi, arena + (size_t)g * kGroupBytes, vo0);
            sxy = xy[slot];
        }
        if (!DECL && tid == 0 && !have) cold = claim_part(cl, g, HALF ? h : 0u, w);
        if constexpr (DECL) claim_wait(cold);            // (the image too: it is needed by the fill next)
        if (tid == 0) flag[3] = claim_lost(cl, cold) ? 1u : 0u;          // read after the fill barrier
        if (!mylen) sxy = 0;
        if constexpr (FRAME) {
            // entries that decrypt nothing are framed by their own thread now
            if (valid && !busy)
                frame_walk(payload + fr.off[e], fr.len[e], fr.bound, fr.maxp, e, fr.npk, fr.used, fr.status,
                           fr.pkt_len);
        }
    } else {
        ent = e;
        slot = valid ? ids[e] : ZRC4_INVALID;
        if (valid && slot >= capacity) {
            latch_fault(err, kErrSlotRange);
            slot = ZRC4_INVALID;
        }
        mylen = slot != ZRC4_INVALID ? len[e] : 0u;
        myoff = slot != ZRC4_INVALID ? off[e] : 0u;
        sxy = mylen ? xy[slot] : (uint16_t)0;
        const uint32_t first = ids[wg * kGroup];
        g = first >> 8;
        if (tid == 0) flag[0] = 1u;
        __syncthreads();
        if (!(slot != ZRC4_INVALID && slot == ((first & ~255u) + j) && (first & 255u) == 0u)) flag[0] = 0u;
        __syncthreads();
        whole = flag[0] != 0u;
        __syncthreads();
    }
    const bool active = slot != ZRC4_INVALID && mylen != 0u;

    uint8_t *msg = payload + myoff;
    uint4 A[4];
    const bool pre = active && mylen >= 64u && head_bytes(msg, mylen) == 0u;
    if constexpr (MODE != kIds) {
        // The image was issued before the entry loads still in flight (kRange:
        // len, off and x/y; kGrouped: x/y).  Waited on every path (the
        // registers must not be reused while it is in flight); the first
        // payload block is issued after this wait, so its round trip overlaps
        // the LDS fill.
        if constexpr (MODE == kRange)
            asm volatile("s_waitcnt vmcnt(3)" : "+{v[160:191]}"(ilo), "+{v[192:223]}"(ihi) :: "memory");
        else   // the x/y load is conditional: wait for everything
            asm volatile("s_waitcnt vmcnt(0)" : "+{v[160:191]}"(ilo), "+{v[192:223]}"(ihi) :: "memory");
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            img[i] = make_uint4(ilo[4 * i], ilo[4 * i + 1], ilo[4 * i + 2], ilo[4 * i + 3]);
            img[i + 8] = make_uint4(ihi[4 * i], ihi[4 * i + 1], ihi[4 * i + 2], ihi[4 * i + 3]);
        }
    }
    if (whole) {
        if constexpr (MODE == kIds) {
            const uint4 *src = reinterpret_cast<const uint4 *>(arena + (size_t)g * kGroupBytes);
#pragma unroll
            for (int i = 0; i < 16; ++i) img[i] = src[i * 256 + tid];
        }
        if (pre) issue_block_asm(A, msg);
#pragma unroll
        for (int i = 0; i < 16; ++i) *reinterpret_cast<uint4 *>(S + i * 4096 + vo0) = img[i];
        if constexpr (PD) pair_meet_d(pdc, pdg);
        else __syncthreads();
        if constexpr (MODE == kGrouped) {
            if (flag[3]) {                               // another bucket of this launch holds the group
                if (tid == 0) latch_fault(err, kErrGroup);
                return;
            }
        }
    } else {
        if (pre) issue_block_asm(A, msg);
        if (active) gather_column(S, col, arena, slot);
    }
    stamp(ts, 1);

    if (active) {
        Rc4Lane st;
        lane_init(st, S, col, sxy);
        crypt_message(S, st, msg, mylen, A, pre);
        xy[slot] = lane_xy(st);
    }
    if constexpr (FRAME) {
        // The lane's own decrypted bytes: its stores must have landed before
        // it reads the headers back.
        const bool mine = MODE == kGrouped ? (ent != ZRC4_INVALID && mylen != 0u) : valid;
        if (mine) {
            __builtin_amdgcn_s_waitcnt(0);
            frame_walk(payload + fr.off[ent], fr.len[ent], fr.bound, fr.maxp, ent, fr.npk, fr.used, fr.status,
                       fr.pkt_len);
        }
    }
    stamp(ts, 2);

    if (whole) {
        if constexpr (PD) pair_meet_d(pdc, pdg);
        else __syncthreads();
        uint8_t *img_out = arena + (size_t)g * kGroupBytes;
#pragma unroll
        for (int i = 0; i < 16; ++i)
            *reinterpret_cast<uint4 *>(img_out + i * 4096 + vo0) = *reinterpret_cast<const uint4 *>(S + i * 4096 + vo0);
    } else if (active) {
        scatter_column(arena, slot, S, col);
    }
#if ZRC4_TIMING
    __builtin_amdgcn_s_waitcnt(0);
    stamp(ts, 3);
    stamps_out(ts, sink, e >> 6);
#endif
}

template <int MODE, bool FRAME = false>
__global__ void __launch_bounds__(256, 2)
crypt_kernel(uint8_t *__restrict__ arena, uint16_t *__restrict__ xy,
             const uint32_t *__restrict__ ids, uint32_t first_slot,
             uint8_t *__restrict__ payload, const uint64_t *__restrict__ off,
             const uint32_t *__restrict__ len, uint32_t n, uint32_t capacity,
             uint32_t *__restrict__ err, uint8_t *__restrict__ sink, FrameArgs fr = FrameArgs{},
             Claim cl = Claim{})
{
    crypt_body<MODE, FRAME, false>(arena, xy, ids, first_slot, payload, off, len, n, capacity, err, sink, fr, cl);
}

// The grouped forms with declared bucket groups (zrc4_crypt_grouped_declared,
// 33..256 buckets): the groups in the kernel arguments.
template <bool FRAME, bool HALF>
__global__ void __launch_bounds__(HALF ? (ZRC4_HALF_PAD ? 256u : 128u) : 256u, HALF ? 1 : 2)
crypt_decl_kernel(uint8_t *__restrict__ arena, uint16_t *__restrict__ xy,
                  const uint32_t *__restrict__ ids, uint8_t *__restrict__ payload,
                  const uint64_t *__restrict__ off, const uint32_t *__restrict__ len, uint32_t n,
                  uint32_t capacity, uint32_t *__restrict__ err, uint8_t *__restrict__ sink, FrameArgs fr,
                  Claim cl, BucketGroups dg)
{
    crypt_body<kGrouped, FRAME, HALF, true>(arena, xy, ids, 0u, payload, off, len, n, capacity, err, sink, fr, cl,
                                            &dg);
}

// Half-group workgroups (kRange / kGrouped, few groups): one per CU;
// workgroup 2w + h runs half h of bucket w.  ZRC4_HALF_PAD: launched with 256
// threads, of which the two waves that work are picked by SIMD (crypt_body);
// A/B knob: 0 launches 128 threads.
constexpr uint32_t kHalfBlock = ZRC4_HALF_PAD ? 256u : 128u;

template <int MODE, bool FRAME = false>
__global__ void __launch_bounds__(kHalfBlock, 1)
crypt_half_kernel(uint8_t *__restrict__ arena, uint16_t *__restrict__ xy,
                  const uint32_t *__restrict__ ids, uint32_t first_slot,
                  uint8_t *__restrict__ payload, const uint64_t *__restrict__ off,
                  const uint32_t *__restrict__ len, uint32_t n, uint32_t capacity,
                  uint32_t *__restrict__ err, uint8_t *__restrict__ sink, FrameArgs fr = FrameArgs{},
                  Claim cl = Claim{})
{
    crypt_body<MODE, FRAME, true>(arena, xy, ids, first_slot, payload, off, len, n, capacity, err, sink, fr, cl);
}

// ---------------------------------------------------------------------------
// crypt_stream_kernel: the throughput-regime crypt (more groups than CUs),
// persistent over groups.
//
// With one group per workgroup every workgroup of a round loads its 64 KiB
// S-box image, runs, and stores the image at the same time, so the HBM idles
// during the keystream and the LDS idles during the image bursts (the
// ablation put the image I/O at 42 us of a 330 us cfg5 launch, r01).  Here
// grid = 2 workgroups per CU and each workgroup walks groups w, w + grid, ...;
// while group w's keystream runs, the next group's image (16 x 16 B per lane,
// in VGPRs), its batch entries and -- once the message loop is done -- its
// first two payload lines are already in flight, and the finished image goes
// back to HBM behind the next group's work.  At a boundary only the LDS
// copies and three barriers remain.  Only line 0 of a group is loaded before
// its S-box fill; line 1 goes out behind the fill (profiles/r02/stream_tl_*:
// the launch prologue, every workgroup loading its image and first lines at
// once, was 12-18 us).
//   PF = range batch with first_slot % 256 == 0: every group is a whole,
//        aligned image and is prefetched; otherwise (ids, unaligned range)
//        each group decides whole/gather as crypt_kernel<kIds> does,
//        unprefetched.
// ---------------------------------------------------------------------------
struct EntryIn {
    uint32_t len;    // 0 for idle lanes
    uint32_t slot;   // ZRC4_INVALID for idle lanes
    uint64_t off;
    uint32_t xy;
};

__device__ __forceinline__ void load_entry(EntryIn &d, uint32_t w, uint32_t j, const uint32_t *ids, uint32_t first_slot,
                                           const uint64_t *off, const uint32_t *len, uint32_t n,
                                           uint32_t capacity, uint32_t *err, const uint16_t *xy)
{
    const uint32_t e = w * kGroup + j;
    const bool valid = e < n;
    uint32_t slot = valid ? (ids ? ids[e] : first_slot + e) : ZRC4_INVALID;
    if (valid && slot >= capacity) {
        latch_fault(err, kErrSlotRange);
        slot = ZRC4_INVALID;
    }
    // No load here depends on another's value (the range path's slot is
    // arithmetic), so prefetching a group never makes the compiler wait.
    d.len = (slot != ZRC4_INVALID) ? len[e] : 0u;
    d.off = (slot != ZRC4_INVALID) ? off[e] : 0u;
    d.slot = slot;
    d.xy = (slot != ZRC4_INVALID) ? xy[slot] : 0u;
}

// Next group's batch entries and S-box image, issued from asm so the compiler
// neither waits for them nor counts them: it would otherwise drain them at
// its next wait for anything younger (in-order vmcnt).  P/Q are passed
// through so the compiler's wait for this group's first lines lands BEFORE
// these loads.  Consumers wait explicitly:
//   entries  "s_waitcnt vmcnt(16)" (the 16 image loads are younger);
//   image    "s_waitcnt vmcnt(24)" (the next group's line-0 loads (8) and
//            this image's 16 stores are younger).
__device__ __forceinline__ void prefetch_group(u32x32 &P, u32x32 &Q, u32x32 &ilo, u32x32 &ihi,
                                               uint32_t &rlen, uint64_t &roff, uint32_t &rxy,
                                               const uint32_t *alen, const uint64_t *aoff,
                                               const uint16_t *axy, const uint8_t *ibase, uint32_t j)
{
    uint32_t vo = img_vo(j);
    asm volatile(
        "global_load_dword %[rlen], %[alen], off\n\t"
        "global_load_dwordx2 %[roff], %[aoff], off\n\t"
        "global_load_ushort %[rxy], %[axy], off\n\t"
        "global_load_dwordx4 v[160:163], %[vo], %[ib]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_load_dwordx4 v[164:167], %[vo], %[ib]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_load_dwordx4 v[168:171], %[vo], %[ib]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_load_dwordx4 v[172:175], %[vo], %[ib]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_load_dwordx4 v[176:179], %[vo], %[ib]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_load_dwordx4 v[180:183], %[vo], %[ib]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_load_dwordx4 v[184:187], %[vo], %[ib]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_load_dwordx4 v[188:191], %[vo], %[ib]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_load_dwordx4 v[192:195], %[vo], %[ib]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_load_dwordx4 v[196:199], %[vo], %[ib]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_load_dwordx4 v[200:203], %[vo], %[ib]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_load_dwordx4 v[204:207], %[vo], %[ib]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_load_dwordx4 v[208:211], %[vo], %[ib]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_load_dwordx4 v[212:215], %[vo], %[ib]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_load_dwordx4 v[216:219], %[vo], %[ib]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_load_dwordx4 v[220:223], %[vo], %[ib]\n\t"
        : "+{v[40:71]}"(P), "+{v[72:103]}"(Q), "=&{v[160:191]}"(ilo), "=&{v[192:223]}"(ihi),
          [rlen] "=&v"(rlen), [roff] "=&v"(roff), [rxy] "=&v"(rxy), [vo] "+v"(vo)
        : [alen] "v"(alen), [aoff] "v"(aoff), [axy] "v"(axy), [ib] "s"(ibase)
        : "memory");
}


// ---------------------------------------------------------------------------
// Grouped batches in the persistent kernel (crypt_stream_kernel<true, true>,
// zrc4_crypt_grouped with more buckets than CUs).  Bucket b holds entries
// b*256 .. b*256+255; its busy entries (a slot id < capacity, length > 0) must
// name ONE group, no slot twice, and no other bucket of the call may name that
// group (include/zrc4.h).  Lane j of the workgroup runs slot g*256 + j, so the
// image moves as one coalesced copy and the LDS columns stay conflict-free.
//
// Pipeline (one group per ~57 us of keystream at 1 KiB): while bucket n runs,
//   * bucket n+1's image, x/y (slot order: g*256 + j), its permuted entries
//     (this lane's length and offset, gathered by the entry index its table
//     names) and its claim are in flight -- exactly the range kernel's
//     prefetch plus one claim -- and
//   * bucket n+2's raw ids and lengths (entry order) are in flight.
// At the boundary into bucket n+1 (in the LDS fill of its image) the raw ids
// of bucket n+2 build its slot -> entry table in LDS; after the fill barrier
// each lane reads its entry and the four waves' group votes, so bucket n+2's
// image address is known a whole group before its keystream starts.  The
// table and the votes are tagged with the bucket (an entry index e belongs
// to bucket e >> 8), so nothing is cleared between buckets.
//
// LDS (after the 64 KiB image at offset 0): 64 B of votes -- per wave its
// group guess (first busy id's group, or ZRC4_INVALID) and a bad word
// (another group or a slot twice) -- plus the claim-lost word, then the
// 256-word table slot & 255 -> entry index.
// Word offsets from gr = smem + kGroupBytes (one base register for all of them).
constexpr uint32_t kGrVote = 0;                          // 4 waves x {guess, bad}
constexpr uint32_t kGrLost = 8;                          // the current bucket's claim was lost
constexpr uint32_t kGrTab = 16;                          // slot & 255 -> entry index
constexpr uint32_t kSmemStreamGr = kGroupBytes + 4u * (kGrTab + 256u);   // 66 624 B: two workgroups per CU

// The table of bucket nb from its raw entries (thread j holds entry nb*256 +
// j), plus this wave's vote.  Call between two barriers that order it after
// every read of the previous table.
// lo (ZRC4_GR_FASTPRO prologue): each busy entry also leaves its length at
// lo[slot & 255] and its offset at lo + 256 (u64) -- the permuted entry the
// lane of that column would otherwise gather from HBM.
__device__ __forceinline__ void bucket_table(uint32_t *gr, uint32_t nb, uint32_t id, uint32_t ln, uint32_t n,
                                             uint32_t capacity, uint32_t *err, uint32_t *lo = nullptr,
                                             uint64_t of = 0)
{
    const uint32_t j = threadIdx.x, e = nb * kGroup + j;
    const bool v = e < n;
    if (v && id >= capacity && id != ZRC4_INVALID) {        // ZRC4_IDLE_SLOT pads buckets
        latch_fault(err, kErrSlotRange);
        id = ZRC4_INVALID;
    }
    const bool busy = v && id != ZRC4_INVALID && ln != 0u;
    const uint64_t bm = __ballot(busy);
    const uint32_t guess = bm ? __builtin_amdgcn_readlane(id, (int)__builtin_ctzll(bm)) >> 8 : ZRC4_INVALID;
    const uint32_t old = busy ? atomicExch(&gr[kGrTab + (id & 255u)], e) : ZRC4_INVALID;
    if (lo && busy) {                        // (a slot named twice refuses the bucket: its values are unused)
        lo[id & 255u] = ln;
        reinterpret_cast<uint64_t *>(lo + 256u)[id & 255u] = of;
    }
    const bool bad = __ballot(busy && ((id >> 8) != guess || (old >> 8) == nb)) != 0u;
    if ((j & 63u) == 0u) {
        const uint32_t wv = __builtin_amdgcn_readfirstlane(j >> 6);   // (an SGPR: no VGPR held across the loop)
        gr[kGrVote + 2u * wv] = guess;
        gr[kGrVote + 2u * wv + 1u] = bad ? 1u : 0u;
    }
}

struct BucketView {
    uint32_t g;      // the bucket's group (0 when idle or refused: an in-bounds address)
    uint32_t ent;    // this lane's entry (valid) or the bucket's first entry
    bool ok;         // busy entries, one group, no slot twice (wave-uniform)
    bool valid;      // this lane's slot g*256 + j has an entry
};

// After the barrier that follows bucket_table(nb): the votes and this lane's
// table entry.  A refused bucket latches kErrGroup (thread 0).
template <int NW = 4>
__device__ __forceinline__ BucketView bucket_read(const uint32_t *gr, uint32_t nb, uint32_t *err)
{
    const uint4 va = *reinterpret_cast<const uint4 *>(gr + kGrVote);
    const uint4 vb = NW > 2 ? *reinterpret_cast<const uint4 *>(gr + kGrVote + 4) : make_uint4(0u, 0u, 0u, 0u);
    const uint32_t vote[8] = {va.x, va.y, va.z, va.w, vb.x, vb.y, vb.z, vb.w};
    uint32_t g = ZRC4_INVALID;
    bool bad = false;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        const uint32_t gw = __builtin_amdgcn_readfirstlane(vote[2 * w]);
        bad = bad || __builtin_amdgcn_readfirstlane(vote[2 * w + 1]) != 0u;
        if (gw != ZRC4_INVALID) {
            if (g == ZRC4_INVALID) g = gw;
            else if (gw != g) bad = true;
        }
    }
    BucketView bv;
    bv.ok = g != ZRC4_INVALID && !bad;
    if (g != ZRC4_INVALID && bad && (threadIdx.x & (NW * 64u - 1u)) == 0u) latch_fault(err, kErrGroup);
    const uint32_t t = gr[kGrTab + threadIdx.x];
    bv.valid = bv.ok && (t >> 8) == nb;
    bv.g = bv.ok ? g : 0u;
    bv.ent = bv.valid ? t : nb * kGroup;
    return bv;
}

// Grouped buckets with wave pairs (ZRC4_PAIR): each pair (waves 2p, 2p+1)
// runs its half of every bucket on its own schedule, so it keeps its own
// votes / claim-lost word / table (region p, kGrPairWords words), claims
// its own part p of the group (so two buckets naming one group can only
// split it by halves, each slot still all or nothing), and builds the table
// of the next bucket from all 256 raw entries: its own lanes' and the other
// pair's, which both pairs publish into an LDS staging buffer one boundary
// ahead (the raw entries are loaded three buckets ahead instead of two).  A
// pair only ever waits for the other to have finished the previous
// boundary -- the staging double buffer's condition -- which a pair never
// a whole group behind does not trigger.
constexpr uint32_t kGrPairCnt = kGrTab + 256u;            // 2 x 256 slot counts (boundary parity)
constexpr uint32_t kGrPairWords = kGrPairCnt + 512u;      // votes, lost, table, counts
constexpr uint32_t kGrMeet = 2u * kGrPairWords;           // 2 pair-meet counters
constexpr uint32_t kGrCnt = kGrMeet + 2u;                 // 2 boundaries-done counters
constexpr uint32_t kGrStg = kGrCnt + 2u;                  // 2 x 256 raw entries {id, len}
// ZRC4_GR_FASTPRO: the first bucket's permuted lengths (256 words) and
// offsets (256 u64), written with its table in the prologue
#ifndef ZRC4_GR_FASTPRO
#define ZRC4_GR_FASTPRO 1
#endif
constexpr uint32_t kGrPro = kGrStg + 1024u;
constexpr uint32_t kSmemStreamGrPair = kGroupBytes + 4u * (kGrPro + (ZRC4_GR_FASTPRO ? 768u : 0u));   // 78 992 B: two workgroups per CU

// Pair version of the bucket table, in two halves around the pair's meet
// so that a boundary pays two LDS round trips (each one queues behind the
// other workgroup's keystream on the CU's LDS) and holds no entry in
// registers across the meet:
//   bucket_table_pair (before the meet): each wave reads ALL 256 raw entries
//     of bucket nb from staging (lane l: l, l+64, l+128, l+192) and votes
//     the group (first busy id) and "a busy entry of another group" by
//     itself -- both waves reach the same answer, nothing to exchange; for
//     its half of the entries it writes the table (slot -> entry) and adds 1
//     to the slot's count (boundary parity cnt, zeroed one boundary ahead);
//   bucket_read_pair (after the meet): a count above 1 anywhere is a slot
//     named twice (each wave reads all 256), plus this lane's own slot.
struct PairVote {
    uint32_t guess;      // the bucket's group (first busy id), or ZRC4_INVALID
    bool bad;            // a busy entry of another group
};

// ocnt / bk: the staging buffer is read only once the other pair has
// finished boundary bk - 1 (its counter read first, in the same round trip).
__device__ __forceinline__ PairVote bucket_table_pair(uint32_t *grp, const uint32_t *stg, uint32_t nb,
                                                      uint32_t capacity, uint32_t *err, const uint32_t *ocnt,
                                                      uint32_t bk)
{
    // (the lane's addresses are recomputed per boundary, not hoisted out of
    // the persistent loop into registers that would be live across it)
    uint32_t tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const uint32_t l = tid & 63u, wv = __builtin_amdgcn_readfirstlane((tid >> 6) & 1u);
    uint32_t *cnt = grp + kGrPairCnt + 256u * (bk & 1u);
    uint32_t *nxt = grp + kGrPairCnt + 256u * ((bk + 1u) & 1u);
    uint2 r[4];
    const uint32_t c = __hip_atomic_load(ocnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    asm volatile("" ::: "memory");
#pragma unroll
    for (int m = 0; m < 4; ++m) r[m] = *reinterpret_cast<const uint2 *>(stg + 2u * (l + 64u * m));
    if (__builtin_amdgcn_readfirstlane(c) < bk) {            // the other pair is a whole group behind
        while (__builtin_amdgcn_readfirstlane(__hip_atomic_load(ocnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) < bk)
            __builtin_amdgcn_s_sleep(1);
        asm volatile("" ::: "memory");
#pragma unroll
        for (int m = 0; m < 4; ++m) r[m] = *reinterpret_cast<const uint2 *>(stg + 2u * (l + 64u * m));
    }
    PairVote pv;
    pv.guess = ZRC4_INVALID;
    uint32_t id[4];
    bool busy[4];
#pragma unroll
    for (int m = 3; m >= 0; --m) {
        id[m] = r[m].x;
        if (id[m] >= capacity && id[m] != ZRC4_INVALID) {      // ZRC4_IDLE_SLOT pads buckets
            latch_fault(err, kErrSlotRange);
            id[m] = ZRC4_INVALID;
        }
        busy[m] = id[m] != ZRC4_INVALID && r[m].y != 0u;
        const uint64_t bm = __ballot(busy[m]);
        if (bm) pv.guess = __builtin_amdgcn_readlane(id[m], (int)__builtin_ctzll(bm)) >> 8;
    }
    bool badl = false;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        badl = badl || (busy[m] && (id[m] >> 8) != pv.guess);
        if (busy[m] && (uint32_t)(m >> 1) == wv) {
            grp[kGrTab + (id[m] & 255u)] = nb * kGroup + l + 64u * m;
            __hip_atomic_fetch_add(cnt + (id[m] & 255u), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
    nxt[wv * 128u + l] = 0u;
    nxt[wv * 128u + 64u + l] = 0u;
    pv.bad = __ballot(badl) != 0u;
    if (l == 0u) {                                           // kept in LDS, not in registers, across the meet
        grp[kGrVote + 2u * wv] = pv.guess;
        grp[kGrVote + 2u * wv + 1u] = pv.bad ? 1u : 0u;
    }
    return pv;
}

// cnt: the counts of the boundary that built nb's table.
__device__ __forceinline__ BucketView bucket_read_pair(const uint32_t *grp, const uint32_t *cnt, uint32_t nb,
                                                       uint32_t *err)
{
    uint32_t tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const uint32_t l = tid & 63u, wv = __builtin_amdgcn_readfirstlane((tid >> 6) & 1u);
    const uint2 vote = *reinterpret_cast<const uint2 *>(grp + kGrVote + 2u * wv);
    PairVote pv;
    pv.guess = __builtin_amdgcn_readfirstlane(vote.x);
    pv.bad = __builtin_amdgcn_readfirstlane(vote.y) != 0u;
    uint32_t most = 0;
#pragma unroll
    for (int m = 0; m < 4; ++m) most = max(most, cnt[l + 64u * m]);
    const uint32_t t = grp[kGrTab + tid];
    const bool bad = pv.bad || __ballot(most > 1u) != 0u;
    BucketView bv;
    bv.ok = pv.guess != ZRC4_INVALID && !bad;
    if (pv.guess != ZRC4_INVALID && bad && (threadIdx.x & 127u) == 0u) latch_fault(err, kErrGroup);
    bv.valid = bv.ok && (t >> 8) == nb;
    bv.g = bv.ok ? pv.guess : 0u;
    bv.ent = bv.valid ? t : nb * kGroup;
    return bv;
}

#ifndef ZRC4_GR_PRECLAIM
#define ZRC4_GR_PRECLAIM 1       // the pair kernel claims the groups of its first buckets in the prologue
#endif
#ifndef ZRC4_GR_PRECLAIM_MAX
#define ZRC4_GR_PRECLAIM_MAX 64  // how many (the lost mask is 64 bits; a test build uses 1)
#endif
static_assert(ZRC4_GR_PRECLAIM_MAX >= 1 && ZRC4_GR_PRECLAIM_MAX <= 64, "pre-claim mask is 64 bits");
// The next bucket's claim (lane 0 of wave 0 swaps the launch epoch into the
// high half of the group's part-0 claim word -- only the epoch decides a
// claim -- and every other wave reads that half instead, so every wave issues
// the same number of VMEM ops and the counted waits hold), its permuted entry
// (an idle lane reads zeros), x/y, the raw ids and lengths of the bucket after
// it, and its image -- in that order, from asm (see prefetch_group).
// Consumers wait:
//   claim, entries, raw  "s_waitcnt vmcnt(16)" (the 16 image loads are younger);
//   image                "s_waitcnt vmcnt(24)".
__device__ __forceinline__ void prefetch_bucket(u32x32 &P, u32x32 &Q, u32x32 &ilo, u32x32 &ihi, uint32_t &cold,
                                                uint32_t &rlen, uint64_t &roff, uint32_t &rxy, uint32_t &qid,
                                                uint32_t &qlen, const uint32_t *cw, uint32_t cv,
                                                uint32_t doclaim, const uint32_t *alen, const uint64_t *aoff,
                                                const uint16_t *axy, const uint32_t *aqid, const uint32_t *aqlen,
                                                const uint8_t *ibase, uint32_t j)
{
    uint32_t vo = img_vo(j);
    uint64_t sv;
    asm volatile(
        "s_mov_b64 %[sv], exec\n\t"
        "s_mov_b64 exec, 1\n\t"
        "s_cmp_eq_u32 %[dc], 0\n\t"
        "s_cbranch_scc1 PB_READ_%=\n\t"
        "global_atomic_swap %[cold], %[cw], %[cv], off sc0\n\t"
        "s_branch PB_CLAIMED_%=\n\t"
        "PB_READ_%=:\n\t"
        "global_load_dword %[cold], %[cw], off\n\t"
        "PB_CLAIMED_%=:\n\t"
        "s_mov_b64 exec, %[sv]\n\t"
        "global_load_dword %[rlen], %[alen], off\n\t"
        "global_load_dwordx2 %[roff], %[aoff], off\n\t"
        "global_load_ushort %[rxy], %[axy], off\n\t"
        "global_load_dword %[qid], %[aqid], off\n\t"
        "global_load_dword %[qlen], %[aqlen], off\n\t"
        "global_load_dwordx4 v[160:163], %[vo], %[ib]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_load_dwordx4 v[164:167], %[vo], %[ib]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_load_dwordx4 v[168:171], %[vo], %[ib]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_load_dwordx4 v[172:175], %[vo], %[ib]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_load_dwordx4 v[176:179], %[vo], %[ib]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_load_dwordx4 v[180:183], %[vo], %[ib]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_load_dwordx4 v[184:187], %[vo], %[ib]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_load_dwordx4 v[188:191], %[vo], %[ib]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_load_dwordx4 v[192:195], %[vo], %[ib]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_load_dwordx4 v[196:199], %[vo], %[ib]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_load_dwordx4 v[200:203], %[vo], %[ib]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_load_dwordx4 v[204:207], %[vo], %[ib]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_load_dwordx4 v[208:211], %[vo], %[ib]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_load_dwordx4 v[212:215], %[vo], %[ib]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_load_dwordx4 v[216:219], %[vo], %[ib]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_load_dwordx4 v[220:223], %[vo], %[ib]\n\t"
        : "+{v[40:71]}"(P), "+{v[72:103]}"(Q), "=&{v[160:191]}"(ilo), "=&{v[192:223]}"(ihi), [cold] "=&v"(cold),
          [rlen] "=&v"(rlen), [roff] "=&v"(roff), [rxy] "=&v"(rxy), [qid] "=&v"(qid), [qlen] "=&v"(qlen),
          [vo] "+v"(vo), [sv] "=&s"(sv)
        : [cw] "v"(cw), [cv] "v"(cv), [dc] "s"(doclaim), [alen] "v"(alen), [aoff] "v"(aoff), [axy] "v"(axy),
          [aqid] "v"(aqid), [aqlen] "v"(aqlen), [ib] "s"(ibase)
        : "memory", "scc");
}

// crypt_stream_kernel's copy-out of a group's S-boxes at a group boundary:
// all 16 LDS reads in flight at once, then the 16 stores (the compiler's
// version paired them, one LDS round trip per pair, while the other
// workgroup on the CU keeps the LDS busy).  v72..v135 (line 1, the transpose
// spares and the store addresses of the line loop) are dead here.
__device__ __forceinline__ void lds_to_image_asm(uint8_t *img, uint32_t tid)
{
    u32x32 d0, d1;
    uint32_t vo = img_vo(tid);
    asm volatile(
        "ds_read_b128 v[72:75], %[vo]\n\t"
        "ds_read_b128 v[76:79], %[vo] offset:4096\n\t"
        "ds_read_b128 v[80:83], %[vo] offset:8192\n\t"
        "ds_read_b128 v[84:87], %[vo] offset:12288\n\t"
        "ds_read_b128 v[88:91], %[vo] offset:16384\n\t"
        "ds_read_b128 v[92:95], %[vo] offset:20480\n\t"
        "ds_read_b128 v[96:99], %[vo] offset:24576\n\t"
        "ds_read_b128 v[100:103], %[vo] offset:28672\n\t"
        "ds_read_b128 v[104:107], %[vo] offset:32768\n\t"
        "ds_read_b128 v[108:111], %[vo] offset:36864\n\t"
        "ds_read_b128 v[112:115], %[vo] offset:40960\n\t"
        "ds_read_b128 v[116:119], %[vo] offset:45056\n\t"
        "ds_read_b128 v[120:123], %[vo] offset:49152\n\t"
        "ds_read_b128 v[124:127], %[vo] offset:53248\n\t"
        "ds_read_b128 v[128:131], %[vo] offset:57344\n\t"
        "ds_read_b128 v[132:135], %[vo] offset:61440\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "global_store_dwordx4 %[vo], v[72:75], %[img]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_store_dwordx4 %[vo], v[76:79], %[img]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_store_dwordx4 %[vo], v[80:83], %[img]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_store_dwordx4 %[vo], v[84:87], %[img]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_store_dwordx4 %[vo], v[88:91], %[img]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_store_dwordx4 %[vo], v[92:95], %[img]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_store_dwordx4 %[vo], v[96:99], %[img]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_store_dwordx4 %[vo], v[100:103], %[img]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_store_dwordx4 %[vo], v[104:107], %[img]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_store_dwordx4 %[vo], v[108:111], %[img]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_store_dwordx4 %[vo], v[112:115], %[img]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_store_dwordx4 %[vo], v[116:119], %[img]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_store_dwordx4 %[vo], v[120:123], %[img]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_store_dwordx4 %[vo], v[124:127], %[img]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_store_dwordx4 %[vo], v[128:131], %[img]\n\t"
        "v_add_u32 %[vo], 0x1000, %[vo]\n\t"
        "global_store_dwordx4 %[vo], v[132:135], %[img]\n\t"
        "s_nop 1\n\t"                          // store-data VGPRs: VMEM store -> VALU write hazard
        : "=&{v[72:103]}"(d0), "=&{v[104:135]}"(d1), [vo] "+v"(vo)
        : [img] "s"(img)
        : "memory");
}

// ZRC4_PAIR (the range form of crypt_stream_kernel): the two wave pairs of a
// workgroup run their groups decoupled.  Pair p (waves 2p, 2p+1) owns the
// columns with bit 7 = p, i.e. bytes [128p, 128p + 128) of every image row,
// and moves exactly those (img_vo), so at a group boundary its waves only
// wait for each other: they meet through an LDS counter instead of the
// workgroup barrier.  Measured first as a timing-only ablation with whole
// images (pair meets, outputs wrong): cfg5 284.5 -> 276.3 us, 262 144 x 1 KiB
// 151.3 -> 148.7 (profiles/r04/ab/ab_pair.log).  0: workgroup barriers.
#ifndef ZRC4_PAIR
#define ZRC4_PAIR 1
#endif
__device__ __forceinline__ void pair_meet(uint32_t *ctr, uint32_t &gen)
{
    ++gen;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if ((threadIdx.x & 63u) == 0u) __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    while (__builtin_amdgcn_readfirstlane(__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) <
           2u * gen)
        __builtin_amdgcn_s_sleep(1);
    asm volatile("" ::: "memory");
}

template <bool PF, bool GR = false, bool FRAME = false>
__global__ void __launch_bounds__(256, 2)
crypt_stream_kernel(uint8_t *__restrict__ arena, uint16_t *__restrict__ xy,
                    const uint32_t *__restrict__ ids, uint32_t first_slot,
                    uint8_t *__restrict__ payload, const uint64_t *__restrict__ off,
                    const uint32_t *__restrict__ len, uint32_t n, uint32_t capacity,
                    uint32_t *__restrict__ err, uint8_t *__restrict__ sink, Claim cl = Claim{},
                    FrameArgs fr = FrameArgs{})
{
    static_assert(PF || !GR, "grouped batches run the prefetching form");
    constexpr bool PG = GR && ZRC4_PAIR;       // grouped buckets by wave pairs
    __shared__ __attribute__((aligned(16))) uint8_t smem[GR ? (PG ? kSmemStreamGrPair : kSmemStreamGr) : kGroupBytes + 16];
    uint8_t *S = smem;
    if (!lds_base_ok(S, err)) return;
    uint32_t *gr = reinterpret_cast<uint32_t *>(smem + kGroupBytes);    // GR: votes, claim word, table
    const uint32_t j = threadIdx.x;
    const uint32_t col = col_of(j);
    const uint32_t nwg = (n + kGroup - 1) / kGroup;
    uint8_t *sk = sink + (size_t)j * kSinkSlot;
    stream_stamp(sink, 0);
    uint32_t k_t = 0;                         // groups done (ZRC4_TIMING stamps)
    bool p_async = false;                     // P = next group's line 0, loaded by the line loop

    uint32_t w = blockIdx.x;
    const uint32_t pr = __builtin_amdgcn_readfirstlane(j >> 7);   // this wave's pair (an SGPR)
#if ZRC4_PAIR
    uint32_t *pctr = gr + (GR ? kGrMeet : 0u) + pr;         // this pair's meet counter
    uint32_t pgen = 0;                                      // meetings so far
    if constexpr (PF && !GR) {
        if (j < 2u) gr[j] = 0u;
        __syncthreads();
    }
#endif
    // PG: this pair's region, the staging buffers, boundaries done so far;
    // the next bucket's vote (before the meet) and view (after it)
    uint32_t *grp = gr + (PG ? pr * kGrPairWords : 0u);
    uint32_t bk = 0;
    EntryIn cur;
    u32x32 ilo, ihi;                          // PF: this group's image, 16 x 16 B per lane
    auto load_image = [&](uint32_t g0) {
        const uint8_t *src = arena + (size_t)g0 * kGroupBytes + img_vo(j);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const u32x4 a = *reinterpret_cast<const u32x4 *>(src + i * 4096),
                        b = *reinterpret_cast<const u32x4 *>(src + (i + 8) * 4096);
#pragma unroll
            for (int d = 0; d < 4; ++d) {
                ilo[4 * i + d] = a[d];
                ihi[4 * i + d] = b[d];
            }
        }
    };
    LineSetup ls;
    u32x32 P, Q = {};
    // GR: this bucket's group and whether it runs (wave-uniform), its claim
    // word's old value (lane 0 of wave 0), and the next bucket's raw entry.
    uint32_t gcur = 0;
    bool cur_ok = false;
    uint32_t cold = 0;
    uint64_t lostm = 0;                       // PG + ZRC4_GR_PRECLAIM: bucket k's claim lost (k < 64)
    bool pre = false;                         // ... pre-claims on (wave-uniform)
    uint32_t qid = ZRC4_INVALID, qlen = 0;
    if constexpr (PG) {
        // Prologue (whole workgroup): bucket w's table in pair 0's region,
        // each pair's claim on its part, the permuted entry, x/y and image;
        // bucket w + grid's raw entries into staging buffer 1 (the table of
        // boundary 0), bucket w + 2 grid's into qid / qlen (published at
        // boundary 0).
        gr[kGrTab + j] = ZRC4_INVALID;
        gr[kGrPairWords + kGrTab + j] = ZRC4_INVALID;
#pragma unroll
        for (uint32_t c = 0; c < 4u; ++c) gr[(c >> 1) * kGrPairWords + kGrPairCnt + 256u * (c & 1u) + j] = 0u;
        if (j < 4u) gr[kGrMeet + j] = 0u;
        // Raw entries of this workgroup's first 8 buckets (w + k grid) in one
        // round trip: bucket 0's table, bucket 1's staging, bucket 2's
        // qid / qlen, and the claims below.
        const uint32_t KB = (nwg - 1u - w) / gridDim.x + 1u;            // this workgroup's buckets (w < nwg)
        const uint32_t K = min((uint32_t)ZRC4_GR_PRECLAIM_MAX, KB);      // ... pre-claimed
        // Pre-claims pay two LDS rounds and a later atomic in the prologue;
        // they win from 3 buckets per workgroup on (cfg5, 4: 293.3 -> 287.4
        // us) and lose below (262 144 / 131 072 x 1 KiB, 2 / 1 bucket: +1.5 /
        // +2.4 us; profiles/r04/claim3), where bucket 0 claims in the prologue
        // and later ones in the loop, as without them.
        pre = ZRC4_GR_PRECLAIM && KB >= 3u;
        const uint32_t wv = __builtin_amdgcn_readfirstlane(j >> 6);
        uint32_t idk[8], lk[8];
        // (unconditional loads from a clamped entry, selected afterwards: a
        // load under a lane mask is merged with its default before the next
        // one is issued, i.e. one round trip per bucket)
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            const uint32_t e = (w + m * gridDim.x) * kGroup + j;
            const uint32_t ec = e < n ? e : n - 1u;
            idk[m] = ids[ec];
            lk[m] = len[ec];
        }
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            const uint32_t e = (w + m * gridDim.x) * kGroup + j;
            const bool v = (uint32_t)m < KB && e < n;
            idk[m] = v ? idk[m] : ZRC4_INVALID;
            lk[m] = v ? lk[m] : 0u;
        }
        qid = idk[2];
        qlen = lk[2];
#if ZRC4_GR_FASTPRO
        // Bucket 0's offsets with its ids: its table hands each column its
        // length and offset through LDS, so line 0 needs no gather round trip
        // (the image itself waits for the table: issued before the claims, its
        // loads would be drained by the wait for the claims' answers)
        const uint64_t of0 = off[w * kGroup + j < n ? w * kGroup + j : n - 1u];   // (unused past n)
#endif
        *reinterpret_cast<uint2 *>(gr + kGrStg + 512u + 2u * j) = make_uint2(idk[1], lk[1]);
#if ZRC4_GR_PRECLAIM
        // Claims up front: each of this workgroup's first 64 buckets whose
        // busy entries all name one group claims that group here -- one
        // atomic per bucket and pair, all in flight together; an atomic
        // issued at a boundary, behind the previous group's image stores,
        // cost ~2 us of boundary each (profiles/r04/gpair4, gpair5).  A
        // bucket naming two groups claims nothing (its table refuses it, as
        // before); one naming a slot twice claims its group and is refused by
        // its table (no other bucket may name that group anyway).  Bit k of
        // lostm: bucket k's claim on part pr was already held.  Buckets from
        // the 65th on claim in the loop.  Scratch: staging buffer 0 (first
        // written at boundary 0) and word 12 of each pair region.
        uint32_t *sv = gr + kGrStg;
        auto votes = [&](const uint32_t (&ik)[8], const uint32_t (&lkk)[8]) {   // each wave's first busy group
#pragma unroll
            for (int m = 0; m < 8; ++m) {
                const uint64_t bm = __ballot(ik[m] < capacity && lkk[m] != 0u);
                const uint32_t gs = bm ? __builtin_amdgcn_readlane(ik[m], (int)__builtin_ctzll(bm)) >> 8 : ZRC4_INVALID;
                if ((j & 63u) == 0u) sv[4u * m + wv] = gs;
            }
        };
        auto first4 = [](uint4 v) {
            return v.x != ZRC4_INVALID ? v.x : v.y != ZRC4_INVALID ? v.y : v.z != ZRC4_INVALID ? v.z : v.w;
        };
        auto mixed = [&](const uint32_t (&ik)[8], const uint32_t (&lkk)[8]) {   // a busy entry of another group?
#pragma unroll
            for (int m = 0; m < 8; ++m) {
                const uint32_t g = __builtin_amdgcn_readfirstlane(first4(*reinterpret_cast<const uint4 *>(sv + 4u * m)));
                const bool mx = __ballot(ik[m] < capacity && lkk[m] != 0u && (ik[m] >> 8) != g) != 0u;
                if ((j & 63u) == 0u) sv[32u + 4u * m + wv] = mx ? 1u : 0u;
            }
        };
        auto claim = [&](uint32_t k0) {                  // lanes 0..7 of each pair's first wave: the old words
            const uint32_t l = j & 127u;
            uint32_t old = 0u;
            if (l < 8u && k0 + l < K) {
                const uint4 mx = *reinterpret_cast<const uint4 *>(sv + 32u + 4u * l);
                const uint32_t g = first4(*reinterpret_cast<const uint4 *>(sv + 4u * l));
                if (g != ZRC4_INVALID && (mx.x | mx.y | mx.z | mx.w) == 0u)
                    old = __hip_atomic_exchange(reinterpret_cast<uint32_t *>(cl.word + (size_t)g * kClaimParts + pr) + 1,
                                                cl.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            return old;
        };
        auto lost_to_lds = [&](uint32_t old) {           // the mask -> word 12 of the pair region
            const uint64_t lb = __ballot(old == cl.epoch);
            if ((j & 127u) == 0u) grp[12] = (uint32_t)lb;
        };
        if (pre) votes(idk, lk);
#endif
        __syncthreads();
#if ZRC4_GR_FASTPRO
        bucket_table(gr, w, idk[0], lk[0], n, capacity, err, gr + kGrPro, of0);
#else
        bucket_table(gr, w, idk[0], lk[0], n, capacity, err);
#endif
#if ZRC4_GR_PRECLAIM
        if (pre) mixed(idk, lk);
#endif
        __syncthreads();
        const BucketView bv = bucket_read(gr, w, err);
        gcur = bv.g;
        cur_ok = bv.ok;
#if ZRC4_GR_PRECLAIM
        // (batch 0's answers are collected after the image loads are issued)
        uint32_t old0 = pre ? claim(0u) : 0u;
        if (!pre && bv.ok && (j & 127u) == 0u)
            cold = __hip_atomic_exchange(reinterpret_cast<uint32_t *>(cl.word + (size_t)bv.g * kClaimParts + pr) + 1,
                                         cl.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (pre && K > 8u) {                             // (more than 4 096 buckets: 8 more per round)
            lost_to_lds(old0);
            __syncthreads();
            lostm = __builtin_amdgcn_readfirstlane(grp[12]);
            for (uint32_t k0 = 8u; k0 < K; k0 += 8u) {
                uint32_t ik[8], lkk[8];
#pragma unroll
                for (int m = 0; m < 8; ++m) {
                    const uint32_t e = (w + (k0 + m) * gridDim.x) * kGroup + j;
                    const uint32_t ec = e < n ? e : n - 1u;
                    ik[m] = ids[ec];
                    lkk[m] = len[ec];
                }
#pragma unroll
                for (int m = 0; m < 8; ++m) {
                    const uint32_t e = (w + (k0 + m) * gridDim.x) * kGroup + j;
                    const bool v = k0 + m < K && e < n;
                    ik[m] = v ? ik[m] : ZRC4_INVALID;
                    lkk[m] = v ? lkk[m] : 0u;
                }
                __syncthreads();                         // the previous round's scratch is read
                votes(ik, lkk);
                __syncthreads();
                mixed(ik, lkk);
                __syncthreads();
                lost_to_lds(claim(k0));
                __syncthreads();
                lostm |= (uint64_t)__builtin_amdgcn_readfirstlane(grp[12]) << k0;
            }
        }
#else
        if (bv.ok && (j & 127u) == 0u)
            cold = __hip_atomic_exchange(reinterpret_cast<uint32_t *>(cl.word + (size_t)bv.g * kClaimParts + (j >> 7)) + 1,
                                         cl.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
#if ZRC4_GR_FASTPRO
        cur.len = bv.valid ? gr[kGrPro + j] : 0u;
        cur.off = bv.valid ? reinterpret_cast<const uint64_t *>(gr + kGrPro + 256u)[j] : 0u;
        cur.slot = bv.valid ? bv.g * 256u + j : ZRC4_INVALID;
        cur.xy = xy[bv.g * 256u + j];
        load_image(gcur);
        // line 0 now, behind the claims and the image, before their answers
        // are waited for below
        line_setup(ls, payload + cur.off, cur.len);
        preload_line0(P, ls, sk);
        // the claims' answers after these loads: compared earlier, the wait
        // for them would drain the loads issued behind them
#if ZRC4_GR_PRECLAIM
        asm volatile("" : "+v"(old0) :: "memory");
#else
        asm volatile("" ::: "memory");
#endif
#else
        cur.len = bv.valid ? len[bv.ent] : 0u;
        cur.off = bv.valid ? off[bv.ent] : 0u;
        cur.slot = bv.valid ? bv.g * 256u + j : ZRC4_INVALID;
        cur.xy = xy[bv.g * 256u + j];
        load_image(gcur);                     // with the entry gathers, not after the barrier
#endif
#if ZRC4_GR_PRECLAIM
        if (pre && K <= 8u) lost_to_lds(old0);
#endif
        __syncthreads();                      // table and votes read before the pairs build their own
#if ZRC4_GR_PRECLAIM
        if (pre && K <= 8u) lostm = __builtin_amdgcn_readfirstlane(grp[12]);
#endif
    } else if constexpr (GR) {
        // Prologue: bucket w's table (compiler loads, waited for once below),
        // its claim, permuted entry, x/y and image; bucket w + grid's raw entry.
        gr[kGrTab + j] = ZRC4_INVALID;
        const uint32_t e0 = w * kGroup + j, e1 = (w + gridDim.x) * kGroup + j;
        const uint32_t id0 = e0 < n ? ids[e0] : ZRC4_INVALID, l0 = e0 < n ? len[e0] : 0u;
        if (e1 < n) {
            qid = ids[e1];
            qlen = len[e1];
        }
        __syncthreads();
        bucket_table(gr, w, id0, l0, n, capacity, err);
        __syncthreads();
        const BucketView bv = bucket_read(gr, w, err);
        gcur = bv.g;
        cur_ok = bv.ok;
        if (bv.ok && j == 0u)
            cold = __hip_atomic_exchange(reinterpret_cast<uint32_t *>(cl.word + (size_t)bv.g * kClaimParts) + 1,
                                         cl.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        cur.len = bv.valid ? len[bv.ent] : 0u;
        cur.off = bv.valid ? off[bv.ent] : 0u;
        cur.slot = bv.valid ? bv.g * 256u + j : ZRC4_INVALID;
        cur.xy = xy[bv.g * 256u + j];
        load_image(gcur);                     // with the entry gathers, not after the barrier
        __syncthreads();                      // table and votes read before the next bucket's are built
    } else {
        load_entry(cur, w, j, ids, first_slot, off, len, n, capacity, err, xy);
    }
#ifndef ZRC4_AB_NOIMG0
#define ZRC4_AB_NOIMG0 0     // timing-only ablation: the first group's image is never loaded (outputs wrong)
#endif
    if constexpr (PF && !GR) {
        if constexpr (ZRC4_AB_NOIMG0) {
#pragma unroll
            for (int i = 0; i < 32; ++i) ilo[i] = ihi[i] = 0u;
        } else {
            load_image((first_slot >> 8) + w);
        }
    }
    if constexpr (!PG || !ZRC4_GR_FASTPRO) {
        line_setup(ls, payload + cur.off, cur.len);
        preload_line0(P, ls, sk);
    }
    // Retire the prologue's loads here, once: inside the loop the compiler's
    // waitcnt analysis merges the first iteration with the back edge, and a
    // value still pending from the prologue would put a vmcnt(0) -- draining
    // the asm prefetch -- into every iteration.
    asm volatile("" : "+v"(cur.len), "+v"(cur.off), "+v"(cur.xy), "+{v[40:71]}"(P),
                 "+{v[160:191]}"(ilo), "+{v[192:223]}"(ihi));
    if constexpr (GR) asm volatile("" : "+v"(cold), "+v"(qid), "+v"(qlen));

    for (;;) {
        // ---- this group's S-boxes into LDS
        bool whole;
        uint32_t g;
        if constexpr (PF) {
            whole = GR ? cur_ok : true;
            g = GR ? gcur : (first_slot >> 8) + w;
            // younger than the prefetched image: at least the next group's
            // line-0 loads (8) and this image's stores (16)
            asm volatile("s_waitcnt vmcnt(24)" : "+{v[160:191]}"(ilo), "+{v[192:223]}"(ihi) :: "memory");
            if (k_t == 1u) stream_stamp(sink, 9);    // ZRC4_TIMING: boundary 0, next image in
            uint8_t *dst = S + img_vo(j);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                *reinterpret_cast<u32x4 *>(dst + i * 4096) = u32x4{ilo[4 * i], ilo[4 * i + 1], ilo[4 * i + 2], ilo[4 * i + 3]};
                *reinterpret_cast<u32x4 *>(dst + (i + 8) * 4096) =
                    u32x4{ihi[4 * i], ihi[4 * i + 1], ihi[4 * i + 2], ihi[4 * i + 3]};
            }
            asm volatile("" ::: "memory");        // the image is in LDS (its registers free) before the tables
            if constexpr (PG) {
                // this pair's claim on the bucket; the next bucket's table
                // from both pairs' raw entries (staging (bk + 1) & 1) once the
                // other pair has finished boundary bk - 1, then bucket
                // w + 2 grid's raw entries published (staging bk & 1)
                const bool lostk = pre && bk < ZRC4_GR_PRECLAIM_MAX ? ((lostm >> bk) & 1u) != 0u : cold == cl.epoch;
                if ((j & 127u) == 0u) grp[kGrLost] = cur_ok && lostk ? 1u : 0u;
                if (w + gridDim.x < nwg)
                    (void)bucket_table_pair(grp, gr + kGrStg + 512u * ((bk + 1u) & 1u), w + gridDim.x, capacity, err,
                                            gr + kGrCnt + (pr ^ 1u), bk);
                else
                    while (__builtin_amdgcn_readfirstlane(__hip_atomic_load(gr + kGrCnt + (pr ^ 1u), __ATOMIC_RELAXED,
                                                                            __HIP_MEMORY_SCOPE_WORKGROUP)) < bk)
                        __builtin_amdgcn_s_sleep(1);
                asm volatile("" ::: "memory");
                const bool qv = (w + 2u * gridDim.x) * kGroup + j < n;
                *reinterpret_cast<uint2 *>(gr + kGrStg + 512u * (bk & 1u) + 2u * j) =
                    make_uint2(qv ? qid : ZRC4_INVALID, qlen);
            } else if constexpr (GR) {
                // this bucket's claim (read back with the entries), and the
                // table of the bucket after next from its raw entries
                if (j == 0u) gr[kGrLost] = cur_ok && cold == cl.epoch ? 1u : 0u;
                if (w + gridDim.x < nwg) bucket_table(gr, w + gridDim.x, qid, qlen, n, capacity, err);
            }
#if ZRC4_PAIR
            if constexpr (!GR || PG) pair_meet(pctr, pgen); else
#endif
            __syncthreads();
            uint32_t lostv = 0;
            if constexpr (PG) {
                // both waves are past their staging accesses of boundary bk
                if ((j & 127u) == 0u)
                    __hip_atomic_fetch_add(gr + kGrCnt + pr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                ++bk;
                lostv = __builtin_amdgcn_readfirstlane(grp[kGrLost]);
            }
            if constexpr (GR) {
                const uint32_t lost = PG ? lostv : __builtin_amdgcn_readfirstlane(grp[kGrLost]);
                if (cur_ok && lost != 0u) {
                    // another bucket of this launch holds the group: skip this one whole
                    if ((j & (PG ? 127u : 255u)) == 0u) latch_fault(err, kErrGroup);
                    cur_ok = false;
                    whole = false;
                    cur.len = 0u;
                    cur.slot = ZRC4_INVALID;
                    line_setup(ls, payload, 0u);
                }
            }
        } else {
            const bool act = cur.slot != ZRC4_INVALID;
            if (!ids) {
                whole = (first_slot & 255u) == 0u;
                g = (first_slot >> 8) + w;
            } else {
                // workgroup AND through a flag word after the image (LDS offset
                // 0 stays the S-box image)
                const uint32_t first = ids[w * kGroup];
                g = first >> 8;
                volatile uint32_t *flag = reinterpret_cast<volatile uint32_t *>(smem + kGroupBytes);
                if (j == 0) flag[0] = 1u;
                __syncthreads();
                if (!(act && cur.slot == ((first & ~255u) + j) && (first & 255u) == 0u)) flag[0] = 0u;
                __syncthreads();
                whole = flag[0] != 0u;
            }
            if (whole) {
                image_to_lds(S, arena + (size_t)g * kGroupBytes);
                __syncthreads();
            } else if (act && cur.len) {
                gather_column(S, col, arena, cur.slot);
            }
        }
        const bool active = cur.slot != ZRC4_INVALID;

        // ---- next group's entries and image, in flight during the keystream (PF)
        const uint32_t wn = w + gridDim.x;
        const bool more = wn < nwg;
        uint32_t rlen = 0, rxy = 0;
        uint64_t roff = 0;
        uint32_t en = 0, nvalid = 0, gn = 0;
        bool nok = false;
        // This group's line 0 is needed now (compiler wait; the previous
        // image's stores are younger); past this point it is asm-defined, so
        // nothing the compiler tracks is pending at the loop.  Line 1 goes out
        // now, behind the fill, and is waited for inside the loop.
#if ZRC4_LINE0_ASM
        if constexpr (PF)
            asm volatile("s_waitcnt vmcnt(16)" : "+{v[40:71]}"(P) :: "memory");   // younger: the 16 image stores
        else
            asm volatile("" : "+{v[40:71]}"(P));
#else
        asm volatile("" : "+{v[40:71]}"(P));
#endif
        p_async = false;
        if (ls.wmax > 2u) issue_line1_asm(Q, ls, sk);
        if (k_t == 1u) stream_stamp(sink, 11);       // ZRC4_TIMING: boundary 0, tables read / met
        if constexpr (GR) {
            if (more) {
                const BucketView bv = PG ? bucket_read_pair(grp, grp + kGrPairCnt + 256u * ((bk - 1u) & 1u), wn, err)
                                         : bucket_read(gr, wn, err);
                if (k_t == 1u) stream_stamp(sink, 10);   // ZRC4_TIMING: boundary 0, next bucket's view read
                gn = bv.g;
                nok = bv.ok;
                // raw entries of the bucket after next (PG: two after next)
                const uint32_t ea = (wn + (PG ? 2u : 1u) * gridDim.x) * kGroup + j;
                const uint32_t eq = ea < n ? ea : n - 1u;
                // the claim: wave 0 (PG: the first wave of each pair) swaps
#ifndef ZRC4_GR_NOSWAP_AB
#define ZRC4_GR_NOSWAP_AB 0      // timing-only: the claim word read, never swapped (claims off)
#endif
                const bool preclaimed = PG && pre && bk < ZRC4_GR_PRECLAIM_MAX;   // (bk: wn's index)
                const uint32_t dc = __builtin_amdgcn_readfirstlane(
                    !ZRC4_GR_NOSWAP_AB && !preclaimed && nok && (j & (PG ? 127u : 255u)) < 64u ? 1u : 0u);
                prefetch_bucket(P, Q, ilo, ihi, cold, rlen, roff, rxy, qid, qlen,
                                reinterpret_cast<const uint32_t *>(cl.word + (size_t)gn * kClaimParts + (PG ? pr : 0u)) + 1,
                                cl.epoch,
                                dc, bv.valid ? len + bv.ent : cl.zero,
                                bv.valid ? off + bv.ent : reinterpret_cast<const uint64_t *>(cl.zero),
                                xy + gn * 256u + j, ids + eq, len + eq, arena + (size_t)gn * kGroupBytes, j);
                nvalid = 1u;                          // idle lanes read length 0
            }
        } else if constexpr (PF) {
            if (more) {
                en = wn * kGroup + j;
                const uint32_t ec = en < n ? en : n - 1u;          // in-bounds address for idle lanes
                nvalid = en < n ? 1u : 0u;
                prefetch_group(P, Q, ilo, ihi, rlen, roff, rxy, len + ec, off + ec, xy + first_slot + ec,
                               arena + (size_t)((first_slot >> 8) + wn) * kGroupBytes, j);
            }
        }

        // ---- keystream over this group's messages
#if ZRC4_PRIO == 1
        {
            const uint32_t hw = hw_id();                 // ZRC4_PRIO (above the line loop)
            if (((hw ^ k_t) & 1u) != 0u)
                __builtin_amdgcn_s_setprio(2);
            else
                __builtin_amdgcn_s_setprio(1);
        }
#endif
        stream_stamp(sink, 1u + 2u * k_t);
        {
            Rc4Lane st;
            lane_init(st, S, col, cur.xy);
            // Before the message's final half (even half counts) the next
            // group's line 0 goes into P (crypt_last_half_next_asm).
            p_async = crypt_message_dpp(S, st, payload + cur.off, cur.len, P, Q, ls, sk, PF && more, rlen, roff,
                                        nvalid, payload);
            if (active && cur.len) xy[cur.slot] = lane_xy(st);
        }
        stream_stamp(sink, 2u + 2u * k_t);
        ++k_t;

        EntryIn nxt = {0u, ZRC4_INVALID, 0u, 0u};
        if (more) {
            if constexpr (PF) {
                // (already waited for when line 0 went out early: a wait here
                // would also wait for it)
                if constexpr (GR) {
                    if (!p_async) {
                        asm volatile("s_waitcnt vmcnt(16)"
                                     : "+v"(rlen), "+v"(roff), "+v"(rxy), "+v"(cold), "+v"(qid), "+v"(qlen) :: "memory");
                    }
                    nxt.len = rlen;           // 0 for lanes without an entry (and for idle / refused buckets)
                    nxt.off = roff;
                    nxt.slot = gn * 256u + j;
                    nxt.xy = rxy;
                } else {
                    if (!p_async)
                        asm volatile("s_waitcnt vmcnt(16)" : "+v"(rlen), "+v"(roff), "+v"(rxy) :: "memory");
                    const bool v = nvalid != 0u;
                    nxt.len = v ? rlen : 0u;
                    nxt.off = v ? roff : 0u;
                    nxt.slot = v ? first_slot + en : ZRC4_INVALID;
                    nxt.xy = v ? rxy : 0u;
                }
            } else {
                load_entry(nxt, wn, j, ids, first_slot, off, len, n, capacity, err, xy);
            }
            // the loop's last two halves issue no loads, so P/Q are free again
            line_setup(ls, payload + nxt.off, nxt.len);
            if (k_t == 1u) stream_stamp(sink, 12);   // ZRC4_TIMING: boundary 0, next entries in
            if (!p_async) {
#if ZRC4_LINE0_ASM
                if constexpr (PF) issue_line0_asm(P, ls, sk);
                else preload_line0(P, ls, sk);
#else
                preload_line0(P, ls, sk);
#endif
            }
        }

        // ---- this group's state back to HBM
        if (whole) {
#if ZRC4_PAIR
            if constexpr (PF && (!GR || PG)) pair_meet(pctr, pgen); else
#endif
            __syncthreads();
            lds_to_image_asm(arena + (size_t)g * kGroupBytes, j);
            if (k_t == 1u) stream_stamp(sink, 13);   // ZRC4_TIMING: boundary 0, image out
        } else if (!PF && active && cur.len) {
            scatter_column(arena, cur.slot, S, col);
        } else if (GR) {
            // An idle or refused bucket stores no image, so the next fill's
            // counted wait (16 image stores younger than the prefetched
            // image) would not cover the image: retire everything here.
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        if (!more) break;
#if ZRC4_PAIR
        if constexpr (PF && (!GR || PG)) pair_meet(pctr, pgen); else
#endif
        __syncthreads();      // every wave has read this image out of LDS before the next fill
        cur = nxt;
        w = wn;
        gcur = gn;
        cur_ok = nok;
    }
    if constexpr (FRAME) {
        // onRecv's framing (§8f row 4) of every entry of this workgroup's
        // chunks, raw or decrypted: every wave's payload stores have landed
        // (same CU) before any lane reads headers back.
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        frame_walk_chunks(payload, fr, blockIdx.x, gridDim.x, nwg, n, j);
    }
#if ZRC4_TIMING
    __builtin_amdgcn_s_waitcnt(0);
    stream_stamp(sink, 15);
#endif
}

// ---------------------------------------------------------------------------
// ksa_kernel: batched RC4Encryption::makeSBox (rc4_encryption.h:46-72).
//
// The swap step is the PRGA swap without the keystream read, plus a key
// byte, so it uses the same 16-bit LDS addresses (index in byte 1) and SDWA
// byte-1 adds.  Per step i (hand-written, ZRC4_KSA_STEP):
//     j += a                      (j already holds j + key[k], added while the
//                                  previous step waited for S[i])
//     b = S[j] ; S[j] = a ; p = S[i+1] ; S[i] = b
//     j += key[k+1]
// 3 VALU + 4 LDS + 2 waits; S[i+1] is read after the S[j] = a write, so no
// forwarding is needed (S[i] = b goes to i != i+1).  Writing S[j] before S[i]
// swaps the reference's order (:63-64); they only collide when i == j, and
// then b == a.
// Key schedule: key lengths dividing 16 keep a 16-byte pattern in 4 VGPRs,
// 32- and 64-byte keys a 64-byte pattern in 16 VGPRs (step u adds pattern
// byte (u+1) mod the chunk length through the SDWA source selector, no key
// loads in the loop); other lengths up to 48 read 17-byte windows of the
// schedule's first 64 bytes from LDS, longer ones fetch the 17 bytes of
// each chunk one chunk ahead (dwords + byte aligns) -- both run the step
// with the key byte taken by SDWA selector from the window's registers.
// In: x0 = &S[i], x1 = &S[i+1], a0 = S[i], ya = &S[j + key[i]].
// ---------------------------------------------------------------------------
#define ZRC4_KSA_STEP_SEL(XC, XN, A, P, KN, SEL)                                                 \
    "v_add_u32_sdwa %[ya], %[ya], %[" #A "] dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE "          \
    "src0_sel:BYTE_1 src1_sel:BYTE_0\n\t"                                                        \
    "ds_read_u8 %[b], %[ya]\n\t"                                                                 \
    "ds_write_b8 %[ya], %[" #A "]\n\t"                                                           \
    "ds_read_u8 %[" #P "], %[" #XN "]\n\t"                                                       \
    "v_add_u32_sdwa %[ya], %[ya], %[" #KN "] dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE "         \
    "src0_sel:BYTE_1 src1_sel:" #SEL "\n\t"                                                      \
    "s_waitcnt lgkmcnt(2)\n\t"                                                                   \
    "ds_write_b8 %[" #XC "], %[b]\n\t"                                                           \
    "v_add_u32_sdwa %[" #XC "], 1, %[" #XN "] dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE "        \
    "src0_sel:DWORD src1_sel:BYTE_1\n\t"                                                         \
    "s_waitcnt lgkmcnt(1)\n\t"
#define ZRC4_KSA_STEP(XC, XN, A, P, KN) ZRC4_KSA_STEP_SEL(XC, XN, A, P, KN, BYTE_0)
#define ZRC4_KSA_QPAIR(K1, S1, K2, S2)                                                           \
    ZRC4_KSA_STEP_SEL(x0, x1, a0, a1, K1, S1) ZRC4_KSA_STEP_SEL(x1, x0, a1, a0, K2, S2)

// 16 KSA steps with the key bytes taken from a 16-byte pattern in registers
// (key lengths 1, 2, 4, 8, 16).  Step u adds pattern byte (u+1) % 16.
__device__ __forceinline__ void ksa16_pattern_asm(uint32_t &x0, uint32_t &x1, uint32_t &a0, uint32_t &ya,
                                                  const uint32_t (&q)[4])
{
    uint32_t a1, b;
    asm volatile(
        ZRC4_KSA_QPAIR(q0, BYTE_1, q0, BYTE_2) ZRC4_KSA_QPAIR(q0, BYTE_3, q1, BYTE_0)
        ZRC4_KSA_QPAIR(q1, BYTE_1, q1, BYTE_2) ZRC4_KSA_QPAIR(q1, BYTE_3, q2, BYTE_0)
        ZRC4_KSA_QPAIR(q2, BYTE_1, q2, BYTE_2) ZRC4_KSA_QPAIR(q2, BYTE_3, q3, BYTE_0)
        ZRC4_KSA_QPAIR(q3, BYTE_1, q3, BYTE_2) ZRC4_KSA_QPAIR(q3, BYTE_3, q0, BYTE_0)
        "s_waitcnt lgkmcnt(0)\n\t"
        : [ya] "+v"(ya), [x0] "+v"(x0), [x1] "+v"(x1), [a0] "+v"(a0), [a1] "=&v"(a1), [b] "=&v"(b)
        : [q0] "v"(q[0]), [q1] "v"(q[1]), [q2] "v"(q[2]), [q3] "v"(q[3])
        : "memory");
}

// 64 KSA steps with the key bytes taken from a 64-byte pattern in registers
// (key lengths 32 and 64: key[k mod len] repeats every 64 steps), so the loop
// issues no key loads at all.  Step u adds pattern byte (u+1) % 64.
#define ZRC4_KSA_Q4(QA, QB) ZRC4_KSA_QPAIR(QA, BYTE_1, QA, BYTE_2) ZRC4_KSA_QPAIR(QA, BYTE_3, QB, BYTE_0)
__device__ __forceinline__ void ksa64_pattern_asm(uint32_t &x0, uint32_t &x1, uint32_t &a0, uint32_t &ya,
                                                  const uint32_t (&q)[16])
{
    uint32_t a1, b;
    asm volatile(
        ZRC4_KSA_Q4(q0, q1) ZRC4_KSA_Q4(q1, q2) ZRC4_KSA_Q4(q2, q3) ZRC4_KSA_Q4(q3, q4)
        ZRC4_KSA_Q4(q4, q5) ZRC4_KSA_Q4(q5, q6) ZRC4_KSA_Q4(q6, q7) ZRC4_KSA_Q4(q7, q8)
        ZRC4_KSA_Q4(q8, q9) ZRC4_KSA_Q4(q9, q10) ZRC4_KSA_Q4(q10, q11) ZRC4_KSA_Q4(q11, q12)
        ZRC4_KSA_Q4(q12, q13) ZRC4_KSA_Q4(q13, q14) ZRC4_KSA_Q4(q14, q15) ZRC4_KSA_Q4(q15, q0)
        "s_waitcnt lgkmcnt(0)\n\t"
        : [ya] "+v"(ya), [x0] "+v"(x0), [x1] "+v"(x1), [a0] "+v"(a0), [a1] "=&v"(a1), [b] "=&v"(b)
        : [q0] "v"(q[0]), [q1] "v"(q[1]), [q2] "v"(q[2]), [q3] "v"(q[3]), [q4] "v"(q[4]),
          [q5] "v"(q[5]), [q6] "v"(q[6]), [q7] "v"(q[7]), [q8] "v"(q[8]), [q9] "v"(q[9]),
          [q10] "v"(q[10]), [q11] "v"(q[11]), [q12] "v"(q[12]), [q13] "v"(q[13]),
          [q14] "v"(q[14]), [q15] "v"(q[15])
        : "memory");
}

// 16 KSA steps with the key bytes of a 17-byte window in registers (q[0..3]
// and byte 0 of q[4]): step u adds window byte u + 1 (the off-pattern key
// lengths, ksa_kernel's window path).
__device__ __forceinline__ void ksa16_window_asm(uint32_t &x0, uint32_t &x1, uint32_t &a0, uint32_t &ya,
                                                 const uint32_t (&q)[5])
{
    uint32_t a1, b;
    asm volatile(
        ZRC4_KSA_QPAIR(q0, BYTE_1, q0, BYTE_2) ZRC4_KSA_QPAIR(q0, BYTE_3, q1, BYTE_0)
        ZRC4_KSA_QPAIR(q1, BYTE_1, q1, BYTE_2) ZRC4_KSA_QPAIR(q1, BYTE_3, q2, BYTE_0)
        ZRC4_KSA_QPAIR(q2, BYTE_1, q2, BYTE_2) ZRC4_KSA_QPAIR(q2, BYTE_3, q3, BYTE_0)
        ZRC4_KSA_QPAIR(q3, BYTE_1, q3, BYTE_2) ZRC4_KSA_QPAIR(q3, BYTE_3, q4, BYTE_0)
        "s_waitcnt lgkmcnt(0)\n\t"
        : [ya] "+v"(ya), [x0] "+v"(x0), [x1] "+v"(x1), [a0] "+v"(a0), [a1] "=&v"(a1), [b] "=&v"(b)
        : [q0] "v"(q[0]), [q1] "v"(q[1]), [q2] "v"(q[2]), [q3] "v"(q[3]), [q4] "v"(q[4])
        : "memory");
}

// 32 KSA steps from a 33-byte window (q[0..7] and byte 0 of q[8]): the window
// path's chunk for key lengths up to 32 (16c mod len + 33 <= 64 then holds
// for 32-step chunks), half the chunk boundaries of ksa16_window_asm.
__device__ __forceinline__ void ksa32_window_asm(uint32_t &x0, uint32_t &x1, uint32_t &a0, uint32_t &ya,
                                                 const uint32_t (&q)[9])
{
    uint32_t a1, b;
    asm volatile(
        ZRC4_KSA_QPAIR(q0, BYTE_1, q0, BYTE_2) ZRC4_KSA_QPAIR(q0, BYTE_3, q1, BYTE_0)
        ZRC4_KSA_QPAIR(q1, BYTE_1, q1, BYTE_2) ZRC4_KSA_QPAIR(q1, BYTE_3, q2, BYTE_0)
        ZRC4_KSA_QPAIR(q2, BYTE_1, q2, BYTE_2) ZRC4_KSA_QPAIR(q2, BYTE_3, q3, BYTE_0)
        ZRC4_KSA_QPAIR(q3, BYTE_1, q3, BYTE_2) ZRC4_KSA_QPAIR(q3, BYTE_3, q4, BYTE_0)
        ZRC4_KSA_QPAIR(q4, BYTE_1, q4, BYTE_2) ZRC4_KSA_QPAIR(q4, BYTE_3, q5, BYTE_0)
        ZRC4_KSA_QPAIR(q5, BYTE_1, q5, BYTE_2) ZRC4_KSA_QPAIR(q5, BYTE_3, q6, BYTE_0)
        ZRC4_KSA_QPAIR(q6, BYTE_1, q6, BYTE_2) ZRC4_KSA_QPAIR(q6, BYTE_3, q7, BYTE_0)
        ZRC4_KSA_QPAIR(q7, BYTE_1, q7, BYTE_2) ZRC4_KSA_QPAIR(q7, BYTE_3, q8, BYTE_0)
        "s_waitcnt lgkmcnt(0)\n\t"
        : [ya] "+v"(ya), [x0] "+v"(x0), [x1] "+v"(x1), [a0] "+v"(a0), [a1] "=&v"(a1), [b] "=&v"(b)
        : [q0] "v"(q[0]), [q1] "v"(q[1]), [q2] "v"(q[2]), [q3] "v"(q[3]), [q4] "v"(q[4]),
          [q5] "v"(q[5]), [q6] "v"(q[6]), [q7] "v"(q[7]), [q8] "v"(q[8])
        : "memory");
}

#ifndef ZRC4_KSA_WIN32
#define ZRC4_KSA_WIN32 1
#endif
#ifndef ZRC4_KSA_EAB
#define ZRC4_KSA_EAB 0       // timing-only: skip assembling E (outputs wrong)
#endif

// ksa_kernel's LDS: the 64 KiB S-box image, then 16 KiB of key schedule
// prefixes (window path: dword w of lane j at kKsaSched + 4 * (w * 256 + j),
// conflict-free for any per-lane w).  80 KiB: two workgroups per CU.
constexpr uint32_t kKsaSched = kGroupBytes;
constexpr uint32_t kKsaWinMax = 48;            // window path: key lengths up to this (16c mod len + 17 <= 64)
constexpr uint32_t kSmemKsa = kGroupBytes + 16384;

__global__ void __launch_bounds__(256, 2)
ksa_kernel(uint8_t *__restrict__ arena, uint16_t *__restrict__ xy,
           const uint32_t *__restrict__ ids, uint32_t first_slot,
           const uint8_t *__restrict__ keys,
           const uint64_t *__restrict__ key_off, const uint32_t *__restrict__ key_len,
           uint32_t n, uint32_t capacity, uint32_t *__restrict__ err)
{
    __shared__ __attribute__((aligned(16))) uint8_t smem[kSmemKsa];
    uint8_t *S = smem;
    if (!lds_base_ok(S, err)) return;

    const uint32_t j = threadIdx.x;
    const uint32_t e = blockIdx.x * kGroup + j;
    const bool valid = e < n;
    uint32_t slot = valid ? (ids ? ids[e] : first_slot + e) : ZRC4_INVALID;
    if (valid && slot >= capacity) {
        latch_fault(err, kErrSlotRange);
        slot = ZRC4_INVALID;
    }
    const bool active = slot != ZRC4_INVALID;
    const uint32_t kl = active ? key_len[e] : 0u;
    const uint8_t *key = active ? keys + key_off[e] : keys;

    bool whole;
    uint32_t g;
    if (!ids) {
        // Entries >= n of the last group are not re-seeded: load the image so
        // their state is written back unchanged.
        whole = (first_slot & 255u) == 0u;
        g = (first_slot >> 8) + blockIdx.x;
    } else {
        const uint32_t first = (blockIdx.x * kGroup < n) ? ids[blockIdx.x * kGroup] : 0u;
        g = first >> 8;
        volatile uint32_t *flag = reinterpret_cast<volatile uint32_t *>(smem + kGroupBytes);
        if (j == 0) flag[0] = 1u;
        __syncthreads();
        if (!(active && slot == ((first & ~255u) + j) && (first & 255u) == 0u)) flag[0] = 0u;
        __syncthreads();
        whole = flag[0] != 0u;
        __syncthreads();
    }
    const bool partial = (blockIdx.x + 1u) * kGroup > n;
    const uint32_t col = col_of(j);

    // Window path (key lengths that do not divide 16 and are not 32 / 64,
    // up to kKsaWinMax): the first 64 bytes of this lane's key schedule,
    // E[i] = key[i mod len] (rc4_encryption.h:67-70), go to LDS once.  The key
    // arrives as the <= 13 dwords that cover it (not 64 per-lane byte loads:
    // each byte-load instruction of a wave touches ~20 cache lines), issued
    // here so that their round trip overlaps the S-box fill; E is built in
    // the lane's schedule rows with dword reads and byte aligns (~100 VALU
    // per lane; assembling it byte by byte cost ~600 and 14 % of the KSA).
    // Layouts are transposed (dword w of lane j at 4 * (w * 256 + j)):
    // conflict-free.
    const bool winpath = active && kl != 0u && kl <= kKsaWinMax && !(kl <= 16u && (16u % kl) == 0u) &&
                         kl != 32u && kl != 64u;
    uint32_t *sch = reinterpret_cast<uint32_t *>(smem + kKsaSched) + j;
    // (32- and 64-byte keys take their 64-byte register pattern from the
    // same dword loads.)
    const bool pat64 = active && (kl == 32u || kl == 64u);
    const uint32_t ksh = (uint32_t)((uintptr_t)key & 3u);
    uint32_t kraw[17];
    if (winpath || pat64) {
        const uint32_t *kw = reinterpret_cast<const uint32_t *>((uintptr_t)key & ~(uintptr_t)3);
        const uint32_t nw = (ksh + kl + 3u) >> 2;           // dwords overlapping the key
#pragma unroll
        for (uint32_t w = 0; w < 17u; ++w) kraw[w] = w < nw ? kw[w] : 0u;
    }

    // Identity boxes (:50-53): a whole, fully re-seeded group fills its 64 KiB
    // image cooperatively (row k = 256 copies of k, 16 x 16 B per lane);
    // otherwise each seeded lane writes its own column.
    if (whole && !partial) {
        uint4 *img = reinterpret_cast<uint4 *>(S);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const uint32_t q = i * 256 + threadIdx.x;
            const uint32_t v = (q >> 4) * 0x01010101u;
            img[q] = make_uint4(v, v, v, v);
        }
        __syncthreads();
    } else {
        if (whole && partial) {
            image_to_lds(S, arena + (size_t)g * kGroupBytes);
            __syncthreads();
        }
        if (active)
            for (int k = 0; k < 256; ++k) S[(k << 8) | col] = (uint8_t)k;
    }

    if (winpath && !ZRC4_KSA_EAB) {
        // X = key || key[0..2] as aligned dwords in the schedule rows, then
        // E dword w = X bytes r .. r+3 with r = 4w mod len (one byte align).
        uint32_t K[12];
#pragma unroll
        for (int w = 0; w < 12; ++w) {
            K[w] = __builtin_amdgcn_alignbyte(kraw[w + 1], kraw[w], ksh);
            sch[w * 256] = K[w];                             // bytes past len: fixed below / never read
        }
        const uint32_t w0 = kl >> 2, m8 = 8u * (kl & 3u);
        const uint32_t kw0 = sch[w0 * 256u];                 // the dword holding byte len (if len % 4)
        sch[w0 * 256u] = (uint32_t)(((uint64_t)kw0 & ((1ull << m8) - 1ull)) | ((uint64_t)K[0] << m8));
        sch[(w0 + 1u) * 256u] = (uint32_t)((uint64_t)K[0] >> (32u - m8));
        uint32_t E[16];
        uint32_t r = 0;
#pragma unroll
        for (int w = 0; w < 16; ++w) {
            const uint32_t *x = sch + (r >> 2) * 256u;
            E[w] = __builtin_amdgcn_alignbyte(x[256], x[0], r & 3u);
            r += 4u;
            if (r >= kl) r -= kl;
            if (r >= kl) r -= kl;                            // len 3
        }
#pragma unroll
        for (int w = 0; w < 16; ++w) sch[w * 256] = E[w];
    }

    if (active && kl) {
        if (kl <= 16u && (16u % kl) == 0u) {
            // the whole key schedule (:67-70) in 16 register bytes, loaded once
            uint32_t q[4] = {0u, 0u, 0u, 0u};
#pragma unroll
            for (int u = 0; u < 16; ++u) q[u >> 2] |= (uint32_t)key[(uint32_t)u & (kl - 1u)] << (8 * (u & 3));
            uint32_t x0 = col, x1 = (1u << 8) | col, a0 = S[col];
            uint32_t ya = col | ((q[0] & 0xFFu) << 8);    // j = 0 + key[0] before step 0
            for (int c = 0; c < 16; ++c) ksa16_pattern_asm(x0, x1, a0, ya, q);
        } else if (kl == 32u || kl == 64u) {
            // 32- and 64-byte keys: the schedule in 64 register bytes (the
            // key's aligned dwords, the first 8 twice for 32 bytes)
            uint32_t q[16];
#pragma unroll
            for (int i = 0; i < 16; ++i)
                q[i] = __builtin_amdgcn_alignbyte(kraw[kl == 32u ? (i & 7) + 1 : i + 1], kraw[kl == 32u ? (i & 7) : i], ksh);
            uint32_t x0 = col, x1 = (1u << 8) | col, a0 = S[col];
            uint32_t ya = col | ((q[0] & 0xFFu) << 8);
            for (int c = 0; c < 4; ++c) ksa64_pattern_asm(x0, x1, a0, ya, q);
        } else if (winpath) {
            // The 17 bytes chunk c needs are E[k .. k+16] with k = 16c mod len
            // (<= 47): 5 dwords + byte aligns, read one chunk ahead (the reads
            // retire ahead of the first step's own LDS round trip).  The
            // per-chunk global byte loads of the fetch path below cost 1.4-2x
            // at 24-40-byte keys.
            uint32_t x0 = col, x1 = (1u << 8) | col, a0 = S[col];
            uint32_t ya = col | ((sch[0] & 0xFFu) << 8);   // j = 0 + key[0] before step 0
            uint32_t k = 0;                                // 16c mod len
#if ZRC4_KSA_WIN32
            if (kl <= 32u) {
                // 32-step chunks: 33 bytes E[k .. k+32], k = 32c mod len <= 31
                uint32_t d[9];
#pragma unroll
                for (int m = 0; m < 9; ++m) d[m] = sch[m * 256];
                for (int c = 0; c < 8; ++c) {
                    const uint32_t sh = 8u * (k & 3u);
                    uint32_t q[9];
#pragma unroll
                    for (int m = 0; m < 8; ++m)
                        q[m] = (uint32_t)(((uint64_t)d[m + 1] << 32 | d[m]) >> sh);
                    q[8] = d[8] >> sh;
                    k += 32u;
                    while (k >= kl) k -= kl;
                    if (c < 7) {
                        const uint32_t i0 = k >> 2;
#pragma unroll
                        for (int m = 0; m < 9; ++m) d[m] = sch[(i0 + m) * 256];
                    }
                    ksa32_window_asm(x0, x1, a0, ya, q);
                }
            } else
#endif
            {
            uint32_t d[5];
#pragma unroll
            for (int m = 0; m < 5; ++m) d[m] = sch[m * 256];
            for (int c = 0; c < 16; ++c) {
                const uint32_t sh = 8u * (k & 3u);
                uint32_t q[5];
#pragma unroll
                for (int m = 0; m < 4; ++m)
                    q[m] = (uint32_t)(((uint64_t)d[m + 1] << 32 | d[m]) >> sh);
                q[4] = d[4] >> sh;
                k += 16u;
                while (k >= kl) k -= kl;
                if (c < 15) {
                    const uint32_t i0 = k >> 2;
#pragma unroll
                    for (int m = 0; m < 5; ++m) d[m] = sch[(i0 + m) * 256];
                }
                ksa16_window_asm(x0, x1, a0, ya, q);
            }
            }
        } else {
            // Longer keys (over 48 bytes but 64): the 17 key bytes of steps
            // 16c .. 16c+16, fetched one chunk ahead -- as the 5 dwords
            // covering them plus byte aligns while they do not wrap past the
            // key's end (all but ~17 / len of the chunks), else byte by byte
            // (r03 fetched every chunk as 17 byte loads: the KSA then ran at
            // the rate of those loads, 2.1x the 16-byte time at 100 bytes).
            uint32_t kk = 0;
            auto fetch = [&](uint32_t (&q)[5]) {
                if (kk + 17u <= kl) {
                    const uintptr_t pa = (uintptr_t)(key + kk);
                    const uint32_t *pw = reinterpret_cast<const uint32_t *>(pa & ~(uintptr_t)3);
                    const uint32_t sh = (uint32_t)(pa & 3u);
                    uint32_t d[5];
#pragma unroll
                    for (int m = 0; m < 5; ++m) d[m] = pw[m];       // (each holds a byte of the window)
#pragma unroll
                    for (int m = 0; m < 4; ++m) q[m] = __builtin_amdgcn_alignbyte(d[m + 1], d[m], sh);
                    q[4] = d[4] >> (8u * sh);
                    kk += 16u;                                      // < len: no wrap here
                } else {
                    uint32_t b[17];
#pragma unroll
                    for (int u = 0; u < 17; ++u) {
                        b[u] = key[kk];
                        if (u < 16 && ++kk >= kl) kk = 0;           // key[k], k cycles mod len (:67-70)
                    }
#pragma unroll
                    for (int m = 0; m < 4; ++m)
                        q[m] = b[4 * m] | (b[4 * m + 1] << 8) | (b[4 * m + 2] << 16) | (b[4 * m + 3] << 24);
                    q[4] = b[16];
                }
            };
            uint32_t cur[5], nxt[5];
            fetch(cur);
            uint32_t x0 = col, x1 = (1u << 8) | col, a0 = S[col];
            uint32_t ya = col | ((cur[0] & 0xFFu) << 8);   // j = 0 + key[0] before step 0
            for (int c = 0; c < 16; ++c) {
                if (c < 15) fetch(nxt);
                ksa16_window_asm(x0, x1, a0, ya, cur);
#pragma unroll
                for (int m = 0; m < 5; ++m) cur[m] = nxt[m];
            }
        }
    }
    if (active) xy[slot] = 0;                        // _x = _y = 0 (:48-49)
    if (whole) {
        __syncthreads();
        lds_to_image(arena + (size_t)g * kGroupBytes, S);
    } else if (active) {
        scatter_column(arena, slot, S, col);
    }
}

// ---------------------------------------------------------------------------
// xor_ring_kernel: payload spans XOR pre-generated keystream from per-slot
// device rings (zrc4_xor_ring).  One workgroup per entry.  Payload is walked
// in dwords aligned to its own address (whole dwords: one 4-byte RMW; the two
// edge dwords: byte RMWs, so no byte outside the span is ever written); the
// ring is read bytewise at (pos + i) mod cap and the bytes used are zeroed,
// so the next zrc4_crypt over them (0 ^ k = k) refills pure keystream.
// Consecutive lanes touch consecutive dwords / ring bytes (coalesced).
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256)
xor_ring_kernel(uint8_t *__restrict__ ring, uint32_t cap, const uint32_t *__restrict__ rid,
                const uint32_t *__restrict__ pos, uint8_t *__restrict__ payload,
                const uint64_t *__restrict__ off, const uint32_t *__restrict__ len, uint32_t n)
{
    const uint32_t e = blockIdx.x;
    if (e >= n) return;
    const uint32_t L = len[e];
    if (L == 0) return;
    uint8_t *d = payload + off[e];
    uint8_t *r = ring + (size_t)rid[e] * cap;
    const uint32_t p0 = pos[e];
    const uint32_t head = (uint32_t)((uintptr_t)d & 3u);
    uint8_t *d0 = d - head;
    const uint32_t nwords = (head + L + 3u) >> 2;
    for (uint32_t w = threadIdx.x; w < nwords; w += blockDim.x) {
        uint32_t ks = 0, mask = 0;
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
            const int32_t idx = (int32_t)(w * 4u + j) - (int32_t)head;   // span byte index
            if (idx >= 0 && (uint32_t)idx < L) {
                uint32_t q = p0 + (uint32_t)idx;
                if (q >= cap) q -= cap;
                ks |= (uint32_t)r[q] << (8u * j);
                r[q] = 0;
                mask |= 0xFFu << (8u * j);
            }
        }
        if (mask == 0xFFFFFFFFu) {
            uint32_t *wp = reinterpret_cast<uint32_t *>(d0) + w;
            *wp ^= ks;
        } else {
            uint8_t *bp = d0 + w * 4u;
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j)
                if (mask & (0xFFu << (8u * j))) bp[j] ^= (uint8_t)(ks >> (8u * j));
        }
    }
}

// frame_scan_kernel: the framing walk (frame_walk) as its own launch over
// already-decrypted, device-resident buffers (zrc4_frame_scan).
__global__ void __launch_bounds__(256)
frame_scan_kernel(const uint8_t *__restrict__ buf, const uint64_t *__restrict__ off,
                  const uint32_t *__restrict__ len, uint32_t bound, uint32_t n, uint32_t maxp,
                  uint32_t *__restrict__ npk, uint32_t *__restrict__ used, uint32_t *__restrict__ status,
                  uint32_t *__restrict__ pkt_len)
{
    const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n) return;
    frame_walk(buf + off[e], len[e], bound, maxp, e, npk, used, status, pkt_len);
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
