// pipe_ubench.hip -- the per-lane PRGA step (zrc4_kernels.hpp ZRC4_CORE)
// against a software-pipelined step that takes the LDS round trips off the
// y chain, on the conflict-free column layout (address = index << 8 | col).
//
// Classic step (product): y += a; b = S[y]; S[y] = a; a' = S[x+1] (read after
// the S[y] write, so no forwarding); wait b; S[x] = b; k = S[a+b]; wait a'.
// Every byte waits for one LDS round trip (a').
//
// Pipelined step s (one lane = one stream; LDS order = program order):
//   1  y_s += a_s                        5  wait b_{s-1}
//   2  read b_s = S[y_s]   (raw)         6  b_{s-1} = c_{s-1} ? b_{s-2} : raw
//   3  x_s + 2 address                   7  S[x_{s-1}] = b_{s-1}   (deferred)
//   4  c_s = (y_s == x_{s-1})            8  t = a_{s-1} + b_{s-1}
//                                        9  read k_{s-1} = S[t]
//   10 S[y_s] = a_s                      11 read raw a_{s+2} = S[x_s + 2]
//   12 wait raw a_{s+1} (read in step s-1)
//   13-14 a_{s+1} = (y_s == x_s + 1) ? a_s : raw     15 XOR k_{s-2}
// b_s is read before the deferred S[x_{s-1}] write (patched by c_s when they
// are the same byte); k_{s-1} is read after S[x_{s-1}] and before S[y_s];
// a_{s+2} is read after S[y_s] and patched against S[y_{s+1}] one step
// later.  The y chain is VALU only; both LDS reads it depends on leave a
// whole step earlier.  Registers rotate with periods 4 (x addresses, a),
// 3 (b), 2 (patch flags, keystream): 12 steps per unrolled block.
//
// Checked bit-exact (final S column, x, y, and the XOR of every keystream
// byte into byte lane step % 4) against the classic step from the same
// state; cycles per byte from s_memtime over the steps alone.
// Build: hipcc --offload-arch=gfx950 -O3 -o pipe_ubench pipe_ubench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <algorithm>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)

__device__ __forceinline__ uint32_t col_of(uint32_t j) {
    const uint32_t w = j >> 6, l = j & 63u;
    return ((l & 31u) << 2) | (l >> 5) | ((w & 1u) << 1) | ((w >> 1) << 7);
}

// ------------------------------------------------------------ classic step
#define ZC(XC, XN, A, P, K)                                                                      \
    "v_add_u32_sdwa %[ya], %[ya], %[" #A "] dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE "          \
    "src0_sel:BYTE_1 src1_sel:BYTE_0\n\t"                                                        \
    "ds_read_u8 %[b], %[ya]\n\t"                                                                 \
    "ds_write_b8 %[ya], %[" #A "]\n\t"                                                           \
    "v_add_u16_e32 %[" #XN "], %[c100], %[" #XC "]\n\t"                                          \
    "ds_read_u8 %[" #P "], %[" #XN "]\n\t"                                                       \
    "s_waitcnt lgkmcnt(2)\n\t"                                                                   \
    "ds_write_b8 %[" #XC "], %[b]\n\t"                                                           \
    "v_add_u32_sdwa %[ta], %[" #A "], %[b] dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE "           \
    "src0_sel:BYTE_0 src1_sel:BYTE_0\n\t"                                                        \
    "ds_read_u8 %[" #K "], %[ta]\n\t"                                                            \
    "s_waitcnt lgkmcnt(2)\n\t"
#define ZX(SEL, K)                                                                               \
    "v_xor_b32_sdwa %[d], %[d], %[" #K "] dst_sel:" #SEL                                         \
    " dst_unused:UNUSED_PRESERVE src0_sel:" #SEL " src1_sel:BYTE_0\n\t"
#define ZE ZC(x0, x1, a0, a1, k0)
#define ZO ZC(x1, x0, a1, a0, k1)
// step s even -> k0 (lane s % 4), XORed at step s + 1
#define ZW ZE ZX(BYTE_3, k1) ZO ZX(BYTE_0, k0) ZE ZX(BYTE_1, k1) ZO ZX(BYTE_2, k0)

// ------------------------------------- classic step with a byte exchange
// b = S[y], S[y] = a in ONE LDS op: ds_mskor_rtn_b32 on the dword holding
// the byte (clear mask m = 0xFF << 8*(col & 3), set a << 8*(col & 3)), the
// old byte extracted with v_bfe.  yd = y's dword address (byte 1 updated
// with y, byte 0 = col & ~3), sh = 8*(col & 3).
#define MC(XC, XN, A, P, K)                                                                      \
    "v_add_u32_sdwa %[ya], %[ya], %[" #A "] dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE "          \
    "src0_sel:BYTE_1 src1_sel:BYTE_0\n\t"                                                        \
    "v_lshlrev_b32 %[tmp], %[sh], %[" #A "]\n\t"                                                \
    "v_and_b32 %[yd], %[ya], %[nm3]\n\t"                                                        \
    "ds_mskor_rtn_b32 %[b], %[yd], %[m], %[tmp]\n\t"                                            \
    "v_add_u16_e32 %[" #XN "], %[c100], %[" #XC "]\n\t"                                          \
    "ds_read_u8 %[" #P "], %[" #XN "]\n\t"                                                       \
    "s_waitcnt lgkmcnt(1)\n\t"                                                                   \
    "v_bfe_u32 %[b], %[b], %[sh], 8\n\t"                                                         \
    "ds_write_b8 %[" #XC "], %[b]\n\t"                                                           \
    "v_add_u32_sdwa %[ta], %[" #A "], %[b] dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE "           \
    "src0_sel:BYTE_0 src1_sel:BYTE_0\n\t"                                                        \
    "ds_read_u8 %[" #K "], %[ta]\n\t"                                                            \
    "s_waitcnt lgkmcnt(2)\n\t"
#define ME MC(x0, x1, a0, a1, k0)
#define MO MC(x1, x0, a1, a0, k1)
#define MW ME ZX(BYTE_3, k1) MO ZX(BYTE_0, k0) ME ZX(BYTE_1, k1) MO ZX(BYTE_2, k0)

// ------------------------------------------------------- pipelined step
#define PS(XP, XC, XN, XF, AP, AC, AN, AF, BPP, BP, BC, SP, SC, KW, KX, LX)                       \
    "v_add_u32_sdwa %[ya], %[ya], %[" #AC "] dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE "         \
    "src0_sel:BYTE_1 src1_sel:BYTE_0\n\t"                                                        \
    "ds_read_u8 %[" #BC "], %[ya]\n\t"                                                           \
    "v_add_u16_e32 %[" #XF "], %[c100], %[" #XN "]\n\t"                                          \
    "v_cmp_eq_u32_e64 " SC ", %[ya], %[" #XP "]\n\t"                                             \
    "s_waitcnt lgkmcnt(5)\n\t"                                                                   \
    "v_cndmask_b32_e64 %[" #BP "], %[" #BP "], %[" #BPP "], " SP "\n\t"                          \
    "ds_write_b8 %[" #XP "], %[" #BP "]\n\t"                                                     \
    "v_add_u32_sdwa %[ta], %[" #AP "], %[" #BP "] dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE "    \
    "src0_sel:BYTE_0 src1_sel:BYTE_0\n\t"                                                        \
    "ds_read_u8 %[" #KW "], %[ta]\n\t"                                                           \
    "ds_write_b8 %[ya], %[" #AC "]\n\t"                                                          \
    "ds_read_u8 %[" #AF "], %[" #XF "]\n\t"                                                      \
    "s_waitcnt lgkmcnt(5)\n\t"                                                                   \
    "v_cmp_eq_u32_e32 vcc, %[ya], %[" #XN "]\n\t"                                                \
    "v_cndmask_b32_e32 %[" #AN "], %[" #AN "], %[" #AC "], vcc\n\t"                              \
    "v_xor_b32_sdwa %[d], %[d], %[" #KX "] dst_sel:" #LX                                         \
    " dst_unused:UNUSED_PRESERVE src0_sel:" #LX " src1_sel:BYTE_0\n\t"

// step s (s = 1 + u, u = 0..11): X/A ring index s % 4, B ring s % 3, flag /
// keystream ring s % 2; XOR lane of k_{s-2} = (s - 2) % 4
#define SG0 "%[sg0]"
#define SG1 "%[sg1]"
#define P1  PS(X0, X1, X2, X3, A0, A1, A2, A3, B2, B0, B1, SG0, SG1, K1, K0, BYTE_3)
#define P2  PS(X1, X2, X3, X0, A1, A2, A3, A0, B0, B1, B2, SG1, SG0, K0, K1, BYTE_0)
#define P3  PS(X2, X3, X0, X1, A2, A3, A0, A1, B1, B2, B0, SG0, SG1, K1, K0, BYTE_1)
#define P4  PS(X3, X0, X1, X2, A3, A0, A1, A2, B2, B0, B1, SG1, SG0, K0, K1, BYTE_2)
#define P5  PS(X0, X1, X2, X3, A0, A1, A2, A3, B0, B1, B2, SG0, SG1, K1, K0, BYTE_3)
#define P6  PS(X1, X2, X3, X0, A1, A2, A3, A0, B1, B2, B0, SG1, SG0, K0, K1, BYTE_0)
#define P7  PS(X2, X3, X0, X1, A2, A3, A0, A1, B2, B0, B1, SG0, SG1, K1, K0, BYTE_1)
#define P8  PS(X3, X0, X1, X2, A3, A0, A1, A2, B0, B1, B2, SG1, SG0, K0, K1, BYTE_2)
#define P9  PS(X0, X1, X2, X3, A0, A1, A2, A3, B1, B2, B0, SG0, SG1, K1, K0, BYTE_3)
#define P10 PS(X1, X2, X3, X0, A1, A2, A3, A0, B2, B0, B1, SG1, SG0, K0, K1, BYTE_0)
#define P11 PS(X2, X3, X0, X1, A2, A3, A0, A1, B0, B1, B2, SG0, SG1, K1, K0, BYTE_1)
#define P12 PS(X3, X0, X1, X2, A3, A0, A1, A2, B1, B2, B0, SG1, SG0, K0, K1, BYTE_2)
#define P12STEPS P1 P2 P3 P4 P5 P6 P7 P8 P9 P10 P11 P12

// ----------------------------------------------- consecutive-index layout
// (r06): four consecutive S indices of one stream in one
// dword, so one ds_read_b32 serves the four a = S[x] reads of a 4-byte block
// and one ds_write_b32 retires its four S[x] = b writes.  Layout per 256-lane
// group (64 KiB): byte (k >> 2) << 10 | lane << 2 | (k & 3), i.e. row m = k/4
// holds one dword per lane: every ds_read_u8 / ds_read_b32 / ds_write_b32 of a
// wave is bank-conflict free for any indices (bank = lane mod 32).
// Registers: W = the current block's dword, kept as the TRUTH for S[4m..4m+3]
// (LDS holds it stale until the block's dword write); XB = the block's dword
// address (m << 10 | lane << 2); y8 = y as a clean byte.  Addresses are no
// longer "index in byte 1" (the SDWA trick of the column layout): addr(v) =
// (v * 0x101 & 0xFC03) | L, two VALU ops per computed index (y and t).
// Exact step j (x = 4m + j), a = W.byte_j:
//   y += a;  R = rotr(W, 8 (y & 3)) (R.b0 = W[y & 3]);  AY = addr(y)
//   ds_read_u8 BR = S[AY];  ds_write_b8 S[AY] = a   (always: an in-block
//   byte is overwritten by the dword write, an out-of-block one is final)
//   c_y = (AY - XB) < 4 (y in this block)
//   b = c_y ? R.b0 : BR;  t = a + b
//   W' = W with byte (y & 3) = a (rotate, replace byte 0, rotate back);
//   W = c_y ? W' : W;  W.byte_j = b      (S[x] = b then S[y] = a: the two
//   bytes differ unless y == x, and then a == b)
//   AT = addr(t);  ds_read_u8 KR = S[AT];  KW = W[t & 3];  c_t = (AT - XB) < 4
//   k = c_t ? KW : KR   (finished in the next step, after its BR wait)
// Block end: ds_write_b32 S[XB] = W; XB += 0x400 (16-bit wrap = index wrap);
// ds_read_b32 W = S[XB] (waited for before the next block's first y add).
// The skeleton (timing bound, outputs wrong) is the same LDS program and the
// same address work without any patch: b = BR, k = KR, no in-block insert.
#define QP_SEL(J) "%[sel" #J "]"
#define QE_STEP(J, WD, JP, KRC, KWC, TCC, KRP, KWP, TCP)                                          \
    "v_add_u32_sdwa %[y8], %[y8], %[w] dst_sel:BYTE_0 dst_unused:UNUSED_PAD "                    \
    "src0_sel:BYTE_0 src1_sel:BYTE_" #J "\n\t"                                                   \
    "v_alignbyte_b32 %[r], %[w], %[w], %[y8]\n\t" /* reads y8[1:0] only */                       \
    QV_##J                                                                                       \
    "v_lshl_or_b32 %[ay], %[y8], 8, %[y8]\n\t"                                                   \
    "v_and_or_b32 %[ay], %[ay], %[msk], %[lb]\n\t"                                               \
    "ds_read_u8 %[br], %[ay]\n\t"                                                                \
    WD                                                                                           \
    "v_sub_u32_e32 %[e], %[ay], %[xb]\n\t"                                                       \
    "v_perm_b32 %[r2], %[w], %[r], " QP_SEL(J) "\n\t"                                            \
    "v_sub_u32_e32 %[ny], 0, %[y8]\n\t"                                                          \
    "v_cmp_gt_u32_e32 vcc, 4, %[e]\n\t"                                                          \
    "v_alignbyte_b32 %[wi], %[r2], %[r2], %[ny]\n\t"                                             \
    "s_waitcnt lgkmcnt(1)\n\t"                                                                   \
    "v_cndmask_b32_e64 %[k], %[" #KRP "], %[" #KWP "], %[" #TCP "]\n\t"                          \
    "v_cndmask_b32_e32 %[b], %[br], %[r], vcc\n\t"                                               \
    "v_xor_b32_sdwa %[d], %[d], %[k] dst_sel:BYTE_" #JP " dst_unused:UNUSED_PRESERVE "           \
    "src0_sel:BYTE_" #JP " src1_sel:BYTE_0\n\t"                                                  \
    "v_add_u32_sdwa %[t8], %[w], %[b] dst_sel:BYTE_0 dst_unused:UNUSED_PAD "                     \
    "src0_sel:BYTE_" #J " src1_sel:BYTE_0\n\t"                                                   \
    "v_cndmask_b32_e32 %[w], %[w], %[wi], vcc\n\t"                                               \
    "v_mov_b32_sdwa %[w], %[b] dst_sel:BYTE_" #J " dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0\n\t" \
    "v_lshl_or_b32 %[at], %[t8], 8, %[t8]\n\t"                                                   \
    "v_and_or_b32 %[at], %[at], %[msk], %[lb]\n\t"                                               \
    "ds_read_u8 %[" #KRC "], %[at]\n\t"                                                          \
    "v_sub_u32_e32 %[et], %[at], %[xb]\n\t"                                                      \
    "v_alignbyte_b32 %[" #KWC "], %[w], %[w], %[t8]\n\t"                                         \
    "v_cmp_gt_u32_e64 %[" #TCC "], 4, %[et]\n\t"
// V = W >> 8 before the odd steps: their a sits in V's byte 0 / byte 2
#define QV_0
#define QV_1 "v_lshrrev_b32_e32 %[v], 8, %[w]\n\t"
#define QV_2
#define QV_3 "v_lshrrev_b32_e32 %[v], 8, %[w]\n\t"
#define QWD_0 "ds_write_b8 %[ay], %[w]\n\t"
#define QWD_1 "ds_write_b8 %[ay], %[v]\n\t"
#define QWD_2 "ds_write_b8_d16_hi %[ay], %[w]\n\t"
#define QWD_3 "ds_write_b8_d16_hi %[ay], %[v]\n\t"
#define QE_BLOCK                                                                                 \
    QE_STEP(0, QWD_0, 3, kr0, kw0, tc0, kr1, kw1, tc1)                                           \
    QE_STEP(1, QWD_1, 0, kr1, kw1, tc1, kr0, kw0, tc0)                                           \
    QE_STEP(2, QWD_2, 1, kr0, kw0, tc0, kr1, kw1, tc1)                                           \
    QE_STEP(3, QWD_3, 2, kr1, kw1, tc1, kr0, kw0, tc0)                                           \
    QBLOCK_END
#define QBLOCK_END                                                                               \
    "ds_write_b32 %[xb], %[w]\n\t"                                                               \
    "v_add_u16_e32 %[xb], %[c400], %[xb]\n\t"                                                    \
    "ds_read_b32 %[w], %[xb]\n\t"                                                                \
    "s_waitcnt lgkmcnt(0)\n\t"
// skeleton: same LDS program and address work, no patches (timing only)
#define QK_STEP(J, WD, JP, KRC, KRP)                                                              \
    "v_add_u32_sdwa %[y8], %[y8], %[w] dst_sel:BYTE_0 dst_unused:UNUSED_PAD "                    \
    "src0_sel:BYTE_0 src1_sel:BYTE_" #J "\n\t"                                                   \
    "v_lshrrev_b32_e32 %[v], 8, %[w]\n\t"                                                        \
    "v_lshl_or_b32 %[ay], %[y8], 8, %[y8]\n\t"                                                   \
    "v_and_or_b32 %[ay], %[ay], %[msk], %[lb]\n\t"                                               \
    "ds_read_u8 %[br], %[ay]\n\t"                                                                \
    WD                                                                                           \
    "s_waitcnt lgkmcnt(1)\n\t"                                                                   \
    "v_xor_b32_sdwa %[d], %[d], %[" #KRP "] dst_sel:BYTE_" #JP " dst_unused:UNUSED_PRESERVE "    \
    "src0_sel:BYTE_" #JP " src1_sel:BYTE_0\n\t"                                                  \
    "v_add_u32_sdwa %[t8], %[w], %[br] dst_sel:BYTE_0 dst_unused:UNUSED_PAD "                    \
    "src0_sel:BYTE_" #J " src1_sel:BYTE_0\n\t"                                                   \
    "v_mov_b32_sdwa %[w], %[br] dst_sel:BYTE_" #J " dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0\n\t" \
    "v_lshl_or_b32 %[at], %[t8], 8, %[t8]\n\t"                                                   \
    "v_and_or_b32 %[at], %[at], %[msk], %[lb]\n\t"                                               \
    "ds_read_u8 %[" #KRC "], %[at]\n\t"
#define QK_BLOCK                                                                                 \
    QK_STEP(0, QWD_0, 3, kr0, kr1) QK_STEP(1, QWD_1, 0, kr1, kr0)                                \
    QK_STEP(2, QWD_2, 1, kr0, kr1) QK_STEP(3, QWD_3, 2, kr1, kr0)                                \
    QBLOCK_END
// skeleton with the next block's dword read issued after step 1 (an exact
// version would have to patch it for steps 1-3's writes into that block):
// no round trip exposed at the block boundary -- the LDS program's best case
#define QK2_BLOCK                                                                                \
    QK_STEP(0, QWD_0, 3, kr0, kr1) QK_STEP(1, QWD_1, 0, kr1, kr0)                                \
    "v_add_u16_e32 %[e], %[c400], %[xb]\n\t"                                                     \
    "ds_read_b32 %[wi], %[e]\n\t"                                                                \
    QK_STEP(2, QWD_2, 1, kr0, kr1) QK_STEP(3, QWD_3, 2, kr1, kr0)                                \
    "ds_write_b32 %[xb], %[w]\n\t"                                                               \
    "v_mov_b32_e32 %[xb], %[e]\n\t"                                                              \
    "v_mov_b32_e32 %[w], %[wi]\n\t"

struct Out { uint64_t cyc; uint32_t d, xy; };

// The same state for every variant: S column = (k * 73 + tid) & 255, x = 0, y = 7.
__device__ __forceinline__ void init_s(uint8_t *S, uint32_t col)
{
    for (int k = 0; k < 256; ++k) S[(k << 8) | col] = (uint8_t)((k * 73 + threadIdx.x) & 255);
}

// classic: steps = 12 * blocks + 1
__global__ void __launch_bounds__(256) classic_kernel(uint8_t *sout, Out *out, int blocks, int active_waves)
{
    __shared__ __attribute__((aligned(16))) uint8_t S[65536];
    const uint32_t col = col_of(threadIdx.x);
    init_s(S, col);
    __syncthreads();
    const bool act = (int)(threadIdx.x >> 6) < active_waves;
    if (act) {
        const uint32_t c100 = 0x100;
        uint32_t ya = (7u << 8) | col, ta = col, x0 = col, x1 = col, a0 = S[x0], d = 0;   // x = 0: a0 = S[0]
        uint32_t a1, b, k0 = 0, k1 = 0;
        const uint64_t t0 = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < blocks; ++i) {
            asm volatile(ZW ZW ZW
                         : [ya] "+v"(ya), [ta] "+v"(ta), [x0] "+v"(x0), [x1] "+v"(x1), [a0] "+v"(a0),
                           [a1] "=&v"(a1), [b] "=&v"(b), [k0] "+v"(k0), [k1] "+v"(k1), [d] "+v"(d)
                         : [c100] "s"(c100) : "memory");
        }
        asm volatile(ZE ZX(BYTE_3, k1) "s_waitcnt lgkmcnt(0)\n\t" ZX(BYTE_0, k0)
                     : [ya] "+v"(ya), [ta] "+v"(ta), [x0] "+v"(x0), [x1] "+v"(x1), [a0] "+v"(a0),
                       [a1] "=&v"(a1), [b] "=&v"(b), [k0] "+v"(k0), [k1] "+v"(k1), [d] "+v"(d)
                     : [c100] "s"(c100) : "memory");
        const uint64_t t1 = __builtin_amdgcn_s_memtime();
        const uint32_t g = blockIdx.x * 256 + threadIdx.x;
        out[g].cyc = t1 - t0;
        out[g].d = d;
        out[g].xy = ((x0 >> 8) & 255u) | (((ya >> 8) & 255u) << 8);   // the last step's x (its XC)
    }
    __syncthreads();
    for (int k = 0; k < 256; ++k) sout[((size_t)blockIdx.x * 256 + threadIdx.x) * 256 + k] = S[(k << 8) | col];
}

// classic with 32-lane waves: 512 threads, lanes 32-63 of every wave idle, so
// a CU's 256 streams run on 8 waves (2 per SIMD) instead of 4: is one wave's
// LDS instruction rate per instruction or per lane?
__global__ void __launch_bounds__(512) half_kernel(uint8_t *sout, Out *out, int blocks, int active_waves)
{
    __shared__ __attribute__((aligned(16))) uint8_t S[65536];
    const uint32_t hj = (threadIdx.x >> 6) * 32u + (threadIdx.x & 31u);   // stream of this lane
    const bool lane_on = (threadIdx.x & 63u) < 32u;
    const uint32_t col = col_of(hj);
    if (lane_on)
        for (int k = 0; k < 256; ++k) S[(k << 8) | col] = (uint8_t)((k * 73 + hj) & 255);
    __syncthreads();
    const bool act = lane_on && (int)(threadIdx.x >> 6) < 2 * active_waves;
    if (act) {
        const uint32_t c100 = 0x100;
        uint32_t ya = (7u << 8) | col, ta = col, x0 = col, x1 = col, a0 = S[x0], d = 0;   // x = 0: a0 = S[0]
        uint32_t a1, b, k0 = 0, k1 = 0;
        const uint64_t t0 = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < blocks; ++i) {
            asm volatile(ZW ZW ZW
                         : [ya] "+v"(ya), [ta] "+v"(ta), [x0] "+v"(x0), [x1] "+v"(x1), [a0] "+v"(a0),
                           [a1] "=&v"(a1), [b] "=&v"(b), [k0] "+v"(k0), [k1] "+v"(k1), [d] "+v"(d)
                         : [c100] "s"(c100) : "memory");
        }
        asm volatile(ZE ZX(BYTE_3, k1) "s_waitcnt lgkmcnt(0)\n\t" ZX(BYTE_0, k0)
                     : [ya] "+v"(ya), [ta] "+v"(ta), [x0] "+v"(x0), [x1] "+v"(x1), [a0] "+v"(a0),
                       [a1] "=&v"(a1), [b] "=&v"(b), [k0] "+v"(k0), [k1] "+v"(k1), [d] "+v"(d)
                     : [c100] "s"(c100) : "memory");
        const uint64_t t1 = __builtin_amdgcn_s_memtime();
        const uint32_t g = blockIdx.x * 256 + hj;
        out[g].cyc = t1 - t0;
        out[g].d = d;
        out[g].xy = ((x0 >> 8) & 255u) | (((ya >> 8) & 255u) << 8);   // the last step's x (its XC)
    }
    __syncthreads();
    if (lane_on)
        for (int k = 0; k < 256; ++k) sout[((size_t)blockIdx.x * 256 + hj) * 256 + k] = S[(k << 8) | col];
}

// classic with the byte exchange (ds_mskor_rtn_b32): steps = 12 * blocks + 1
__global__ void __launch_bounds__(256) mskor_kernel(uint8_t *sout, Out *out, int blocks, int active_waves)
{
    __shared__ __attribute__((aligned(16))) uint8_t S[65536];
    const uint32_t col = col_of(threadIdx.x);
    init_s(S, col);
    __syncthreads();
    const bool act = (int)(threadIdx.x >> 6) < active_waves;
    if (act) {
        const uint32_t c100 = 0x100;
        uint32_t ya = (7u << 8) | col, ta = col, x0 = col, x1 = col, a0 = S[x0], d = 0;   // x = 0: a0 = S[0]
        uint32_t a1, b, k0 = 0, k1 = 0, tmp, yd;
        const uint32_t sh = 8u * (col & 3u), m = 0xFFu << sh, nm3 = ~3u;
        const uint64_t t0 = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < blocks; ++i) {
            asm volatile(MW MW MW
                         : [ya] "+v"(ya), [ta] "+v"(ta), [x0] "+v"(x0), [x1] "+v"(x1), [a0] "+v"(a0),
                           [a1] "=&v"(a1), [b] "=&v"(b), [k0] "+v"(k0), [k1] "+v"(k1), [d] "+v"(d),
                           [tmp] "=&v"(tmp), [yd] "=&v"(yd)
                         : [c100] "s"(c100), [sh] "v"(sh), [m] "v"(m), [nm3] "v"(nm3) : "memory");
        }
        asm volatile(ME ZX(BYTE_3, k1) "s_waitcnt lgkmcnt(0)\n\t" ZX(BYTE_0, k0)
                     : [ya] "+v"(ya), [ta] "+v"(ta), [x0] "+v"(x0), [x1] "+v"(x1), [a0] "+v"(a0),
                       [a1] "=&v"(a1), [b] "=&v"(b), [k0] "+v"(k0), [k1] "+v"(k1), [d] "+v"(d),
                       [tmp] "=&v"(tmp), [yd] "=&v"(yd)
                     : [c100] "s"(c100), [sh] "v"(sh), [m] "v"(m), [nm3] "v"(nm3) : "memory");
        const uint64_t t1 = __builtin_amdgcn_s_memtime();
        const uint32_t g = blockIdx.x * 256 + threadIdx.x;
        out[g].cyc = t1 - t0;
        out[g].d = d;
        out[g].xy = ((x0 >> 8) & 255u) | (((ya >> 8) & 255u) << 8);   // the last step's x (its XC)
    }
    __syncthreads();
    for (int k = 0; k < 256; ++k) sout[((size_t)blockIdx.x * 256 + threadIdx.x) * 256 + k] = S[(k << 8) | col];
}

// pipelined: step 0 classic (in C++), steps 1 .. 12 * blocks pipelined, tail
__global__ void __launch_bounds__(256) pipe_kernel(uint8_t *sout, Out *out, int blocks, int active_waves)
{
    __shared__ __attribute__((aligned(16))) uint8_t S[65536];
    const uint32_t col = col_of(threadIdx.x);
    init_s(S, col);
    __syncthreads();
    const bool act = (int)(threadIdx.x >> 6) < active_waves;
    if (act) {
        const uint32_t c100 = 0x100;
        // step 0: x_0 = 0, y = 7
        uint32_t X0 = col, X1 = (1u << 8) | col, X2 = (2u << 8) | col, X3 = 0;
        uint32_t A0 = S[X0];
        uint32_t ya = (((7u + A0) & 255u) << 8) | col;
        uint32_t B0 = S[ya];
        S[ya] = (uint8_t)A0;
        S[X0] = (uint8_t)B0;
        uint32_t A1 = S[X1], A2 = S[X2], A3 = 0, B1 = 0, B2 = 0, K0 = 0, K1 = 0, d = 0, ta = col;
        uint64_t sg0 = 0, sg1 = 0;     // the b patch flags (SGPR pairs), carried across the asm blocks
        const uint64_t t0 = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < blocks; ++i) {
            asm volatile(P12STEPS
                         : [ya] "+v"(ya), [ta] "+v"(ta), [X0] "+v"(X0), [X1] "+v"(X1), [X2] "+v"(X2), [X3] "+v"(X3),
                           [A0] "+v"(A0), [A1] "+v"(A1), [A2] "+v"(A2), [A3] "+v"(A3), [B0] "+v"(B0), [B1] "+v"(B1),
                           [B2] "+v"(B2), [K0] "+v"(K0), [K1] "+v"(K1), [d] "+v"(d), [sg0] "+s"(sg0), [sg1] "+s"(sg1)
                         : [c100] "s"(c100) : "memory", "vcc");
        }
        // tail after step s = 12 * blocks (P12): b_s raw in B0, its flag in sg0, b_{s-1}
        // final in B2 -> b_s = sg0 ? B2 : B0; S[x_s] (X0) = b_s; k_s = S[a_s (A0) + b_s];
        // k_{s-1} is in K0 (lane 3), k_s lane 0.
        asm volatile("s_waitcnt lgkmcnt(0)\n\t"
                     "v_cndmask_b32_e64 %[B0], %[B0], %[B2], %[sg0]\n\t"
                     "ds_write_b8 %[X0], %[B0]\n\t"
                     "v_add_u32_sdwa %[ta], %[A0], %[B0] dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE "
                     "src0_sel:BYTE_0 src1_sel:BYTE_0\n\t"
                     "ds_read_u8 %[K1], %[ta]\n\t"
                     "s_waitcnt lgkmcnt(0)\n\t"
                     "v_xor_b32_sdwa %[d], %[d], %[K0] dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_3 src1_sel:BYTE_0\n\t"
                     "s_nop 1\n\t"                      // (an SDWA byte write read by the next VALU op)
                     "v_xor_b32_sdwa %[d], %[d], %[K1] dst_sel:BYTE_0 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0 src1_sel:BYTE_0\n\t"
                     : [ta] "+v"(ta), [B0] "+v"(B0), [K0] "+v"(K0), [K1] "+v"(K1), [d] "+v"(d)
                     : [X0] "v"(X0), [A0] "v"(A0), [B2] "v"(B2), [sg0] "s"(sg0) : "memory");
        const uint64_t t1 = __builtin_amdgcn_s_memtime();
        const uint32_t g = blockIdx.x * 256 + threadIdx.x;
        out[g].cyc = t1 - t0;
        out[g].d = d;
        out[g].xy = ((X0 >> 8) & 255u) | (((ya >> 8) & 255u) << 8);
    }
    __syncthreads();
    for (int k = 0; k < 256; ++k) sout[((size_t)blockIdx.x * 256 + threadIdx.x) * 256 + k] = S[(k << 8) | col];
}

// consecutive-index layout: steps 0 .. 12 * blocks - 1 in 4-byte blocks, then
// step 12 * blocks (j = 0 of the next block) and the final dword write.
__device__ __forceinline__ uint32_t qaddr(uint32_t k, uint32_t j) { return ((k >> 2) << 10) | (j << 2) | (k & 3u); }

#define QREGS                                                                                    \
    [y8] "+v"(y8), [w] "+v"(w), [xb] "+v"(xb), [v] "+v"(v), [d] "+v"(d), [k] "+v"(k),          \
    [kr0] "+v"(kr0), [kr1] "+v"(kr1), [kw0] "+v"(kw0), [kw1] "+v"(kw1), [tc0] "+s"(tc0),        \
    [tc1] "+s"(tc1), [br] "=&v"(br), [b] "=&v"(b), [r] "=&v"(r), [r2] "=&v"(r2), [ny] "=&v"(ny), \
    [wi] "=&v"(wi), [e] "=&v"(e), [t8] "=&v"(t8), [at] "=&v"(at), [et] "=&v"(et), [ay] "=&v"(ay)
#define QINS                                                                                     \
    [lb] "v"(lb), [msk] "s"(msk), [c400] "s"(c400), [sel0] "s"(sel0), [sel1] "s"(sel1),         \
    [sel2] "s"(sel2), [sel3] "s"(sel3)

template <int QMODE>   // 0 skeleton, 1 exact, 2 skeleton with the next block's read ahead
__global__ void __launch_bounds__(256) quad_kernel(uint8_t *sout, Out *out, int blocks, int active_waves)
{
    __shared__ __attribute__((aligned(16))) uint8_t S[65536];
    const uint32_t jl = threadIdx.x;
    for (int kk = 0; kk < 256; ++kk) S[qaddr(kk, jl)] = (uint8_t)((kk * 73 + jl) & 255);
    __syncthreads();
    const bool act = (int)(threadIdx.x >> 6) < active_waves;
    if (act) {
        const uint32_t lb = jl << 2, msk = 0xFC03u, c400 = 0x400u;
        const uint32_t sel0 = 0x03020104u, sel1 = 0x03020105u, sel2 = 0x03020106u, sel3 = 0x03020107u;
        uint32_t xb = lb, y8 = 7, d = 0, v = 0, k = 0, kr0 = 0, kr1 = 0, kw0 = 0, kw1 = 0;
        uint32_t br, b, r, r2, ny, wi, e, t8, at, et, ay;
        uint64_t tc0 = 0, tc1 = 0;
        uint32_t w = *reinterpret_cast<const uint32_t *>(&S[xb]);      // x = 0: S[0..3]
        const uint64_t t0 = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < blocks; ++i) {
            if (QMODE == 1)
                asm volatile(QE_BLOCK QE_BLOCK QE_BLOCK : QREGS : QINS : "memory", "vcc");
            else if (QMODE == 2)
                asm volatile(QK2_BLOCK QK2_BLOCK QK2_BLOCK : QREGS : QINS : "memory", "vcc");
            else
                asm volatile(QK_BLOCK QK_BLOCK QK_BLOCK : QREGS : QINS : "memory", "vcc");
        }
        if (QMODE == 1)
            asm volatile(QE_STEP(0, QWD_0, 3, kr0, kw0, tc0, kr1, kw1, tc1)
                         "s_waitcnt lgkmcnt(0)\n\t"
                         "v_cndmask_b32_e64 %[k], %[kr0], %[kw0], %[tc0]\n\t"
                         "s_nop 1\n\t"
                         "v_xor_b32_sdwa %[d], %[d], %[k] dst_sel:BYTE_0 dst_unused:UNUSED_PRESERVE "
                         "src0_sel:BYTE_0 src1_sel:BYTE_0\n\t"
                         "ds_write_b32 %[xb], %[w]\n\t"
                         "s_waitcnt lgkmcnt(0)\n\t"
                         : QREGS : QINS : "memory", "vcc");
        else
            asm volatile(QK_STEP(0, QWD_0, 3, kr0, kr1)
                         "s_waitcnt lgkmcnt(0)\n\t"
                         "v_xor_b32_sdwa %[d], %[d], %[kr0] dst_sel:BYTE_0 dst_unused:UNUSED_PRESERVE "
                         "src0_sel:BYTE_0 src1_sel:BYTE_0\n\t"
                         "ds_write_b32 %[xb], %[w]\n\t"
                         "s_waitcnt lgkmcnt(0)\n\t"
                         : QREGS : QINS : "memory", "vcc");
        const uint64_t t1 = __builtin_amdgcn_s_memtime();
        const uint32_t g = blockIdx.x * 256 + threadIdx.x;
        out[g].cyc = t1 - t0;
        out[g].d = d;
        out[g].xy = (((xb >> 10) & 63u) << 2) | ((y8 & 255u) << 8);
    }
    __syncthreads();
    for (int kk = 0; kk < 256; ++kk) sout[((size_t)blockIdx.x * 256 + threadIdx.x) * 256 + kk] = S[qaddr(kk, jl)];
}

// CPU reference for one lane (tid t): same init, steps 12 * blocks + 1.
static void cpu_ref(uint32_t t, int steps, uint8_t *S, uint32_t &d, uint32_t &xy)
{
    for (int k = 0; k < 256; ++k) S[k] = (uint8_t)((k * 73 + t) & 255);
    uint32_t x = 0, y = 7;
    d = 0;
    // our step s processes index x_s = s (x starts at 0 for step 0)
    for (int s = 0; s < steps; ++s) {
        const uint8_t a = S[x];
        y = (y + a) & 255;
        const uint8_t b = S[y];
        S[x] = b;
        S[y] = a;
        const uint8_t k = S[(a + b) & 255];
        d ^= (uint32_t)k << (8 * (s % 4));
        if (s + 1 < steps) x = (x + 1) & 255;
    }
    xy = x | (y << 8);
}

int main(int argc, char **argv)
{
    const int blocks = argc > 1 ? atoi(argv[1]) : 86;   // 12 * 86 + 1 = 1 033 steps
    int ncu = 0;
    CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    const int steps = 12 * blocks + 1;
    struct Cfg { int wg_per_cu, waves; const char *name; } cfgs[] = {{1, 1, "1wave_per_cu"}, {1, 4, "4waves_per_cu"},
                                                                    {2, 4, "8waves_per_cu"}};
    printf("{\"steps\": %d", steps);
    for (auto &c : cfgs) {
        const int grid = ncu * c.wg_per_cu, n = grid * 256;
        uint8_t *ds; Out *dout;
        CHECK(hipMalloc(&ds, (size_t)n * 256)); CHECK(hipMalloc(&dout, (size_t)n * sizeof(Out)));
        std::vector<uint8_t> s0((size_t)n * 256), s1((size_t)n * 256);
        std::vector<Out> o0(n), o1(n);
        std::vector<uint8_t> s2((size_t)n * 256), s3((size_t)n * 256), s4((size_t)n * 256), s5((size_t)n * 256), s6((size_t)n * 256);
        std::vector<Out> o2(n), o3(n), o4(n), o5(n), o6(n);
        double med[7];
        // QUAD_ONLY: the classic step and the two consecutive-index kernels only
        const bool quad_only = getenv("QUAD_ONLY") != nullptr;
        for (int v = 0; v < 7; ++v) {
            if (quad_only && v >= 1 && v <= 3) { med[v] = 0; continue; }
            CHECK(hipMemset(dout, 0, (size_t)n * sizeof(Out)));
            for (int r = 0; r < 3; ++r) {
                if (v == 0) hipLaunchKernelGGL(classic_kernel, dim3(grid), dim3(256), 0, 0, ds, dout, blocks, c.waves);
                else if (v == 1) hipLaunchKernelGGL(pipe_kernel, dim3(grid), dim3(256), 0, 0, ds, dout, blocks, c.waves);
                else if (v == 2) hipLaunchKernelGGL(mskor_kernel, dim3(grid), dim3(256), 0, 0, ds, dout, blocks, c.waves);
                else if (v == 3) hipLaunchKernelGGL(half_kernel, dim3(grid), dim3(512), 0, 0, ds, dout, blocks, c.waves);
                else if (v == 4) hipLaunchKernelGGL(quad_kernel<1>, dim3(grid), dim3(256), 0, 0, ds, dout, blocks, c.waves);
                else if (v == 5) hipLaunchKernelGGL(quad_kernel<0>, dim3(grid), dim3(256), 0, 0, ds, dout, blocks, c.waves);
                else hipLaunchKernelGGL(quad_kernel<2>, dim3(grid), dim3(256), 0, 0, ds, dout, blocks, c.waves);
                CHECK(hipDeviceSynchronize());
            }
            std::vector<uint8_t> &sv = v == 0 ? s0 : v == 1 ? s1 : v == 2 ? s2 : v == 3 ? s3 : v == 4 ? s4 : v == 5 ? s5 : s6;
            std::vector<Out> &ov = v == 0 ? o0 : v == 1 ? o1 : v == 2 ? o2 : v == 3 ? o3 : v == 4 ? o4 : v == 5 ? o5 : o6;
            CHECK(hipMemcpy(sv.data(), ds, (size_t)n * 256, hipMemcpyDeviceToHost));
            CHECK(hipMemcpy(ov.data(), dout, (size_t)n * sizeof(Out), hipMemcpyDeviceToHost));
            std::vector<double> cyc;
            for (int g = 0; g < n; ++g)
                if ((int)((g % 256) >> 6) < c.waves) cyc.push_back((double)ov[g].cyc / steps);
            std::sort(cyc.begin(), cyc.end());
            med[v] = cyc[cyc.size() / 2];
        }
        // bit-exactness: classic vs CPU on a sample, pipelined vs classic everywhere (active lanes)
        long bad_cpu = 0, bad_pipe = 0, bad_mskor = 0, bad_half = 0, bad_quad = 0, bad_quad_cpu = 0;
        std::vector<uint8_t> S(256);
        for (int g = 0; g < n; ++g) {
            if ((int)((g % 256) >> 6) >= c.waves) continue;
            if (g % 97 == 0) {
                uint32_t d, xy;
                cpu_ref((uint32_t)(g % 256), steps, S.data(), d, xy);
                if (memcmp(S.data(), &s0[(size_t)g * 256], 256) || d != o0[g].d || xy != o0[g].xy) ++bad_cpu;
                if (memcmp(S.data(), &s4[(size_t)g * 256], 256) || d != o4[g].d || xy != o4[g].xy) ++bad_quad_cpu;
            }
            if (memcmp(&s0[(size_t)g * 256], &s4[(size_t)g * 256], 256) || o0[g].d != o4[g].d || o0[g].xy != o4[g].xy)
                ++bad_quad;
            if (quad_only) continue;
            if (memcmp(&s0[(size_t)g * 256], &s1[(size_t)g * 256], 256) || o0[g].d != o1[g].d || o0[g].xy != o1[g].xy)
                ++bad_pipe;
            if (memcmp(&s0[(size_t)g * 256], &s2[(size_t)g * 256], 256) || o0[g].d != o2[g].d || o0[g].xy != o2[g].xy)
                ++bad_mskor;
            if (memcmp(&s0[(size_t)g * 256], &s3[(size_t)g * 256], 256) || o0[g].d != o3[g].d || o0[g].xy != o3[g].xy)
                ++bad_half;
        }
        if (getenv("PIPE_DEBUG")) {
            for (int g = 0; g < 3; ++g) {
                uint32_t d, xy;
                cpu_ref((uint32_t)(g % 256), steps, S.data(), d, xy);
                int fs0 = -1, fs1 = -1, fs4 = -1;
                for (int k = 0; k < 256; ++k) {
                    if (fs0 < 0 && s0[(size_t)g * 256 + k] != S[k]) fs0 = k;
                    if (fs1 < 0 && s1[(size_t)g * 256 + k] != S[k]) fs1 = k;
                    if (fs4 < 0 && s4[(size_t)g * 256 + k] != S[k]) fs4 = k;
                }
                printf("\n  lane %d cpu d %08x xy %04x | classic d %08x xy %04x firstbadS %d | pipe d %08x xy %04x firstbadS %d"
                       " | quad d %08x xy %04x firstbadS %d", g, d, xy,
                       o0[g].d, o0[g].xy, fs0, o1[g].d, o1[g].xy, fs1, o4[g].d, o4[g].xy, fs4);
            }
        }
        printf(", \"%s\": {\"classic_cyc_per_byte\": %.1f, \"pipelined_cyc_per_byte\": %.1f, \"classic_vs_cpu_bad\": %ld, "
               "\"pipelined_vs_classic_bad\": %ld, \"mskor_cyc_per_byte\": %.1f, \"mskor_vs_classic_bad\": %ld, "
               "\"half_lanes_2x_waves_cyc_per_byte\": %.1f, \"half_vs_classic_bad\": %ld, "
               "\"quad_exact_cyc_per_byte\": %.1f, \"quad_exact_vs_classic_bad\": %ld, \"quad_exact_vs_cpu_bad\": %ld, "
               "\"quad_skeleton_cyc_per_byte\": %.1f, \"quad_skeleton_read_ahead_cyc_per_byte\": %.1f}",
               c.name, med[0], med[1], bad_cpu, bad_pipe, med[2], bad_mskor, med[3], bad_half,
               med[4], bad_quad, bad_quad_cpu, med[5], med[6]);
        CHECK(hipFree(ds)); CHECK(hipFree(dout));
    }
    printf("}\n");
    return 0;
}
