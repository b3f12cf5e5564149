// win64_loop.hpp -- A/B only (tools/ubench/win_ubench.hip mode 7): speculative
// RC4 windows with ONE stream per wave (W = 64), not used by the library.
// Measured on MI355X: bit-exact, 11.49 bytes per window
// against 10.14 at W = 16, but ~470 cycles per window against ~420, so the
// per-stream rate equals the product loop's (zrc4::win_windows) and it was not
// kept.
#pragma once
#include "../../zsummerx_amd/csrc/zrc4_win.hpp"

namespace zrc4 {

// One stream per wave, W = 64 (launches of at most kWin64MaxGroups groups, one
// wave per SIMD at most).  The same rules over 64 lanes (11.45 bytes commit per
// window against 10.58 at W = 16, tools/window_sim.py), and with one stream
// per wave every rule becomes a per-lane "cut <= my lane" flag, so the cut is
// scalar work on a 64-bit ballot instead of a DPP OR chain:
//   d_l < l (j_l is an earlier step's i)                   -> v_cmp
//   j_k == j_l, k < l (duplicate j)                        -> M[j_l] >  v_l
//   j_k == i_l, k < l (an earlier step swaps my i: the
//   "l < d_k < W -> cut <= d_k" rule seen from lane d_k)   -> M[i_l] >  v_l
//   l >= rem                                               -> v_cmp
// commit mask = (P - 1) & ~P (lanes below the first flagged one), cut =
// popcount; x, y (readlane of the last committed j), rem and the ring position
// are SGPRs.  The scan of a runs over the whole wave (row_shr 1, 2, 4, 8, then
// row_bcast 15 and 31).  Lane 0 is never flagged while rem > 0, so cut >= 1.
// `xa` = x + 1, `rp` = stream position; the asm needs rem > 0.
// gfx950 forwards an SDWA result with dst_sel BYTE_0 to the NEXT VALU op
// before the byte select (measured: the unmasked sum reached the marker
// address), so every such result is read at least one op later.
#ifdef ZW64_DEBUG_CAP
#define ZW64_DBG_OUT , [d0] "=&v"(dbg[0]), [d1] "=&v"(dbg[1]), [d2] "=&v"(dbg[2]), [d3] "=&v"(dbg[3])
#define ZW64_DBG_ASM "v_mov_b32 %[d0], v112\n\tv_mov_b32 %[d1], v117\n\tv_mov_b32 %[d2], v115\n\tv_mov_b32 %[d3], v118\n\t"
#define ZW64_DBG_PARAM , uint32_t *dbg
#else
#define ZW64_DBG_OUT
#define ZW64_DBG_ASM
#define ZW64_DBG_PARAM
#endif
__device__ __forceinline__ void win64_windows(uint32_t &xa, uint32_t &y, uint32_t &v, uint32_t rem, uint32_t &rp,
                                              uint32_t l, uint32_t sb, uint32_t mb, uint32_t rbv ZW64_DBG_PARAM)
{
    asm volatile(
        "s_mov_b64 s[46:47], 0\n\t"                             // no window n-1 yet: empty commit mask
        "s_mov_b64 s[44:45], 0\n\t"
#ifdef ZW64_DEBUG_CAP
        "s_mov_b32 s53, " ZW64_DEBUG_CAP "\n\t"
#endif
        "v_mov_b32 v123, 0\n\t"
        "v_mov_b32 v106, %[sb]\n\t"                             // S base (256-aligned) in bytes 1-3
        "v_mov_b32 v114, %[sb]\n\t"
        "v_mov_b32 v126, %[sb]\n\t"
        "v_mov_b32 v131, %[sb]\n\t"
        "v_add_u32_sdwa v106, %[xa], %[l] dst_sel:BYTE_0 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n\t"
        "ds_read_u8 v107, v106\n\t"                             // a_l of window 0
        "ZW64_LOOP_%=:\n\t"
        // 1. tail of window n-1 (keystream select, ring store) in the wait
        //    slots of the scan of a over the wave (>= 2 VALU ops or an s_nop 1
        //    between a VALU write of v112 and its DPP read)
        "s_waitcnt lgkmcnt(0)\n\t"
        "v_mov_b32 v112, v107\n\t"
        "v_cmp_ge_u32_e64 s[42:43], v123, %[v]\n\t"             // M[t]: a committed lane <= l wrote t
        "v_and_b32 v113, 0xff, v106\n\t"                        // i_l
        "v_add_u32_dpp v112, v112, v112 row_shr:1 row_mask:0xf bank_mask:0xf\n\t"
        "s_or_b64 s[42:43], s[42:43], s[44:45]\n\t"             // or t is the i of a step <= l
        "v_add_u32 %[v], 0x100, %[v]\n\t"                       // window tag
        "v_cndmask_b32_e64 v124, v121, v122, s[42:43]\n\t"      // keystream byte of window n-1
        "v_add_u32_dpp v112, v112, v112 row_shr:2 row_mask:0xf bank_mask:0xf\n\t"
        "s_mov_b64 s[40:41], exec\n\t"
        "s_mov_b64 exec, s[46:47]\n\t"
        "ds_write_b8 v125, v124\n\t"
        "s_mov_b64 exec, s[40:41]\n\t"
        "v_lshl_add_u32 v113, v113, 2, %[mb]\n\t"               // &M[i_l]
        "s_nop 0\n\t"
        "v_add_u32_dpp v112, v112, v112 row_shr:4 row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_add_u32_dpp v112, v112, v112 row_shr:8 row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_add_u32_dpp v112, v112, v112 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_add_u32_dpp v112, v112, v112 row_bcast:31 row_mask:0xc bank_mask:0xf\n\t"
        // 2. b / marker round trip, d rule and the rem cap under it
        "v_add_u32_sdwa v114, %[y], v112 dst_sel:BYTE_0 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n\t"
        "ds_read_u8 v116, v114\n\t"                             // b_l = S0[J]
        "v_add_u32_sdwa v112, %[y], v112 dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:DWORD\n\t"   // J
        "v_cmp_le_u32_e64 s[50:51], %[rem], %[l]\n\t"           // (the SDWA byte result needs one op before a VALU reads it)
        "v_lshl_add_u32 v115, v112, 2, %[mb]\n\t"
        "ds_max_u32 v115, %[v]\n\t"
        "ds_read_b32 v117, v115\n\t"                            // lowest lane with this J
        "ds_read_b32 v113, v113\n\t"                            // lowest lane whose J is my i
        "v_subrev_u32_sdwa v118, %[xa], v112 dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:DWORD\n\t"   // d
        "s_nop 0\n\t"
        "v_cmp_lt_u32_e64 s[48:49], v118, %[l]\n\t"
        "s_or_b64 s[48:49], s[48:49], s[50:51]\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        // 3. S0[t] read, cut, commit, window n+1's a_l read
        "v_add_u32_sdwa v126, v107, v116 dst_sel:BYTE_0 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n\t"   // &S[t]
        "ds_read_u8 v121, v126\n\t"                             // S0[t]
        "v_max_u32 v117, v117, v113\n\t"
        "v_cmp_gt_u32_e64 s[50:51], v117, %[v]\n\t"
        "s_or_b64 s[48:49], s[48:49], s[50:51]\n\t"             // P: lanes that bound the cut
        "s_sub_u32 s46, s48, 1\n\t"
        "s_subb_u32 s47, s49, 0\n\t"
        "s_andn2_b64 s[46:47], s[46:47], s[48:49]\n\t"          // commit = lanes below P's lowest bit
        "s_bcnt1_i32_b64 s54, s[46:47]\n\t"                     // cut
        "s_mov_b32 s55, %[xa]\n\t"
        "s_add_u32 %[xa], %[xa], s54\n\t"
        "s_and_b32 %[xa], %[xa], 0xff\n\t"
        "v_add_u32_sdwa v131, %[xa], %[l] dst_sel:BYTE_0 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n\t"
        "s_mov_b64 s[40:41], exec\n\t"
        "s_mov_b64 exec, s[46:47]\n\t"
        "ds_write_b8 v106, v116\n\t"                            // S[i_l] = b_l
        "ds_write_b8 v114, v107\n\t"                            // S[J_l] = a_l
        "s_mov_b64 exec, s[40:41]\n\t"
        "ds_read_u8 v107, v131\n\t"                             // a_l of window n+1
        // 4. keystream bookkeeping of window n under that round trip (v107
        //    is in flight: t comes from &S[t])
        "v_and_b32 v128, 0xff, v126\n\t"                        // t
        "v_lshl_add_u32 v129, v128, 2, %[mb]\n\t"
        "ds_read_u8 v122, v126\n\t"                             // S_final[t]
        "ds_read_b32 v123, v129\n\t"                            // lowest lane whose J == t
        "v_subrev_u32_sdwa v130, s55, v128 dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:DWORD\n\t"   // e = t - x - 1
        "v_add_u32 v119, %[rp], %[l]\n\t"
        "v_cmp_le_u32_e64 s[44:45], v130, %[l]\n\t"             // t is the i of a step <= l
        "v_bfi_b32 v125, %[rmask], v119, %[rb]\n\t"             // ring slot of window n (stored next iteration)
        "s_add_u32 s55, s54, -1\n\t"
        "v_readlane_b32 %[y], v112, s55\n\t"                    // y' = J of the last committed lane
        "v_mov_b32 v106, v131\n\t"
        "s_sub_u32 %[rem], %[rem], s54\n\t"
        "s_add_u32 %[rp], %[rp], s54\n\t"
#ifdef ZW64_DEBUG_CAP
        "s_sub_u32 s53, s53, 1\n\t"
        "s_cmp_eq_u32 s53, 0\n\t"
        "s_cbranch_scc1 ZW64_OUT_%=\n\t"
#endif
        "s_cmp_lg_u32 %[rem], 0\n\t"
        "s_cbranch_scc1 ZW64_LOOP_%=\n\t"
        "ZW64_OUT_%=:\n\t"
        // drain: tail of the last window (window n+1's a_l read is harmless)
        "s_waitcnt lgkmcnt(0)\n\t"
        "v_cmp_ge_u32_e64 s[42:43], v123, %[v]\n\t"
        "s_or_b64 s[42:43], s[42:43], s[44:45]\n\t"
        "v_cndmask_b32_e64 v124, v121, v122, s[42:43]\n\t"
        "s_mov_b64 s[40:41], exec\n\t"
        "s_mov_b64 exec, s[46:47]\n\t"
        "ds_write_b8 v125, v124\n\t"
        "s_mov_b64 exec, s[40:41]\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        ZW64_DBG_ASM
        : [xa] "+s"(xa), [y] "+s"(y), [v] "+v"(v), [rem] "+s"(rem), [rp] "+s"(rp) ZW64_DBG_OUT
        : [l] "v"(l), [sb] "s"(sb), [mb] "s"(mb), [rb] "v"(rbv), [rmask] "s"(kWinRing - 1)
        : "memory", "scc", "v106", "v107", "v112", "v113", "v114", "v115", "v116", "v117", "v118", "v121", "v122",
          "v119", "v123", "v124", "v125", "v126", "v128", "v129", "v130", "v131", "s40", "s41", "s42", "s43", "s44", "s45", "s46",
          "s47", "s48", "s49", "s50", "s51", "s53", "s54", "s55");
}

}  // namespace zrc4
