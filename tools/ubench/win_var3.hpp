// Variant S of the product window loop (zrc4::win_windows): three byte
// masks folded into SDWA byte writes (J, d and x + 1), with one op between
// each SDWA byte write and its first reader (the gfx950 forwarding hazard,
// DESIGN.md §3.8): 3 instructions less per window.  Sae / Sbe: two of the
// three (J and x + 1; d and x + 1).
#pragma once
#include "../../zsummerx_amd/csrc/zrc4_win.hpp"
namespace zrc4 {
__device__ __forceinline__ void win_windows_S(WinLane &w, uint32_t rem, uint32_t l, uint32_t sb, uint32_t mb,
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
        "v_add_u32_sdwa v112, v112, v120 dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0\n\t"   // J = scan + y' (mod 256)
        // 2. b / marker round trip, d rule and rem cap under it
        "v_and_b32 %[y], 0xff, v120\n\t"                      // (one op between the SDWA byte write and its readers)
        "v_add_u32 v114, %[sb], v112\n\t"
        "v_lshl_add_u32 v115, v112, 2, %[mb]\n\t"
        "ds_read_u8 v116, v114\n\t"                             // b_l = S0[J]
        "ds_max_u32 v115, %[v]\n\t"
        "ds_read_b32 v117, v115\n\t"                            // lowest lane with this J
        "s_mov_b64 s[40:41], exec\n\t"
        "s_mov_b64 exec, s[46:47]\n\t"
        "ds_write_b8 v125, v124\n\t"                            // window n-1's ring store, behind the round trip
        "s_mov_b64 exec, s[40:41]\n\t"
        "v_sub_u32_sdwa v118, v112, %[xa] dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:DWORD\n\t"   // d
        "v_or_b32 v130, %[l1], v112\n\t"                        // y' candidate of this lane (between)
        "v_med3_u32 v119, v118, %[l], 16\n\t"
        "v_cmp_ne_u32 vcc, v118, %[l]\n\t"
        "v_cndmask_b32 v119, 16, v119, vcc\n\t"
        "v_lshlrev_b32 v118, v119, 1\n\t"                       // bit 16 = no d conflict
        "v_min_u32 v119, 16, %[rem]\n\t"
        "v_lshlrev_b32 v119, v119, 1\n\t"
        "v_or_b32 v118, v118, v119\n\t"                        // + bit min(rem, 16): cut <= rem
        "v_or_b32 v119, v118, %[bitl]\n\t"                     // the same if this lane's J repeats
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
        "v_add_u32_sdwa %[xa], %[xa], v118 dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:DWORD\n\t"
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

__device__ __forceinline__ void win_windows_Sae(WinLane &w, uint32_t rem, uint32_t l, uint32_t sb, uint32_t mb,
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
        "v_add_u32_sdwa v112, v112, v120 dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0\n\t"
        // 2. b / marker round trip, d rule and rem cap under it
        "v_and_b32 %[y], 0xff, v120\n\t"
        "v_add_u32 v114, %[sb], v112\n\t"
        "v_lshl_add_u32 v115, v112, 2, %[mb]\n\t"
        "ds_read_u8 v116, v114\n\t"                             // b_l = S0[J]
        "ds_max_u32 v115, %[v]\n\t"
        "ds_read_b32 v117, v115\n\t"                            // lowest lane with this J
        "s_mov_b64 s[40:41], exec\n\t"
        "s_mov_b64 exec, s[46:47]\n\t"
        "ds_write_b8 v125, v124\n\t"                            // window n-1's ring store, behind the round trip
        "s_mov_b64 exec, s[40:41]\n\t"
        "v_sub_u32 v118, v112, %[xa]\n\t"
        "v_and_b32 v118, 0xff, v118\n\t"                       // d
        "v_med3_u32 v119, v118, %[l], 16\n\t"
        "v_cmp_ne_u32 vcc, v118, %[l]\n\t"
        "v_cndmask_b32 v119, 16, v119, vcc\n\t"
        "v_lshlrev_b32 v118, v119, 1\n\t"                       // bit 16 = no d conflict
        "v_min_u32 v119, 16, %[rem]\n\t"
        "v_lshlrev_b32 v119, v119, 1\n\t"
        "v_or_b32 v118, v118, v119\n\t"                        // + bit min(rem, 16): cut <= rem
        "v_or_b32 v119, v118, %[bitl]\n\t"                     // the same if this lane's J repeats
        "v_or_b32 v130, %[l1], v112\n\t"                        // y' candidate of this lane
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
        "v_add_u32_sdwa %[xa], %[xa], v118 dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:DWORD\n\t"
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

__device__ __forceinline__ void win_windows_Sbe(WinLane &w, uint32_t rem, uint32_t l, uint32_t sb, uint32_t mb,
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
        "v_add_u32 v112, v112, v120\n\t"                       // + y' (byte 0 of v120; J is masked below)
        // 2. b / marker round trip, d rule and rem cap under it
        "v_add_u32_sdwa v114, %[sb], v112 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0\n\t"
        "v_and_b32 v112, 0xff, v112\n\t"                       // J
        "v_lshl_add_u32 v115, v112, 2, %[mb]\n\t"
        "ds_read_u8 v116, v114\n\t"                             // b_l = S0[J]
        "ds_max_u32 v115, %[v]\n\t"
        "ds_read_b32 v117, v115\n\t"                            // lowest lane with this J
        "s_mov_b64 s[40:41], exec\n\t"
        "s_mov_b64 exec, s[46:47]\n\t"
        "ds_write_b8 v125, v124\n\t"                            // window n-1's ring store, behind the round trip
        "s_mov_b64 exec, s[40:41]\n\t"
        "v_and_b32 %[y], 0xff, v120\n\t"
        "v_sub_u32_sdwa v118, v112, %[xa] dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:DWORD\n\t"
        "v_or_b32 v130, %[l1], v112\n\t"
        "v_med3_u32 v119, v118, %[l], 16\n\t"
        "v_cmp_ne_u32 vcc, v118, %[l]\n\t"
        "v_cndmask_b32 v119, 16, v119, vcc\n\t"
        "v_lshlrev_b32 v118, v119, 1\n\t"                       // bit 16 = no d conflict
        "v_min_u32 v119, 16, %[rem]\n\t"
        "v_lshlrev_b32 v119, v119, 1\n\t"
        "v_or_b32 v118, v118, v119\n\t"                        // + bit min(rem, 16): cut <= rem
        "v_or_b32 v119, v118, %[bitl]\n\t"                     // the same if this lane's J repeats
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
        "v_add_u32_sdwa %[xa], %[xa], v118 dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:DWORD\n\t"
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

}  // namespace zrc4
