#!/usr/bin/env python3
"""Generate zsummerx_amd/csrc/zrc4_line_loop.inc: the throughput-regime message
loop of crypt_kernel as gfx950 asm text (see zrc4_kernels.hpp,
crypt_message_dpp, for the C++ side and the register contract).

One iteration ("half") handles one 128-byte line per lane (blocks b, b+1 of
the lane's own session):
  1. wait for the line's loads (counted vmcnt: every VMEM op of the loop is
     issued with the full exec mask, so the counts are static; the first
     half is entered past this wait, at LL_PSTART: its line is retired by the
     caller and the second line is still in flight);
  2. RC4 keystream XOR over the two 64-byte blocks (ZL_BLOCK, exec = lanes
     whose session has that block);
  3. 8x8 transpose of 16-byte chunks inside each group of 8 consecutive lanes
     with v_cndmask_b32_dpp butterflies (XOR 1 / 2 via quad_perm, XOR 4 via
     row_shr/row_shl:4) -- afterwards lane 8g+i holds chunk i of the lines of
     sessions 8g .. 8g+7, so each store instruction writes 8 whole 128-byte
     lines (8 lanes per line);
  4. 8 stores (address per lane = line chunk, or the sink for chunks past
     their session's last block -- ragged batches);
  5. loads of the line two iterations ahead (blocks b+4, b+5) into the freed registers
     (clamped to the sink when the session has no such block).
Two halves (register sets P and Q) ping-pong; X is the transpose spare set.

Stores are nt (the streamed lines stop competing for L2 with the S-box
images: cfg5 306.6 -> 291.6 us, r01); loads use the default policy.  The
whole-line-load variant (a second transpose) was 4 % slower and is only in
git revision 849e847.

The script also simulates the butterflies lane by lane with the DPP
semantics used (quad_perm, row_shr:4, row_shl:4, bound_ctrl -> 0) and
asserts that the result is the transpose.

  python tools/gen_line_loop.py          # rewrites the .inc
"""
from __future__ import annotations

import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
OUT = ROOT / "zsummerx_amd" / "csrc" / "zrc4_line_loop.inc"
OUT_AB = ROOT / "zsummerx_amd" / "csrc" / "ab" / "zrc4_line_loop_ab.inc"

P_BASE, Q_BASE, X_BASE = 40, 72, 104      # 8 + 8 + 4 tuples of 4 VGPRs
ADDR_BASE = 120                            # 8 x 64-bit store addresses (chunk i of session 8g+q)
LIM_BASE = 136                             # 8 x u32 store limits
LA, LB, SA0, SA1, SINK = 144, 146, 148, 150, 152   # 64-bit load / store address temps, sink

CLEAR = {1: 0x55555555, 2: 0x33333333, 4: 0x0F0F0F0F}
CTRL_A = {1: "quad_perm:[1,0,3,2]", 2: "quad_perm:[2,3,0,1]", 4: "row_shr:4"}   # bit-set lanes read lane-m
CTRL_B = {1: "quad_perm:[1,0,3,2]", 2: "quad_perm:[2,3,0,1]", 4: "row_shl:4"}   # bit-clear lanes read lane+m
DPP_TAIL = "row_mask:0xf bank_mask:0xf bound_ctrl:1"


def transpose_plan(start, free):
    """Emit the 3 butterfly stages over chunk tuples start[c] (c = 0..7) with
    the spare tuples `free`; return (lines, final chunk -> tuple map, ops,
    tuples left free)."""
    reg = dict(start)
    free = list(free)
    lines, ops = [], []
    for m in (1, 2, 4):
        pairs = [(c, c | m) for c in range(8) if not c & m]
        lines += [f"s_mov_b32 vcc_lo, 0x{CLEAR[m]:08x}", f"s_mov_b32 vcc_hi, 0x{CLEAR[m]:08x}", "s_nop 1"]
        new = {}
        for ca, cb in pairs:
            t = free.pop(0)
            new[ca] = t
            for d in range(4):
                lines.append(f"v_cndmask_b32_dpp v{t + d}, v{reg[cb] + d}, v{reg[ca] + d}, vcc {CTRL_A[m]} {DPP_TAIL}")
            ops.append(("a", m, t, reg[cb], reg[ca]))
        inv = 0xFFFFFFFF ^ CLEAR[m]
        lines += [f"s_mov_b32 vcc_lo, 0x{inv:08x}", f"s_mov_b32 vcc_hi, 0x{inv:08x}", "s_nop 1"]
        for ca, cb in pairs:
            for d in range(4):
                lines.append(f"v_cndmask_b32_dpp v{reg[cb] + d}, v{reg[ca] + d}, v{reg[cb] + d}, vcc {CTRL_B[m]} {DPP_TAIL}")
            ops.append(("b", m, reg[cb], reg[ca], reg[cb]))
        for ca, _ in pairs:
            free.append(reg[ca])
            reg[ca] = new[ca]
        lines.append("s_nop 1")
    return lines, reg, ops, free


def simulate(ops, start, final):
    """Lane-level model of the emitted ops (tuple granularity, one value per
    (lane, chunk)): checks that lane 8g+i ends with chunk i of lane 8g+c in
    chunk slot c."""
    regs = {}
    for lane in range(64):
        for c in range(8):
            regs[(start[c], lane)] = (lane, c)

    def src(ctrl, lane):
        if ctrl.startswith("quad_perm"):
            perm = [int(v) for v in ctrl[ctrl.index("[") + 1:-1].split(",")]
            return (lane & ~3) + perm[lane & 3]
        n = int(ctrl.split(":")[1])
        s = lane - n if ctrl.startswith("row_shr") else lane + n
        return s if (s >> 4) == (lane >> 4) else None     # outside the row: bound_ctrl -> 0

    for kind, m, dst, s0, s1 in ops:
        ctrl = CTRL_A[m] if kind == "a" else CTRL_B[m]
        clear = CLEAR[m]
        vcc = [((clear if kind == "a" else ~clear) >> (lane & 31)) & 1 for lane in range(64)]
        out = {}
        for lane in range(64):
            if vcc[lane]:
                out[lane] = regs[(s1, lane)]
            else:
                sl = src(ctrl, lane)
                out[lane] = regs[(s0, sl)] if sl is not None else None
        for lane in range(64):
            regs[(dst, lane)] = out[lane]
    for lane in range(64):
        g, i = lane >> 3, lane & 7
        for c in range(8):
            got = regs[(final[c], lane)]
            assert got == (8 * g + c, i), (lane, c, got)


def zl_block(base: int) -> str:
    return "ZL_BLOCK(" + ", ".join(f"v{base + d}" for d in range(16)) + ")"


def half(name: str, cur: int, ab: int = 0, last: bool = False) -> str:
    """ab (timing-only A/B builds, zrc4_line_loop_ab.inc; outputs are wrong):
    1 stores to the lane's sink slot (one 64 KiB sink for the whole chip:
    contended), 2 loads from it, 3 no transpose, 4 both sinks.  (r02's 5 / 6,
    a sink load in place of each store, were removed in r03: those loads
    landed in the store-address temporaries v144-v151 asynchronously, and
    crypt_last_half_next_asm ends on vmcnt(8), so they could still be in
    flight when the compiler reused those registers -- a cfg5 A/B run with
    them faulted the GPU.)"""
    start = {c: cur + 4 * c for c in range(8)}
    tl, final, ops, _ = transpose_plan(start, [X_BASE + 4 * t for t in range(4)])
    simulate(ops, start, final)
    q = lambda s: f'"{s}\\n\\t"'
    out = []
    w = out.append
    # 1-2. keystream over blocks b and b+1 (line loaded two halves ago)
    # Younger VMEM ops than this line's first block: its second block (4),
    # the previous half's stores (8) and loads (8) -> vmcnt(20).  Halves whose
    # line-after-next does not exist issue no loads, so the LAST half has
    # only 12 younger ops: it waits vmcnt(8) (both blocks) instead.
    # last (crypt_last_half_next_asm): the message's last half.  Its
    # previous half never loads (no line after this one), so the wait is
    # vmcnt(8) unconditionally -- the count the branch below always picks
    # there -- and section 5 (loads of a line after this one) is absent, so
    # every load this statement leaves is one the statement itself waits for
    # (checkable without the relation between sb and wmax,
    # tools/vmem_hazard_check.py).
    if last:
        w(q("s_waitcnt vmcnt(8)"))
    else:
        w(q("s_add_u32 %[s1], %[sb], 2"))
        w(q("s_cmp_ge_u32 %[s1], %[wmax]"))
        w(q(f"s_cbranch_scc0 LL_{name}W_%="))
        w(q("s_waitcnt vmcnt(8)"))
        w(q(f"LL_{name}W_%=:"))
        w(q("s_waitcnt vmcnt(20)"))
    if name == "P":
        # entry of the first half: line 0 (P) was retired by the caller and
        # line 1 (Q) may still be in flight (issued after the S-box fill)
        w(q("LL_PSTART_%=:"))
    w(q("v_cmp_lt_u32_e64 %[msk], %[sb], %[nblk]"))
    w(q("s_and_b64 exec, %[full], %[msk]"))
    w(q(f"s_cbranch_execz LL_{name}1_%="))
    w(zl_block(cur))
    w(q(f"LL_{name}1_%=:"))
    w(q("s_waitcnt vmcnt(16)"))
    w(q("s_add_u32 %[s1], %[sb], 1"))
    w(q("v_cmp_lt_u32_e64 %[msk], %[s1], %[nblk]"))
    w(q("s_and_b64 exec, %[full], %[msk]"))
    w(q(f"s_cbranch_execz LL_{name}2_%="))
    w(zl_block(cur + 16))
    w(q(f"LL_{name}2_%=:"))
    w(q("s_mov_b64 exec, %[full]"))
    w(q("s_nop 4"))                                    # exec write -> DPP
    # 3. transpose
    if ab != 3:
        for line in tl:
            w(q(line))
    else:
        final = dict(start)
    # 4. stores: chunk i of session 8g+q's line, or the sink past its last block
    for qq in range(8):
        sa = SA0 if qq % 2 == 0 else SA1
        a = ADDR_BASE + 2 * qq
        w(q(f"v_cmp_gt_u32_e64 %[msk], v{LIM_BASE + qq}, %[sb]"))
        w(q(f"v_cndmask_b32_e64 v{sa}, v{SINK}, v{a}, %[msk]"))
        w(q(f"v_cndmask_b32_e64 v{sa + 1}, v{SINK + 1}, v{a + 1}, %[msk]"))
        if ab in (1, 4):
            sa = SINK
        if ab == 5:
            # the round-2 "sink load in place of each store" ablation that
            # faulted the GPU in round 3: the load lands in the store-address
            # temporaries asynchronously (--hazard-demo only: never built into
            # a library that runs; tests/test_vmem_hazards.py checks that
            # tools/vmem_hazard_check.py flags it)
            w(f'"global_load_dwordx2 v[{sa}:{sa + 1}], v[{SINK}:{SINK + 1}], off\\n\\t"')
            continue
        w(f'"global_store_dwordx4 v[{sa}:{sa + 1}], v[{final[qq]}:{final[qq] + 3}], off nt\\n\\t"')
    for qq in range(8):
        a = ADDR_BASE + 2 * qq
        w(q(f"v_lshl_add_u64 v[{a}:{a + 1}], 8, 4, v[{a}:{a + 1}]"))     # += 8 << 4 (shift must be 0..4)
    if last:
        return f"#define ZRC4_LL_HALF_{name}F \\\n    " + " \\\n    ".join(out) + "\n"
    # 5. loads of the line two halves ahead (blocks b+4, b+5) into this set;
    #    palo:pahi = own payload + 64 * (b + 4) on entry
    w(q("s_add_u32 %[s1], %[sb], 4"))
    w(q("s_cmp_ge_u32 %[s1], %[wmax]"))
    w(q(f"s_cbranch_scc1 LL_{name}L_%="))             # no line b+4 in this wave: no loads
    w(q("v_cmp_lt_u32_e64 %[msk], %[s1], %[nblk]"))
    w(q(f"v_cndmask_b32_e64 v{LA}, v{SINK}, %[palo], %[msk]"))
    w(q(f"v_cndmask_b32_e64 v{LA + 1}, v{SINK + 1}, %[pahi], %[msk]"))
    la = SINK if ab in (2, 4) else LA
    lb = SINK if ab in (2, 4) else LB
    for d in range(4):
        w(f'"global_load_dwordx4 v[{cur + 4 * d}:{cur + 4 * d + 3}], v[{la}:{la + 1}], off offset:{16 * d}\\n\\t"')
    w(q("s_add_u32 %[s1], %[sb], 5"))
    w(q("v_cmp_lt_u32_e64 %[msk], %[s1], %[nblk]"))
    w(q(f"v_cndmask_b32_e64 v{LB}, v{SINK}, %[palo], %[msk]"))
    w(q(f"v_cndmask_b32_e64 v{LB + 1}, v{SINK + 1}, %[pahi], %[msk]"))
    for d in range(4):
        w(f'"global_load_dwordx4 v[{cur + 16 + 4 * d}:{cur + 16 + 4 * d + 3}], v[{lb}:{lb + 1}], off offset:{64 + 16 * d}\\n\\t"')
    w(q("v_add_co_u32_e32 %[palo], vcc, 0x80, %[palo]"))
    w(q("v_addc_co_u32_e32 %[pahi], vcc, 0, %[pahi], vcc"))
    w(q(f"LL_{name}L_%=:"))
    w(q("s_add_u32 %[sb], %[sb], 2"))
    w(q("s_cmp_ge_u32 %[sb], %[wend]"))               # wend = wmax, or 2 less: stop before the last half
    w(q("s_cbranch_scc1 LL_DONE_%="))
    return f"#define ZRC4_LL_HALF_{name} \\\n    " + " \\\n    ".join(out) + "\n"


def transpose_only(name: str, cur: int) -> str:
    """The butterflies alone + the final chunk -> tuple map, for
    tools/ubench/dpp_transpose_check.hip."""
    tl, final, _, _ = transpose_plan({c: cur + 4 * c for c in range(8)}, [X_BASE + 4 * t for t in range(4)])
    body = " \\\n    ".join(f'"{line}\\n\\t"' for line in tl)
    fin = ", ".join(str(final[c]) for c in range(8))
    return (f"#define ZRC4_LL_TRANSPOSE_{name} \\\n    {body}\n"
            f"#define ZRC4_LL_FINAL_{name} {fin}\n")


def main(ab_only: bool = False):
    if ab_only:
        write_ab()
        return
    text = [
        "// GENERATED by tools/gen_line_loop.py -- do not edit by hand.\n",
        "// Throughput-regime message loop of crypt_kernel (zrc4_kernels.hpp,\n",
        "// crypt_message_dpp): keystream XOR, 8x8 DPP transpose of 16-byte chunks\n",
        "// per 8-lane group, whole-line stores, loads two lines ahead.\n",
        f"// Pinned VGPRs: P v[{P_BASE}:{P_BASE + 31}], Q v[{Q_BASE}:{Q_BASE + 31}], X v[{X_BASE}:{X_BASE + 15}],\n",
        f"// store addresses v[{ADDR_BASE}:{ADDR_BASE + 15}], limits v[{LIM_BASE}:{LIM_BASE + 7}],\n",
        f"// temps v[{LA}:{SA1 + 1}], sink v[{SINK}:{SINK + 1}].\n",
        "#pragma once\n",
        half("P", P_BASE),
        half("Q", Q_BASE),
        half("Q", Q_BASE, last=True),
        transpose_only("P", P_BASE),
    ]
    OUT.write_text("".join(text))
    print("wrote", OUT)


def write_hazard_demo(out_dir: Path) -> Path:
    """The removed round-2 ablation 5 as THE line loop, into a scratch dir
    (tests/test_vmem_hazards.py builds it next to copies of the kernels and
    expects tools/vmem_hazard_check.py to flag it).  Never run on a GPU."""
    out_dir.mkdir(parents=True, exist_ok=True)
    text = ["// GENERATED by tools/gen_line_loop.py --hazard-demo: BROKEN on purpose (never run it).\n",
            "#pragma once\n", half("P", P_BASE, 5), half("Q", Q_BASE, 5), half("Q", Q_BASE, 5, last=True),
            transpose_only("P", P_BASE)]
    out = out_dir / "zrc4_line_loop.inc"
    out.write_text("".join(text))
    return out


def write_ab():
    """The timing-only variants are generated on demand (build_variant runs
    this for ZRC4_LL_AB builds) and kept out of the tree."""
    ab = ["// GENERATED by tools/gen_line_loop.py -- do not edit by hand.\n",
          "// Timing-only A/B variants of zrc4_line_loop.inc (outputs are WRONG), selected by\n",
          "// ZRC4_LL_AB: 1 stores to the sink, 2 loads from the sink, 3 no transpose, 4 both sinks.\n",
          "#pragma once\n"]
    for v in (1, 2, 3, 4):
        ab += [f"#if ZRC4_LL_AB == {v}\n", half("P", P_BASE, v), half("Q", Q_BASE, v), "#endif\n"]
    OUT_AB.parent.mkdir(exist_ok=True)
    OUT_AB.write_text("".join(ab))
    print("wrote", OUT_AB)


if __name__ == "__main__":
    if "--hazard-demo" in sys.argv[1:]:
        print("wrote", write_hazard_demo(Path(sys.argv[sys.argv.index("--hazard-demo") + 1])))
    else:
        main(ab_only="--ab" in sys.argv[1:])
