#!/usr/bin/env python3
"""Static check of the asm-issued-load discipline in the shipped gfx950 code.

The hand-written kernels issue global loads from inline asm into registers
(pinned ranges such as v[40:71], v[148:151], v[160:223], and compiler-chosen
ones such as the prefetched entries) and retire them later with counted
`s_waitcnt vmcnt(N)` waits.  The compiler cannot see those loads, so nothing
but convention stops compiler code between two asm statements from reading or
overwriting such a register while its load is still in flight -- which is what
faulted the GPU in round 3 (timing-only sink loads into
v148/v150 were still in flight when ZRC4_NEXT_LINE0 rewrote v[148:149]).

This tool checks the property on the final machine code, for every kernel of
a library (`libzrc4.so` by default):

  1. the gfx950 code object is unbundled from the library's .hip_fatbin and
     disassembled with llvm-objdump;
  2. each kernel is split into basic blocks (branch targets, fall-throughs);
  3. a forward dataflow analysis tracks, for every load that may be in
     flight, its destination VGPRs and a lower bound on the VMEM operations
     issued after it (stores and non-returning atomics count too): gfx9
     VMEM operations retire in order, so `s_waitcnt vmcnt(N)` retires
     exactly those with at least N younger ones, and the counter saturates
     at 63; at control-flow joins pending loads are united and the bounds
     take the minimum, so no path's in-flight load is missed;
  4. branches on the kernels' uniform control flow are pruned when they
     cannot be taken: difference constraints between SGPRs (x - y in
     [lo, hi], closed transitively, every SGPR an unsigned value that does
     not wrap) through moves, constant adds and compares; the compiler's
     uniform booleans (s_cselect_b64 -1/0, their s_and / s_xor, 0/1 copies
     in VGPRs, VCC branches on them) and the selects made on them; block
     states are kept apart by pending loads and decided compares.  This
     is what proves the counted waits of the line loop (e.g. "the last
     half's previous half issued no loads"), not an assumption;
  5. any instruction other than a VMEM load that names (reads or writes) a
     VGPR whose load may still be in flight on some path is a HAZARD.  A new
     load into such a register is allowed (in-order returns: the younger
     value lands last).

Exit status 1 when a hazard is found.  tests/test_vmem_hazards.py runs it on
the product build and on a deliberately broken build (the removed round-2
"sink load in place of each store" line loop, regenerated into a scratch
directory by tools/gen_line_loop.py --hazard-demo), which must fail.

  python tools/vmem_hazard_check.py [lib.so] [--kernel SUBSTR] [--max-report N]
"""
from __future__ import annotations

import argparse
import functools
import re
import subprocess
import sys
import tempfile
from dataclasses import dataclass, field
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
LLVM = Path("/opt/rocm/llvm/bin")
VMCNT_MAX = 63

_REG = re.compile(r"\bv(\d+)\b|\bv\[(\d+):(\d+)\]")
_ADDR = re.compile(r"//\s*([0-9A-Fa-f]+):")
_FUNC = re.compile(r"^[0-9a-fA-F]+ <(\S+)>:$")


@dataclass
class Insn:
    addr: int
    mnem: str
    ops: str
    text: str
    target: int | None = None
    regs: frozenset = field(default_factory=frozenset)



def _unbundle(lib: Path, td: str) -> Path:
    fb, co = Path(td) / "fb.bin", Path(td) / "co.o"
    subprocess.run([str(LLVM / "llvm-objcopy"), f"--dump-section=.hip_fatbin={fb}", str(lib), str(Path(td) / "x")],
                   check=True, capture_output=True)
    subprocess.run([str(LLVM / "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={fb}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True, capture_output=True)
    return co


def disassemble(lib: Path) -> str:
    """The gfx950 code object of a HIP shared library, disassembled."""
    with tempfile.TemporaryDirectory() as td:
        co = _unbundle(lib, td)
        return subprocess.run([str(LLVM / "llvm-objdump"), "-d", "--mcpu=gfx950", str(co)], check=True,
                              capture_output=True, text=True).stdout


def kernel_resources(lib: Path) -> dict:
    """Per kernel: VGPRs, VGPR / SGPR spills, scratch and LDS bytes, from the code
    object's AMDGPU metadata note."""
    with tempfile.TemporaryDirectory() as td:
        co = _unbundle(lib, td)
        notes = subprocess.run([str(LLVM / "llvm-readelf"), "--notes", str(co)], check=True, capture_output=True,
                               text=True).stdout
    out, cur = {}, {}
    for line in notes.splitlines():
        m = re.match(r"\s*(?:- )?\.(agpr_count|name|vgpr_count|vgpr_spill_count|sgpr_spill_count|"
                     r"group_segment_fixed_size|private_segment_fixed_size):\s+(\S+)", line)
        if not m:
            continue
        k, v = m.groups()
        if k == "agpr_count":                       # first key of a kernel's block
            cur = {}
        cur[k] = v if k == "name" else int(v)
        if k == "name":
            out[v] = cur
    return out


def regs_of(ops: str) -> frozenset:
    out = set()
    for m in _REG.finditer(ops):
        if m.group(1) is not None:
            out.add(int(m.group(1)))
        else:
            out.update(range(int(m.group(2)), int(m.group(3)) + 1))
    return frozenset(out)


def parse(text: str) -> dict[str, list[Insn]]:
    """Kernels (mangled C++ symbols) and their instructions; asm labels inside
    a kernel (LL_LOOP_11, ...) are symbols too but stay part of it.  Branch
    targets come from the instruction encoding."""
    funcs: dict[str, list[Insn]] = {}
    sym_addr: dict[str, int] = {}
    cur = None
    for line in text.splitlines():
        m = _FUNC.match(line.strip())
        if m:
            addr = int(line.strip().split()[0], 16)
            sym_addr[m.group(1)] = addr
            if m.group(1).startswith("_Z"):
                cur = funcs.setdefault(m.group(1), [])
            continue
        if cur is None or not line.startswith("\t"):
            continue
        body, _, comment = line.strip().partition("//")
        am = _ADDR.search(line)
        if not am or not body.strip():
            continue
        parts = body.split(None, 1)
        mnem, ops = parts[0], (parts[1] if len(parts) > 1 else "")
        ins = Insn(int(am.group(1), 16), mnem, ops.strip(), body.strip(), regs=regs_of(ops))
        if mnem.startswith("s_branch") or mnem.startswith("s_cbranch"):
            # SOPP encoding: target = next instruction + 4 * simm16 (the
            # disassembler prints the operand as a number or a label name)
            enc = re.search(r"//\s*[0-9A-Fa-f]+:\s*([0-9A-Fa-f]{8})", line)
            simm = int(enc.group(1), 16) & 0xFFFF
            simm -= 0x10000 if simm & 0x8000 else 0
            ins.target = ins.addr + 4 + 4 * simm
        cur.append(ins)
    return funcs


def is_vmem(m: str) -> bool:
    return m.startswith(("global_", "buffer_", "scratch_", "flat_", "tbuffer_"))


def vmem_dest(ins: Insn) -> frozenset:
    """Destination VGPRs of a VMEM op (empty for stores, non-returning atomics,
    loads straight to LDS and cache maintenance)."""
    m = ins.mnem
    if "_lds" in m or m.startswith(("buffer_wbl2", "buffer_inv", "buffer_wbinvl1")):
        return frozenset()
    first = ins.ops.split(",")[0]
    if "_load" in m:
        return regs_of(first)
    if "_atomic" in m and re.search(r"\bsc0\b", ins.ops):
        return regs_of(first)
    return frozenset()


def vmcnt_of(ins: Insn):
    m = re.search(r"vmcnt\((\d+)\)", ins.ops)
    return int(m.group(1)) if m else None


_SREG = re.compile(r"^s(\d+)$|^s\[(\d+):(\d+)\]$")


def _sregs(op: str) -> set:
    m = _SREG.match(op.strip())
    if not m:
        return set()
    if m.group(1) is not None:
        return {int(m.group(1))}
    return set(range(int(m.group(2)), int(m.group(3)) + 1))


_NO_DEST = ("s_cmp", "s_bitcmp", "s_cbranch", "s_branch", "s_setpc", "s_waitcnt", "s_sleep", "s_setprio", "s_nop",
            "s_barrier", "s_endpgm", "s_setreg", "s_ttracedata", "s_sendmsg", "s_icache")


def sgpr_dest(ins: Insn) -> set:
    """SGPRs an instruction writes through its first operand."""
    if ins.mnem.startswith(_NO_DEST) or not ins.ops:
        return set()
    if not (ins.mnem.startswith("s_") or ins.mnem.startswith("v_")):
        return set()
    return _sregs(ins.ops.split(",")[0])


def exec_step(ins: Insn, full: bool, sg: dict):
    """EXEC tracking: is EXEC the whole wave after `ins`, and which SGPR
    operands hold the whole-wave mask (saved by s_mov / s_*_saveexec)."""
    m = ins.mnem
    ops = [o.strip() for o in ins.ops.split(",")] if ins.ops else []
    if not ops:
        return full, sg
    dst = ops[0]
    if dst == "exec":
        srcs = ops[1:]
        if m == "s_mov_b64":
            return (srcs[0] == "-1" or sg.get(srcs[0], False)), sg
        if m == "s_or_b64":
            return (full and "exec" in srcs) or any(x == "-1" or sg.get(x, False) for x in srcs), sg
        return False, sg
    if "saveexec" in m:
        clobber = _sregs(dst)
        sg = {k: v for k, v in sg.items() if not (_sregs(k) & clobber)}
        sg[dst] = full
        return (m.startswith("s_or_saveexec") and ops[1] == "-1"), sg
    if m.startswith("v_cmpx"):
        return False, sg
    clobber = sgpr_dest(ins)
    if clobber:
        sg = {k: v for k, v in sg.items() if not (_sregs(k) & clobber)}
        if m == "s_mov_b64" and len(ops) > 1:
            if ops[1] == "exec":
                sg[dst] = full
            elif ops[1] in sg:
                sg[dst] = sg[ops[1]]
    return full, sg


U32 = (1 << 32) - 1
M64 = (1 << 64) - 1


INF = float("inf")


def _term(op: str):
    """A scalar operand as (variable, constant): an SGPR is ("sN", 0), an
    inline or literal constant ("0", c).  None for anything else."""
    op = op.strip()
    try:
        return ("0", int(op, 0) & U32)
    except ValueError:
        pass
    return (op, 0) if re.match(r"^s\d+$", op) else None


def _upper(D: dict, x: str, y: str) -> float:
    """Least upper bound of x - y implied by the constraints (shortest path,
    Bellman-Ford: difference constraints plus "every SGPR >= 0", i.e.
    0 - v <= 0)."""
    if x == y:
        return 0
    return _upper_cached(frozenset(D.items()), x, y)


@functools.lru_cache(maxsize=1 << 16)
def _upper_cached(items: frozenset, x: str, y: str) -> float:
    D = dict(items)
    nodes = {"0", x, y}
    edges = []
    for (a, b), (lo, hi) in D.items():
        nodes.update((a, b))
        if hi < INF:
            edges.append((a, b, hi))        # a - b <= hi
        if lo > -INF:
            edges.append((b, a, -lo))       # b - a <= -lo
    edges += [("0", v, 0) for v in nodes if v != "0"]
    dist = {v: INF for v in nodes}
    dist[x] = 0
    for _ in range(len(nodes)):
        changed = False
        for a, b, w in edges:
            # path x -> .. -> a -> b bounds x - b: x - b = (x - a) + (a - b)
            if dist[a] + w < dist[b]:
                dist[b] = dist[a] + w
                changed = True
        if not changed:
            break
    return dist[y]


def dbm_bounds(D: dict, x: str, y: str):
    """Bounds of x - y: the tightest the difference constraints imply
    (transitively, with every SGPR >= 0 as an unsigned value that does not
    wrap); None when unbounded both ways."""
    if x == y:
        return (0, 0)
    hi = _upper(D, x, y)
    lo = -_upper(D, y, x)
    if (lo, hi) == (-INF, INF):
        return None
    return (lo, hi)


def _diff(D: dict, A, B):
    """Bounds of A - B for terms A, B."""
    bd = dbm_bounds(D, A[0], B[0])
    if bd is None:
        return None
    k = A[1] - B[1]
    return (bd[0] + k, bd[1] + k)


def _decide(op, d):
    """Does `A op B` hold for every / no value, given bounds d of A - B?"""
    if d is None or op.startswith("bit"):
        return None
    lo, hi = d
    return {"lt": True if hi < 0 else False if lo >= 0 else None,
            "le": True if hi <= 0 else False if lo > 0 else None,
            "gt": True if lo > 0 else False if hi <= 0 else None,
            "ge": True if lo >= 0 else False if hi < 0 else None,
            "eq": True if lo == hi == 0 else False if hi < 0 or lo > 0 else None,
            "lg": False if lo == hi == 0 else True if hi < 0 or lo > 0 else None}[op]


_NEG = {"lt": "ge", "le": "gt", "gt": "le", "ge": "lt", "eq": "lg", "lg": "eq", "bit0": "bit1", "bit1": "bit0",
        "opq": "nopq", "nopq": "opq"}
_SWAP = {"lt": "gt", "le": "ge", "gt": "lt", "ge": "le", "eq": "eq", "lg": "lg", "bit0": None, "bit1": None,
         "opq": None, "nopq": None}


def _consistent(D: dict, a: str) -> bool:
    """No negative cycle through `a` (Bellman-Ford from a)."""
    nodes = {"0", a}
    edges = []
    for (x, y), (lo, hi) in D.items():
        nodes.update((x, y))
        if hi < INF:
            edges.append((x, y, hi))
        if lo > -INF:
            edges.append((y, x, -lo))
    edges += [("0", v, 0) for v in nodes if v != "0"]
    dist = {v: INF for v in nodes}
    dist[a] = 0
    for _ in range(len(nodes) + 1):
        changed = False
        for x, y, w in edges:
            if dist[x] + w < dist[y]:
                dist[y] = dist[x] + w
                changed = True
        if dist[a] < 0:
            return False
        if not changed:
            return True
    return False


def _refine(D: dict, cond, holds: bool):
    """Add the compare `A op B` (or its negation) as a constraint on the
    difference of the two variables; None when that is infeasible."""
    op, xa, xb = cond
    A, B = _term(xa), _term(xb)
    if A is None or B is None or op.startswith("bit"):
        return D
    if not holds:
        op = _NEG[op]
    if A[0] == B[0]:
        return D if _decide(op, (A[1] - B[1],) * 2) is not False else None
    k = B[1] - A[1]                         # A op B  <=>  a - b op k
    lo, hi = {"lt": (-INF, k - 1), "le": (-INF, k), "gt": (k + 1, INF), "ge": (k, INF), "eq": (k, k),
              "lg": (-INF, INF)}[op]
    if (lo, hi) == (-INF, INF):
        return D
    key, sign = ((A[0], B[0]), 1) if (B[0], A[0]) not in D else ((B[0], A[0]), -1)
    if sign < 0:
        lo, hi = -hi, -lo
    olo, ohi = D.get(key, (-INF, INF))
    nlo, nhi = max(lo, olo), min(hi, ohi)
    if nlo > nhi:
        return None
    D = dict(D)
    D[key] = (nlo, nhi)
    return D if _consistent(D, key[0]) else None


def _assign(D: dict, d: str, src, k: int = 0):
    """d := src + k (src a variable, or "0" for a constant), or unknown
    (src None): constraints are renamed, not lost, when d is written from
    itself (the loop counters' s_add sN, sN, 2)."""
    if src == d:
        out = {}
        for (x, y), (lo, hi) in D.items():
            if x == d:
                out[(x, y)] = (lo + k, hi + k)
            elif y == d:
                out[(x, y)] = (lo - k, hi - k)
            else:
                out[(x, y)] = (lo, hi)
        return out
    # d dies: keep what it implied between the other variables (projection
    # of the difference constraints: x - d and d - y bound x - y)
    out = {key: v for key, v in D.items() if d not in key}
    rel = []                                       # (z, lo, hi) for d - z
    for (x, y), (lo, hi) in D.items():
        if x == d and y != d:
            rel.append((y, lo, hi))
        elif y == d and x != d:
            rel.append((x, -hi, -lo))
    for i, (z1, l1, h1) in enumerate(rel):
        for z2, l2, h2 in rel[i + 1:]:
            if z1 == z2:
                continue
            lo, hi = l2 - h1, h2 - l1              # z1 - z2 = (d - z2) - (d - z1)
            key, sg = ((z1, z2), 1) if (z2, z1) not in out else ((z2, z1), -1)
            if sg < 0:
                lo, hi = -hi, -lo
            olo, ohi = out.get(key, (-INF, INF))
            nlo, nhi = max(lo, olo), min(hi, ohi)
            if (nlo, nhi) != (-INF, INF) and nlo <= nhi:
                out[key] = (nlo, nhi)
    if src is None:
        return out
    if src == "0":
        out[(d, "0")] = (k, k)
        return out
    for (x, y), (lo, hi) in list(out.items()):
        if x == src and y != d:
            out[(d, y)] = (lo + k, hi + k)
        elif y == src and x != d:
            out[(x, d)] = (lo - k, hi - k)
    out[(d, src)] = (k, k)
    return out


def scalar_step(ins: Insn, D: dict, cond):
    """Difference constraints between SGPRs (and the constant 0) through the
    scalar code the kernels' uniform control flow uses: moves, adds and
    subtracts of constants (renaming constraints), bounds through shifts /
    ands / selects, compares; any other write to an SGPR forgets it.
    Values are treated as unbounded integers (loop counters and sizes stay
    far from the 32-bit wrap).  Returns (D, scc condition)."""
    m = ins.mnem
    ops = [o.strip() for o in ins.ops.split(",")] if ins.ops else []
    mm = re.match(r"^s_cmp_(\w+?)_[ui]32$", m)
    if mm and mm.group(1) in _NEG and len(ops) == 2:
        return D, (mm.group(1), ops[0], ops[1])
    mm = re.match(r"^s_bitcmp([01])_b32$", m)
    if mm and len(ops) == 2:
        return D, ("bit" + mm.group(1), ops[0], ops[1])
    if not ops:
        return D, cond
    clobber = sgpr_dest(ins)
    writes_scc = m.startswith("s_") and not m.startswith(("s_mov", "s_cselect", "s_cmov", "s_waitcnt", "s_nop",
                                                           "s_barrier", "s_setprio", "s_sleep", "s_branch",
                                                           "s_cbranch", "s_load", "s_buffer_load", "s_getreg",
                                                           "s_memtime", "s_memrealtime", "s_movk"))
    cond = None if writes_scc else cond
    if not clobber:
        return D, cond
    names = ["s%d" % r for r in sorted(clobber)]
    if len(names) != 1:
        for n in names:
            D = _assign(D, n, None)
        return D, cond
    d = names[0]
    A = _term(ops[1]) if len(ops) > 1 else None
    B = _term(ops[2]) if len(ops) > 2 else None
    if m in ("s_mov_b32", "s_movk_i32") and A:
        return _assign(D, d, A[0], A[1]), cond
    if m in ("s_add_u32", "s_add_i32") and A and B and (A[0] == "0" or B[0] == "0"):
        v, c = (B, A[1]) if A[0] == "0" else (A, B[1])
        return _assign(D, d, v[0], v[1] + c), cond
    if m in ("s_sub_u32", "s_sub_i32") and A and B and B[0] == "0":
        return _assign(D, d, A[0], A[1] - B[1]), cond
    # bounds only
    def rng(T):
        if T is None:
            return None
        b = dbm_bounds(D, T[0], "0")
        return None if b is None else (b[0] + T[1], b[1] + T[1])
    ra, rb = rng(A), rng(B)
    r = None
    if m in ("s_add_u32", "s_add_i32") and ra and rb:
        r = (ra[0] + rb[0], ra[1] + rb[1])
    elif m == "s_lshl_b32" and ra and rb and rb[0] == rb[1]:
        r = (ra[0] * 2 ** rb[0], ra[1] * 2 ** rb[0])
    elif m == "s_lshr_b32" and ra and rb and rb[0] == rb[1] and ra[0] >= 0:
        r = (ra[0] // 2 ** rb[0], ra[1] // 2 ** rb[0] if ra[1] != INF else INF)
    elif m == "s_and_b32" and (ra and ra[0] >= 0 or rb and rb[0] >= 0):
        r = (0, min(x[1] for x in (ra, rb) if x and x[0] >= 0))
    elif m == "s_cselect_b32" and ra and rb:
        r = (min(ra[0], rb[0]), max(ra[1], rb[1]))
    elif m in ("s_min_u32", "s_max_u32") and ra and rb:
        f = min if m == "s_min_u32" else max
        r = (f(ra[0], rb[0]), f(ra[1], rb[1]))
    D = _assign(D, d, None)
    if r and (r[0] > -INF or r[1] < INF):
        D[(d, "0")] = r
    return D, cond


def fact_status(bc: dict, op, x, y):
    """A compare already decided on this path: True / False / None."""
    if ("F", op, x, y) in bc or (_SWAP[op] and ("F", _SWAP[op], y, x) in bc):
        return True
    n = _NEG[op]
    if ("F", n, x, y) in bc or (_SWAP[n] and ("F", _SWAP[n], y, x) in bc):
        return False
    return None


def conj_status(bc: dict, lits) -> bool | None:
    """A conjunction of compares: True when all hold, False when one fails."""
    sts = [fact_status(bc, *l) for l in lits]
    if any(x is False for x in sts):
        return False
    return True if all(sts) else None


def _neg_sym(v):
    """Negation of a symbolic boolean (only a single compare negates into
    one); None when not representable."""
    if isinstance(v, int):
        return ~v
    if len(v[1]) == 1:
        (op, x, y), = v[1]
        return ("c", frozenset({(_NEG[op], x, y)}))
    return None


def _lit_regs(l) -> set:
    return set() if l[0] in ("opq", "nopq") else (_sregs(l[1]) | _sregs(l[2]))


def _stale(sym, regs: set):
    """A symbolic boolean whose compares read a register that is being
    overwritten keeps its identity (an opaque literal named after the
    compares) but can no longer be decided from new facts."""
    if not any(_lit_regs(l) & regs for l in sym[1]):
        return sym
    return ("c", frozenset({("opq", repr(sorted(sym[1])), "")}))


def _touches(k, regs: set) -> bool:
    if isinstance(k, tuple) and k[0] == "sel":   # ("sel", d): its operands are checked with the value
        return bool(_sregs(k[1]) & regs)
    if isinstance(k, tuple):                     # ("F", op, a, b)
        return bool(_lit_regs(k[1:]) & regs)
    return bool(_sregs(k) & regs)


def bool_step(ins: Insn, bc: dict, cond) -> dict:
    """Uniform booleans of the compiler's scalar control flow:
      * SGPR-pair values: constants (s_mov_b64 sX, -1 / 0, folded through
        s_xor / s_and / s_or) or a compare (s_cselect_b64 sX, -1, 0 after
        s_cmp: ("c", op, a, b));
      * facts ("F", op, a, b): compares decided on this path by a branch;
      * VCC: known zero / non-zero, or "vcc_src" = the pair sX a
        s_and(n2)_b64 vcc, exec, sX copied -- a VCC branch on it tells sX
        (the compiler lowers uniform conditions that way).
    Any write to an SGPR forgets what depends on it."""
    m = ins.mnem
    ops = [o.strip() for o in ins.ops.split(",")] if ins.ops else []
    if not ops:
        return bc
    dst = ops[0]
    writes_vcc = (dst == "vcc" and not m.startswith(_NO_DEST)) or \
        (m.startswith("v_") and ("_e32" in m and ("v_cmp" in m or "_co_" in m or "addc" in m or "subb" in m)))
    clobber = sgpr_dest(ins)
    before = bc                                   # sources are read before the write
    vdst = regs_of(dst) if (m.startswith("v_") or "_load" in m or m.startswith("ds_read")) and not \
        m.startswith("v_cmp") else frozenset()
    if vdst:
        bc = {k: v for k, v in bc.items() if not (isinstance(k, str) and re.match(r"^v\d+$", k)
                                                  and int(k[1:]) in vdst)}
        # a 0/1 lane value from a uniform boolean: v_cndmask_b32_e64 vD, 0, 1, sX
        if m == "v_cndmask_b32_e64" and len(ops) == 4 and {ops[1], ops[2]} == {"0", "1"} and len(vdst) == 1:
            src = bc.get(ops[3])
            if src is not None and ops[1] == "1":   # 1 where sX is clear
                src = _neg_sym(src)
            if src is not None:
                bc["v%d" % next(iter(vdst))] = src
        if not clobber and not writes_vcc:
            return bc
    if not clobber and not writes_vcc:
        return bc
    out = {}
    for k, v in bc.items():
        if k == "vcc":
            if writes_vcc:
                continue
        elif k == "vcc_src":
            if writes_vcc or _sregs(v[0]) & clobber:
                continue
        elif k == "vcc_sym":
            if writes_vcc:
                continue
            v = _stale(v, clobber)
        elif isinstance(k, tuple) and k[0] == "sel":
            if _touches(k, clobber):
                continue
            v = (_stale(v[0], clobber),) + tuple(v[1:])
            # an overwritten operand no longer names the selected value
            v = (v[0], None if v[1] and _sregs(v[1]) & clobber else v[1],
                 None if v[2] and _sregs(v[2]) & clobber else v[2])
            if v[1] is None and v[2] is None:
                continue
        elif isinstance(k, tuple) and k[0] == "F":
            if k[1] not in ("opq", "nopq") and _touches(k, clobber):
                continue
        elif _touches(k, clobber):
            continue
        elif isinstance(v, tuple):
            v = _stale(v, clobber)
        out[k] = v
    bc = out

    def const(o):
        v = before.get(o)
        if isinstance(v, int):
            return v & M64
        try:
            return int(o, 0) & M64
        except ValueError:
            return None

    def fresh(sym):
        # a boolean computed again (the next loop iteration): facts and
        # selects about its previous instance's opaque name are dropped
        tok = repr(sorted(sym[1]))
        for k_ in [k_ for k_ in bc if isinstance(k_, tuple) and k_[0] == "F" and k_[2] == tok]:
            del bc[k_]
        for k_ in [k_ for k_, v_ in bc.items() if isinstance(v_, tuple) and v_ and isinstance(v_[0], tuple)
                   and v_[0][0] == "c" and any(l[1] == tok for l in v_[0][1])]:
            del bc[k_]
        for k_ in [k_ for k_, v_ in bc.items() if isinstance(v_, tuple) and v_ and v_[0] == "c"
                   and any(l[1] == tok for l in v_[1])]:
            del bc[k_]
        return sym

    fold = {"s_xor_b64": lambda a, b: a ^ b, "s_and_b64": lambda a, b: a & b, "s_or_b64": lambda a, b: a | b,
            "s_andn2_b64": lambda a, b: a & ~b & M64, "s_orn2_b64": lambda a, b: (a | ~b) & M64}
    if m == "s_mov_b64" and len(ops) == 2:
        if const(ops[1]) is not None:
            c = const(ops[1])
            bc[dst] = -1 if c == M64 else c
        elif isinstance(before.get(ops[1]), tuple):
            bc[dst] = before[ops[1]]
    elif m == "s_cselect_b64" and len(ops) == 3 and cond is not None and {ops[1], ops[2]} == {"-1", "0"}:
        op = cond[0] if ops[1] == "-1" else _NEG[cond[0]]
        st = fact_status(bc, op, cond[1], cond[2])
        bc[dst] = (-1 if st else 0) if st is not None else fresh(("c", frozenset({(op, cond[1], cond[2])})))
    elif m in fold and len(ops) == 3 and dst != "vcc" and const(ops[1]) is not None and const(ops[2]) is not None:
        c = fold[m](const(ops[1]), const(ops[2]))
        bc[dst] = -1 if c == M64 else c
    elif re.match(r"^v_cmp_(eq|ne)_u32_e64$", m) and len(ops) == 3 and clobber and \
            {ops[1], ops[2]} & {"0", "1"} and ("v" + (ops[2] if ops[1] in ("0", "1") else ops[1]).lstrip("v")) in bc:
        k = ops[1] if ops[1] in ("0", "1") else ops[2]
        vb = bc["v" + (ops[2] if ops[1] in ("0", "1") else ops[1]).lstrip("v")]
        # lanes hold 1 where vb is set: (v == 1) is vb, (v != 1) / (v == 0) its negation
        neg = (m == "v_cmp_ne_u32_e64") == (k == "1")
        r = _neg_sym(vb) if neg else vb
        if isinstance(r, int):
            r &= M64
            r = -1 if r == M64 else r
        if r is not None:
            bc[dst] = r
    elif m == "s_xor_b64" and len(ops) == 3 and dst != "vcc" and "-1" in ops[1:] and \
            isinstance(before.get(ops[1] if ops[2] == "-1" else ops[2]), tuple):
        r = _neg_sym(before[ops[1] if ops[2] == "-1" else ops[2]])
        if r is not None:
            bc[dst] = r
    elif m == "s_and_b64" and len(ops) == 3 and dst != "vcc":
        # conjunction of uniform booleans (EXEC stands for "true")
        parts = [(-1 if o == "exec" else before.get(o, const(o))) for o in ops[1:]]
        if all(p_ is not None for p_ in parts):
            if any(p_ == 0 for p_ in parts):
                bc[dst] = 0
            else:
                lits = frozenset().union(*[p_[1] for p_ in parts if isinstance(p_, tuple)])
                if lits:
                    st = conj_status(bc, lits)
                    bc[dst] = fresh(("c", lits)) if st is None else (-1 if st else 0)
                elif all(p_ == -1 for p_ in parts):
                    bc[dst] = -1
    elif re.match(r"^v_cmp_(eq|ne)_u32_e32$", m) and len(ops) == 3 and dst == "vcc" and \
            {ops[1], ops[2]} & {"0", "1"} and ("v" + (ops[2] if ops[1] in ("0", "1") else ops[1]).lstrip("v")) in bc:
        k = ops[1] if ops[1] in ("0", "1") else ops[2]
        vb = bc["v" + (ops[2] if ops[1] in ("0", "1") else ops[1]).lstrip("v")]
        neg = (m == "v_cmp_ne_u32_e32") == (k == "1")
        r = _neg_sym(vb) if neg else vb
        if isinstance(r, int):
            bc["vcc"] = (r & M64) != 0
        elif r is not None:
            st = conj_status(bc, r[1])
            if st is not None:
                bc["vcc"] = st
            else:
                bc["vcc_sym"] = r
    elif dst == "vcc" and m in ("s_and_b64", "s_andn2_b64") and len(ops) == 3 and ops[1] == "exec":
        v = before.get(ops[2])
        if isinstance(v, tuple):
            st = conj_status(bc, v[1])
            v = None if st is None else (-1 if st else 0)
        if v in (0, -1):
            nz = v == -1
            bc["vcc"] = nz if m == "s_and_b64" else not nz
        elif _sregs(ops[2]):
            bc["vcc_src"] = (ops[2], m == "s_and_b64")
    return bc


def check_function(name: str, insns: list[Insn], max_states: int = 400000, debug: dict | None = None,
                   track_partial: bool = False):
    if not insns:
        return [], 0
    idx = {i.addr: k for k, i in enumerate(insns)}
    leaders = {0}
    for k, i in enumerate(insns):
        if i.mnem.startswith(("s_branch", "s_cbranch", "s_endpgm", "s_setpc", "s_swappc")):
            if k + 1 < len(insns):
                leaders.add(k + 1)
            if i.target is not None and i.target in idx:
                leaders.add(idx[i.target])
    starts = sorted(leaders)
    blocks = {s: (s, (starts[n + 1] if n + 1 < len(starts) else len(insns))) for n, s in enumerate(starts)}

    def succs(end_k):
        """(successor, sense): sense = True / False for the taken / fall-through
        edge of an SCC branch, None otherwise."""
        last = insns[end_k - 1]
        m = last.mnem
        if m.startswith("s_endpgm") or m.startswith(("s_setpc", "s_swappc")):
            return []
        if m.startswith("s_branch"):
            return [(idx[last.target], None)] if last.target in idx else []
        scc = m in ("s_cbranch_scc0", "s_cbranch_scc1")
        out = [(end_k, (m == "s_cbranch_scc0") if scc else None)] if end_k < len(insns) else []
        if m.startswith("s_cbranch") and last.target in idx:
            out.append((idx[last.target], (m == "s_cbranch_scc1") if scc else None))
        return out

    # State: (pending, full, sg).
    #   pending: for every tracked load that may be in flight, its destination
    #     set -> a LOWER bound on the VMEM ops issued after it.  vmcnt(N)
    #     retires exactly the ops with at least N younger ones (in-order
    #     retirement); at a join the pending loads are united and the bounds
    #     take the minimum (sound: never retires a load some path may still
    #     have in flight).
    #   full: EXEC holds every lane of the wave (all launches use whole waves).
    #   sg: SGPR operands known to hold the full mask (saved EXEC).
    # Loads issued with the full EXEC are tracked; with track_partial, every
    # load is, whatever EXEC held: a load under a partial mask (the grouped
    # claim, issued by lane 0 alone) writes its lanes of the destination when
    # it returns, so a copy or move of that register by the compiler before
    # the covering wait would read a stale value in those lanes.  Any access
    # to a tracked register by any lane before the covering wait is a hazard
    # (conservative for the other lanes).  Partial tracking multiplies the
    # pending sets of compiler code with many per-lane loads, so it is asked
    # for on the persistent kernels, where the asm-issued claim lives.
    def merge(x, y, widen):
        px, fx, sx, ix, bx = x
        py, fy, sy, iy, by = y
        out = dict(px)
        for d, n in py.items():
            out[d] = min(n, out.get(d, n))
        iv = {}
        keys = set(ix) | {k for k in iy if (k[1], k[0]) not in ix}
        for r in keys:
            a_, b_ = dbm_bounds(ix, *r), dbm_bounds(iy, *r)      # direct, reversed or through 0
            if a_ is None or b_ is None:
                continue
            lo, hi = a_
            o = b_
            nl, nh = min(lo, o[0]), max(hi, o[1])
            if widen:                                  # loops: growing bounds go to infinity
                nl = lo if nl == lo else -INF
                nh = hi if nh == hi else INF
            if (nl, nh) != (-INF, INF):
                iv[r] = (nl, nh)
        return (out, fx and fy, {k: v for k, v in sx.items() if sy.get(k) == v}, iv,
                {k: v for k, v in bx.items() if by.get(k) == v})

    # Block entry states are kept apart by which loads are pending (the key),
    # so a join does not lose the link between "line 1 was issued" and the
    # scalar facts that make its consumer run (disjunctive completion over
    # the pending sets; within one key the states merge).
    hazards = {}
    first_load: dict[frozenset, int] = {}
    entry: dict[int, dict] = {0: {(frozenset(), frozenset()): ({}, True, {}, {}, {})}}
    nvis: dict[tuple, int] = {}
    work = [(0, (frozenset(), frozenset()))]
    visits = 0
    while work:
        s, key = work.pop()
        visits += 1
        nvis[(s, key)] = nvis.get((s, key), 0) + 1
        if visits > max_states:
            raise RuntimeError(f"{name}: no fixpoint after {max_states} block visits")
        st, full, sg, iv, bc = entry[s][key]
        st, sg, iv, bc = dict(st), dict(sg), dict(iv), dict(bc)
        cond = None
        scc_bool = None
        a, b = blocks[s]
        for k in range(a, b):
            ins = insns[k]
            if ins.mnem == "s_waitcnt":
                n = vmcnt_of(ins)
                if n is not None:
                    st = {d: y for d, y in st.items() if y < n}
                continue
            full, sg = exec_step(ins, full, sg)
            sel = None
            if ins.mnem == "s_cselect_b32" and scc_bool is not None:
                o = [x.strip() for x in ins.ops.split(",")]
                if len(o) == 3 and _term(o[1]) and _term(o[2]):
                    if isinstance(scc_bool, bool):       # SCC known: d is that operand
                        t_ = _term(o[1] if scc_bool else o[2])
                        iv = _assign(iv, o[0], t_[0], t_[1])
                        bc = bool_step(ins, bc, cond)
                        continue
                    sel = (o[0], scc_bool, o[1], o[2])
            iv, cond = scalar_step(ins, iv, cond)
            bc = bool_step(ins, bc, cond)
            if ins.mnem.startswith("s_") and ins.mnem.endswith("_b64") and not ins.mnem.startswith(
                    ("s_mov", "s_cselect", "s_cmp")) and sgpr_dest(ins):
                # SALU 64-bit logic sets SCC = (result != 0): a uniform boolean
                v_ = bc.get(ins.ops.split(",")[0].strip())
                scc_bool = v_ if isinstance(v_, tuple) else ((v_ & M64) != 0) if isinstance(v_, int) else None
            elif ins.mnem.startswith("s_") and not ins.mnem.startswith(("s_mov", "s_cselect", "s_waitcnt", "s_nop",
                                                                        "s_barrier", "s_setprio", "s_load", "s_getreg",
                                                                        "s_branch", "s_cbranch")):
                scc_bool = None
            if sel is not None:
                # d = SCC ? a : b, SCC the boolean: remembered until the
                # boolean is decided by a branch (then d equals one of them)
                bc[("sel", sel[0])] = sel[1:]
            pending = set().union(*st) if st else set()
            if is_vmem(ins.mnem):
                dest = vmem_dest(ins)
                bad = (ins.regs - dest) & pending if "_load" in ins.mnem else ins.regs & pending
                if bad:
                    hazards.setdefault(ins.addr, (ins, sorted(bad), next(first_load[d] for d in st if d & bad)))
                st = {d: y + 1 for d, y in st.items() if y + 1 < VMCNT_MAX}
                if dest and (full or track_partial):
                    first_load.setdefault(dest, ins.addr)
                    st[dest] = 0
                if dest and debug is not None:
                    debug.setdefault("loads", {}).setdefault(ins.addr, set()).add(full)
            else:
                bad = ins.regs & pending
                if bad:
                    hazards.setdefault(ins.addr, (ins, sorted(bad), next(first_load[d] for d in st if d & bad)))
                    if debug is not None:
                        debug.setdefault("where", {}).setdefault(ins.addr, (s, key))
        last = insns[b - 1].mnem
        for t, sense in succs(b):
            tbc = bc
            tiv = iv
            if last in ("s_cbranch_vccnz", "s_cbranch_vccz"):
                is_taken = t == idx.get(insns[b - 1].target) and t != b
                if "vcc" in bc:
                    if is_taken != (bc["vcc"] == (last == "s_cbranch_vccnz")):
                        continue                           # infeasible edge
                elif "vcc_src" in bc or "vcc_sym" in bc:
                    vcc_nz = is_taken == (last == "s_cbranch_vccnz")
                    tbc = dict(bc)
                    if "vcc_src" in bc:
                        src, pos = bc["vcc_src"]
                        val = -1 if vcc_nz == pos else 0
                        sym = bc.get(src)
                        tbc[src] = val
                    else:
                        sym, val = bc["vcc_sym"], (-1 if vcc_nz else 0)
                    tbc["vcc"] = vcc_nz
                    if isinstance(sym, tuple):             # selects made on this boolean
                        for k_, sv in bc.items():
                            if not (isinstance(k_, tuple) and k_[0] == "sel"):
                                continue
                            bs, ta, tb = sv
                            if bs == sym:
                                tsel = ta if val else tb
                            elif bs == _neg_sym(sym):
                                tsel = tb if val else ta
                            else:
                                continue
                            if tsel is not None:
                                tiv = _refine(tiv, ("eq", k_[1], tsel), True) if tiv is not None else None
                        if tiv is None:
                            continue
                    if isinstance(sym, tuple):             # the compares behind the boolean
                        if val:
                            for l in sym[1]:
                                tbc[("F",) + l] = True
                        else:
                            open_ = [l for l in sym[1] if fact_status(bc, *l) is not True]
                            if any(fact_status(bc, *l) is False for l in sym[1]):
                                pass
                            elif len(open_) == 1:
                                op, x, y = open_[0]
                                tbc[("F", _NEG[op], x, y)] = True
                            elif not open_:
                                continue                   # infeasible: all hold, yet false
            if sense is not None and cond is not None:
                st_ = fact_status(bc, *cond)
                if st_ is not None and st_ != sense:
                    continue                               # infeasible edge
                A, B = _term(cond[1]), _term(cond[2])
                dec = _decide(cond[0], _diff(iv, A, B)) if A and B else None
                if dec is not None and dec != sense:
                    continue                               # infeasible edge
                tiv = _refine(iv, cond, sense)
                if tiv is None:
                    continue
                tbc = dict(tbc)
                tbc[("F", cond[0] if sense else _NEG[cond[0]], cond[1], cond[2])] = True
            out = (st, full, sg, tiv, tbc)
            # states are kept apart by the pending loads and by the compares
            # decided on the way (a join would intersect those facts away)
            tkey = (frozenset(st), frozenset(k for k in tbc if isinstance(k, tuple)))
            cur = entry.setdefault(t, {}).get(tkey)
            new = merge(cur, out, nvis.get((t, tkey), 0) > 6) if cur is not None else out
            if cur is None or new != cur:
                if debug is not None and cur is None:
                    debug.setdefault("parent", {})[(t, tkey)] = (s, key)
                entry[t][tkey] = new
                if (t, tkey) not in work:
                    work.append((t, tkey))
    if debug is not None:
        debug.update(entry=entry, blocks=blocks, succs=succs)
    return list(hazards.values()), visits


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("lib", nargs="?", default=str(ROOT / "zsummerx_amd" / "libzrc4.so"))
    ap.add_argument("--kernel", default="", help="only kernels whose mangled name contains this")
    ap.add_argument("--max-report", type=int, default=20)
    ap.add_argument("--disasm", help="read this llvm-objdump output instead of the library")
    args = ap.parse_args(argv)
    text = Path(args.disasm).read_text() if args.disasm else disassemble(Path(args.lib))
    funcs = parse(text)
    total = 0
    for name, insns in funcs.items():
        if args.kernel and args.kernel not in name:
            continue
        hz, visits = check_function(name, insns)
        status = "HAZARD" if hz else "ok"
        print(f"{status:6s} {name} ({len(insns)} instructions, {visits} block visits)")
        for ins, regs, load_addr in sorted(hz, key=lambda h: h[0].addr)[: args.max_report]:
            print(f"    0x{ins.addr:x}: {ins.text}    <- v{regs[0]}{'..' if len(regs) > 1 else ''} "
                  f"still loading from the VMEM op at 0x{load_addr:x}")
        total += len(hz)
    print(f"{total} hazard(s)")
    return 1 if total else 0


if __name__ == "__main__":
    sys.exit(main())
