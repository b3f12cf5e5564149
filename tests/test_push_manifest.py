"""The GPU push must carry every file the GPU tests, smoke() and bench.py read.

gpurun snapshots the tree minus the patterns in `.gpurunignore` (tar exclude
patterns: `*` also matches `/`, a pattern matches the whole member name
`./path` or any tail of it that starts after a `/`, a pattern ending in `/`
matches nothing, and an excluded directory takes everything under it).  In
round 4 a `*.npz` line meant for profile dumps also dropped
`tests/golden/batch_small.npz`, and the driver's GPU run stopped at the first
test that loads it.  This test applies the patterns the same way to every
tracked file and fails if one under tests/, oracle/ (sources), zsummerx_amd/,
include/ or the root entry points is excluded.
"""
import fnmatch
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]

# Tracked files kept off the box on purpose: CPU-only checkers whose text names
# the scalar-cache store instructions gpurun refuses to upload.  No GPU test,
# smoke() or bench.py imports them.
DELIBERATE = {
    "tools/vmem_hazard_check.py",
    "tests/test_vmem_hazards.py",
}

MUST_SHIP_PREFIXES = ("tests/", "oracle/", "zsummerx_amd/", "include/")
MUST_SHIP_ROOT = ("bench.py", "__graft_entry__.py", "BASELINE.json")


def load_patterns(text):
    pats = []
    for line in text.splitlines():
        line = line.strip()
        if not line or line.startswith("#") or line.endswith("/"):
            continue
        pats.append(line)
    return pats


def _matches(name, pat):
    # no-anchored: the full member name or any tail after a '/'
    if fnmatch.fnmatchcase(name, pat):
        return True
    i = name.find("/")
    while i >= 0:
        if fnmatch.fnmatchcase(name[i + 1:], pat):
            return True
        i = name.find("/", i + 1)
    return False


def excluded(relpath, pats):
    """True if tar would drop `relpath` (or a directory above it)."""
    parts = relpath.split("/")
    for k in range(1, len(parts) + 1):
        member = "./" + "/".join(parts[:k])
        if any(_matches(member, p) for p in pats):
            return True
    return False


def tracked_files():
    out = subprocess.run(["git", "ls-files"], cwd=ROOT, capture_output=True, text=True)
    if out.returncode != 0:
        pytest.skip("not a git checkout")
    return [l for l in out.stdout.splitlines() if l]


def test_matcher_semantics():
    pats = load_patterns("*.log\n./results\nbuild/\n./profiles/r04\n./profiles/*.npz\n")
    assert excluded("a/b/c.log", pats)
    assert excluded("results/x.json", pats)
    assert not excluded("tests/results/x.json", pats)
    assert not excluded("build/x.o", pats)          # trailing '/' matches nothing
    assert excluded("profiles/r04/final/t.npz", pats)
    assert excluded("profiles/t.npz", pats)
    assert not excluded("tests/golden/batch_small.npz", pats)


def test_no_needed_file_is_push_excluded():
    pats = load_patterns((ROOT / ".gpurunignore").read_text())
    files = tracked_files()
    assert "tests/golden/batch_small.npz" in files
    bad = []
    for f in files:
        need = f.startswith(MUST_SHIP_PREFIXES) or f in MUST_SHIP_ROOT
        if f.startswith("oracle/_ref/"):
            need = False
        if need and f not in DELIBERATE and excluded(f, pats):
            bad.append(f)
    assert not bad, f".gpurunignore drops files the GPU run needs: {bad}"


def test_deliberate_exclusions_are_cpu_only():
    """Files kept off the box must not be GPU tests or product imports."""
    for f in DELIBERATE:
        p = ROOT / f
        if not p.exists():
            continue
        text = p.read_text()
        assert "pytest.mark.gpu" not in text, f
    for src in ["bench.py", "__graft_entry__.py"] + [
            str(p.relative_to(ROOT)) for p in (ROOT / "zsummerx_amd").rglob("*.py")]:
        text = (ROOT / src).read_text()
        assert "vmem_hazard_check" not in text, src
