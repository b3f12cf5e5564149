import json
import os
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
GOLDEN = ROOT / "tests" / "golden"
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")


def soak_seeds(default=(1,)):
    """Seeds of the randomised GPU sweeps' soak cases: $ZRC4_SOAK_SEEDS as
    'a-b' and/or 'a,b,c' (scripts/r06_soak.sh), else `default`."""
    spec = os.environ.get("ZRC4_SOAK_SEEDS", "").strip()
    if not spec:
        return list(default)
    out = []
    for part in spec.split(","):
        a, _, b = part.strip().partition("-")
        out.extend(range(int(a), int(b) + 1) if b else [int(a)])
    return out


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) device")


@pytest.fixture(scope="session")
def kat():
    return json.loads((GOLDEN / "kat.json").read_text())


@pytest.fixture(scope="session")
def edge():
    return json.loads((GOLDEN / "edge.json").read_text())["cases"]


@pytest.fixture(scope="session")
def batch_small():
    with np.load(GOLDEN / "batch_small.npz", allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def synth_digests():
    return json.loads((GOLDEN / "synth_digests.json").read_text())


@pytest.fixture(scope="session")
def built():
    from zsummerx_amd import build
    build.build_all()
    return True
