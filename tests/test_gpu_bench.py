"""bench.py's GPU runner against the CPU oracle (test infrastructure: the
oracle is the checker).  Every slot-addressing mode the bench can time --
range, grouped, declared and scattered ids (scattered with a ragged last
group) -- must crypt exactly the sessions a plain range crypt of
the same batches would, so the bench never times a path that differs from
the parity-tested one."""
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))
sys.path.insert(0, str(ROOT / "tests"))


@pytest.mark.gpu
@pytest.mark.parametrize("ids,S", [("range", 300), ("scattered", 300), ("scattered", 512),
                                   ("grouped", 512), ("declared", 512)])
def test_bench_runner_matches_oracle(built, ids, S):
    import torch
    import bench
    from oracle_runner import OracleRunner
    L, R, steps = 64, 2, 3
    run = bench.GpuRunner(torch, 0, S, L, R, 0, ids)
    ref = OracleRunner(S, L, R, 0)
    try:
        for i in range(steps):
            run.step(i)
            ref.step(i)
        run.check()
        got = run.payload.cpu().numpy()
        want = ref.w.payload
        bad = np.flatnonzero(got != want)
        assert bad.size == 0, (f"{ids}: {bad.size} bytes differ, first at {bad[:8].tolist()} "
                               f"(sessions {sorted(set((bad[:64] // L).tolist()))[:8]})")
    finally:
        run.close()
