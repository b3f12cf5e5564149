"""One rank of bench.py's self-launched job, on the CPU (gloo) with the oracle
runner: what bench.self_launch starts N times when `--gpus N` runs without
torchrun, minus the GPU.  tests/test_multirank.py::test_self_launch_two_ranks
drives it through bench.self_launch, the same function `python bench.py
--gpus N` uses.  Test shapes: tiny = 256 x 64 B per rank (weak), tiny2 =
512 x 64 B job (its strong companion)."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT, ROOT / "oracle", ROOT / "tests"):
    sys.path.insert(0, str(p))

import bench  # noqa: E402
from oracle_runner import OracleRunner  # noqa: E402

bench.CONFIG_SHAPES["tiny"] = (256, 64)
bench.CONFIG_TEXT["tiny"] = "256 sessions x 64 B (test shape)"
bench.CONFIG_SHAPES["tiny2"] = (512, 64)
bench.CONFIG_TEXT["tiny2"] = "512 sessions x 64 B job (test shape)"
bench.COMPANION_BASES.add("tiny")

if __name__ == "__main__":
    bench.rank_main(bench.parse(sys.argv[1:]), backend="gloo", make_runner=OracleRunner)
