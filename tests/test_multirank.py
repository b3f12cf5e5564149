"""CPU multi-rank tests (gloo, world_size 2) of bench.py's distributed path.

The GPU bench shards sessions across ranks by global id with no data-path
collective; torch.distributed carries only the start/stop
barrier and the max-over-ranks time.  Here the same orchestration
(bench.run_bench) runs on two CPU processes with a test-side runner that
crypts its shard with the oracle, and we check: disjoint, complete shards;
each rank's ciphertext equals the single-process result for those global
sessions; rank 0 reports the whole-job aggregate from the MAX rank time.
"""
import hashlib
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT

sys.path.insert(0, str(ROOT))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class OracleRunner:
    """Runner with the GpuRunner interface, backed by the CPU oracle."""

    def __init__(self, S, L, R, first):
        import pyoracle
        from zsummerx_amd import synth
        self.S, self.L, self.R, self.first = S, L, R, first
        w = synth.make(first, S * R, L)
        self.w = w
        self.ob = pyoracle.Batch(S * R)
        self.ob.make_sbox(w.keys, w.key_off, w.key_len)
        self.ob.crypt(np.zeros(1000, dtype=np.uint8), np.zeros(S * R, dtype=np.uint64), w.adv)
        self.steps_done = []

    def step(self, i):
        import pyoracle  # noqa: F401
        b = i % self.R
        sl = slice(b * self.S, (b + 1) * self.S)
        # crypt only batch b's sessions (others keep their state)
        sub_off = self.w.off.copy()
        sub_len = np.zeros_like(self.w.length)
        sub_len[sl] = self.w.length[sl]
        self.ob.crypt(self.w.payload, sub_off, sub_len)
        self.steps_done.append(i)

    def sync(self):
        pass

    def check(self):
        pass

    # bench.GpuRunner's timing interface: events made before the timed
    # region, launches, then per-segment ms per step
    def make_events(self, k, every=16):
        return [None] * (-(-k // every) + 1)

    def launch_steps(self, first, k, every, marks):
        import time
        for seg, d in enumerate(range(0, k, every)):
            t0 = time.perf_counter()
            m = min(every, k - d)
            for i in range(first + d, first + d + m):
                self.step(i)
            marks[seg] = (time.perf_counter() - t0) * 1e3 / m

    @staticmethod
    def segment_ms(k, every, marks):
        return [v for v in marks if v is not None]


def _worker(rank, ws, port, q, workload, steps, warmup, footprint, strong=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(ws), LOCAL_RANK=str(rank))
    sys.path.insert(0, str(ROOT / "oracle"))
    import bench
    bench.CONFIG_SHAPES["tiny"] = (256, 64)
    bench.CONFIG_TEXT["tiny"] = "256 sessions x 64 B (test shape)"
    bench.CONFIG_SHAPES["tiny2"] = (512, 64)
    bench.CONFIG_TEXT["tiny2"] = "512 sessions x 64 B job (test shape)"
    args = bench.parse(["--workload", "cfg2", "--steps", str(steps), "--warmup", str(warmup),
                        "--footprint-mib", str(footprint), "--cpu-seconds", "0"])
    args.workload = workload
    args.strong = strong
    res, runner = bench.run_bench(args, ws, rank, rank, backend="gloo", make_runner=OracleRunner)
    q.put((rank, res, runner.first, runner.S * runner.R,
           hashlib.sha256(runner.w.payload.tobytes()).hexdigest(), len(runner.steps_done)))


@pytest.mark.timeout(300)
def test_two_rank_gloo_sharding_and_aggregate():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ws, steps, warmup = 2, 3, 1
    procs = [ctx.Process(target=_worker, args=(r, ws, port, q, "tiny", steps, warmup, 0))
             for r in range(ws)]
    for p in procs:
        p.start()
    got = [q.get(timeout=240) for _ in range(ws)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    got.sort()
    (r0, res, first0, n0, dig0, nsteps0), (r1, res1, first1, n1, dig1, nsteps1) = got
    assert res1 is None and res is not None
    # disjoint, contiguous shards of global session ids
    assert (first0, first1) == (0, n0) and n0 == n1
    assert nsteps0 == nsteps1 == steps + warmup
    # each rank's result equals a single-process run over the same global ids
    sys.path.insert(0, str(ROOT / "oracle"))
    for first, n, dig in ((first0, n0, dig0), (first1, n1, dig1)):
        r = OracleRunner(256, 64, 1, first)
        for i in range(steps + warmup):
            r.step(i)
        assert hashlib.sha256(r.w.payload.tobytes()).hexdigest() == dig
    # aggregate: whole-job payload over the max rank time, weak scaling
    assert res["n_gpus"] == 2 and res["scaling"] == "weak"
    total = ws * steps * 256 * 64
    expect = total / (res["ms_per_step"] * steps * 1e-3) / 2**30   # both fields are rounded
    assert abs(res["value"] - expect) <= 0.02 * expect + 2e-3
    assert res["config"]["global_sessions_per_step"] == 512
    # per-GPU breakdown: one entry per rank, the slowest sets ms_per_step
    assert [g["rank"] for g in res["per_gpu"]] == [0, 1]
    slowest = min(g["payload_gibs"] for g in res["per_gpu"])
    assert abs(slowest * ws - res["value"]) <= 0.05 * res["value"] + 2e-3


@pytest.mark.timeout(300)
def test_two_rank_gloo_strong_scaling():
    """--strong (BASELINE configs[4]): the workload's sessions are the whole
    job; two ranks split them into disjoint halves and the aggregate counts the
    job once."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ws, steps, warmup = 2, 2, 1
    procs = [ctx.Process(target=_worker, args=(r, ws, port, q, "tiny2", steps, warmup, 0, True))
             for r in range(ws)]
    for p in procs:
        p.start()
    got = [q.get(timeout=240) for _ in range(ws)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    got.sort()
    (r0, res, first0, n0, _, _), (r1, res1, first1, n1, _, _) = got
    assert res1 is None and res is not None
    assert n0 == n1 == 256 and (first0, first1) == (0, 256)
    assert res["scaling"] == "strong" and res["config"]["global_sessions_per_step"] == 512
    assert res["config"]["sessions_per_gpu"] == 256
    total = steps * 512 * 64                                   # the job once, not per rank
    expect = total / (res["ms_per_step"] * steps * 1e-3) / 2**30
    assert abs(res["value"] - expect) <= 0.02 * expect + 2e-3
