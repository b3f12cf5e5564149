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
import json
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT
from oracle_runner import OracleRunner

sys.path.insert(0, str(ROOT))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


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


@pytest.mark.timeout(300)
def test_self_launch_two_ranks(capsys):
    """`python bench.py --gpus 2` without torchrun: bench.self_launch starts
    the two rank processes itself (here tests/bench_child_cpu.py: the same
    rank_main over gloo with the oracle runner) and relays rank 0's line,
    which names the weak curve, the world size the process group saw, one
    per_gpu entry per rank, and the strong configs[4]-style companion split
    over the same ranks."""
    import bench
    argv = ["--gpus", "2", "--workload", "tiny", "--steps", "3", "--warmup", "1", "--footprint-mib", "0",
            "--cpu-seconds", "0", "--companion-workload", "tiny2", "--companion-steps", "2",
            "--companion-warmup", "1"]
    rc = bench.self_launch(argv, 2, entry=ROOT / "tests" / "bench_child_cpu.py", timeout=240)
    out = capsys.readouterr().out
    assert rc == 0, out
    res = json.loads([ln for ln in out.splitlines() if ln.startswith("{")][-1])
    assert res["n_gpus"] == 2 and res["scaling"] == "weak"
    assert res["config"]["world_size_seen"] == 2 and res["config"]["dist_backend"] == "gloo"
    assert res["config"]["curve"].startswith("weak")
    assert [g["rank"] for g in res["per_gpu"]] == [0, 1]
    rf = res["roofline"]              # the device span per step: launches and gaps, no host wake-up
    assert 0 < rf["device_us_per_step"] <= res["ms_per_step"] * 1e3 * 1.05
    comp = res["configs4_strong"]
    assert comp["n_gpus"] == 2 and comp["scaling"] == "strong"
    assert comp["config"]["sessions_per_gpu"] == 256 and comp["config"]["global_sessions_per_step"] == 512
    assert comp["config"]["world_size_seen"] == 2
    assert [g["rank"] for g in comp["per_gpu"]] == [0, 1]
    expect = comp["steps"] * 512 * 64 / (comp["ms_per_step"] * comp["steps"] * 1e-3) / 2**30
    assert abs(comp["value"] - expect) <= 0.02 * expect + 2e-3


@pytest.mark.timeout(300)
def test_self_launch_rehearsal_puts_every_rank_on_device_0(capsys, monkeypatch):
    """`--rehearse-one-gpu` (scripts/r06_rehearse.sh: the multi-rank path on a
    one-GPU box): every rank takes device 0 whatever LOCAL_RANK says, the
    group is gloo, and the line says it is a rehearsal."""
    import bench
    argv = ["--gpus", "2", "--workload", "tiny", "--steps", "2", "--warmup", "1", "--footprint-mib", "0",
            "--cpu-seconds", "0", "--companion-workload", "none", "--rehearse-one-gpu"]
    rc = bench.self_launch(argv, 2, entry=ROOT / "tests" / "bench_child_cpu.py", timeout=240)
    out = capsys.readouterr().out
    assert rc == 0, out
    res = json.loads([ln for ln in out.splitlines() if ln.startswith("{")][-1])
    assert res["n_gpus"] == 2 and res["config"]["dist_backend"] == "gloo"
    assert "rehearsal" in res["config"]
    seen = []
    monkeypatch.setenv("WORLD_SIZE", "1")
    monkeypatch.setenv("LOCAL_RANK", "3")
    monkeypatch.setattr(bench, "run_bench", lambda a, ws, rank, local, backend, *r, **k: (
        seen.append((local, backend)), ({"config": {}}, None))[1])
    bench.rank_main(bench.parse(["--rehearse-one-gpu", "--companion-workload", "none"]))
    assert seen == [(0, "gloo")]


@pytest.mark.timeout(120)
def test_self_launch_reports_a_failing_rank(capsys):
    """A rank that fails makes the job fail (non-zero exit), and the other
    rank is stopped rather than left waiting at the barrier."""
    import bench
    argv = ["--gpus", "2", "--workload", "no-such-shape"]
    rc = bench.self_launch(argv, 2, entry=ROOT / "tests" / "bench_child_cpu.py", timeout=100)
    assert rc != 0


def test_usable_cpus_caps_affinity_by_quota(monkeypatch):
    import bench
    monkeypatch.setattr(bench.os, "sched_getaffinity", lambda pid: set(range(256)))
    monkeypatch.setattr(bench, "cgroup_cpu_quota", lambda: 16.0)
    assert bench.usable_cpus() == (16, 256, 16.0)
    monkeypatch.setattr(bench, "cgroup_cpu_quota", lambda: 2.5)
    assert bench.usable_cpus()[0] == 3
    monkeypatch.setattr(bench, "cgroup_cpu_quota", lambda: None)
    assert bench.usable_cpus()[0] == 256


def test_cpu_baseline_times_the_reference(monkeypatch):
    """bench.py's cpu_baseline leg times the reference's own RC4Encryption
    (oracle/_ref, kind "reference") when that build is present, else the
    restatement (kind "port"); the reported threads are the usable CPUs."""
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "oracle"))
    import bench
    import pyoracle
    monkeypatch.setattr(bench, "usable_cpus", lambda: (2, 8, 2.0))
    args = bench.parse(["--cpu-seconds", "0.2", "--workload", "cfg2"])
    r = bench.cpu_baseline(args, 512, 1024)
    assert r["kind"] == ("reference" if pyoracle.ref_lib() is not None else "port")
    assert r["cores"] == r["threads"] == 2 and r["value"] > 0 and r["value_1thread"] > 0
    assert r["sample"].startswith("RC4Encryption" if r["kind"] == "reference" else "the oracle")


def test_reference_batch_matches_the_restatement():
    """The reference-timed baseline crypts the same bytes as the restatement."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import ctypes as C
    import pyoracle
    if pyoracle.ref_lib() is None:
        pytest.skip("oracle/_ref not built")
    from zsummerx_amd import synth
    S, L = 64, 300
    w = synth.make(0, S, L, threads=1)
    rb = pyoracle.RefBatch(S)
    rb.make_sbox(w.keys, w.key_off, w.key_len)
    rb.advance(w.adv)
    ob = pyoracle.Batch(S)
    ob.make_sbox(w.keys, w.key_off, w.key_len)
    ob.crypt(np.zeros(1000, dtype=np.uint8), np.zeros(S, dtype=np.uint64), w.adv)
    p1, p2 = w.payload.copy(), w.payload.copy()
    for i in range(S):
        rb.R.zrc4_ref_encryption(C.c_void_p(rb.base + i * rb.sz), C.c_void_p(p1.ctypes.data + int(w.off[i])),
                                 int(w.length[i]))
    ob.crypt(p2, w.off, w.length)
    assert np.array_equal(p1, p2)


class _ShardRunner:
    """bench.GpuRunner's interface for shard_projection, on the CPU: every
    launch records (first_slot, n) and 'takes' n * 1e-6 ms, so a shard of
    S/N sessions times N times faster than the whole batch."""
    class _Fn:
        __name__ = "zrc4_crypt_range"

        def __init__(self, log):
            self.log = log

        def __call__(self, h, first, pay, offp, lenp, n, st):
            self.log.append((first, offp.value, lenp.value, n))
            return 0

    def __init__(self, S, L):
        import ctypes as C
        self.S, self.L, self.R, self.log = S, L, 1, []
        self._fn = self._Fn(self.log)
        self._args = [(None, 0, C.c_void_p(1 << 20), C.c_void_p(2 << 20), C.c_void_p(3 << 20), S, None)]

    def step(self, i):
        self._fn(*self._args[i % self.R])

    def sync(self):
        pass

    def check(self):
        pass

    def make_events(self, k, every=16):
        return [None] * (-(-k // every) + 1)

    def launch_steps(self, first, k, every, marks):
        for seg, d in enumerate(range(0, k, every)):
            m = min(every, k - d)
            for i in range(first + d, first + d + m):
                self.step(i)
            marks[seg] = self._args[0][5] * 1e-6       # ms per launch, proportional to the shard

    @staticmethod
    def segment_ms(k, every, marks):
        return [v for v in marks if v is not None]


def test_shard_projection_splits_the_batch_into_contiguous_shards():
    """configs4_strong.shard_projection (N = 1 only): shard k of N is slots
    [k S/N, (k+1) S/N) with its offsets / lengths advanced to match, the
    shards rotate, the runner is restored afterwards, and the speed-ups are
    the 1-GPU kernel time over each shard's."""
    import argparse
    import bench
    S, L = 524288, 1024
    run = _ShardRunner(S, L)
    saved = list(run._args)
    c = argparse.Namespace(workload="cfg5", warmup=2, steps=32, event_every=16)
    res = {"roofline": {"kernel_avg_us": S * 1e-3}, "ms_per_step": S * 1e-6}
    proj = bench.shard_projection(c, run, res)
    assert [s["gpus"] for s in proj["shards"]] == [2, 4, 8]
    for s in proj["shards"]:
        n = s["gpus"]
        assert s["sessions_per_gpu"] == S // n
        assert abs(s["projected_speedup_kernel"] - n) < 1e-6
    assert run._args == saved and run.R == 1
    shards8 = {(f, o, ln, n) for f, o, ln, n in run.log if n == S // 8}
    assert shards8 == {(k * S // 8, (2 << 20) + 8 * k * S // 8, (3 << 20) + 4 * k * S // 8, S // 8) for k in range(8)}
