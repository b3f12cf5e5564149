#!/usr/bin/env python3
"""bench.py -- device-resident batched RC4 throughput on MI355X.

Metric (BASELINE.json): "RC4 GiB/s device-resident (batched session payloads)
at 1/2/4/8 MI355X".  One step = one zrc4_crypt pass (batched
RC4Encryption::encryption, depends/rc4/rc4_encryption.h:74-93) over one batch
of the chosen workload:

  cfg2 (default, BASELINE configs[1]): 4 096 sessions x 1 KiB per GPU
  cfg3: 65 536 x 256 B   cfg4: 1 024 x 64 KiB   cfg5: 524 288 x 1 KiB

Multi-GPU: one process per GPU, sessions shard across ranks with no
collective on the data path; each rank runs the same per-GPU
batch over its own global session ids -> "scaling": "weak"; with --strong the
workload's sessions are the whole job and ranks split them (BASELINE
configs[4]: --workload cfg5 --strong).  torch.distributed
is used only for the start/stop barrier and the max-over-ranks time.  Ranks
come from torchrun's environment, or -- `--gpus N` with no WORLD_SIZE set --
bench.py starts its own N rank processes (self_launch: child processes with
RANK/LOCAL_RANK/WORLD_SIZE/MASTER_*; the parent never touches the GPU).
Which curve a line is: config.curve.  The weak cfg2 line also carries the
strong configs[4] split measured in the same job ("configs4_strong": 524 288
x 1 KiB over the same ranks), so a 1/2/4/8 sweep yields both curves.

HBM honesty: each rank rotates over R distinct batches (distinct sessions,
states and payload buffers) totalling >= --footprint-mib (default 640 MiB, i.e.
beyond the 256 MiB Infinity Cache), so successive steps do not re-hit caches.

Inputs are synthetic (zsummerx_amd/synth.py): mt19937_64 keys
and payload, states pre-advanced (sid*37)%1000 bytes; KSA and pre-advance run
before the timed region.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import math
import os
import statistics
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "RC4 GiB/s device-resident (batched session payloads) at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
STATE_BYTES = 516              # 258-B state load + store per session
GIB = float(1 << 30)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return ws, rank, local


def algorithmic_bytes(S: int, L: int) -> int:
    """B = 2*sum(L) + 516*S  (payload read+write + state load+store)."""
    return 2 * S * L + STATE_BYTES * S


def per_rank_sessions(S_job: int, ws: int) -> int:
    """Strong scaling: rank r owns sessions [r*S, (r+1)*S) of the job (whole
    256-session groups; every BASELINE total divides evenly at 1/2/4/8)."""
    if S_job % (256 * ws):
        raise SystemExit(f"--strong: {S_job} sessions do not split into whole groups over {ws} ranks")
    return S_job // ws


def rotation_batches(S: int, L: int, footprint_mib: int) -> int:
    per_batch = S * L + S * 256
    return max(1, math.ceil(footprint_mib * (1 << 20) / per_batch))


def shard_first(rank: int, R: int, S: int) -> int:
    """Global id of rank r's first session: ranks own disjoint session ranges."""
    return rank * R * S


# ------------------------------------------------------------------ GPU leg
class GpuRunner:
    """Owns the device buffers of R rotating batches on one GPU."""

    def __init__(self, torch, device: int, S: int, L: int, R: int, first: int, ids_mode: str = "range"):
        from zsummerx_amd import Context, synth
        self.torch, self.S, self.L, self.R = torch, S, L, R
        dev = torch.device("cuda", device)
        self.ctx = Context(device, S * R)
        self.stream = torch.cuda.current_stream(dev)
        t0 = time.time()
        keys = synth.keys(first, S * R).reshape(-1)
        adv = synth.advance(first, S * R)
        payload = synth.payload(first * L, S * R * L, threads=8)
        log(f"[rank gen] {S*R} sessions, {payload.nbytes/2**20:.0f} MiB payload in {time.time()-t0:.1f}s")
        T = lambda a: torch.from_numpy(a).to(dev)
        n = S * R
        key_len = T(np.full(n, 16, dtype=np.int32))
        key_off = T(np.arange(n, dtype=np.int64) * 16)
        self.ctx.ksa(key_len, key_off, T(keys), stream=self.stream)
        scratch = torch.zeros(1000, dtype=torch.uint8, device=dev)
        self.ctx.crypt(scratch, torch.zeros(n, dtype=torch.int64, device=dev),
                       T(adv.view(np.int32)), stream=self.stream)
        self.payload = T(payload)
        self.off = T((np.arange(n, dtype=np.int64) * L))
        self.len = T(np.full(n, L, dtype=np.int32))
        self.ctx.sync(self.stream)
        # batch b = slots [b*S, (b+1)*S): zrc4_crypt_range(ctx, first_slot, payload, off, len, n, stream)
        lib, h, st = self.ctx._lib, self.ctx._h, C.c_void_p(self.stream.cuda_stream)
        self._args = []
        if ids_mode == "range":
            self._fn = lib.zrc4_crypt_range
            for b in range(R):
                self._args.append((h, b * S, C.c_void_p(self.payload.data_ptr()),
                                   C.c_void_p(self.off.data_ptr() + 8 * b * S),
                                   C.c_void_p(self.len.data_ptr() + 4 * b * S), S, st))
        else:
            # Entry i of batch b crypts session b*S + i with the slot the
            # session was seeded in; slots are a random permutation inside each
            # 256-slot group and the groups come in random order ("scattered"
            # ids, as an engine's free list hands them out).  grouped: entries
            # bucketed by group -> zrc4_crypt_grouped (coalesced images);
            # scattered: the same ids unbucketed -> zrc4_crypt (per-lane gathers).
            # (grouped / declared: whole groups only -- a short group placed
            # mid-batch would make later buckets straddle two groups; scattered
            # ids are unbucketed, so a ragged last group is fine there)
            if S % 256 and ids_mode != "scattered":
                raise SystemExit(f"--ids {ids_mode} needs a multiple of 256 sessions per batch, not {S}")
            rng = np.random.default_rng(77)
            perm = np.empty(n, dtype=np.int64)
            bgroups = []
            ng = -(-S // 256)
            for b in range(R):
                order = rng.permutation(ng)
                bgroups.append(np.ascontiguousarray((b * ng + order).astype(np.uint32)))
                pos = b * S
                for g in order:
                    lo = b * S + g * 256
                    hi = min(lo + 256, (b + 1) * S)
                    perm[pos:pos + hi - lo] = lo + rng.permutation(hi - lo)
                    pos += hi - lo
            # entry e of batch b -> session perm[e]: keys/state/payload follow the session
            self.ids = T(perm.astype(np.int32))
            self.off = T((perm * L).astype(np.int64))
            self._bgroups = bgroups          # declared: each bucket's group (host memory)
            for b in range(R):
                common = (C.c_void_p(self.payload.data_ptr()), C.c_void_p(self.off.data_ptr() + 8 * b * S),
                          C.c_void_p(self.len.data_ptr() + 4 * b * S), S)
                idp = C.c_void_p(self.ids.data_ptr() + 4 * b * S)
                if ids_mode == "declared":
                    self._fn = lib.zrc4_crypt_grouped_declared
                    self._args.append((h, idp, C.c_void_p(bgroups[b].ctypes.data), *common, None, st))
                else:
                    self._fn = lib.zrc4_crypt_grouped if ids_mode == "grouped" else lib.zrc4_crypt
                    self._args.append((h, idp, *common, st))

    def step(self, i: int) -> None:
        rc = self._fn(*self._args[i % self.R])
        if rc:
            raise RuntimeError(f"zrc4 crypt ({self._fn.__name__}) failed: {rc}")

    def sync(self) -> None:
        self.torch.cuda.synchronize()

    def check(self) -> None:
        self.ctx.sync(self.stream)

    def close(self) -> None:
        """Free the batches and the arena (before the companion measurement)."""
        self.torch.cuda.synchronize()
        self._args = []
        self.payload = self.off = self.len = self.ids = None
        self.ctx.close()
        self.torch.cuda.empty_cache()

    def make_events(self, k: int, every: int = 16):
        """The HIP events of timed_steps, created BEFORE the timed region
        (creating one costs host time that is not part of a step)."""
        return [self.torch.cuda.Event(enable_timing=True) for _ in range(-(-k // every) + 1)]

    def timed_steps(self, first: int, k: int, every: int = 16, marks=None):
        """Launch steps first..first+k-1 back to back; HIP events on the launch
        stream bracket consecutive segments of `every` launches, and each
        segment's duration / its launch count is returned (ms per launch).
        (An event pair around EVERY launch adds ~7 us of queue work per step
        and reads ~3 us high on a 50 us kernel -- tools/launch_gap.py; a
        16-launch segment amortises that to <0.2 us and agrees with the
        rocprofv3 kernel average.)"""
        if marks is None:
            marks = self.make_events(k, every)
        self.launch_steps(first, k, every, marks)
        self.sync()
        return self.segment_ms(k, every, marks)

    def launch_steps(self, first: int, k: int, every: int, marks) -> None:
        marks[0].record(self.stream)
        done, seg = 0, 0
        while done < k:
            m = min(every, k - done)
            for i in range(m):
                self.step(first + done + i)
            seg += 1
            marks[seg].record(self.stream)
            done += m

    @staticmethod
    def segment_ms(k: int, every: int, marks):
        counts = [min(every, k - d) for d in range(0, k, every)]
        return [a.elapsed_time(b) / m for a, b, m in zip(marks, marks[1:], counts)]


def ensure_process_group(ws, local, backend):
    """One process group per job (RCCL on the GPU box, gloo in the CPU tests);
    returns True when this call created it."""
    import torch
    import torch.distributed as dist
    if ws <= 1 or dist.is_initialized():
        return False
    if backend == "nccl":
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist.init_process_group(backend)
    return True


def run_bench(args, ws, rank, local, backend="nccl", make_runner=None, own_pg=True):
    """Shared orchestration (GPU bench and the gloo CPU test): W untimed steps,
    barrier + sync, K timed steps, sync + barrier, max over ranks.  Sessions
    shard across ranks by global id (shard_first); no data-path collective.
    own_pg: tear the process group down at the end (main() keeps it for the
    configs[4] companion measurement and tears it down itself)."""
    import torch
    import torch.distributed as dist

    on_gpu = backend == "nccl"
    ensure_process_group(ws, local, backend)
    seen_ws = dist.get_world_size() if dist.is_initialized() else 1
    S_job, L = CONFIG_SHAPES[args.workload]
    # --strong: the workload's sessions are the WHOLE job (BASELINE configs[4]:
    # 524 288 sessions sharded across the GPUs); otherwise every rank runs it
    S = per_rank_sessions(S_job, ws) if args.strong else S_job
    R = rotation_batches(S, L, args.footprint_mib) if args.footprint_mib > 0 else 1
    if make_runner is None:
        runner = GpuRunner(torch, local, S, L, R, shard_first(rank, R, S), getattr(args, "ids", "range"))
    else:
        runner = make_runner(S, L, R, shard_first(rank, R, S))
    dev = "cuda" if on_gpu else "cpu"

    def barrier():
        if ws > 1:
            dist.barrier()

    for i in range(args.warmup):
        runner.step(i)
    runner.sync()

    marks = runner.make_events(args.steps, args.event_every)
    barrier()
    runner.sync()
    t0 = time.perf_counter()
    runner.launch_steps(args.warmup, args.steps, args.event_every, marks)
    runner.sync()
    barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = runner.segment_ms(args.steps, args.event_every, marks)
    runner.check()

    t = torch.tensor([elapsed, statistics.mean(kern_ms)], dtype=torch.float64, device=dev)
    if ws > 1:
        parts = [torch.zeros_like(t) for _ in range(ws)]
        dist.all_gather(parts, t)
        per_rank = [(float(p[0].item()), float(p[1].item())) for p in parts]
    else:
        per_rank = [(elapsed, statistics.mean(kern_ms))]
    tmax = max(e for e, _ in per_rank)
    kern_avg_ms = max(k for _, k in per_rank)

    res = None
    if rank == 0:
        total_payload = (args.steps * S_job * L) if args.strong else (ws * args.steps * S * L)
        res = build_result(args, ws, S, L, R, tmax, kern_avg_ms, kern_ms, total_payload)
        res["config"]["world_size_seen"] = seen_ws
        res["config"]["dist_backend"] = (dist.get_backend() if dist.is_initialized() else "none (one process)")
        # per-GPU achieved B/t separates a latency bound from a scaling bug
        B = algorithmic_bytes(S, L)
        res["per_gpu"] = [{"rank": r, "payload_gibs": round(args.steps * S * L / e / GIB, 3),
                           "kernel_avg_us": round(k * 1e3, 3),
                           "achieved_gbs": round(B / (k * 1e-3) / 1e9, 2)}
                          for r, (e, k) in enumerate(per_rank)]
        if args.cpu_seconds > 0 and ws == 1 and make_runner is None:
            res["cpu_baseline"] = cpu_baseline(args, S, L)
        else:
            res["cpu_baseline"] = None
    if ws > 1:
        dist.barrier()
        if own_pg:
            dist.destroy_process_group()
    return res, runner


CONFIG_SHAPES = {"cfg2": (4096, 1024), "cfg3": (65536, 256), "cfg4": (1024, 65536),
                 "cfg5": (524288, 1024)}
COMPANION_BASES = {"cfg2"}     # workloads whose line carries the configs[4] companion
CONFIG_TEXT = {"cfg2": "4096 sessions x 1 KiB per GPU (BASELINE configs[1])",
               "cfg3": "65536 sessions x 256 B per GPU (BASELINE configs[2])",
               "cfg4": "1024 sessions x 64 KiB per GPU (BASELINE configs[3])",
               "cfg5": "524288 sessions x 1 KiB per GPU (BASELINE configs[4] total)"}


def latency_ceiling(S: int, L: int, cyc_per_byte: float, clock_ghz: float = 2.4,
                    resident: int = 131072) -> float:
    """Chain-bound payload rate (GiB/s): min(S, resident) chains x clock / cycles-per-byte."""
    return min(S, resident) * clock_ghz * 1e9 / cyc_per_byte / GIB


def build_result(args, ws, S, L, R, tmax, kern_avg_ms, kern_ms, total_payload):
    value = total_payload / tmax / GIB
    B = algorithmic_bytes(S, L)
    achieved = B / (kern_avg_ms * 1e-3) / 1e9
    ids = getattr(args, "ids", "range")
    traffic, traffic_src = load_traffic(args.workload if ids == "range" else f"{args.workload}-{ids}")
    return {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": ws,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(tmax / args.steps * 1e3, 5),
        "higher_is_better": True,
        "scaling": "strong" if args.strong else "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (mt19937_64 keys seed 1, payload seed 42, pre-advance (sid*37)%1000)",
        "config": {"workload": (f"{args.workload}: {S * ws} sessions x {L} B job total, {S} per GPU "
                                f"(strong scaling; BASELINE configs[4] when cfg5)" if args.strong
                                else f"{args.workload}: {CONFIG_TEXT[args.workload]}"),
                   "sessions_per_gpu": S, "payload_bytes_per_session": L,
                   "global_sessions_per_step": S * ws, "rotation_batches_per_gpu": R,
                   "job": ("fixed total split across ranks (strong)" if args.strong
                           else "per-GPU batch replicated over ranks' own sessions (weak)"),
                   "footprint_mib_per_gpu": round(R * S * (L + 256) / 2**20, 1),
                   "parallelism": f"shard{ws} (sessions split across GPUs, no collective)",
                   "curve": (f"strong: {args.workload}'s {S * ws} sessions split over {ws} GPU(s)" if args.strong
                             else f"weak: {args.workload} per GPU on each of {ws} GPU(s); the strong configs[4] "
                                  f"split is 'configs4_strong' (or --workload cfg5 --strong)"),
                   "slot_ids": getattr(args, "ids", "range")},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                     "traffic": traffic,
                     "traffic_source": traffic_src,
                     "kernel": kernel_name(S, getattr(args, "ids", "range")),
                     "algorithmic_bytes_per_launch": B,
                     "kernel_avg_us": round(kern_avg_ms * 1e3, 3),
                     "kernel_min_segment_us": round(min(kern_ms) * 1e3, 3),
                     # the first event to the last over the whole timed region, per step:
                     # every launch and inter-launch gap, not the host's first-launch
                     # latency or its wake-up after the last kernel (ms_per_step has both)
                     "device_us_per_step": round(sum(k * min(args.event_every, args.steps - i * args.event_every)
                                                     for i, k in enumerate(kern_ms)) / args.steps * 1e3, 3),
                     "kernel_timing": f"HIP events bracketing {len(kern_ms)} segments of "
                                      f"{args.event_every} back-to-back timed launches (per-launch average)"},
        "latency_ceiling_gibs": {"note": "chain-bound payload rate min(S,131072 resident)*2.4GHz/L_cyc per "
                                         "stream: L46 = 16 lanes per stream (crypt_win_kernel, <= 32 groups), "
                                         "L96 = one lane per stream, L130 = one lane at 8 waves/CU",
                                 "L46": round(latency_ceiling(S, L, 46), 1),
                                 "L96": round(latency_ceiling(S, L, 96), 1),
                                 "L130": round(latency_ceiling(S, L, 130), 1)},
    }


WIN_MAX_GROUPS = 32   # zrc4.hip ZRC4_WIN_MAX_GROUPS


def kernel_name(S: int, ids: str = "range") -> str:
    """The kernel the bench's crypt call launches for S sessions (zrc4.hip
    launch_crypt): at most WIN_MAX_GROUPS groups (range batches from an
    aligned first slot, or grouped buckets) -> 16 lanes per stream
    (crypt_win_kernel); 2G <= CUs -> half-group workgroups; G <= CUs -> one
    group per workgroup; more groups than CUs -> the persistent throughput
    kernel (grouped buckets: its grouped form).  Scattered ids run the
    per-lane gather forms."""
    try:
        import torch
        cus = torch.cuda.get_device_properties(0).multi_processor_count
    except Exception:
        cus = 256
    groups = -(-S // 256)
    mode = {"range": 1, "grouped": 2, "declared": 2, "scattered": 0}[ids]
    if ids == "scattered":
        return "zrc4::crypt_stream_kernel<false, false, false>" if groups > cus else "zrc4::crypt_kernel<0, false>"
    if groups <= WIN_MAX_GROUPS:
        return f"zrc4::crypt_win_kernel<{mode}, false, {'true' if ids == 'declared' else 'false'}>"
    if ids == "declared" and groups <= 256:
        return f"zrc4::crypt_decl_kernel<false, {'true' if 2 * groups <= cus else 'false'}>"
    if 2 * groups <= cus:
        return f"zrc4::crypt_half_kernel<{mode}, false>"
    if groups <= cus:
        return f"zrc4::crypt_kernel<{mode}, false>"
    return ("zrc4::crypt_stream_kernel<true, true, false>" if ids in ("grouped", "declared")
            else "zrc4::crypt_stream_kernel<true, false, false>")


def load_traffic(workload: str):
    """HBM bytes per launch from the committed rocprofv3 PMC summary, if any:
    (bytes, where they come from).  The PMC passes run in their own rocprofv3
    processes (scripts/pmc_traffic.sh), never inside this bench run."""
    p = ROOT / "profiles" / f"pmc_{workload}.json"
    if not p.exists():
        return None, None
    try:
        d = json.loads(p.read_text())
        src = (f"profiles/pmc_{workload}.json (round {d.get('round', '?')}, builder's rocprofv3 FETCH_SIZE + "
               f"WRITE_SIZE passes over bench.py --workload {d.get('workload', workload)}; kernel "
               f"{d.get('kernel', '?')}; not measured in this run)")
        return d.get("hbm_bytes_per_launch"), src
    except Exception:
        return None, None


# ------------------------------------------------------------- CPU baseline
def cgroup_cpu_quota():
    """The container's CPU quota (cgroup v2 cpu.max / v1 cfs), or None."""
    try:
        q, per = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except Exception:
        pass
    try:
        q = int(Path("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read_text())
        per = int(Path("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read_text())
        return None if q <= 0 else round(q / per, 2)
    except Exception:
        return None


def usable_cpus():
    """CPUs this process can run on at once: the affinity mask, capped by the
    cgroup CPU quota (a 16-CPU quota on a 256-core host is 16, not 256).
    Returns (usable, affinity_cores, quota)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except Exception:
        aff = os.cpu_count() or 1
    quota = cgroup_cpu_quota()
    usable = aff if quota is None else max(1, min(aff, math.ceil(quota)))
    return usable, aff, quota


def cpu_baseline(args, S, L):
    """The reference's own RC4 (RC4Encryption from depends/rc4/rc4_encryption.h,
    compiled -O3 from where it lies into oracle/_ref/libzrc4_ref.so; kind
    "reference") -- or, where that build is absent, the oracle restatement (a
    -O3 C port of rc4_encryption.h:74-93; kind "port") -- timed on this host
    on a bounded sample of the same workload (same keys, payload and
    pre-advance as rank 0's first batch): 1 thread (the reference's single
    event-loop thread), then one worker per CPU the process can use at once
    (usable_cpus: affinity mask capped by the cgroup quota), each re-crypting
    its contiguous share for the whole window.  Reported, not optimised
    against."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import pyoracle  # cpu_baseline leg only
    from zsummerx_amd import synth

    cores, aff, quota = usable_cpus()
    if args.cpu_threads > 0:
        cores = min(cores, args.cpu_threads)
    w = synth.make(0, S, L, threads=8)
    if pyoracle.ref_lib() is not None:
        kind, ob = "reference", pyoracle.RefBatch(S)
        ob.make_sbox(w.keys, w.key_off, w.key_len)
        ob.advance(w.adv)
        what = "RC4Encryption::encryption, the reference header compiled -O3 (oracle/_ref)"
    else:
        kind, ob = "port", pyoracle.Batch(S)
        ob.make_sbox(w.keys, w.key_off, w.key_len)
        ob.crypt(np.zeros(1000, dtype=np.uint8), np.zeros(S, dtype=np.uint64), w.adv)
        what = "the oracle restatement of rc4_encryption.h:74-93 (-O3); oracle/_ref absent"
    pay = w.payload.copy()
    reps = 5
    win = args.cpu_seconds / 2 / reps

    def rate(threads):
        return statistics.median(ob.crypt_rate(pay, w.off, w.length, threads, win) for _ in range(reps)) / GIB

    one = rate(1)
    many = rate(cores) if cores > 1 else one
    return {"value": round(many, 4), "unit": "GiB/s", "cores": cores, "threads": cores, "kind": kind,
            "value_1thread": round(one, 4), "hardware_concurrency": os.cpu_count(),
            "affinity_cores": aff, "cgroup_cpu_quota": quota,
            "sample": f"{what}: {args.workload} batch ({S} x {L} B) re-crypted for {win:.1f} s windows, median of "
                      f"{reps}: 1 thread, then {cores} threads (min(affinity {aff}, ceil(cgroup quota {quota})))"}


# ------------------------------------------------------- host-inclusive rate
def host_chunks(nbytes: int) -> int:
    """Default pipelining depth of the copy path (r03, tools/hostinc_sweep.py,
    profiles/r03/hostinc_sweep.log and hostinc/): the box's pinned copies run
    at ~57 GB/s whether one direction or both are busy, so chunking only hides
    the kernel (25 us to 0.3 ms against 0.15-19 ms of copies) and costs a
    per-copy latency: whole batches up to 32 MiB (cfg2 18.4 GiB/s whole vs
    11.1 in 8 chunks), one chunk per 32 MiB above, at most 16 (cfg5 29.9 in
    16 chunks on 4 streams vs 26.2 whole)."""
    mib = nbytes >> 20
    return 1 if mib <= 32 else max(1, min(16, mib // 32))


def host_inclusive(args):
    """The path starts in a socket recv buffer and ends in a send buffer, so
    the rate including PCIe is measured too (reported in DESIGN.md, never as
    `value`): pinned host payload, sessions split into --chunks chunks pipelined
    over --streams HIP streams (H2D -> zrc4_crypt_range -> D2H per chunk), wall
    clock from the first H2D to the last D2H, median of --steps passes."""
    import torch
    from zsummerx_amd import Context, synth
    S, L = CONFIG_SHAPES[args.workload]
    dev = torch.device("cuda", 0)
    ctx = Context(0, S)
    w = synth.make(0, S, L, threads=8)
    T = lambda a: torch.from_numpy(a).to(dev)
    ctx.ksa(T(w.key_len.view(np.int32)), T(w.key_off.view(np.int64)), T(w.keys))
    ctx.crypt(torch.zeros(1000, dtype=torch.uint8, device=dev), torch.zeros(S, dtype=torch.int64, device=dev),
              T(w.adv.view(np.int32)))
    ctx.sync()
    host = torch.from_numpy(w.payload).pin_memory()
    devbuf = torch.empty(S * L, dtype=torch.uint8, device=dev)
    off = T(w.off.view(np.int64))
    ln = T(w.length.view(np.int32))
    chunks = args.chunks or host_chunks(S * L)
    nchunk = max(1, min(chunks, S // 256))
    per = -(-S // nchunk)
    per = -(-per // 256) * 256                      # whole 256-slot groups per chunk
    streams = [torch.cuda.Stream(dev) for _ in range(max(1, args.streams))]
    times = []
    if getattr(args, "ids", "range") != "range" and args.zero_copy:
        # The session engine's own path: its receive / send blocks live in a
        # pinned SessionBlock pool, and each event-loop iteration runs ONE
        # zrc4_crypt_grouped_declared over them in place (buckets built and
        # declared on the host; device ids / offsets / lengths).  Slots in
        # random order inside each group, groups in random order.
        if S % 256:
            raise SystemExit("--ids declared --zero-copy needs whole groups")
        rng = np.random.default_rng(77)
        order = rng.permutation(S // 256)
        ids = np.concatenate([g * 256 + rng.permutation(256) for g in order]).astype(np.uint32)
        d_ids = T(ids.view(np.int32))
        d_off = T((ids.astype(np.int64) * L))
        d_len = T(np.full(S, L, dtype=np.int32))
        groups = order.astype(np.uint32)
        st = streams[0]
        # as the engine's hooks do (rc4_hooks_device.cpp): declared up to 256
        # buckets, zrc4_crypt_grouped above (the buckets are the same)
        launch = ((lambda: ctx.crypt_grouped_declared(host, d_off, d_len, d_ids, groups, stream=st))
                  if groups.size <= 256 else (lambda: ctx.crypt_grouped(host, d_off, d_len, d_ids, stream=st)))
        for it in range(args.warmup + args.steps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            launch()
            torch.cuda.synchronize()
            if it >= args.warmup:
                times.append(time.perf_counter() - t0)
        ctx.sync(st)
        t = statistics.median(times)
        return {"metric": "RC4 GiB/s host-inclusive (engine path: grouped buckets, declared up to 256, on pinned host blocks)",
                "value": round(S * L / t / GIB, 3), "unit": "GiB/s", "ms_per_pass": round(t * 1e3, 4),
                "workload": args.workload, "ids": "declared buckets, random slot and group order",
                "pcie_bytes_per_pass": 2 * S * L, "note": "not the headline value (DESIGN.md)"}
    if getattr(args, "ids", "range") != "range":
        # The engine's shape through the host-pointer C-ABI: zrc4_crypt_host
        # with the sessions' slot ids in random order; the library buckets
        # them by group on the host, declares each bucket's group
        # (zrc4_crypt_grouped_declared) and moves the payload through its
        # pinned staging (zero-copy up to 256 KiB, device copies above).
        rng = np.random.default_rng(77)
        ids = rng.permutation(S).astype(np.uint32)
        hoff = (ids.astype(np.uint64) * L)
        hlen = np.full(S, L, dtype=np.uint32)
        buf = w.payload.copy()
        for it in range(args.warmup + args.steps):
            t0 = time.perf_counter()
            ctx.crypt_host(buf, hoff, hlen, ids=ids)
            if it >= args.warmup:
                times.append(time.perf_counter() - t0)
        t = statistics.median(times)
        return {"metric": "RC4 GiB/s host-inclusive (zrc4_crypt_host: host ids bucketed and declared by the library)",
                "value": round(S * L / t / GIB, 3), "unit": "GiB/s", "ms_per_pass": round(t * 1e3, 4),
                "workload": args.workload, "ids": "random slot order, bucketed on the host",
                "pcie_bytes_per_pass": 2 * S * L, "note": "not the headline value (DESIGN.md)"}
    if args.zero_copy:
        # the kernels read and write the pinned host buffer in place over PCIe
        # (the session engine's pinned SessionBlock pool does the same)
        st = streams[0]
        for it in range(args.warmup + args.steps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ctx.crypt_range(0, host, off, ln, n=S, stream=st)
            torch.cuda.synchronize()
            if it >= args.warmup:
                times.append(time.perf_counter() - t0)
        ctx.sync(st)
        t = statistics.median(times)
        return {"metric": "RC4 GiB/s host-inclusive (zero-copy: kernels on pinned host memory)",
                "value": round(S * L / t / GIB, 3), "unit": "GiB/s", "ms_per_pass": round(t * 1e3, 4),
                "workload": args.workload, "pcie_bytes_per_pass": 2 * S * L,
                "note": "not the headline value (DESIGN.md)"}
    for it in range(args.warmup + args.steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for c, s0 in enumerate(range(0, S, per)):
            n = min(per, S - s0)
            st = streams[c % len(streams)]
            a, z = s0 * L, (s0 + n) * L
            with torch.cuda.stream(st):
                devbuf[a:z].copy_(host[a:z], non_blocking=True)
                ctx.crypt_range(s0, devbuf, off[s0:], ln[s0:], n=n, stream=st)
                host[a:z].copy_(devbuf[a:z], non_blocking=True)
        torch.cuda.synchronize()
        if it >= args.warmup:
            times.append(time.perf_counter() - t0)
    ctx.sync()
    t = statistics.median(times)
    return {"metric": "RC4 GiB/s host-inclusive (pinned H2D -> kernel -> D2H)",
            "value": round(S * L / t / GIB, 3), "unit": "GiB/s", "ms_per_pass": round(t * 1e3, 4),
            "workload": args.workload, "chunks": nchunk, "streams": len(streams),
            "pcie_bytes_per_pass": 2 * S * L, "note": "not the headline value (DESIGN.md)"}


# ------------------------------------------------- connection-storm KSA rate
def ksa_storm(args):
    """a connection storm re-seeds every session at once
    (RC4Encryption::makeSBox, rc4_encryption.h:46-72; two streams per session,
    src/frame/session.cpp:110-111).  K launches of zrc4_ksa_range over all S
    slots of the workload with device-resident 16-byte keys, timed with HIP
    events over 16-launch segments; the CPU baseline is the oracle's
    make_sbox on a bounded sample (1 thread, like the event-loop thread).
    Reported in DESIGN.md; never the headline `value`."""
    import torch
    from zsummerx_amd import Context, synth
    S, _ = CONFIG_SHAPES[args.workload]
    KL = int(getattr(args, "key_len", 16))
    dev = torch.device("cuda", 0)
    ctx = Context(0, S)
    # 16-byte keys: the synthetic sessions' own keys; other lengths: seeded
    # random bytes (the key schedule's register / window / fetch paths,
    # DESIGN.md §3.7)
    keys = synth.keys(0, S).reshape(-1) if KL == 16 else \
        np.random.default_rng(5).integers(0, 256, S * KL, dtype=np.uint8)
    T = lambda a: torch.from_numpy(a).to(dev)
    kl = T(np.full(S, KL, dtype=np.int32))
    ko = T(np.arange(S, dtype=np.int64) * KL)
    kd = T(keys)
    st = torch.cuda.current_stream(dev)
    for _ in range(args.warmup):
        ctx.ksa_range(0, kl, ko, kd, n=S, stream=st)
    torch.cuda.synchronize()
    seg = []
    done = 0
    t0 = time.perf_counter()
    while done < args.steps:
        m = min(args.event_every, args.steps - done)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        for _ in range(m):
            ctx.ksa_range(0, kl, ko, kd, n=S, stream=st)
        b.record(st)
        seg.append((a, b, m))
        done += m
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ctx.sync()
    per = statistics.median(a.elapsed_time(b) / m for a, b, m in seg) * 1e-3   # s per launch
    out = {"metric": "RC4 KSA streams/s (batched makeSBox, connection storm)",
           "value": round(S / per, 1), "unit": "streams/s", "workload": args.workload,
           "streams_per_launch": S, "key_bytes": KL, "kernel_us": round(per * 1e6, 3),
           "ns_per_stream": round(per * 1e9 / S, 4), "wall_streams_per_s": round(S * args.steps / wall, 1),
           "algorithmic_bytes_per_launch": S * (KL + 8 + 4 + STATE_BYTES // 2),
           "note": "key + offset/len read, 258-B state written per stream; not the headline value"}
    if args.cpu_seconds > 0:
        sys.path.insert(0, str(ROOT / "oracle"))
        import pyoracle  # cpu_baseline leg only
        n = min(S, 65536)
        ob = pyoracle.Batch(n)
        kh = keys[: KL * n]
        offs = np.arange(n, dtype=np.uint64) * KL
        lens = np.full(n, KL, dtype=np.uint32)
        runs, t_end = [], time.perf_counter() + args.cpu_seconds
        while len(runs) < 5 or time.perf_counter() < t_end:
            t1 = time.perf_counter()
            ob.make_sbox(kh, offs, lens)
            runs.append(n / (time.perf_counter() - t1))
            if len(runs) >= 50:
                break
        cpu = statistics.median(runs)
        out["cpu_baseline"] = {"value": round(cpu, 1), "unit": "streams/s", "cores": 1, "kind": "port",
                               "sample": f"{n} x {KL}-byte keys, oracle make_sbox batch, median of {len(runs)} runs"}
        out["speedup_vs_1_core"] = round(S / per / cpu, 1)
    return out


# ------------------------------------------------- device-side framing scan
def frame_payload(S: int, L: int, seed: int = 7):
    """S session buffers of L bytes of proto4z packets (length fields drawn
    from 6..min(700, L/2+6)), the last packet cut at the buffer end: what a
    recv block holds after the decrypt.  Returns (buffers, complete packets)."""
    rng = np.random.default_rng(seed)
    buf = np.zeros(S * L, dtype=np.uint8)
    hi = min(700, L // 2 + 6)
    lens = rng.integers(6, hi + 1, size=(S, max(4, 2 * L // 6)))
    complete = 0
    for s in range(S):
        pos, k = 0, 0
        while pos + 4 <= L:
            ln = int(lens[s, k % lens.shape[1]])
            k += 1
            buf[s * L + pos: s * L + pos + 4] = np.frombuffer(ln.to_bytes(4, "little"), np.uint8)
            complete += pos + ln <= L
            pos += ln
    return buf, complete


def frame_bench(args):
    """zrc4_frame_scan (TcpSession::onRecv's framing loop,
    src/frame/session.cpp:329-371, over HasRawPacket, proto4z.h:704-748) on
    decrypted, device-resident buffers shaped like the workload; K launches
    timed with HIP events over 16-launch segments, next to the crypt kernel on
    the same batch.  CPU baseline: the oracle's scan, 1 thread (the reference
    frames on its single event-loop thread).  Reported in DESIGN.md; never the
    headline `value`."""
    import torch
    from zsummerx_amd import Context
    S, L = CONFIG_SHAPES[args.workload]
    S = min(S, 524288)
    dev = torch.device("cuda", 0)
    buf, npk_total = frame_payload(S, L)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    d_buf = T(buf)
    d_off = T(np.arange(S, dtype=np.int64) * L)
    d_len = T(np.full(S, L, dtype=np.int32))
    npk, used, status = (torch.zeros(S, dtype=torch.int32, device=dev) for _ in range(3))
    st = torch.cuda.current_stream(dev)
    with Context(0, S) as ctx:
        def timed(fn):
            for _ in range(args.warmup):
                fn()
            torch.cuda.synchronize()
            seg, done = [], 0
            while done < args.steps:
                m = min(args.event_every, args.steps - done)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(st)
                for _ in range(m):
                    fn()
                b.record(st)
                seg.append((a, b, m))
                done += m
            torch.cuda.synchronize()
            return statistics.median(a.elapsed_time(b) / m for a, b, m in seg) * 1e-3
        bound = max(20480, L)          # SESSION_BLOCK_SIZE (config.h:100); cfg4's 64 KiB needs a larger block
        scan = lambda: ctx.frame_scan(d_buf, d_off, d_len, bound, npk, used, status, stream=st)
        t_scan = timed(scan)
        ctx.sync(st)
        got_npk = int(npk.sum().item())
        scratch = T(np.zeros(S * L, dtype=np.uint8))
        # Decrypt + frame: each session's block = [L bytes of packets | L-byte
        # fresh tail]; the tail is decrypted, the packet part framed (kept out
        # of the decrypt so repeated launches frame the same packets).  Fused
        # (zrc4_crypt_range_frame / zrc4_crypt_grouped_frame: one launch) vs
        # two launches (the crypt, then zrc4_frame_scan).  --ids grouped:
        # entries bucketed by group, slots permuted inside each group and the
        # groups in random order (the session engine's shape).
        blk = np.zeros(S * 2 * L, dtype=np.uint8)
        blk.reshape(S, 2 * L)[:, :L] = buf.reshape(S, L)
        d_blk = T(blk)
        perm = np.arange(S, dtype=np.int64)
        if args.ids == "grouped":
            rng = np.random.default_rng(77)
            pos = 0
            for g in rng.permutation(-(-S // 256)):
                lo, hi = g * 256, min((g + 1) * 256, S)
                perm[pos:pos + hi - lo] = lo + rng.permutation(hi - lo)
                pos += hi - lo
        d_ids = T(perm.astype(np.int32))
        f_off = T(perm * 2 * L)
        t_off = T(perm * 2 * L + L)
        if args.ids == "grouped":
            crypt = lambda p, o: ctx.crypt_grouped(p, o, d_len, d_ids, n=S, stream=st)
            fused = lambda fr: ctx.crypt_grouped_frame(d_blk, t_off, d_len, d_ids, fr, n=S, stream=st)
        else:
            crypt = lambda p, o: ctx.crypt_range(0, p, o, d_len, n=S, stream=st)
            fused = lambda fr: ctx.crypt_range_frame(0, d_blk, t_off, d_len, fr, n=S, stream=st)
        d_off_e = T(perm * L)                            # entry e -> session perm[e]'s L bytes of scratch
        t_crypt = timed(lambda: crypt(scratch, d_off_e))
        ctx.sync(st)
        frame = {"off": f_off, "len": d_len, "bound": bound, "npk": npk, "used": used, "status": status}
        t_fused = timed(lambda: fused(frame))
        ctx.sync(st)
        fused_npk = int(npk.sum().item())

        def two_launches():
            crypt(d_blk, t_off)
            ctx.frame_scan(d_blk, f_off, d_len, bound, npk, used, status, stream=st)
        t_two = timed(two_launches)
        ctx.sync(st)
    out = {"metric": "proto4z frame scan (device-resident, decrypted buffers)", "workload": args.workload,
           "ids": args.ids, "sessions": S, "bytes_per_session": L, "packets_per_launch": got_npk,
           "packets_expected": npk_total, "kernel_us": round(t_scan * 1e6, 3),
           "framed_gib_s": round(S * L / t_scan / GIB, 2), "packets_per_s": round(got_npk / t_scan, 1),
           "crypt_kernel_us_same_batch": round(t_crypt * 1e6, 3),
           "scan_share_of_decrypt_plus_scan": round(t_scan / (t_scan + t_crypt), 4),
           "fused_decrypt_frame_us": round(t_fused * 1e6, 3), "two_launches_us": round(t_two * 1e6, 3),
           "fused_saves_us": round((t_two - t_fused) * 1e6, 3),
           "note": "scan reads 4 header bytes per packet; latency-bound chain of header reads per session"}
    if args.cpu_seconds > 0:
        sys.path.insert(0, str(ROOT / "oracle"))
        import pyoracle  # cpu_baseline leg only
        off = np.arange(S, dtype=np.uint64) * L
        ln = np.full(S, L, dtype=np.uint32)
        runs, t_end = [], time.perf_counter() + args.cpu_seconds
        while len(runs) < 5 or time.perf_counter() < t_end:
            t1 = time.perf_counter()
            pyoracle.frame_scan(buf, off, ln, max(20480, L), 0)
            runs.append(time.perf_counter() - t1)
            if len(runs) >= 50:
                break
        cpu = statistics.median(runs)
        out["cpu_baseline"] = {"value": round(S * L / cpu / GIB, 3), "unit": "GiB/s framed", "cores": 1,
                               "kind": "port", "sample": f"the same {S} buffers, oracle_frame_scan, median of {len(runs)}"}
        out["speedup_vs_1_core"] = round(cpu / t_scan, 1)
    assert got_npk == npk_total, (got_npk, npk_total)
    assert fused_npk == npk_total, (fused_npk, npk_total)
    return out


def parse(argv=None):
    p = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--workload", choices=sorted(CONFIG_SHAPES), default="cfg2")
    p.add_argument("--strong", action="store_true",
                   help="the workload's sessions are the whole job, split across ranks (BASELINE configs[4])")
    p.add_argument("--footprint-mib", type=int, default=640,
                   help="rotate over distinct batches totalling this many MiB per GPU (0 = one batch)")
    p.add_argument("--cpu-seconds", type=float, default=10.0,
                   help="CPU baseline time budget on rank 0 at N=1 (0 disables)")
    p.add_argument("--cpu-threads", type=int, default=0,
                   help="cap on CPU-baseline threads (0 = every core in the affinity mask)")
    p.add_argument("--ids", choices=["range", "grouped", "declared", "scattered"], default="range",
                   help="slot addressing: contiguous range (zrc4_crypt_range), scattered slots bucketed by group "
                        "(zrc4_crypt_grouped), the same with each bucket's group declared from the host "
                        "(zrc4_crypt_grouped_declared, the engine's path) or the same ids unbucketed (zrc4_crypt)")
    p.add_argument("--event-every", type=int, default=16,
                   help="launches per HIP-event segment (kernel duration = segment time / N)")
    p.add_argument("--host-inclusive", action="store_true",
                   help="measure the PCIe-inclusive rate instead (DESIGN.md), one JSON line")
    p.add_argument("--key-len", type=int, default=16, help="with --ksa: key bytes per session")
    p.add_argument("--ksa", action="store_true",
                   help="measure the connection-storm KSA rate instead (DESIGN.md), one JSON line")
    p.add_argument("--frame", action="store_true",
                   help="measure the device-side proto4z framing scan instead (DESIGN.md), one JSON line")
    p.add_argument("--zero-copy", action="store_true",
                   help="with --host-inclusive: run the kernels directly on the pinned host buffer")
    p.add_argument("--companion-workload", choices=sorted(CONFIG_SHAPES) + ["none"], default="cfg5",
                   help="with the default weak cfg2 line: also measure this workload split over the same ranks "
                        "(strong scaling, BASELINE configs[4]) as 'configs4_strong'; none disables")
    p.add_argument("--no-shard-projection", dest="shard_projection", action="store_false",
                   help="N=1 only: skip timing the companion's 2/4/8-GPU shards on this GPU "
                        "(configs4_strong.shard_projection)")
    p.add_argument("--companion-steps", type=int, default=100)
    p.add_argument("--companion-warmup", type=int, default=120)
    p.add_argument("--chunks", type=int, default=0,
                   help="with --host-inclusive: chunks of the batch (0 = by size, host_chunks: one up to 32 MiB, "
                        "else one per 32 MiB, at most 16; tools/hostinc_sweep.py)")
    p.add_argument("--streams", type=int, default=4)
    p.add_argument("--rehearse-one-gpu", action="store_true",
                   help="N > 1 on a one-GPU box: every rank on cuda:0 over gloo (scripts/r06_rehearse.sh); "
                        "exercises the multi-rank path end to end, its times are no scaling measurement")
    return p.parse_args(argv)


def free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def self_launch(argv, n: int, entry=None, timeout: float | None = None) -> int:
    """`--gpus N` without torchrun: start N rank processes of `entry` (default
    this file) with the environment torchrun would give them (RANK,
    LOCAL_RANK, WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT), relay rank
    0's JSON line to stdout and return the first non-zero exit code (0 when
    every rank succeeded).  The parent never touches the GPU and never execs:
    the ranks are child processes.  When one rank fails the others are
    terminated (they would otherwise wait at the barrier)."""
    import subprocess
    import tempfile
    entry = str(entry or Path(__file__).resolve())
    port = free_port()
    out0 = tempfile.TemporaryFile(mode="w+")
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, entry, *argv], env=env,
                                      stdout=out0 if r == 0 else 2))      # other ranks: stdout -> our stderr
    log(f"[self_launch] {n} ranks of {Path(entry).name}, master 127.0.0.1:{port}, pids {[p.pid for p in procs]}")
    deadline = None if timeout is None else time.time() + timeout
    rc = 0
    while True:
        codes = [p.poll() for p in procs]
        bad = [c for c in codes if c not in (None, 0)]
        if bad or all(c is not None for c in codes):
            rc = bad[0] if bad else 0
            break
        if deadline is not None and time.time() > deadline:
            rc = 124
            break
        time.sleep(0.1)
    if rc:
        log(f"[self_launch] a rank exited with {rc}: stopping the others")
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(15)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    out0.seek(0)
    lines = [ln for ln in out0.read().splitlines() if ln.startswith("{")]
    if not rc and not lines:
        log("[self_launch] rank 0 printed no JSON line")
        rc = 1
    if lines:
        print(lines[-1], flush=True)
    return rc


def companion_strong(args, ws, rank, local, backend="nccl", make_runner=None):
    """BASELINE configs[4] -- 524 288 sessions x 1 KiB split over the job's
    ranks (strong scaling) -- measured in the same job as the weak cfg2 line,
    so one 1/2/4/8 sweep yields both curves.  Same barrier / max-over-ranks
    timing; steady-state warmup (the clock dips over the first ~100 cfg5
    launches)."""
    c = argparse.Namespace(**vars(args))
    c.workload, c.strong, c.cpu_seconds, c.ids = args.companion_workload, True, 0.0, "range"
    c.steps = max(args.steps, args.companion_steps)
    c.warmup = max(args.warmup, args.companion_warmup)
    res, runner = run_bench(c, ws, rank, local, backend, make_runner, own_pg=False)
    proj = None
    if ws == 1 and make_runner is None and getattr(args, "shard_projection", True) and res is not None:
        proj = shard_projection(c, runner, res)
    if hasattr(runner, "close"):
        runner.close()
    if res is None:
        return None
    keep = ("value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "scaling")
    out = {k: res[k] for k in keep}
    out["config"] = {k: res["config"][k] for k in ("workload", "sessions_per_gpu", "global_sessions_per_step",
                                                   "rotation_batches_per_gpu", "world_size_seen", "curve")}
    out["roofline"] = {k: res["roofline"][k] for k in ("achieved", "peak", "unit", "frac", "kernel",
                                                       "algorithmic_bytes_per_launch", "kernel_avg_us")}
    out["per_gpu"] = res["per_gpu"]
    if proj is not None:
        out["shard_projection"] = proj
    return out


def shard_projection(c, runner, res, gpus=(2, 4, 8)):
    """SURVEY.md §8e on one GPU: the per-GPU shard of the strong configs[4]
    split at N = 2, 4, 8 (524 288 / N sessions x 1 KiB), timed in the same
    job as the 1-GPU line with the same method (warmup, then HIP events over
    16-launch segments plus the sync-bracketed wall clock).  The shards are
    contiguous slot ranges of the companion's own batch, launched in rotation
    (shard k of N = slots [k S/N, (k+1) S/N)), so the rotation still covers the
    whole >= 640 MiB footprint.  Speed-ups are against the 1-GPU value measured
    just before: what N GPUs give if each runs its shard as this GPU does (no
    collective on the data path; the driver's SCALE run measures the real
    node)."""
    if runner.R != 1 or runner._fn.__name__ != "zrc4_crypt_range":
        return None
    h, first, pay, offp, lenp, S, st = runner._args[0]
    one_kern = res["roofline"]["kernel_avg_us"]
    one_step = res["ms_per_step"] * 1e3
    out = {"method": (f"{c.workload} shards of the 1-GPU batch on this GPU, rotated; {c.warmup} warmup "
                      f"launches, then {c.steps} timed: HIP events over {c.event_every}-launch segments"),
           "one_gpu_kernel_avg_us": one_kern, "one_gpu_us_per_step": round(one_step, 3), "shards": []}
    saved = (runner._args, runner.R)
    try:
        for n in gpus:
            if S % (256 * n):
                continue
            sn = S // n
            runner._args = [(h, first + k * sn, pay, C.c_void_p(offp.value + 8 * k * sn),
                             C.c_void_p(lenp.value + 4 * k * sn), sn, st) for k in range(n)]
            runner.R = n
            for i in range(c.warmup):
                runner.step(i)
            runner.sync()
            marks = runner.make_events(c.steps, c.event_every)
            t0 = time.perf_counter()
            runner.launch_steps(c.warmup, c.steps, c.event_every, marks)
            runner.sync()
            wall = time.perf_counter() - t0
            kern = statistics.mean(runner.segment_ms(c.steps, c.event_every, marks)) * 1e3
            B = algorithmic_bytes(sn, runner.L)
            out["shards"].append({
                "gpus": n, "sessions_per_gpu": sn, "kernel_avg_us": round(kern, 3),
                "us_per_step": round(wall / c.steps * 1e6, 3),
                "achieved_gbs": round(B / (kern * 1e-6) / 1e9, 2),
                "projected_speedup_kernel": round(one_kern / kern, 3),
                "projected_speedup_step": round(one_step / (wall / c.steps * 1e6), 3),
                "projected_job_gibs": round(n * sn * runner.L / (wall / c.steps) / GIB, 1)})
        runner.check()
    finally:
        runner._args, runner.R = saved
    return out


def rank_main(args, backend="nccl", make_runner=None):
    """One rank of the bench (torchrun's, self_launch's or the only one)."""
    import torch.distributed as dist
    ws, rank, local = dist_env()
    if getattr(args, "rehearse_one_gpu", False):
        backend, local = "gloo", 0
    if ws != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={ws}; using WORLD_SIZE")
    res, runner = run_bench(args, ws, rank, local, backend, make_runner, own_pg=False)
    if hasattr(runner, "close"):
        runner.close()
    del runner
    if args.companion_workload != "none" and not args.strong and args.workload in COMPANION_BASES \
            and getattr(args, "ids", "range") == "range":
        comp = companion_strong(args, ws, rank, local, backend, make_runner)
        if rank == 0:
            res["configs4_strong"] = comp
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        if getattr(args, "rehearse_one_gpu", False):
            res["config"]["rehearsal"] = "gloo, every rank on cuda:0: the multi-rank path, not a scaling measurement"
        print(json.dumps(res), flush=True)
    return res


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse(argv)
    if args.host_inclusive:
        print(json.dumps(host_inclusive(args)), flush=True)
        return
    if args.ksa:
        print(json.dumps(ksa_storm(args)), flush=True)
        return
    if args.frame:
        print(json.dumps(frame_bench(args)), flush=True)
        return
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(self_launch(argv, args.gpus))
    rank_main(args)


if __name__ == "__main__":
    main()
