"""Test-side bench runner: bench.GpuRunner's interface, backed by the CPU
oracle (test infrastructure: the oracle is the checker, never the product).
Used by the gloo multi-rank tests (tests/test_multirank.py) and by the
self-launched rank processes of tests/bench_child_cpu.py."""
import numpy as np


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
