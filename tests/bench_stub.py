"""A stub of fluidframework_amd.engine.Engine for the CPU tests of bench.py's multi-rank plumbing (test
infrastructure only: it records and "replays" its documents with the CPU oracle, so the counters, digests and
timing the bench reduces are real).  bench.py loads it only when MTR_BENCH_STUB_ENGINE names it, and then marks its
line `"engine": "stub"`.

BENCH_STUB_CORRUPT_RANK=r makes rank r report a wrong digest for its first document (the per-rank oracle sample
must catch it)."""
import os
import time

import numpy as np


class StubEngine:
    """The Engine methods bench.py's timed loop and its checker leg use, over oracle-recorded documents."""

    ops_per_doc = None

    def __init__(self, max_docs, **kw):
        self.n = max_docs
        self.hs = np.zeros(0, np.uint64)
        self.steps = 0

    def generate(self, cfg, tabs, grow=0):
        from oracle.oracle import generate, replay_batch
        self.batch, self.hs, st = generate(cfg, tabs, 0, int(cfg.n_docs), threads=2)
        assert not st.any()
        self.cfg = cfg
        # the replay the timed steps stand for (its digests must equal the recorded ones)
        _, h, st = replay_batch(self.batch, 0, int(cfg.n_docs), 2)
        assert (h == self.hs).all() and not st.any()
        bad = os.environ.get("BENCH_STUB_CORRUPT_RANK")
        if bad is not None and bad == os.environ.get("RANK"):
            self.hs = self.hs.copy()
            self.hs[0] ^= np.uint64(1)

    def download(self, lo, hi, pinned_memory=False):
        assert lo == 0
        return self.batch

    def reset(self):
        pass

    def run(self):
        time.sleep(0.02)  # (a step long enough for ms_per_step's 3 decimals)
        self.steps += 1

    def summarize(self):
        pass

    def sync(self):
        pass

    def timing(self):
        return {"apply_ms": 1.0, "summary_ms": 0.5, "apply_launches": 2, "apply_kernel_ms": 0.8}

    def stats(self):
        n = int(self.cfg.n_docs)
        return {"bad_docs": 0, "ops": n * (int(self.cfg.ops_per_doc) + 1), "sum_leaves_before_op": 1000 * n,
                "text_units_inserted": 10 * n, "max_leaves": 100, "max_heap": 10}

    def hashes(self, n=None):
        return self.hs[: n if n is not None else len(self.hs)]

    def summary_bytes(self):
        return 1234
