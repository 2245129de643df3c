"""Test-only stand-ins for bench.py's measured path (CPU, no GPU): the rank's
"device" output is the oracle's, optionally with one token corrupted.  Used by
tests/test_multirank.py, directly (OracleCutter under bench.run) and through
bench.py's own N-rank launcher (OracleBackend via JB_BENCH_TEST_BACKEND)."""
import os


class OracleCutter:
    """Stands in for bench.GpuCutter on CPU."""

    def __init__(self, o, buf, off, hmm, corrupt=False):
        self.o, self.buf, self.off, self.hmm, self.corrupt = o, buf, off, hmm, corrupt
        self.steps = 0

    def step(self):
        self.steps += 1

    def sync(self):
        pass

    def profile(self, steps):
        return {}, None

    def results(self):
        s, e, d = self.o.cut_batch(self.buf, self.off, bool(self.hmm), nthreads=2)
        s = s.copy()
        if self.corrupt and len(s):
            s[len(s) // 2] += 1
        return s, e, d

    def ties(self):
        return 0


class OracleBackend:
    """bench.GpuBackend's interface over OracleCutter.  JB_TEST_DEVICES: the
    device count it reports (default 8); JB_TEST_CORRUPT_RANK: the rank whose
    output gets one wrong token (default none)."""
    name = "oracle-stand-in"

    def device_count(self):
        return int(os.environ.get("JB_TEST_DEVICES", "8"))

    def open(self, cfg_kw, local):
        import oracle as O
        self.o = O.Oracle.from_files(cfg_kw["dict_path"], cfg_kw["emit_path"], cfg_kw["kind"],
                                     cfg_kw["size_override"])
        return self.o

    def make_cutter(self, buf, off, hmm, local):
        bad = int(os.environ.get("JB_TEST_CORRUPT_RANK", "-1"))
        return OracleCutter(self.o, buf, off, hmm, corrupt=int(os.environ.get("RANK", "0")) == bad)

    def close(self):
        pass
