"""Shared fixtures.  CPU tests: oracle vs the reference's golden vectors, host
logic, library exports.  GPU tests (marked `gpu`): the MI355X path through the
C ABI against the oracle."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("oracle", "gen", os.path.join("jieba-go_amd", "python")):
    p = os.path.join(ROOT, sub)
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD Instinct GPU (gfx950) and the built HIP library")
    # the two CPU-side helper libraries build in a second; the HIP library is built by build()
    for d in ("oracle", "gen"):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, d)])


@pytest.fixture(scope="session")
def kats():
    with open(os.path.join(GOLDEN, "reference_kats.json"), encoding="utf-8") as f:
        return json.load(f)


@pytest.fixture(scope="session")
def mini_paths():
    return os.path.join(GOLDEN, "mini_dict.txt"), os.path.join(GOLDEN, "mini_emit.json")


def _syn_files(tmp_path_factory, nwords, name):
    import synth
    d = str(tmp_path_factory.mktemp(name))
    s = synth.Synth(nwords=nwords)
    dp, ep = s.write_files(d)
    return dp, ep, s


@pytest.fixture(scope="session")
def syn_small(tmp_path_factory):
    """20k-word synthetic dictionary + emission (fast)."""
    return _syn_files(tmp_path_factory, 20_000, "syn_small")


@pytest.fixture(scope="session")
def syn_full(tmp_path_factory):
    """350k-word D_syn + E_syn."""
    return _syn_files(tmp_path_factory, 350_000, "syn_full")


def real_data_dir():
    """Directory holding the genuine jieba LFS objects (checked by sha256), or None."""
    import hashlib
    d = os.environ.get("JIEBA_DATA_DIR")
    if not d:
        return None
    with open(os.path.join(GOLDEN, "reference_kats.json"), encoding="utf-8") as f:
        want = json.load(f)["real_data_sha256"]
    for name in ("dict.txt", "prob_emit.json"):
        p = os.path.join(d, name)
        if not os.path.exists(p):
            return None
        with open(p, "rb") as f:
            if hashlib.sha256(f.read()).hexdigest() != want[name]:
                return None
    return d


@pytest.fixture(scope="session")
def syn_golden(tmp_path_factory):
    """Committed golden vectors (tests/golden/syn_golden.json) and the regenerated
    synthetic data files they were made on (checked by sha256)."""
    import base64
    import hashlib
    with open(os.path.join(GOLDEN, "syn_golden.json")) as f:
        g = json.load(f)
    dp, ep, _ = _syn_files(tmp_path_factory, g["nwords"], "syn_golden")
    for name, p in (("dict.txt", dp), ("prob_emit.json", ep)):
        with open(p, "rb") as f:
            assert hashlib.sha256(f.read()).hexdigest() == g["sha256"][name], f"generator output changed: {name}"
    docs = [base64.b64decode(d) for d in g["docs_b64"]]
    return g, docs, dp, ep
