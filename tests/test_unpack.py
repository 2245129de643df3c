"""The host half of the packed spans (jb_capi.cpp unpack_spans): the decoder's
source is cut out of jb_capi.cpp, compiled on the CPU with stand-ins for the few library
names it uses (tests/host/unpack_harness_*.cpp), and run on random spans with escaped gaps
and lengths, escapes in bulk and none, outputs misaligned against each other and aligned
alike: the AVX-512 path (where the CPU has it) and the scalar path (JB_DECODE_AVX512=0)
must both give every span.  The packing itself runs on the GPU (test_packed_spans_escapes)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLANG = "/opt/rocm/lib/llvm/bin/clang++"


@pytest.mark.skipif(not os.path.exists(CLANG) and not shutil.which("clang++"), reason="no clang")
def test_unpack_spans_paths(tmp_path):
    src = open(os.path.join(ROOT, "jieba-go_amd", "csrc", "jb_capi.cpp")).read()
    a = src.index("// One token of a packed piece")
    b = src.index("// Text already in pinned memory (jb_host_alloc)")
    h = os.path.join(ROOT, "tests", "host")
    prog = tmp_path / "unpack.cpp"
    prog.write_text(open(os.path.join(h, "unpack_harness_head.cpp")).read() + src[a:b] +
                    open(os.path.join(h, "unpack_harness_main.cpp")).read())
    exe = str(tmp_path / "unpack")
    cc = CLANG if os.path.exists(CLANG) else shutil.which("clang++")
    subprocess.run([cc, "-O2", "-std=c++17", "-pthread", "-o", exe, str(prog)], check=True)
    for avx in ("1", "0"):
        r = subprocess.run([exe], capture_output=True, text=True, timeout=300,
                           env=dict(os.environ, JB_DECODE_AVX512=avx))
        assert r.returncode == 0 and r.stdout.strip() == "ok", (avx, r.stdout, r.stderr)
