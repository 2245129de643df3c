"""CPU: the library's host code under AddressSanitizer + UndefinedBehaviorSanitizer.

Two programs, each built here with -fsanitize=address,undefined -fno-sanitize-recover=all:
- tests/host/image_fuzz.cpp over jieba-go_amd/csrc/jb_image.cpp (the dict.txt, gob and emission
  parsers, the image builder, its hot rows, save/load, lookups), one full pass on the synthetic
  dictionary and then mutation rounds against every parser and the image loader;
- the packed-spans decoder of jb_capi.cpp in its test harness (tests/test_unpack.py's program).
A report from either sanitizer fails the run.  (The GPU kernels cannot run under a sanitizer on
this pool; the host code they are fed by can.)"""
import os
import shutil
import subprocess

import pytest

import gobenc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]
CLANG = "/opt/rocm/lib/llvm/bin/clang++"
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")


def _gob_of(dict_path, out_path):
    items = {}
    with open(dict_path, encoding="utf-8") as f:
        for line in f:
            p = line.split()
            if len(p) >= 2:
                items[p[0]] = int(p[1])
    with open(out_path, "wb") as f:
        f.write(gobenc.encode_map(sorted(items.items())))


@pytest.mark.skipif(not shutil.which("g++"), reason="no g++")
def test_image_code_under_asan_ubsan(tmp_path, syn_small):
    dp, ep, _ = syn_small
    gob = str(tmp_path / "dict.gob")
    _gob_of(dp, gob)
    exe = str(tmp_path / "image_fuzz")
    src = os.path.join(ROOT, "jieba-go_amd", "csrc")
    subprocess.run(["g++", "-std=c++17", *SAN, "-I", os.path.join(ROOT, "include"), "-I", src,
                    "-I/opt/rocm/include", "-D__HIP_PLATFORM_AMD__", "-o", exe,
                    os.path.join(ROOT, "tests", "host", "image_fuzz.cpp"), os.path.join(src, "jb_image.cpp")],
                   check=True)
    r = subprocess.run([exe, dp, ep, gob, "400", "7"], capture_output=True, text=True, timeout=600, env=ENV)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stderr[-4000:]


@pytest.mark.skipif(not os.path.exists(CLANG), reason="no clang")
def test_span_decoder_under_asan_ubsan(tmp_path):
    src = open(os.path.join(ROOT, "jieba-go_amd", "csrc", "jb_capi.cpp")).read()
    a = src.index("// One token of a packed piece")
    b = src.index("// Text already in pinned memory (jb_host_alloc)")
    h = os.path.join(ROOT, "tests", "host")
    prog = tmp_path / "unpack.cpp"
    prog.write_text(open(os.path.join(h, "unpack_harness_head.cpp")).read() + src[a:b] +
                    open(os.path.join(h, "unpack_harness_main.cpp")).read())
    exe = str(tmp_path / "unpack_san")
    subprocess.run([CLANG, "-std=c++17", "-pthread", *SAN, "-o", exe, str(prog)], check=True)
    for avx in ("1", "0"):
        r = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=dict(ENV, JB_DECODE_AVX512=avx))
        assert r.returncode == 0 and r.stdout.strip() == "ok", (avx, r.stderr[-4000:])
