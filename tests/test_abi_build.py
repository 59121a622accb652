"""The C ABI header compiles as C99 and C++17 and a C++ program links and
runs against libkmws_gpu.so (the way kuma's C++ would consume it)."""
import os
import subprocess

import pytest

from kuma_amd import build as kb

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = os.path.join(ROOT, "include")


def test_header_is_plain_c(tmp_path):
    src = tmp_path / "t.c"
    src.write_text('#include "kmws_gpu.h"\nint main(void){ kmws_desc d; (void)d; '
                   'return kmws_make_flags(1,0,0,0,2,1) == 0x182 ? 0 : 1; }\n')
    subprocess.check_call(["gcc", "-std=c99", "-Wall", "-Werror", "-pedantic", "-I", INC, "-fsyntax-only",
                           str(src)])


def _build_and_run(tmp_path):
    lib = kb.build()
    exe = tmp_path / "abi_smoke"
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-Wall", "-I", INC,
                           os.path.join(ROOT, "tests", "cpp", "abi_smoke.cpp"),
                           "-L", os.path.dirname(lib), "-lkmws_gpu",
                           "-Wl,-rpath," + os.path.dirname(lib), "-o", str(exe)])
    return subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)


def test_cpp_consumer_host_paths(tmp_path):
    r = _build_and_run(tmp_path)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK" in r.stdout


@pytest.mark.gpu
def test_cpp_consumer_on_gpu(tmp_path):
    r = _build_and_run(tmp_path)
    assert r.returncode == 0, r.stdout + r.stderr
