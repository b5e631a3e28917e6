"""The C++ restatement of eazy_test.go (tests/cpp/eazy_test.cpp) over the C++
host side (eazy_amd/cpp/eazy.hpp): host-only tests here, all of it on the GPU."""

import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
CPP = os.path.join(HERE, "cpp")


def _build():
    p = subprocess.run(["make", "-s", "-C", CPP], capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-2000:]
    return os.path.join(CPP, "eazy_test")


def _run(*args):
    p = subprocess.run([_build(), *args], capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stdout[-4000:] + p.stderr[-2000:]
    return p.stdout


def test_cpp_host_only():
    out = _run("--cpu")
    assert "6/6 passed" in out


@pytest.mark.gpu
def test_cpp_full(cuda):
    out = _run()
    assert "FAIL" not in out and "22/22 passed" in out
