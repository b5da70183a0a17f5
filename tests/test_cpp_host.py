"""The C++ host mirror (dag_rider_amd/host/process.hpp) running the reference's own
tests (TestPath, TestStack) ported to C++ -- tests/cpp/process_internal_test.cpp."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "build", "process_internal_test")


@pytest.mark.gpu
def test_cpp_process_internal(gpu_device):
    assert os.path.exists(BIN), "build/process_internal_test missing: run make"
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=120)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "FAIL" not in r.stdout
