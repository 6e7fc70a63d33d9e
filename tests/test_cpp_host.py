"""The C++ host mirror of the reference's IndexSystem interface
(include/mosaic_index_system.hpp), driven by its own test program
tests/cpp/test_host_api (built by __graft_entry__.build(); known answers from the
reference's tests and docs, see the program's header)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "cpp", "test_host_api")


def _run(mode):
    if not os.path.exists(EXE):
        pytest.skip("tests/cpp/test_host_api not built (run __graft_entry__.build())")
    r = subprocess.run([EXE, mode], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def test_cpp_host_cpu():
    assert "0 failure" in _run("--cpu")


@pytest.mark.gpu
def test_cpp_host_gpu(gpu):
    assert "0 failure" in _run("--gpu")
