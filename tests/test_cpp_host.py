"""The C++ host mirror of the reference's IndexSystem interface
(include/mosaic_index_system.hpp), driven by its own test program
tests/cpp/test_host_api (built by __graft_entry__.build(); known answers from the
reference's tests and docs, see the program's header)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "cpp", "test_host_api")


def _run(mode, exe=EXE):
    if not os.path.exists(exe):
        pytest.skip("%s not built (run __graft_entry__.build())" % exe)
    r = subprocess.run([exe] + ([mode] if mode else []), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def test_cpp_host_cpu():
    assert "0 failure" in _run("--cpu")


@pytest.mark.gpu
def test_cpp_host_gpu(gpu):
    assert "0 failure" in _run("--gpu")


def test_h3_fast_digit_encoding_equals_restatement():
    """face_ijk_to_h3_fast (axial walk + bit-plane rotations, used by the kernels) ==
    face_ijk_to_h3 (the _faceIjkToH3 restatement) on 6.4M lattice positions."""
    out = _run(None, os.path.join(ROOT, "tests", "cpp", "test_h3_digits"))
    assert "mismatches 0" in out
