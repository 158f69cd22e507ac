"""The C++ adapter (include/dlsm_bloom_adapter.hpp) compiled as a reference-side
caller would compile it, run on the GPU, checked against the oracle."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _compile(tmp_path):
    exe = tmp_path / "adapter_test"
    cmd = ["g++", "-std=c++17", "-O2", "-I", os.path.join(ROOT, "include"),
           os.path.join(ROOT, "tests", "cpp", "adapter_test.cc"),
           "-L", os.path.join(ROOT, "dlsm_amd", "lib"), "-ldlsm_bloom",
           "-L", os.path.join(ROOT, "oracle"), "-loracle",
           "-Wl,-rpath," + os.path.join(ROOT, "dlsm_amd", "lib"),
           "-Wl,-rpath," + os.path.join(ROOT, "oracle"),
           "-Wl,-rpath,/opt/rocm/lib", "-L/opt/rocm/lib", "-o", str(exe)]
    subprocess.run(cmd, check=True)
    return exe


def test_adapter_compiles_without_hip_headers(tmp_path):
    """A reference-side C++ caller needs only the C header (no HIP, no torch)."""
    _compile(tmp_path)


@pytest.mark.gpu
def test_adapter_on_gpu(tmp_path):
    exe = _compile(tmp_path)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0 and "OK adapter" in out.stdout, out.stdout + out.stderr
