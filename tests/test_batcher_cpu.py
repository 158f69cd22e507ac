"""The batcher's queue logic (dlsm_amd/csrc/batcher.hip) on the CPU under
ThreadSanitizer, against a stubbed C ABI (tests/cpp/batcher_cpu_test.cc): two
or more executors with gathering windows, bursty submitters whose queue
drains to empty while an executor still waits, per-job status
isolation, and the exact-count flag.  No GPU needed."""
import os
import shutil
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLANG = "/opt/rocm/lib/llvm/bin/clang++"  # its TSan intercepts pthread_cond_clockwait (gcc 11's does not)


def test_batcher_queue_under_tsan(tmp_path):
    exe = tmp_path / "batcher_cpu_test"
    cxx = CLANG if os.path.exists(CLANG) else shutil.which("clang++")
    assert cxx, "clang++ (ROCm LLVM) is needed for the ThreadSanitizer build"
    subprocess.run([cxx, "-std=c++17", "-O1", "-g", "-fsanitize=thread", "-pthread",
                    "-I", os.path.join(ROOT, "include"),
                    "-x", "c++", os.path.join(ROOT, "dlsm_amd", "csrc", "batcher.hip"),
                    "-x", "c++", os.path.join(ROOT, "tests", "cpp", "batcher_cpu_test.cc"),
                    "-o", str(exe)], check=True)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66")
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0 and "OK batcher cpu" in out.stdout, out.stdout + out.stderr[-4000:]
    assert "ThreadSanitizer" not in out.stderr, out.stderr[-4000:]
