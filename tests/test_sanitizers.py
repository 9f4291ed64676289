"""Race detection / memory safety for the native host code.

The C++ TCP transport (csrc/comm/tcp_transport.cpp: epoll reader thread, queued writer
thread with reconnect, status queries from the caller's thread) is built together with a
multi-threaded stress driver (csrc/tests/transport_stress.cpp) under
  * AddressSanitizer + UndefinedBehaviorSanitizer, and
  * ThreadSanitizer
with the ROCm LLVM clang++ (its TSan runtime intercepts pthread_cond_clockwait, which GCC 11's
does not - that produces false "double lock" reports for std::condition_variable::wait_for).
TSan found a real race here: ``Push::fd`` / fault-injection knobs written by the writer
thread while ``lsa_push_connected`` / ``lsa_push_fault`` touched them from the caller
(fixed with atomics). GPU sanitizers are not available on the MI355X pool; device code is
covered by the host-side shape checks in ops/hip.py and by the numerics tests.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLANG = "/opt/rocm/lib/llvm/bin/clang++"
SRCS = [os.path.join(ROOT, "csrc", "tests", "transport_stress.cpp"),
        os.path.join(ROOT, "csrc", "comm", "tcp_transport.cpp")]


def _compiler():
    if os.path.exists(CLANG):
        return CLANG
    return shutil.which("clang++")


@pytest.mark.parametrize("san,env", [
    ("address,undefined", {"ASAN_OPTIONS": "detect_leaks=1:halt_on_error=1:verify_asan_link_order=0",
                           "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1"}),
    ("thread", {"TSAN_OPTIONS": "halt_on_error=1"}),
])
def test_transport_under_sanitizer(san, env, tmp_path):
    cxx = _compiler()
    if cxx is None:
        pytest.skip("no clang++")
    exe = tmp_path / f"stress_{san.split(',')[0]}"
    b = subprocess.run([cxx, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", f"-fsanitize={san}",
                        *SRCS, "-o", str(exe), "-lpthread"], capture_output=True, text=True, timeout=300)
    if b.returncode != 0 and "cannot find" in (b.stderr + b.stdout) and "libclang_rt" in (b.stderr + b.stdout):
        pytest.skip(f"sanitizer runtime for {san} not installed")
    assert b.returncode == 0, b.stderr[-3000:]
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600, env=dict(os.environ, **env))
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-6000:]
    assert "transport stress OK" in out
    assert "Sanitizer" not in out, out[-6000:]
