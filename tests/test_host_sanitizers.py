"""Host-code sanitizers: the native host code that is not a GPU kernel — C++ sequence
packing (csrc/packing_core.h) and the threaded host AdamW of optimizer offload (csrc/cpu_adam_core.h) —
built into a standalone harness under AddressSanitizer + UndefinedBehaviorSanitizer and under
ThreadSanitizer, run, and required to finish clean (a sanitizer report aborts with a non-zero code).
GPU sanitizers are not available on the MI355X pool; the kernels' index safety is covered by the
device-side checks instead (ops/native.py check_kernel_errors)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "native", "host_sanitize.cpp")
INC = os.path.join(ROOT, "llm_training_amd", "csrc")


def _build_and_run(tmp_path, flags, env_extra):
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("g++ not available")
    exe = tmp_path / "host_sanitize"
    r = subprocess.run([cxx, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", *flags, "-I", INC, SRC,
                        "-o", str(exe), "-pthread"], capture_output=True, text=True, timeout=300)
    if r.returncode != 0 and ("cannot find" in r.stderr or "-lasan" in r.stderr or "-ltsan" in r.stderr):
        pytest.skip("sanitizer runtime not installed: " + r.stderr[-300:])
    assert r.returncode == 0, r.stderr[-3000:]
    env = dict(os.environ, **env_extra)
    out = subprocess.run([str(exe), "4"], capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0 and "ok" in out.stdout, (out.stdout[-2000:], out.stderr[-4000:])
    assert "runtime error" not in out.stderr and "WARNING: ThreadSanitizer" not in out.stderr, out.stderr[-4000:]


def test_host_code_under_asan_ubsan(tmp_path):
    _build_and_run(tmp_path, ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"],
                   {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=1"})


def test_host_adamw_threads_under_tsan(tmp_path):
    _build_and_run(tmp_path, ["-fsanitize=thread"], {"TSAN_OPTIONS": "halt_on_error=1"})
