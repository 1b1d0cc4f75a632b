"""Host-code sanitizers: the HBM-limit shim's budget accounting is exercised by a
multithreaded self-test against a malloc-backed stand-in for the HIP allocation API, built with
AddressSanitizer + UndefinedBehaviorSanitizer and, separately, ThreadSanitizer (GPU sanitizers are
not available on the MI355X pool; host code is where these run)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")


def _build_and_run(tmp_path, flags):
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("no g++")
    lib = tmp_path / "libfake_hip.so"
    exe = tmp_path / "selftest"
    base = [cxx, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer"] + flags
    subprocess.run(base + ["-shared", "-fPIC", os.path.join(CSRC, "tests", "fake_hip.cpp"), "-o", str(lib)], check=True)
    subprocess.run(base + [os.path.join(CSRC, "tests", "hbm_limit_selftest.cpp"), os.path.join(CSRC, "hbm_limit.cpp"),
                           "-o", str(exe), f"-L{tmp_path}", "-lfake_hip", f"-Wl,-rpath,{tmp_path}", "-ldl", "-pthread"],
                   check=True)
    env = dict(os.environ, NOS_HBM_LIMIT_BYTES=str(64 << 20))
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([str(exe)], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "selftest ok" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr and "WARNING: ThreadSanitizer" not in r.stderr
    assert "runtime error" not in r.stderr  # UBSan


def test_hbm_limit_shim_asan_ubsan(tmp_path):
    _build_and_run(tmp_path, ["-fsanitize=address,undefined"])


def test_hbm_limit_shim_tsan(tmp_path):
    _build_and_run(tmp_path, ["-fsanitize=thread"])
