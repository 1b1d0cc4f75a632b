"""The xGMI commit barrier's host code (csrc/p2p_barrier_host.h, the code nos_p2p_barrier runs on
the GPU) on a multi-device fake of the HIP runtime (csrc/tests/fake_hip_multi.*) at 8 and 64
devices: full ring, peer-enable failures re-planned, missing peer paths (local writes), corrupted
tokens and no-votes vetoed, a hung device returning -3 within NOS_BARRIER_DEADLINE_MS — plain, under
AddressSanitizer + UndefinedBehaviorSanitizer, and under ThreadSanitizer (the fake's devices are
threads writing memory the host reads back). VERDICT r4 next-round #4: every hardware run had one
device, so these paths had never executed anywhere."""
import json
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
SCENARIOS = {"full_ring", "enable_fails_replan", "no_peer_path_local_write", "corrupt_token_vetoes",
             "no_vote_vetoes", "hung_device_deadline", "repeat_reuses_links", "fake_catches_write_without_peer_access"}


def _build(tmp_path, flags, tag):
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("no g++")
    exe = tmp_path / f"p2p_selftest_{tag}"
    subprocess.run([cxx, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-Wall", "-Werror"] + flags +
                   [os.path.join(CSRC, "tests", "p2p_barrier_selftest.cpp"),
                    os.path.join(CSRC, "tests", "fake_hip_multi.cpp"), "-o", str(exe), "-pthread"], check=True)
    return exe


@pytest.mark.parametrize("flags,tag", [([], "plain"), (["-fsanitize=address,undefined"], "asan"),
                                       (["-fsanitize=thread"], "tsan")])
@pytest.mark.parametrize("n", [8, 64])
def test_barrier_host_paths_on_a_multi_device_fake(tmp_path, flags, tag, n):
    exe = _build(tmp_path, flags, tag)
    env = {k: v for k, v in os.environ.items() if k not in ("LD_PRELOAD", "NOS_BARRIER_NO_PEER",
                                                            "NOS_BARRIER_DEADLINE_MS")}
    env["TSAN_OPTIONS"] = "halt_on_error=1"
    r = subprocess.run([str(exe), str(n)], env=env, capture_output=True, text=True, timeout=300)
    rows = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
    assert "ERROR: AddressSanitizer" not in r.stderr and "WARNING: ThreadSanitizer" not in r.stderr, r.stderr[-3000:]
    assert "runtime error" not in r.stderr, r.stderr[-3000:]
    got = {row["scenario"]: row for row in rows if "scenario" in row}
    assert set(got) == SCENARIOS and all(row["ok"] for row in got.values()), rows
    assert got["full_ring"]["peer"] == n and got["hung_device_deadline"]["rc"] == -3
    assert got["hung_device_deadline"]["ms"] < 5000   # the 200 ms deadline, not the 10 s default
