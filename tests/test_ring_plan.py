"""Commit-barrier ring planning (``csrc/ring_plan.h``): the host logic that turns the
node's peer matrix into the token writes of the xGMI barrier, built here with g++ as a host-only
library and driven through its C entry point. The same header is compiled into ``nos-gpuhelper``.

A missing peer path must never veto a commit (it only drops that link's fabric check): every device
writes exactly one token, into the next device it reaches or into its own memory, and no two writes
share a destination."""
import ctypes
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")


@pytest.fixture(scope="module")
def ringplan(tmp_path_factory):
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("no g++")
    out = tmp_path_factory.mktemp("ringplan") / "libnos_ringplan.so"
    subprocess.run([cxx, "-std=c++17", "-O1", "-g", "-Wall", "-Werror", "-shared", "-fPIC", f"-I{CSRC}",
                    os.path.join(CSRC, "ring_plan_capi.cpp"), "-o", str(out)], check=True)
    lib = ctypes.CDLL(str(out))
    P = ctypes.POINTER(ctypes.c_int)
    lib.nos_ring_plan.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_uint8), P, P, P, P, P, P]
    lib.nos_ring_plan.restype = ctypes.c_int

    def plan(n, can):
        m = (ctypes.c_uint8 * (n * n))(*[1 if can(i, j) else 0 for i in range(n) for j in range(n)])
        src, dst, reg = (ctypes.c_int * n)(), (ctypes.c_int * n)(), (ctypes.c_int * n)()
        peer, local, closed = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        k = lib.nos_ring_plan(n, m, src, dst, reg, ctypes.byref(peer), ctypes.byref(local), ctypes.byref(closed))
        assert k == n
        steps = [(src[i], dst[i], reg[i]) for i in range(k)]
        return steps, peer.value, local.value, closed.value
    return plan


def _check(n, steps, can):
    assert sorted(s for s, _, _ in steps) == list(range(n))            # every device writes exactly once
    assert len({(d, r) for _, d, r in steps}) == n                      # no shared destination
    for s, d, r in steps:
        assert (r == 1 and d == s) or (r == 0 and d != s and can(s, d))  # peer writes only over real paths


def test_fully_connected_node_is_the_plain_ring(ringplan):
    for n in (1, 2, 8, 64):
        can = lambda i, j: i != j  # noqa: E731
        steps, peer, local, closed = ringplan(n, can)
        _check(n, steps, can)
        if n == 1:
            assert steps == [(0, 0, 1)] and local == 1 and peer == 0    # the one-GPU box: a local write
        else:
            assert steps == [(d, (d + 1) % n, 0) for d in range(n)] and peer == n and closed == 1


def test_two_devices_that_cannot_reach_each_other_still_commit(ringplan):
    """VERDICT r3 #4's done-criterion: a topology with an unreachable pair plans a full set of
    writes (the helper then commits if every token reads back) instead of a veto."""
    n = 8
    can = lambda i, j: i != j and {i, j} != {3, 4}  # noqa: E731
    steps, peer, local, closed = ringplan(n, can)
    _check(n, steps, can)
    assert local == 0 and peer == n                      # the ring simply goes around the gap


def test_isolated_device_writes_locally_and_the_rest_keep_their_ring(ringplan):
    n = 8
    can = lambda i, j: i != j and 5 not in (i, j)  # noqa: E731
    steps, peer, local, closed = ringplan(n, can)
    _check(n, steps, can)
    assert (5, 5, 1) in steps and local == 1 and peer == 7 and closed == 1


def test_no_peer_paths_at_all_is_all_local(ringplan):
    n = 4
    can = lambda i, j: False  # noqa: E731
    steps, peer, local, closed = ringplan(n, can)
    _check(n, steps, can)
    assert local == 4 and peer == 0


def test_one_way_links_and_two_islands(ringplan):
    """Two islands of four fully connected devices (e.g. two groups of GPUs), plus a device that can
    only write out: each island closes its own ring; one-way links are used only forwards."""
    n = 9
    island = lambda i: 0 if i < 4 else 1  # noqa: E731
    can = lambda i, j: i != j and ((i < 8 and j < 8 and island(i) == island(j)) or (i == 8 and j == 0))  # noqa: E731
    steps, peer, local, closed = ringplan(n, can)
    _check(n, steps, can)
    assert closed == 2
    assert (8, 8, 1) in steps or (8, 0, 0) in steps


def test_random_topologies_always_plan_one_write_per_device(ringplan):
    import random
    rng = random.Random(7)
    for _ in range(200):
        n = rng.randint(1, 16)
        p = rng.random()
        m = {(i, j): rng.random() < p for i in range(n) for j in range(n)}
        can = lambda i, j: i != j and m[(i, j)]  # noqa: E731
        steps, peer, local, closed = ringplan(n, can)
        _check(n, steps, can)
        assert peer + local == n
