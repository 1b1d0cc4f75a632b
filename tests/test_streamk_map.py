"""The stream-K work split (csrc/streamk.h) the GEMM producer and the LayerNorm consumer share,
checked on the host through the library's own map function: every K stage of every tile is owned by
exactly one workgroup, a tile's segments land on distinct planes below the reported depth, and the
consumer's per-tile segment count equals the number of workgroups that wrote the tile."""
import ctypes
import os

import pytest

from walkai_nos_amd.ops import build


@pytest.fixture(scope="module")
def lib():
    path = os.path.join(build.OUT, "libnos_kernels.so")
    if not os.path.exists(path):
        pytest.skip("libnos_kernels.so not built")
    L = ctypes.CDLL(path)
    L.nos_gemm_x3_streamk_map.argtypes = [ctypes.c_int] * 5 + [ctypes.c_void_p]
    return L


def _map(L, M, N, K, cfg, P):
    out = (ctypes.c_int * 7)()
    rc = L.nos_gemm_x3_streamk_map(M, N, K, cfg, P, out)
    return rc, tuple(out)


def owner(u, P, U):
    return ((u + 1) * P - 1) // U


@pytest.mark.parametrize("M,N,K", [(3401, 384, 1536), (3401, 384, 384), (300, 768, 256), (33, 128, 64)])
@pytest.mark.parametrize("cfg", range(6))
@pytest.mark.parametrize("P", [1, 7, 256, 512, 100000])
def test_every_stage_owned_once_and_segments_fit_the_planes(lib, M, N, K, cfg, P):
    rc, m = _map(lib, M, N, K, cfg, P)
    bm, bn = m[3], m[4]
    if N % bn:
        assert rc != 0
        return
    assert rc == 0
    Pe, U, nk, _, _, tiles_n, planes = m
    tiles = -(-M // bm) * tiles_n
    assert U == tiles * nk and Pe == min(P, U) and tiles_n * bn == N
    # the producer: workgroup w owns [w*U/P, (w+1)*U/P); segment = w - owner(first stage of the tile)
    seen = [0] * U
    segs = {}
    for w in range(Pe):
        u0, u1 = w * U // Pe, (w + 1) * U // Pe
        assert u1 > u0
        for u in range(u0, u1):
            seen[u] += 1
            assert owner(u, Pe, U) == w
            t = u // nk
            segs.setdefault(t, set()).add(w - owner(t * nk, Pe, U))
    assert all(c == 1 for c in seen)
    assert max(max(s) for s in segs.values()) + 1 == planes
    # the consumer: tile t adds planes 0 .. segments(t) - 1, exactly the ones written
    for t, s in segs.items():
        n = owner((t + 1) * nk - 1, Pe, U) - owner(t * nk, Pe, U) + 1
        assert s == set(range(n))


def test_bad_arguments_are_refused(lib):
    assert _map(lib, 3401, 384, 1536, 6, 256)[0] != 0     # no such config
    assert _map(lib, 3401, 384, 1536, 0, 0)[0] != 0       # no workgroups
    assert _map(lib, 3401, 384, 1000, 1, 256)[0] != 0     # K not a multiple of the 64-deep stage
