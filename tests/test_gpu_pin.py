"""Partition pinning on the GPU (csrc/pin.h): the emulation of CPX/QPX/DPX partitions runs each
partition's kernels on its own XCDs only.

* census: under 8 concurrent streams, every logical block of a pinned launch runs exactly once and
  only on an XCD of its mask (the dispatcher's round-robin XCD placement, read back from
  HW_REG_XCC_ID);
* numerics: every pinned hot op (split3, LayerNorm, x3 GEMM tiles incl. persistent ones, x3
  attention, the whole model) is bit-identical to its unpinned launch — pinning changes only where
  workgroups run, never what they compute.
"""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu

MASKS = [1 << 3, 0b1100, 0xF0, 0xFF]


@pytest.fixture(scope="module")
def K():
    from walkai_nos_amd.ops import kernels as K
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    K.set_backend("hip")
    L = K._L()
    L.nos_pin_census.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_uint, ctypes.c_void_p]
    yield K
    K.set_slice_pin(0)
    K.set_slice_cus(None)


def test_pin_census_every_block_once_on_its_xcds_under_concurrency(K):
    L = K._L()
    n = 4099
    streams = [torch.cuda.Stream() for _ in range(8)]
    for rep in range(3):
        bufs = []
        for k, s in enumerate(streams):
            mask = (1 << k) if rep == 0 else MASKS[k % len(MASKS)]
            counts = torch.zeros(n, dtype=torch.int32, device="cuda")
            xcc = torch.full((n,), -1, dtype=torch.int32, device="cuda")
            torch.cuda.synchronize()
            bufs.append((mask, counts, xcc))
        for (mask, counts, xcc), s in zip(bufs, streams):
            with torch.cuda.stream(s):
                for _ in range(4):  # 4 launches per stream, all streams in flight together
                    assert L.nos_pin_census(counts.data_ptr(), xcc.data_ptr(), n, mask, s.cuda_stream) == 0
        torch.cuda.synchronize()
        for mask, counts, xcc in bufs:
            assert torch.all(counts == 4), (mask, int((counts != 4).sum()))
            seen = set(xcc.unique().tolist())
            assert seen and all((mask >> x) & 1 for x in seen), (mask, seen)
            assert seen == {x for x in range(8) if (mask >> x) & 1}, (mask, seen)


def _pinned(K, mask, cus, fn):
    K.set_slice_cus(cus)
    K.set_slice_pin(mask)
    try:
        out = fn()
        torch.cuda.synchronize()
        return out
    finally:
        K.set_slice_pin(0)
        K.set_slice_cus(None)


@pytest.mark.parametrize("mask", [1 << 5, 0b0011, 0x0F])
def test_pinned_ops_bit_identical_to_unpinned(K, mask):
    from walkai_nos_amd.ops import gemm as G
    torch.manual_seed(11)
    cus = 32 * bin(mask).count("1")
    T, D, H = 3401, 384, 6
    x = torch.randn(T, D, device="cuda")
    w = torch.randn(D, device="cuda")
    b = torch.randn(D, device="cuda")
    ref = _pinned(K, 0, cus, lambda: (K.split3(x), K.layernorm_x3(x[None], w, b, 1e-12),
                                      K.layernorm(x[None], w, b, 1e-12)))
    got = _pinned(K, mask, cus, lambda: (K.split3(x), K.layernorm_x3(x[None], w, b, 1e-12),
                                         K.layernorm(x[None], w, b, 1e-12)))
    for r, g in zip(ref, got):
        assert torch.equal(r, g)
    # x3 GEMM: one tile of every kind (register-staged, LDS-DMA, 16x16 MFMA, persistent)
    a3 = K.split3(torch.randn(T, D, device="cuda"))
    wt = torch.randn(3 * D, D, device="cuda") * 0.05
    bt = torch.randn(3 * D, device="cuda")
    res = torch.randn(T, 3 * D, device="cuda")
    cfgs = [c for c in (3, 11, 14, 24, 29, 102, 107) if c in G.x3_eligible(3 * D, D)]
    assert len(cfgs) >= 6
    for cfg in cfgs:
        r = _pinned(K, 0, cus, lambda: G.gemm_x3(a3, wt, bt, residual=res, tile=cfg, out_f32=True, out_x3=True))
        g = _pinned(K, mask, cus, lambda: G.gemm_x3(a3, wt, bt, residual=res, tile=cfg, out_f32=True, out_x3=True))
        assert torch.equal(r[0], g[0]) and torch.equal(r[1], g[1]), cfg
    # x3 attention from fp32 QKV, grid sized to the slice
    qkv = torch.randn(1, T, 3 * D, device="cuda")
    r = _pinned(K, 0, cus, lambda: K.attention_qkv_x3f(qkv, H, 64, 0.125))
    g = _pinned(K, mask, cus, lambda: K.attention_qkv_x3f(qkv, H, 64, 0.125))
    assert torch.equal(r, g)


def test_pinned_model_matches_unpinned_on_a_cpx_slice(K):
    from walkai_nos_amd.models.workload.yolos import YolosSmall, demo_input
    torch.manual_seed(0)
    m = YolosSmall().cuda().eval()
    x = demo_input(1, (800, 1066), "cuda")
    with torch.no_grad():
        ref = _pinned(K, 0, 32, lambda: m(x))
        got = _pinned(K, 1 << 6, 32, lambda: m(x))
    # the autotuner may pick different tiles per key, so compare to fp32-accurate tolerance
    for r, g in zip(ref, got):
        assert (r - g).abs().max().item() < 1e-4


def test_landing_mask_places_work_on_own_xcd_and_one_cu_elsewhere(K):
    """The "landing" emulation's CU mask (bench_core.slice_cus): a CPX partition's workgroups run on
    31 CUs of one XCD, and on exactly one (the landing) CU of every other XCD; under the partition's
    pin (census above) the latter are the exit-only ones."""
    import collections

    from walkai_nos_amd.bench_core import slice_cus, slice_pin
    from walkai_nos_amd.ops import probe
    cus = slice_cus("cpx_nps1", 3, emulation="landing")
    assert len(cus) == 31 + 7 and slice_pin("cpx_nps1", 3, "landing") == 1 << 3
    with probe.Stream(0, cus) as s:
        placements = probe.census(0, s, n_wg=2048, spin=200)
    per_xcc = collections.defaultdict(set)
    for p in placements:
        per_xcc[p["xcc"]].add((p["se"], p["sh"], p["cu"]))
    sizes = sorted(len(v) for v in per_xcc.values())
    assert sizes == [1] * 7 + [31], dict((x, len(v)) for x, v in per_xcc.items())
