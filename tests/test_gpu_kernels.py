"""Numerics of the HIP workload kernels vs plain PyTorch fp32 references (GPU only)."""
import math
import os

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def K():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from walkai_nos_amd.ops import kernels
    assert kernels.hip_available(), "libnos_kernels.so must be built on a GPU box"
    kernels.set_backend("hip")
    return kernels


def _ref_attention(qkv, H, Dh, scale):
    B, T, _ = qkv.shape
    q, k, v = qkv.double().view(B, T, 3, H, Dh).permute(2, 0, 3, 1, 4)
    s = (q @ k.transpose(-1, -2)) * scale
    p = torch.softmax(s, dim=-1)
    return (p @ v).transpose(1, 2).reshape(B, T, H * Dh).float()


@pytest.mark.parametrize("B,T,H", [(1, 32, 1), (1, 77, 2), (2, 300, 3), (1, 3401, 6)])
def test_attention_matches_fp64_reference(K, B, T, H):
    torch.manual_seed(0)
    qkv = torch.randn(B, T, 3 * H * 64, device="cuda")
    out = K.attention_qkv(qkv, H, 64, 1.0 / 8.0)
    torch.cuda.synchronize()
    ref = _ref_attention(qkv, H, 64, 1.0 / 8.0)
    err = (out - ref).abs().max().item()
    assert err < 2e-5, err


def test_attention_asymmetric_values_catch_transposes(K):
    # V with distinct per-(key, dim) values and a peaked softmax: a swapped layout cannot pass
    T, H = 96, 1
    qkv = torch.zeros(1, T, 3 * 64, device="cuda")
    qkv[0, :, :64] = torch.randn(T, 64, device="cuda") * 4
    qkv[0, :, 64:128] = torch.randn(T, 64, device="cuda") * 4
    qkv[0, :, 128:] = torch.arange(T * 64, device="cuda", dtype=torch.float32).view(T, 64) / 1000
    out = K.attention_qkv(qkv, H, 64, 0.125)
    ref = _ref_attention(qkv, H, 64, 0.125)
    assert (out - ref).abs().max().item() < 1e-4


@pytest.mark.parametrize("T,H,B", [(1000, 2, 1), (3401, 6, 1), (77, 1, 2)])
def test_attention_stream_k_any_grid_matches_reference(K, T, H, B):
    # every grid size exercises a different partial-segment pattern: a wave inside one tile,
    # waves spanning tile boundaries, more waves than units, one wave doing everything
    torch.manual_seed(1)
    qkv = torch.randn(B, T, 3 * H * 64, device="cuda")
    ref = _ref_attention(qkv, H, 64, 0.125)
    units = B * H * ((T + 31) // 32) ** 2
    try:
        for variant in (0, 2, 3):
            K.set_attention_variant(variant)
            for waves in (1, 3, 7, 64, 333, 1024, 3072, units + 5):
                out = torch.full((B, T, H * 64), float("nan"), device="cuda")
                K.attention_sk(qkv, out, H, 64, 0.125, waves)
                torch.cuda.synchronize()
                assert (out - ref).abs().max().item() < 2e-5, (variant, waves)
    finally:
        K.set_attention_variant(0)
    un = K.attention_unsplit(qkv, H, 64, 0.125)
    assert (un - ref).abs().max().item() < 2e-5


def test_attention_concurrent_streams_stream_k(K):
    # two slices running stream-K launches at once must not share scratch
    torch.manual_seed(2)
    qa = torch.randn(1, 700, 3 * 2 * 64, device="cuda")
    qb = torch.randn(1, 900, 3 * 2 * 64, device="cuda")
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    outs = []
    torch.cuda.synchronize()
    for _ in range(3):
        with torch.cuda.stream(sa):
            oa = K.attention_sk(qa, torch.empty(1, 700, 128, device="cuda"), 2, 64, 0.125, 300)
        with torch.cuda.stream(sb):
            ob = K.attention_sk(qb, torch.empty(1, 900, 128, device="cuda"), 2, 64, 0.125, 512)
        outs.append((oa, ob))
    torch.cuda.synchronize()
    ra, rb = _ref_attention(qa, 2, 64, 0.125), _ref_attention(qb, 2, 64, 0.125)
    for oa, ob in outs:
        assert (oa - ra).abs().max().item() < 2e-5
        assert (ob - rb).abs().max().item() < 2e-5


@pytest.mark.parametrize("D", [384, 768, 1024])
def test_layernorm(K, D):
    torch.manual_seed(0)
    x = torch.randn(3401, D, device="cuda") * 3 + 1
    w = torch.randn(D, device="cuda")
    b = torch.randn(D, device="cuda")
    out = K.layernorm(x, w, b, 1e-12)
    ref = F.layer_norm(x.double(), (D,), w.double(), b.double(), 1e-12).float()
    assert (out - ref).abs().max().item() < 1e-4


def test_linear_gelu(K):
    torch.manual_seed(0)
    x = torch.randn(3401, 384, device="cuda")
    w = torch.randn(1536, 384, device="cuda") * 0.05
    b = torch.randn(1536, device="cuda")
    out = K.linear_gelu(x, w, b)
    h = x.double() @ w.double().t() + b.double()
    ref = (0.5 * h * (1 + torch.erf(h / math.sqrt(2)))).float()
    assert (out - ref).abs().max().item() < 1e-3


def test_linear_residual(K):
    torch.manual_seed(0)
    x = torch.randn(1, 3401, 1536, device="cuda")
    w = torch.randn(384, 1536, device="cuda") * 0.02
    b = torch.randn(384, device="cuda")
    r = torch.randn(1, 3401, 384, device="cuda")
    out = K.linear_residual(x, w, b, r)
    ref = (r.double() + x.double() @ w.double().t() + b.double()).float()
    assert (out - ref).abs().max().item() < 1e-3


@pytest.mark.parametrize("M,N,Kd", [(3401, 384, 384), (3401, 1152, 384), (3401, 1536, 384), (3401, 384, 1536),
                                    (100, 128, 64), (1, 128, 32)])
def test_mfma_gemm_every_tile_and_epilogue(K, M, N, Kd):
    from walkai_nos_amd.ops import gemm as G
    torch.manual_seed(0)
    x = torch.randn(M, Kd, device="cuda")
    w = torch.randn(N, Kd, device="cuda") * 0.05
    b = torch.randn(N, device="cuda")
    r = torch.randn(M, N, device="cuda")
    h = x.double() @ w.double().t()
    refs = {"plain": (h, {}), "bias": (h + b.double(), {"bias": b}),
            "gelu": (None, {"bias": b, "gelu": True}), "res": (h + b.double() + r.double(), {"bias": b, "residual": r})}
    hb = h + b.double()
    refs["gelu"] = (0.5 * hb * (1 + torch.erf(hb / math.sqrt(2))), refs["gelu"][1])
    for cfg in G.eligible(M, N, Kd):
        for name, (ref, kw) in refs.items():
            out = G.gemm(x, w, tile=cfg, **kw)
            torch.cuda.synchronize()
            err = (out.double() - ref).abs().max().item()
            assert err < 2e-3 * max(1.0, Kd / 384), (cfg, name, err)


def test_gemm_autotune_picks_and_caches(K):
    from walkai_nos_amd.ops import gemm as G
    x = torch.randn(3401, 384, device="cuda")
    w = torch.randn(1536, 384, device="cuda") * 0.05
    b = torch.randn(1536, device="cuda")
    out = K.linear_gelu(x, w, b)
    hb = x.double() @ w.double().t() + b.double()
    ref = 0.5 * hb * (1 + torch.erf(hb / math.sqrt(2)))
    assert (out.double() - ref).abs().max().item() < 2e-3
    assert G.choose(3401, 1536, 384, G.EPI_BIAS | G.EPI_GELU, K.slice_cus()) is not None
    assert G.tuning_table()


def test_yolos_hip_matches_torch_backend(K):
    from walkai_nos_amd.models.workload.yolos import YolosSmall, demo_input
    m = YolosSmall().cuda().eval()
    x = demo_input(1, (800, 1066), "cuda")
    with torch.no_grad():
        K.set_backend("torch")
        ref_l, ref_b = m(x)
        K.set_backend("hip")
        l, bx = m(x)
    torch.cuda.synchronize()
    assert (l - ref_l).abs().max().item() < 1e-3
    assert (bx - ref_b).abs().max().item() < 1e-4


def test_gemm_second_residual_broadcast_and_out_view(K):
    from walkai_nos_amd.ops import gemm as G
    torch.manual_seed(3)
    T, N, Kd = 300, 128, 64
    x = torch.randn(2 * T, Kd, device="cuda")
    w = torch.randn(N, Kd, device="cuda") * 0.1
    b = torch.randn(N, device="cuda")
    r = torch.randn(2 * T, N, device="cuda")
    r2 = torch.randn(1, T, N, device="cuda")
    ref = x.double() @ w.double().t() + b.double() + r.double() + r2.double().repeat(2, 1, 1).reshape(2 * T, N)
    for cfg in G.eligible(2 * T, N, Kd):
        buf = torch.zeros(2 * T + 7, N, device="cuda")
        out = G.gemm(x, w, b, residual=r, residual2=r2, tile=cfg, out=buf[3:3 + 2 * T])
        torch.cuda.synchronize()
        assert (out.double() - ref).abs().max().item() < 1e-3, cfg
        assert buf[:3].abs().max().item() == 0 and buf[-4:].abs().max().item() == 0  # no stray writes


def test_patch_embed_matches_conv(K):
    torch.manual_seed(4)
    px = torch.randn(1, 3, 800, 1066, device="cuda")
    w = torch.randn(384, 3, 16, 16, device="cuda") * 0.02
    b = torch.randn(384, device="cuda")
    pos = torch.randn(50 * 66, 384, device="cuda")
    out = K.patch_embed(px, w, b, 16, pos)
    ref = torch.nn.functional.conv2d(px.double(), w.double(), b.double(), stride=16).flatten(2).transpose(1, 2) \
        + pos.double()
    torch.cuda.synchronize()
    assert out.shape == (1, 3300, 384)
    assert (out.double() - ref).abs().max().item() < 1e-3


def test_split3_is_exact(K):
    torch.manual_seed(5)
    x = torch.randn(1 << 16, device="cuda") * torch.logspace(-20, 20, 1 << 16, device="cuda")
    p = K.split3(x)
    assert p.dtype == torch.bfloat16 and p.shape == (3,) + x.shape
    recon = p[0].double() + p[1].double() + p[2].double()
    assert torch.equal(recon, x.double())
    # the GPU split is the CPU reference split bit for bit
    assert torch.equal(p.cpu(), K.split3(x.cpu()))


@pytest.mark.parametrize("T,H,B", [(1000, 2, 1), (3401, 6, 1), (77, 1, 2)])
def test_attention_x3_fp32_accurate_any_grid(K, T, H, B):
    # the x3 path must be as accurate as the f32-input MFMA path (both vs fp64), for every
    # stream-K partial-segment pattern
    torch.manual_seed(1)
    qkv = torch.randn(B, T, 3 * H * 64, device="cuda")
    ref = _ref_attention(qkv, H, 64, 0.125)
    planes = K.split3(qkv)
    units = B * H * (((T + 31) // 32 + 3) // 4) * ((T + 31) // 32)
    f32 = torch.empty(B, T, H * 64, device="cuda")
    K.attention_sk(qkv, f32, H, 64, 0.125, 256)
    torch.cuda.synchronize()
    err_f32 = (f32 - ref).abs().max().item()
    try:
        for pipelined, group in ((True, 4), (True, 8), (False, 4)):
            K.set_attention_x3_pipelined(pipelined)
            K.set_attention_x3_group(group)
            for waves in (1, 3, 7, 64, 333, 512, units + 5):
                out = torch.full((B, T, H * 64), float("nan"), device="cuda")
                K.attention_x3(planes, out, H, 64, 0.125, waves)
                torch.cuda.synchronize()
                err = (out - ref).abs().max().item()
                assert err < max(2.0 * err_f32, 2e-6), (pipelined, group, waves, err, err_f32)
    finally:
        K.set_attention_x3_pipelined(True)
        K.set_attention_x3_group(8)


@pytest.mark.parametrize("group", [4, 8])
def test_attention_x3_head_blocks_match_one_launch(K, group):
    # heads in blocks (one launch per block, x3 planes out) must equal the all-heads launch and fp64
    T, H, B = 1000, 6, 2
    torch.manual_seed(3)
    qkv = torch.randn(B, T, 3 * H * 64, device="cuda")
    ref = _ref_attention(qkv, H, 64, 0.125)
    planes = K.split3(qkv)
    K.set_attention_x3_group(group)
    try:
        for hb, waves in ((1, 32), (2, 7), (4, 64), (6, 256)):
            o3 = torch.full((3, B, T, H * 64), float("nan"), dtype=torch.bfloat16, device="cuda")
            K.attention_x3(planes, o3, H, 64, 0.125, waves, head_block=hb)
            torch.cuda.synchronize()
            out = o3[0].float() + o3[1].float() + o3[2].float()
            assert (out - ref).abs().max().item() < 2e-6, (hb, waves)
    finally:
        K.set_attention_x3_group(8)


def test_attention_x3_asymmetric_values(K):
    T, H = 96, 1
    qkv = torch.zeros(1, T, 3 * 64, device="cuda")
    qkv[0, :, :64] = torch.randn(T, 64, device="cuda") * 4
    qkv[0, :, 64:128] = torch.randn(T, 64, device="cuda") * 4
    qkv[0, :, 128:] = torch.arange(T * 64, device="cuda", dtype=torch.float32).view(T, 64) / 1000
    out = torch.empty(1, T, 64, device="cuda")
    K.attention_x3(K.split3(qkv), out, H, 64, 0.125, 5)
    ref = _ref_attention(qkv, H, 64, 0.125)
    assert (out - ref).abs().max().item() < 1e-4


@pytest.mark.parametrize("M,N,Kd", [(3401, 384, 384), (3401, 1152, 384), (3401, 1536, 384), (3401, 384, 1536),
                                    (3300, 384, 768), (100, 128, 64), (1, 128, 32)])
def test_gemm_x3_every_tile_epilogue_and_output(K, M, N, Kd, monkeypatch):
    # fp32-accurate: the x3 GEMM's error vs fp64 stays within 2x the f32-input MFMA GEMM's (every
    # tile, the opt-in staggered one included)
    from walkai_nos_amd.ops import gemm as G
    monkeypatch.setenv("NOS_X3_STAGGER", "1")
    torch.manual_seed(0)
    x = torch.randn(M, Kd, device="cuda")
    w = torch.randn(N, Kd, device="cuda") * 0.05
    b = torch.randn(N, device="cuda")
    r = torch.randn(M, N, device="cuda")
    x3 = K.split3(x)
    hb = x.double() @ w.double().t() + b.double()
    cases = {"bias": (hb, {"bias": b}),
             "gelu": (0.5 * hb * (1 + torch.erf(hb / math.sqrt(2))), {"bias": b, "gelu": True}),
             "res": (hb + r.double(), {"bias": b, "residual": r})}
    for name, (ref, kw) in cases.items():
        f32 = G.gemm(x, w, tile=G.eligible(M, N, Kd)[0], **kw)
        err_f32 = (f32.double() - ref).abs().max().item()
        for cfg in G.x3_eligible(N, Kd):
            y, y3 = G.gemm_x3(x3, w, tile=cfg, out_f32=True, out_x3=True, **kw)
            torch.cuda.synchronize()
            err = (y.double() - ref).abs().max().item()
            assert err <= max(2.0 * err_f32, 1e-5), (cfg, name, err, err_f32)
            assert torch.equal(y3[0].double() + y3[1].double() + y3[2].double(), y.double()), (cfg, name)
            only3 = G.gemm_x3(x3, w, tile=cfg, out_f32=False, out_x3=True, **kw)
            assert torch.equal(only3, y3), (cfg, name)


def test_gemm_x3_second_residual_and_out_view(K):
    from walkai_nos_amd.ops import gemm as G
    torch.manual_seed(3)
    T, N, Kd = 300, 128, 64
    x = torch.randn(2 * T, Kd, device="cuda")
    w = torch.randn(N, Kd, device="cuda") * 0.1
    b = torch.randn(N, device="cuda")
    r = torch.randn(2 * T, N, device="cuda")
    r2 = torch.randn(1, T, N, device="cuda")
    ref = x.double() @ w.double().t() + b.double() + r.double() + r2.double().repeat(2, 1, 1).reshape(2 * T, N)
    for cfg in G.x3_eligible(N, Kd):
        buf = torch.zeros(2 * T + 7, N, device="cuda")
        out = G.gemm_x3(K.split3(x), w, b, residual=r, residual2=r2, tile=cfg, out=buf[3:3 + 2 * T])
        torch.cuda.synchronize()
        assert (out.double() - ref).abs().max().item() < 1e-4, cfg
        assert buf[:3].abs().max().item() == 0 and buf[-4:].abs().max().item() == 0


def test_layernorm_and_attention_x3_outputs(K):
    torch.manual_seed(6)
    x = torch.randn(1, 3401, 384, device="cuda")
    w, b = torch.randn(384, device="cuda"), torch.randn(384, device="cuda")
    y = K.layernorm(x, w, b, 1e-12)
    y3 = K.layernorm_x3(x, w, b, 1e-12)
    assert torch.equal(y3[0].double() + y3[1].double() + y3[2].double(), y.double())
    qkv = torch.randn(1, 1000, 3 * 2 * 64, device="cuda")
    o3 = K.attention_qkv_x3(K.split3(qkv), 2, 64, 0.125)
    ref = _ref_attention(qkv, 2, 64, 0.125)
    o = (o3[0].double() + o3[1].double() + o3[2].double())
    assert (o - ref.double()).abs().max().item() < 2e-6


def test_yolos_x3_matches_f32_mode(K):
    from walkai_nos_amd.models.workload.yolos import YolosSmall, demo_input
    m = YolosSmall().cuda().eval()
    x = demo_input(1, (800, 1066), "cuda")
    try:
        with torch.no_grad():
            K.set_fp32_matmul("f32")
            l32, b32 = m(x)
            K.set_fp32_matmul("x3")
            l3, b3 = m(x)
            K.set_backend("torch")
            lt, bt = m(x)
    finally:
        K.set_backend("hip")
        K.set_fp32_matmul("x3")
    torch.cuda.synchronize()
    # both HIP modes sit at fp32 rounding distance from the PyTorch fp32 reference
    e3, e32 = (l3 - lt).abs().max().item(), (l32 - lt).abs().max().item()
    assert e3 < 1e-3 and e32 < 1e-3, (e3, e32)
    assert (b3 - bt).abs().max().item() < 1e-4


@pytest.mark.parametrize("T,H,B", [(1000, 2, 1), (3401, 6, 1), (77, 1, 2)])
def test_attention_x3_fp32_input_equals_planes_input(K, T, H, B):
    # the fp32-input kernel splits Q/K/V in-kernel exactly as split3 does: bit-identical planes out
    torch.manual_seed(4)
    qkv = torch.randn(B, T, 3 * H * 64, device="cuda")
    ref = _ref_attention(qkv, H, 64, 0.125)
    for waves, hb in ((7, None), (252, None), (64, 1)):
        a = torch.empty(3, B, T, H * 64, dtype=torch.bfloat16, device="cuda")
        b = torch.empty_like(a)
        K.attention_x3(K.split3(qkv), a, H, 64, 0.125, waves, head_block=hb)
        K.attention_x3f(qkv, b, H, 64, 0.125, waves, head_block=hb)
        torch.cuda.synchronize()
        assert torch.equal(a, b), (waves, hb)
        out = b[0].float() + b[1].float() + b[2].float()
        assert (out - ref).abs().max().item() < 2e-6


def test_detection_heads_fused_match_torch(K):
    # final LayerNorm + class/box MLPs (csrc/head.hip, three launches) vs the torch modules in fp32
    import torch.nn.functional as F
    from walkai_nos_amd.models.workload.yolos import YolosSmall
    torch.manual_seed(4)
    m = YolosSmall().cuda().eval()
    for p in list(m.cls_head.parameters()) + list(m.box_head.parameters()) + list(m.ln_f.parameters()):
        p.data.normal_(0, 0.05)
    det = torch.randn(100, 384, device="cuda")
    with torch.no_grad():
        logits, boxes = K.detection_heads(det, m.ln_f, m.cls_head.layers, m.box_head.layers)
        h = F.layer_norm(det.double(), (384,), m.ln_f.weight.double(), m.ln_f.bias.double(), m.ln_f.eps)

        def mlp(layers, x):
            for i, l in enumerate(layers):
                x = x @ l.weight.double().t() + l.bias.double()
                if i < len(layers) - 1:
                    x = torch.relu(x)
            return x
        ref_l, ref_b = mlp(m.cls_head.layers, h), torch.sigmoid(mlp(m.box_head.layers, h))
    torch.cuda.synchronize()
    assert logits.shape == (100, 92) and boxes.shape == (100, 4)
    assert (logits.double() - ref_l).abs().max().item() < 1e-5
    assert (boxes.double() - ref_b).abs().max().item() < 1e-6


def test_patch_planes_equal_im2col_split(K):
    torch.manual_seed(6)
    for (B, H, W, p) in [(1, 800, 1066, 16), (2, 64, 98, 16), (1, 36, 40, 4)]:
        px = torch.randn(B, 3, H, W, device="cuda")
        gh, gw = H // p, W // p
        cols = px[:, :, :gh * p, :gw * p].reshape(B, 3, gh, p, gw, p).permute(0, 2, 4, 1, 3, 5) \
            .reshape(B * gh * gw, 3 * p * p)
        planes = K.patch_planes(px, p)
        torch.cuda.synchronize()
        assert torch.equal(planes, K.split3(cols.contiguous())), (B, H, W, p)


@pytest.mark.parametrize("M,N,Kd", [(3401, 384, 1536), (3401, 384, 384), (300, 768, 256)])
def test_splitk_partials_and_combine_layernorm(K, M, N, Kd, monkeypatch):
    # split-K partial GEMM (every offered tile x split count, the opt-in staggered tile included) +
    # the combine/residual/LayerNorm kernel vs fp64; the partial planes sum to the unsplit product
    import torch.nn.functional as F
    from walkai_nos_amd.ops import gemm as G
    monkeypatch.setenv("NOS_X3_STAGGER", "1")
    torch.manual_seed(8)
    x3 = K.split3(torch.randn(M, Kd, device="cuda"))
    w = torch.randn(N, Kd, device="cuda") * 0.05
    b = torch.randn(N, device="cuda")
    r = torch.randn(M, N, device="cuda")
    r2 = torch.randn(1, 97, N, device="cuda")
    lw, lb = torch.randn(N, device="cuda"), torch.randn(N, device="cuda")
    a = x3.double().sum(0)
    hb = a @ G.weight_planes(w).double().sum(0).t()
    ref_x = hb + b.double() + r.double() + r2.double().reshape(97, N)[torch.arange(M) % 97]
    ref_ln = F.layer_norm(ref_x, (N,), lw.double(), lb.double(), 1e-12)
    cands = G.split_candidates(N, Kd)
    assert cands
    for cfg, sp in cands:
        part = G.gemm_x3_partials(x3, w, cfg, sp)
        x, planes = K.splitk_layernorm(part, b, r, r2, (lw, lb, 1e-12))
        torch.cuda.synchronize()
        assert (part.double().sum(0) - hb).abs().max().item() < 1e-4, (cfg, sp)
        assert (x.double() - ref_x).abs().max().item() < 1e-4, (cfg, sp)
        assert (planes.double().sum(0) - ref_ln).abs().max().item() < 1e-4, (cfg, sp)
        x_only, none = K.splitk_layernorm(part, b, r, None)
        torch.cuda.synchronize()
        assert none is None
        assert (x_only.double() - (hb + b.double() + r.double())).abs().max().item() < 1e-4, (cfg, sp)


@pytest.mark.parametrize("M,N,Kd", [(3401, 384, 1536), (3401, 384, 384), (300, 768, 256)])
def test_streamk_partials_and_combine_layernorm(K, M, N, Kd):
    # stream-K partials over every config and grids that cut tiles into 1..many segments (P = 1,
    # a prime, the chip's slots, more workgroups than units) + the combine/LayerNorm vs fp64
    import torch.nn.functional as F
    from walkai_nos_amd.ops import gemm as G
    torch.manual_seed(18)
    x3 = K.split3(torch.randn(M, Kd, device="cuda"))
    w = torch.randn(N, Kd, device="cuda") * 0.05
    b = torch.randn(N, device="cuda")
    r = torch.randn(M, N, device="cuda")
    r2 = torch.randn(1, 97, N, device="cuda")
    lw, lb = torch.randn(N, device="cuda"), torch.randn(N, device="cuda")
    hb = x3.double().sum(0) @ G.weight_planes(w).double().sum(0).t()
    ref_x = hb + b.double() + r.double() + r2.double().reshape(97, N)[torch.arange(M) % 97]
    ref_ln = F.layer_norm(ref_x, (N,), lw.double(), lb.double(), 1e-12)
    ran = 0
    for cfg, (bm, bn, bk, _) in G.X3K_TILES.items():
        if N % bn or Kd % bk:
            continue
        for P in (1, 7, 256, 512, 1 << 20):
            m = G.streamk_map(M, N, Kd, cfg, P)
            # planes a tile does not own stay NaN: the combine must never read them
            part, m2 = G.gemm_x3_streamk(x3, w, cfg, P, out=torch.full((m[6], M, N), float("nan"), device="cuda"))
            assert m2 == m
            x, planes = K.streamk_layernorm(part, m, b, r, r2, (lw, lb, 1e-12))
            torch.cuda.synchronize()
            assert (x.double() - ref_x).abs().max().item() < 1e-4, (cfg, P, m)
            assert (planes.double().sum(0) - ref_ln).abs().max().item() < 1e-4, (cfg, P, m)
            ran += 1
    assert ran >= 10


@pytest.mark.parametrize("M,N,Kd", [(3401, 1152, 384), (3401, 1536, 384), (300, 256, 64), (1, 128, 32)])
def test_gemm_x3_fp32_activation_matches_the_planes_kernel(K, M, N, Kd):
    # the fp32-A kernel splits the activation in registers exactly as split3 does: bit-identical
    # to the planes-in 16x16x32 8-wave tile of the same shape (29: 128x128, 36: 256x128)
    from walkai_nos_amd.ops import gemm as G
    torch.manual_seed(21)
    x = torch.randn(M, Kd, device="cuda")
    w = torch.randn(N, Kd, device="cuda") * 0.05
    b = torch.randn(N, device="cuda")
    for cfg, tile in ((0, 29), (1, 36)):
        if N % G.X3A_TILES[cfg][1]:
            continue
        y, y3 = G.gemm_x3_f32a(x, w, b, gelu=True, out_x3=True, cfg=cfg)
        r, r3 = G.gemm_x3(K.split3(x), w, b, gelu=True, out_f32=True, out_x3=True, tile=tile)
        torch.cuda.synchronize()
        assert torch.equal(y, r) and torch.equal(y3, r3), (cfg, (y - r).abs().max().item())


def test_linear_residual_ln_x3_tuned_pipeline(K):
    # whichever pipeline the tuner picks, the result matches the unfused ops
    from walkai_nos_amd.ops import gemm as G
    torch.manual_seed(9)
    M, N, Kd = 3401, 384, 1536
    f3 = K.split3(torch.randn(M, Kd, device="cuda"))
    w = torch.randn(N, Kd, device="cuda") * 0.05
    b = torch.randn(N, device="cuda")
    r = torch.randn(1, M, N, device="cuda")
    lw, lb = torch.ones(N, device="cuda"), torch.zeros(N, device="cuda")
    x, h3 = K.linear_residual_ln_x3(f3, w, b, r, ln=(lw, lb, 1e-12))
    x_ref = G.gemm_x3(f3, w, b, residual=r)
    h_ref = K.layernorm_x3(x_ref, lw, lb, 1e-12)
    torch.cuda.synchronize()
    assert x.shape == r.shape and h3.shape == (3,) + r.shape
    assert (x - x_ref).abs().max().item() < 1e-4
    assert (h3.double().sum(0) - h_ref.double().sum(0)).abs().max().item() < 1e-4
    assert G.fused_table()


@pytest.mark.parametrize("B,T,waves", [(1, 3401, None), (1, 3401, 32), (1, 3401, 126), (1, 3401, 500),
                                       (2, 77, 5), (2, 200, None), (3, 45, 7)])
def test_attention_merge_proj_layernorm_fused(K, B, T, waves):
    # attention partials + the fused merge / projection / residual / LayerNorm kernel vs fp64, over
    # stream-K grids that split query tiles 2-4 ways, leave whole groups to one workgroup, and
    # batches whose rows straddle the kernel's 32-row tiles; and vs the unfused fixup + GEMM + LN
    import torch.nn.functional as F
    from walkai_nos_amd.ops import gemm as G
    torch.manual_seed(12)
    H, Dh = 6, 64
    D = H * Dh
    qkv = torch.randn(B, T, 3 * D, device="cuda")
    w = torch.randn(D, D, device="cuda") * 0.05
    b = torch.randn(D, device="cuda")
    r = torch.randn(B, T, D, device="cuda")
    lw, lb = torch.randn(D, device="cuda"), torch.randn(D, device="cuda")
    x, h3 = K.attention_proj_ln_x3f(qkv, H, Dh, 0.125, w, b, r, (lw, lb, 1e-12), waves=waves)
    torch.cuda.synchronize()
    o = _ref_attention(qkv, H, Dh, 0.125).double()
    ref_x = o @ G.weight_planes(w).double().sum(0).t() + b.double() + r.double()
    ref_ln = F.layer_norm(ref_x, (D,), lw.double(), lb.double(), 1e-12)
    assert x.shape == r.shape and h3.shape == (3,) + r.shape
    assert (x.double() - ref_x).abs().max().item() < 1e-4
    assert (h3.double().sum(0) - ref_ln).abs().max().item() < 1e-4
    o3 = K.attention_qkv_x3f(qkv, H, Dh, 0.125)
    x2, h2 = K.linear_residual_ln_x3(o3, w, b, r, ln=(lw, lb, 1e-12))
    torch.cuda.synchronize()
    assert (x - x2).abs().max().item() < 1e-4
    assert (h3.double().sum(0) - h2.double().sum(0)).abs().max().item() < 1e-4


@pytest.mark.parametrize("B,T,waves", [(1, 3401, None), (1, 3401, 32), (2, 300, 7), (1, 77, 3)])
def test_attention_reciprocal_bookkeeping_bit_identical(K, B, T, waves):
    # the stream-K bookkeeping through f32-reciprocal divisions (default) and through 64-bit
    # divisions (flag bit 3) must place every unit identically: the outputs are bit-identical
    torch.manual_seed(13)
    H, Dh = 6, 64
    qkv = torch.randn(B, T, 3 * H * Dh, device="cuda")
    w = waves or K.attention_x3_waves(K.slice_cus(), B, T, H)
    outs = []
    L = K._L()
    try:
        for flags in (0, 8):
            L.nos_attention_x3_set_flags(flags)
            out = torch.empty(3, B, T, H * Dh, dtype=torch.bfloat16, device="cuda")
            outs.append(K.attention_x3f(qkv, out, H, Dh, 0.125, w).clone())
        torch.cuda.synchronize()
    finally:
        L.nos_attention_x3_set_flags(int(os.environ.get("NOS_ATTN_X3_FLAGS", "0")))
    assert torch.equal(outs[0], outs[1])
    ref = _ref_attention(qkv, H, Dh, 0.125).double()
    assert (outs[0].double().sum(0) - ref).abs().max().item() < 1e-5


@pytest.mark.parametrize("B,T,H,waves", [(1, 3401, 6, None), (1, 3401, 6, 7), (2, 300, 3, 64), (1, 77, 1, 3),
                                         (1, 1000, 2, 333)])
def test_attention_wide_kernel_bit_identical_to_two_wave_kernel(K, B, T, H, waves):
    # attn_fwd_x3w (one wave per SIMD, two query tiles per wave) runs each tile's arithmetic in the
    # order of attn_fwd_x3p<8> and writes the same partial slots: fp32 and x3-plane outputs are
    # bit-identical for every stream-K split, and fp32-accurate against fp64
    torch.manual_seed(21)
    qkv = torch.randn(B, T, 3 * H * 64, device="cuda")
    w = waves or K.attention_x3_waves(K.slice_cus(), B, T, H)
    ref = _ref_attention(qkv, H, 64, 0.125)
    try:
        for x3 in (False, True):
            outs = []
            for wide in (True, False):
                K.set_attention_x3_wide(wide)
                out = (torch.full((3, B, T, H * 64), float("nan"), dtype=torch.bfloat16, device="cuda") if x3
                       else torch.full((B, T, H * 64), float("nan"), device="cuda"))
                outs.append(K.attention_x3f(qkv, out, H, 64, 0.125, w))
            torch.cuda.synchronize()
            assert torch.equal(outs[0], outs[1]), (x3, w)
            o = outs[0].double().sum(0) if x3 else outs[0].double()
            assert (o - ref.double()).abs().max().item() < 2e-6, (x3, w)
            if x3:
                # the planes are the exact split of the fp32 output (direct and merged tiles alike)
                assert torch.equal(outs[0], K.split3(f32)), w
            else:
                f32 = outs[0]
    finally:
        K.set_attention_x3_wide(K.attention_x3_wide_default())


@pytest.mark.parametrize("B,T,H,waves,hb", [(1, 3401, 6, None, None), (1, 3401, 6, 32, 2), (2, 300, 3, 64, None),
                                            (1, 77, 1, 3, None), (1, 1000, 2, 333, 1)])
def test_attention_in_kernel_merge_matches_fixup_launch(K, B, T, H, waves, hb):
    # the wide kernel's in-kernel stream-K merge (the last workgroup of a row to finish merges its
    # partials) against the separate attn_sk_lds_fixup launch: bit-identical, fp32 and x3 planes,
    # for grids with empty ranges (333 workgroups for 256 units), head blocks, and back-to-back
    # launches that reuse the row counters (each launch leaves them zero)
    torch.manual_seed(22)
    qkv = torch.randn(B, T, 3 * H * 64, device="cuda")
    w = waves or K.attention_x3_waves(K.slice_cus(), B, T, H)
    try:
        K.set_attention_x3_wide(True)
        for x3 in (False, True):
            outs = []
            for merge in (True, False, True):
                K.set_attention_merge(merge)
                out = (torch.full((3, B, T, H * 64), float("nan"), dtype=torch.bfloat16, device="cuda") if x3
                       else torch.full((B, T, H * 64), float("nan"), device="cuda"))
                outs.append(K.attention_x3f(qkv, out, H, 64, 0.125, w, head_block=hb))
            torch.cuda.synchronize()
            assert torch.equal(outs[0], outs[1]), (x3, w)
            assert torch.equal(outs[2], outs[1]), (x3, w)
        assert int(K._row_counters(qkv.device, 1).abs().sum().item()) == 0
    finally:
        K.set_attention_merge(None)
        K.set_attention_x3_wide(K.attention_x3_wide_default())


@pytest.mark.parametrize("B,T,H,waves,hb", [(1, 3401, 6, None, None), (1, 3401, 6, 126, None), (1, 3401, 6, 32, 2),
                                            (2, 300, 3, 64, None), (1, 77, 1, 3, None), (1, 1000, 2, 333, 1)])
def test_attention_fixup_xcd_local_order_is_bit_identical(K, B, T, H, waves, hb):
    # the stream-K fixup merges every split tile once whichever order its blocks take them in: the
    # plain order (default) against the XCD-local one (flag bit 6), fp32 and x3 planes
    torch.manual_seed(23)
    qkv = torch.randn(B, T, 3 * H * 64, device="cuda")
    w = waves or K.attention_x3_waves(K.slice_cus(), B, T, H)
    L = K._L()
    try:
        for x3 in (False, True):
            outs = []
            for flags in (0, 64):
                L.nos_attention_x3_set_flags(flags)
                out = (torch.full((3, B, T, H * 64), float("nan"), dtype=torch.bfloat16, device="cuda") if x3
                       else torch.full((B, T, H * 64), float("nan"), device="cuda"))
                outs.append(K.attention_x3f(qkv, out, H, 64, 0.125, w, head_block=hb))
            torch.cuda.synchronize()
            assert not torch.isnan(outs[0].float()).any(), (x3, w)
            assert torch.equal(outs[0], outs[1]), (x3, w)
    finally:
        L.nos_attention_x3_set_flags(int(os.environ.get("NOS_ATTN_X3_FLAGS", "0")))
