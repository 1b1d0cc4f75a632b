"""Hot-op dispatch for the workload model: hand-written HIP kernels on the GPU, PyTorch reference
math on the CPU.

On a GPU tensor the HIP path is mandatory unless the caller explicitly selects the ``torch``
backend (used only as the measured baseline in the benchmark's A/B mode): a missing
``libnos_kernels.so`` raises instead of silently falling back.

Kernels (``csrc/kernels.hip``, ``csrc/gemm_x3.hip``, ``csrc/gemm.hip``):

* fp32 matmuls run in the **x3** form by default (``set_fp32_matmul``): every fp32 operand as three
  exact bf16 planes, six bf16 MFMAs per block, fp32-accurate; producers emit planes directly
  (``layernorm_x3``, ``linear_x3(..., out_x3=True)``, ``attention_qkv_x3``);
* ``layernorm`` / ``layernorm_x3`` — one wave per row, two-pass mean/var in registers;
* ``linear_x3`` — x3 GEMM with bias / exact GELU / residual(s) fused into the store, tile and
  pipeline (register-staged, LDS-DMA ring, persistent) autotuned per (shape, slice);
* ``linear`` / ``linear_gelu`` / ``linear_residual`` — the f32-input-MFMA GEMM (``f32`` mode), tuned
  against hipBLASLt;
* ``attention_qkv_x3`` / ``attention_qkv`` — stream-K flash attention over the packed QKV tensor
  (software-pipelined x3 kernel, or the f32-MFMA kernel), persistent grid sized to the slice.
"""
from __future__ import annotations

import ctypes
import math
import os
import threading
from typing import Dict, Optional, Tuple

import torch
import torch.nn.functional as F

from .native import NativeUnavailable, available, load

LIB = "libnos_kernels.so"
_backend = threading.local()
_lib: Optional[ctypes.CDLL] = None
_lock = threading.Lock()


_slice = threading.local()


def set_slice_cus(n: Optional[int]) -> None:
    """Tell the kernels how many CUs the current stream may use (its CU mask / partition size), so
    launch decompositions fit the slice instead of assuming the whole 256-CU device."""
    _slice.cus = n


def env_mask_cus(mask: Optional[str] = None, device: int = 0) -> Optional[int]:
    """CUs the process-wide ``HSA_CU_MASK`` (``<dev>:<ranges>[;<dev>:<ranges>]``, what the nos device
    plugin's ``Allocate`` hands a container) leaves device ``device``; None when it does not mask it."""
    mask = os.environ.get("HSA_CU_MASK", "") if mask is None else mask
    for part in mask.split(";"):
        dev, _, ranges = part.partition(":")
        if not dev.strip().isdigit() or int(dev) != device or not ranges.strip():
            continue
        n = 0
        for r in ranges.split(","):
            lo, _, hi = r.strip().partition("-")
            n += (int(hi) - int(lo) + 1) if hi else 1
        return n
    return None


def slice_cus() -> int:
    """CUs the current stream may use: the thread's slice, else the process's ``HSA_CU_MASK``
    (a pod run as its own process), else the whole device."""
    return getattr(_slice, "cus", None) or env_mask_cus() or total_cus()


def set_slice_pin(mask: int) -> None:
    """Pin the current thread's launches to the XCDs in ``mask`` (bit x = XCD x; 0 = unpinned): the
    emulation of a compute partition on an SPX device (``csrc/pin.h``). The pin is thread-local on
    both sides, like the slice's CU count, and a captured HIP graph keeps the pin it was captured with."""
    mask = int(mask or 0)
    if not 0 <= mask <= 0xFF:
        raise ValueError("pin: XCD mask must fit 8 bits")
    _slice.pin = mask
    if hip_available():
        _check(_L().nos_set_pin(mask))


def slice_pin() -> int:
    return getattr(_slice, "pin", 0)


def total_cus() -> int:
    """CUs of the whole device (256 on MI355X; the device query when a GPU is visible)."""
    global _total_cus
    if _total_cus is None:
        try:
            import torch
            _total_cus = int(torch.cuda.get_device_properties(0).multi_processor_count) \
                if torch.cuda.is_available() else 256
        except Exception:  # noqa: BLE001 - CPU-only hosts, early import
            _total_cus = 256
    return _total_cus


_total_cus: Optional[int] = None


_waves_per_cu: Optional[int] = None
_variant = 0


def set_attention_variant(variant: int) -> None:
    """0 = LDS-shared K/V workgroup kernel (default); 2 / 3 = one-wave-per-tile stream-K kernel
    with 2 or 3 resident waves per SIMD (A/B reference)."""
    global _waves_per_cu, _variant
    _check(_L().nos_attention_set_variant(variant))
    _waves_per_cu = None
    _variant = variant


def attention_waves(cus: int, B: int = 0, T: int = 0, H: int = 0) -> int:
    """Persistent stream-K grid for a slice of ``cus`` CUs: every resident workgroup slot, once —
    except when that leaves fewer than ~30 (128-query x 32-key) units per workgroup (the whole
    256-CU GPU at T = 3401): then one slot per CU stays empty, so fewer tiles are split across
    workgroups and the partial/fixup traffic drops (measured: 164 vs 179 us on SPX)."""
    global _waves_per_cu
    if _waves_per_cu is None:
        _waves_per_cu = int(_L().nos_attention_waves_per_cu())
    per_cu = _waves_per_cu
    if T and _variant == 0:
        nk = (T + 31) // 32
        units = B * H * ((nk + 3) // 4) * nk
        while per_cu > 1 and units / (per_cu * cus) < 30:
            per_cu -= 1
    return per_cu * cus


_fp32 = threading.local()


def set_fp32_matmul(mode: str) -> None:
    """How fp32 products run on the matrix cores: ``x3`` (default) splits each fp32 operand
    exactly into three bf16 planes and sums the six significant cross products on the bf16 MFMA
    (fp32-accurate: the dropped terms are 2^-24 relative, the fp32 rounding level) at 6/16 of the
    f32-input MFMA's cycles; ``f32`` uses the f32-input MFMA (v_mfma_f32_32x32x2_f32)."""
    if mode not in ("x3", "f32"):
        raise ValueError(mode)
    _fp32.mode = mode


def get_fp32_matmul() -> str:
    return getattr(_fp32, "mode", "x3")


def split3(x: torch.Tensor) -> torch.Tensor:
    """fp32 tensor -> ``[3, *x.shape]`` bf16 planes with ``x == p0 + p1 + p2`` (exact for normal
    numbers): round-to-nearest-even bf16 of x, then of each exact f32 residual."""
    x = x.contiguous()
    out = torch.empty((3,) + tuple(x.shape), dtype=torch.bfloat16, device=x.device)
    if not x.is_cuda:
        r = x
        for i in range(3):
            out[i] = r.to(torch.bfloat16)
            r = r - out[i].float()
        return out
    _check(_L().nos_split3_f32(x.data_ptr(), out.data_ptr(), x.numel(), _stream()))
    return out


_x3_wg: Optional[int] = None


def set_attention_x3_pipelined(on: bool) -> None:
    """True (default): the software-pipelined x3 attention kernel; False: block-at-a-time (A/B)."""
    global _x3_wg
    _check(_L().nos_attention_x3_set_pipelined(1 if on else 0))
    _x3_wg = None


def set_attention_x3_group(g: int) -> None:
    """Query tiles per workgroup of the pipelined x3 kernel: 4 (two 256-thread workgroups per CU)
    or 8 (one 512-thread workgroup per CU sharing every K/V block: half the K/V traffic)."""
    global _x3_wg
    _check(_L().nos_attention_x3_set_group(int(g)))
    _x3_wg = None


def set_attention_x3_wide(on: bool) -> None:
    """fp32-input 8-tile attention: True (default) runs ``attn_fwd_x3w`` (``csrc/attn_wide.hip``) —
    one wave per SIMD carrying two 32-query tiles — False (``NOS_ATTN_WIDE=0``) the
    two-waves-per-SIMD ``attn_fwd_x3p<8>``. Same units, partials and per-tile arithmetic: the
    outputs are bit-identical (``profiles/attn_wide_ab_r6.json``: the wide kernel 4-8% faster)."""
    _check(_L().nos_attention_x3_set_wide(1 if on else 0))


def attention_x3_wide_default() -> bool:
    """The process's setting at load time (``NOS_ATTN_WIDE``; A/B code restores it)."""
    return os.environ.get("NOS_ATTN_WIDE", "1").strip() != "0"


def attention_x3_wide() -> bool:
    return bool(_L().nos_attention_x3_wide())


def attention_x3_group() -> int:
    return int(_L().nos_attention_x3_group())


def attention_x3_waves(cus: int, B: int = 0, T: int = 0, H: int = 0) -> int:
    """Persistent grid of the x3 attention kernel (same sizing rule as the f32 LDS kernel), trimmed
    to the largest multiple of half the query-group count when that keeps >= 90% of the slots: then
    stream-K segment boundaries fall on (or halfway through) query groups, so each workgroup runs
    one or two whole key ranges with one prologue each. Measured on the whole GPU (T = 3401, 84
    groups): 252 workgroups 100 us vs 256 120 us (`profiles/attn_grid_r2.json`); DPX 126 vs 128:
    145 vs 153 us; smaller slices keep every slot."""
    global _x3_wg
    if _x3_wg is None:
        _x3_wg = int(_L().nos_attention_x3_wg_per_cu())
    per_cu = _x3_wg
    if not T:
        return per_cu * cus
    nk = (T + 31) // 32
    g = attention_x3_group()
    groups = B * H * ((nk + g - 1) // g)
    units = groups * nk
    while per_cu > 1 and units / (per_cu * cus) < 30:
        per_cu -= 1
    slots = per_cu * cus
    half = max(1, groups // 2) if groups % 2 == 0 else groups
    aligned = (slots // half) * half
    return aligned if aligned >= 0.9 * slots else slots


_head_block: Optional[int] = None


def set_attention_head_block(n: Optional[int]) -> None:
    """Heads per x3 attention launch (None = the slice-size rule of :func:`attention_head_block`)."""
    global _head_block
    _head_block = n


def attention_head_block(cus: int, heads: int) -> int:
    """Heads per x3 attention launch on a slice of ``cus`` CUs. All heads in one launch puts every
    head's K/V planes in the L2 working set at once; on a small slice the heads run in blocks so
    its workgroups share one block's K/V (``NOS_ATTN_HEAD_BLOCK`` / :func:`set_attention_head_block`
    override the rule for A/B runs)."""
    env = os.environ.get("NOS_ATTN_HEAD_BLOCK")
    n = _head_block if _head_block is not None else (int(env) if env else heads)
    return max(1, min(heads, n))


def attention_x3(planes: torch.Tensor, out: torch.Tensor, heads: int, head_dim: int, scale: float,
                 waves: int, head_block: Optional[int] = None) -> torch.Tensor:
    """Stream-K attention over the x3 planes ``[3, B, T, 3*H*64]`` of a packed QKV tensor. ``out`` is
    fp32 ``[B, T, H*64]`` or bf16 ``[3, B, T, H*64]`` (the output leaves as x3 planes); the heads run
    ``head_block`` at a time (default: all)."""
    _, B, T, _ = planes.shape
    ws = torch.empty(waves * 2 * (64 * 32 + 64) * attention_x3_group(), dtype=torch.float32, device=planes.device)
    x3_out = out.dtype == torch.bfloat16
    hb = heads if head_block is None else max(1, min(heads, int(head_block)))
    for h0 in range(0, heads, hb):
        _check(_L().nos_attention_x3_sk_heads(planes.data_ptr(), planes[0].numel(),
                                              None if x3_out else out.data_ptr(), out.data_ptr() if x3_out else None,
                                              ws.data_ptr(), B, T, heads, h0, min(hb, heads - h0), head_dim, scale,
                                              waves, _stream()))
    return out


def attention_input_f32() -> bool:
    """True: the model hands attention an fp32 QKV tensor (the QKV GEMM writes 4 B per element instead
    of three bf16 planes; the kernel splits Q, K and V itself). ``NOS_ATTN_F32IN=0`` keeps planes."""
    return os.environ.get("NOS_ATTN_F32IN", "1") != "0" and attention_x3_group() == 8


_merge: Optional[bool] = None
_row_cnt: Dict[Tuple[int, int], torch.Tensor] = {}


def set_attention_merge(on: Optional[bool]) -> None:
    """True: the wide kernel merges split query tiles itself (the last workgroup of a row to finish
    merges the row's partials, ``csrc/attn_wide.hip``); False: the separate ``attn_sk_lds_fixup``
    launch. None: ``NOS_ATTN_MERGE`` (default off). Bit-identical outputs either way. Off because
    it measured slower (``profiles/attn_merge_ab_r6.json``: 149 vs 96 us on the whole GPU); the
    likely cause is the device-scope release / acquire around the hand-off, which compile to a
    write-back and an invalidate of the XCD's L2 (the per-XCD L2s are not coherent)."""
    global _merge
    _merge = on


def attention_merge_in_kernel() -> bool:
    if _merge is not None:
        return _merge
    return os.environ.get("NOS_ATTN_MERGE", "0").strip() == "1"


def _row_counters(device: torch.device, n: int) -> torch.Tensor:
    """The in-kernel merge's row counters for the current stream: zeroed once, left zero by every
    launch; one array per stream, because launches that share one must not overlap (launches on one
    stream never do)."""
    key = (device.index if device.index is not None else torch.cuda.current_device(), _stream())
    with _lock:
        c = _row_cnt.get(key)
        if c is None or c.numel() < n:
            c = torch.zeros(max(n, 1024), dtype=torch.int32, device=device)
            _row_cnt[key] = c
        return c


def attention_x3f(qkv: torch.Tensor, out: torch.Tensor, heads: int, head_dim: int, scale: float, waves: int,
                  head_block: Optional[int] = None) -> torch.Tensor:
    """:func:`attention_x3` from an fp32 packed QKV tensor ``[B, T, 3*H*64]`` (split in-kernel)."""
    B, T, _ = qkv.shape
    qkv = qkv.contiguous()
    ws = torch.empty(waves * 2 * (64 * 32 + 64) * attention_x3_group(), dtype=torch.float32, device=qkv.device)
    x3_out = out.dtype == torch.bfloat16
    hb = heads if head_block is None else max(1, min(heads, int(head_block)))
    L = _L()
    rows = B * hb * (((T + 31) // 32 + 7) // 8)
    cnt = _row_counters(qkv.device, rows) if attention_merge_in_kernel() and attention_x3_wide() else None
    for h0 in range(0, heads, hb):
        o, op = (None, out.data_ptr()) if x3_out else (out.data_ptr(), None)
        if cnt is not None:
            _check(L.nos_attention_x3f_sk_heads_merged(qkv.data_ptr(), o, op, ws.data_ptr(), cnt.data_ptr(),
                                                       cnt.numel(), B, T, heads, h0, min(hb, heads - h0), head_dim,
                                                       scale, waves, _stream()))
        else:
            _check(L.nos_attention_x3f_sk_heads(qkv.data_ptr(), o, op, ws.data_ptr(), B, T, heads, h0,
                                                min(hb, heads - h0), head_dim, scale, waves, _stream()))
    return out


def attention_qkv_x3f(qkv: torch.Tensor, heads: int, head_dim: int, scale: float) -> torch.Tensor:
    """fp32 packed QKV in, x3 planes ``[3, B, T, H*64]`` of the attention output out."""
    B, T, _ = qkv.shape
    if not _use_hip(qkv):
        return split3(attention_ref(qkv, heads, head_dim, scale))
    out = torch.empty(3, B, T, heads * head_dim, dtype=torch.bfloat16, device=qkv.device)
    cus = slice_cus()
    hb = attention_head_block(cus, heads)
    return attention_x3f(qkv, out, heads, head_dim, scale, attention_x3_waves(cus, B, T, hb), head_block=hb)


def attn_proj_fusable(heads: int, head_dim: int) -> bool:
    """``NOS_ATTN_PROJ_FUSED=1``: the attention -> projection -> LayerNorm step as two launches
    (attention partials, then csrc/attn_proj.hip's merge + projection + residual + LayerNorm) for the
    384-wide model with fp32 QKV in. Off by default: measured slower than fixup + tuned GEMM +
    LayerNorm (38 vs 29 us per layer on the whole GPU, ``profiles/attn_proj_fused_r3.json``) — a
    workgroup that owns whole rows must stream the whole x3 weight (884 KB) per 32 rows through the
    texture path, which is busy 80% of the kernel."""
    return (os.environ.get("NOS_ATTN_PROJ_FUSED", "0") == "1" and head_dim == 64 and heads * head_dim == 384
            and attention_input_f32())


def attention_proj_ln_x3f(qkv: torch.Tensor, heads: int, head_dim: int, scale: float, w: torch.Tensor,
                          b: torch.Tensor, residual: torch.Tensor, ln, waves: Optional[int] = None):
    """``x = residual + attention(qkv) @ w^T + b`` and the x3 planes of ``LayerNorm(x)`` (``ln =
    (weight, bias, eps)``): the x3 attention leaves its stream-K partials in the workspace and one
    kernel merges them, projects, adds bias and residual and normalises (csrc/attn_proj.hip), instead
    of the fixup, the projection GEMM and a LayerNorm kernel. Returns ``(x, planes)``."""
    B, T, _ = qkv.shape
    D = heads * head_dim
    if not _use_hip(qkv):
        o = attention_ref(qkv, heads, head_dim, scale)
        x = (residual.double() + o.double() @ w.double().t() + b.double()).float()
        return x, split3(F.layer_norm(x, (D,), ln[0], ln[1], ln[2]))
    from .gemm import weight_planes
    qkv = qkv.contiguous()
    if waves is None:
        waves = attention_x3_waves(slice_cus(), B, T, heads)
    ws = torch.empty(waves * 2 * (64 * 32 + 64) * 8, dtype=torch.float32, device=qkv.device)
    odirect = torch.empty(B, T, D, dtype=torch.float32, device=qkv.device)
    L = _L()
    _check(L.nos_attention_x3f_partials(qkv.data_ptr(), odirect.data_ptr(), ws.data_ptr(), B, T, heads, head_dim,
                                        scale, waves, _stream()))
    w3 = weight_planes(w)
    res = residual.contiguous()
    if res.shape != (B, T, D) and res.numel() != B * T * D:
        raise ValueError("attention_proj_ln_x3f: residual must hold B*T*D elements")
    x = torch.empty_like(res)
    planes = torch.empty((3,) + tuple(res.shape), dtype=torch.bfloat16, device=qkv.device)
    rc = L.nos_attn_merge_proj_ln(ws.data_ptr(), waves, odirect.data_ptr(), B, T, heads, w3.data_ptr(),
                                  w3[0].numel(), b.data_ptr(), res.data_ptr(), ln[0].data_ptr(), ln[1].data_ptr(),
                                  float(ln[2]), x.data_ptr(), planes.data_ptr(), _stream())
    if rc != 0:
        raise RuntimeError(f"nos kernel failed: {L.nos_attn_proj_last_error().decode()} (rc={rc})")
    return x, planes


def attention_qkv_x3(planes: torch.Tensor, heads: int, head_dim: int, scale: float) -> torch.Tensor:
    """x3 planes of packed QKV in, x3 planes ``[3, B, T, H*64]`` of the attention output out."""
    _, B, T, _ = planes.shape
    if not _use_hip(planes):
        qkv = (planes[0].double() + planes[1].double() + planes[2].double()).float()
        return split3(attention_ref(qkv, heads, head_dim, scale))
    out = torch.empty(3, B, T, heads * head_dim, dtype=torch.bfloat16, device=planes.device)
    cus = slice_cus()
    hb = attention_head_block(cus, heads)
    return attention_x3(planes, out, heads, head_dim, scale, attention_x3_waves(cus, B, T, hb), head_block=hb)


def set_backend(name: str) -> None:
    """``hip`` (default) or ``torch`` (reference math, GPU A/B baseline only)."""
    if name not in ("hip", "torch"):
        raise ValueError(name)
    _backend.name = name


def get_backend() -> str:
    return getattr(_backend, "name", "hip")


def hip_available() -> bool:
    return available(LIB)


def _L() -> ctypes.CDLL:
    global _lib
    with _lock:
        if _lib is None:
            L = load(LIB)
            vp, i32, f32 = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
            L.nos_layernorm_f32.argtypes = [vp, vp, vp, vp, vp, i32, i32, f32, vp]
            L.nos_layernorm_f32_grid.argtypes = [vp, vp, vp, vp, vp, i32, i32, f32, i32, vp]
            L.nos_bias_gelu_f32.argtypes = [vp, vp, i32, i32, vp]
            L.nos_attention_f32.argtypes = [vp, vp, i32, i32, i32, i32, f32, vp]
            L.nos_attention_f32_sk.argtypes = [vp, vp, vp, i32, i32, i32, i32, f32, i32, vp]
            L.nos_attention_ws_bytes.argtypes = [i32]
            L.nos_attention_ws_bytes.restype = ctypes.c_size_t
            L.nos_kernels_last_error.restype = ctypes.c_char_p
            L.nos_set_pin.argtypes = [ctypes.c_uint]
            L.nos_splitk_layernorm_f32.argtypes = [vp, i32, vp, vp, vp, i32, vp, vp, vp, vp, i32, i32, f32, i32, vp]
            L.nos_streamk_layernorm_f32.argtypes = [vp, vp, vp, vp, vp, i32, vp, vp, vp, vp, i32, i32, f32, i32, vp]
            L.nos_pin_mask.restype = ctypes.c_uint
            L.nos_split3_f32.argtypes = [vp, vp, ctypes.c_size_t, vp]
            L.nos_attention_x3_set_pipelined.argtypes = [i32]
            L.nos_attention_x3_set_group.argtypes = [i32]
            L.nos_attention_x3_set_wide.argtypes = [i32]
            L.nos_attention_x3_sk.argtypes = [vp, ctypes.c_size_t, vp, vp, vp, i32, i32, i32, i32, f32, i32, vp]
            L.nos_attention_x3_sk_heads.argtypes = [vp, ctypes.c_size_t, vp, vp, vp, i32, i32, i32, i32, i32, i32, f32,
                                                    i32, vp]
            L.nos_attention_x3f_sk_heads.argtypes = [vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, f32, i32, vp]
            L.nos_attention_x3f_sk_heads_merged.argtypes = [vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, f32,
                                                            i32, vp]
            L.nos_attention_x3f_partials.argtypes = [vp, vp, vp, i32, i32, i32, i32, f32, i32, vp]
            L.nos_attn_merge_proj_ln.argtypes = [vp, i32, vp, i32, i32, i32, vp, ctypes.c_size_t, vp, vp, vp, vp, f32,
                                                 vp, vp, vp]
            L.nos_attn_proj_last_error.restype = ctypes.c_char_p
            L.nos_attention_x3_set_flags.argtypes = [i32]
            L.nos_attention_x3_set_flags(int(os.environ.get("NOS_ATTN_X3_FLAGS", "0")))
            group = os.environ.get("NOS_ATTN_X3_GROUP")  # A/B switch for whole-model runs
            if group and L.nos_attention_x3_set_group(int(group)) != 0:
                raise RuntimeError(f"NOS_ATTN_X3_GROUP={group}: {L.nos_kernels_last_error().decode()}")
            _lib = L
        return _lib


def _use_hip(t: torch.Tensor) -> bool:
    if not t.is_cuda:
        return False
    if get_backend() == "torch":
        return False
    if not hip_available():
        raise NativeUnavailable(f"{LIB} is not built but a GPU tensor reached the HIP op path")
    return True


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _check(rc: int) -> None:
    if rc != 0:
        raise RuntimeError(f"nos kernel failed: {_L().nos_kernels_last_error().decode()} (rc={rc})")


def layernorm_wgs(rows: int) -> int:
    """LayerNorm workgroups (4 rows each, grid-stride): one per 4 rows on the whole GPU; a slice that
    shares the GPU launches ``NOS_LN_WG_PER_CU`` (default 4) per CU of the slice."""
    cus = slice_cus()
    if cus >= total_cus():
        return 0
    return cus * int(os.environ.get("NOS_LN_WG_PER_CU", "4"))


def layernorm(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, eps: float) -> torch.Tensor:
    if not _use_hip(x) or x.dtype != torch.float32:
        return F.layer_norm(x, (x.shape[-1],), w, b, eps)
    x = x.contiguous()
    D = x.shape[-1]
    rows = x.numel() // D
    if D % 4 != 0 or D > 64 * 4 * 8:
        return F.layer_norm(x, (D,), w, b, eps)
    out = torch.empty_like(x)
    _check(_L().nos_layernorm_f32_grid(x.data_ptr(), w.data_ptr(), b.data_ptr(), out.data_ptr(), None, rows, D, eps,
                                       layernorm_wgs(rows), _stream()))
    return out


def splitk_layernorm(part: torch.Tensor, bias: torch.Tensor, res: torch.Tensor, res2: Optional[torch.Tensor],
                     ln=None, shape=None):
    """``x = sum(part) + bias + res (+ res2 broadcast by row)`` from split-K partials ``[S, M, N]``
    (planes added in order), and with ``ln = (weight, bias, eps)`` LayerNorm(x) as x3 planes, in
    one kernel. Returns ``(x, planes or None)`` shaped like ``shape`` (default ``res.shape``)."""
    S, M, N = part.shape
    shape = tuple(shape if shape is not None else res.shape)
    x = torch.empty(shape, dtype=torch.float32, device=part.device)
    planes = torch.empty((3,) + shape, dtype=torch.bfloat16, device=part.device) if ln is not None else None
    r2 = res2.reshape(-1, N).contiguous() if res2 is not None else None
    res = res.contiguous()
    _check(_L().nos_splitk_layernorm_f32(part.data_ptr(), S, bias.data_ptr(), res.data_ptr(),
                                         r2.data_ptr() if r2 is not None else None, r2.shape[0] if r2 is not None else 0,
                                         x.data_ptr(), ln[0].data_ptr() if ln is not None else None,
                                         ln[1].data_ptr() if ln is not None else None,
                                         planes.data_ptr() if planes is not None else None, M, N,
                                         float(ln[2]) if ln is not None else 0.0, layernorm_wgs(M), _stream()))
    return x, planes


def streamk_layernorm(part: torch.Tensor, sk_map, bias: torch.Tensor, res: torch.Tensor,
                      res2: Optional[torch.Tensor], ln=None, shape=None):
    """:func:`splitk_layernorm` over stream-K partials (``gemm.gemm_x3_streamk``): ``sk_map`` is the
    launch's ``(P, U, nk, bm, bn, tiles_n, planes)``; tile t's first ``segments(t)`` planes are added
    in order (``csrc/streamk.h``)."""
    _, M, N = part.shape
    shape = tuple(shape if shape is not None else res.shape)
    x = torch.empty(shape, dtype=torch.float32, device=part.device)
    planes = torch.empty((3,) + shape, dtype=torch.bfloat16, device=part.device) if ln is not None else None
    r2 = res2.reshape(-1, N).contiguous() if res2 is not None else None
    res = res.contiguous()
    m = (ctypes.c_int * 6)(*[int(v) for v in sk_map[:6]])
    _check(_L().nos_streamk_layernorm_f32(part.data_ptr(), m, bias.data_ptr(), res.data_ptr(),
                                          r2.data_ptr() if r2 is not None else None, r2.shape[0] if r2 is not None else 0,
                                          x.data_ptr(), ln[0].data_ptr() if ln is not None else None,
                                          ln[1].data_ptr() if ln is not None else None,
                                          planes.data_ptr() if planes is not None else None, M, N,
                                          float(ln[2]) if ln is not None else 0.0, layernorm_wgs(M), _stream()))
    return x, planes


def linear_residual_ln_x3(a3: torch.Tensor, w: torch.Tensor, b: torch.Tensor, residual: torch.Tensor,
                          residual2: Optional[torch.Tensor] = None, ln=None):
    """``x = a @ w^T + b + residual (+ residual2)`` and (``ln = (weight, bias, eps)``) the x3 planes of
    LayerNorm(x); on the GPU the faster of the fused-epilogue GEMM + LayerNorm and the split-K
    partial GEMM + combine-and-LayerNorm kernel (``gemm.linear_residual_ln_x3``)."""
    if not _use_hip(a3) or a3.shape[-1] % 32 or residual.shape[-1] not in (384, 768):
        x = linear_x3(a3, w, b, residual=residual, residual2=residual2)
        return x, (layernorm_x3(x, ln[0], ln[1], ln[2]) if ln is not None else None)
    from .gemm import linear_residual_ln_x3 as fused
    return fused(a3, w, b, residual, residual2, ln)


def layernorm_x3(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, eps: float) -> torch.Tensor:
    """LayerNorm whose output leaves as x3 planes ``[3, *x.shape]`` bf16 (the next GEMM's operand)."""
    if not _use_hip(x):
        return split3(F.layer_norm(x, (x.shape[-1],), w, b, eps))
    x = x.contiguous()
    D = x.shape[-1]
    rows = x.numel() // D
    out = torch.empty((3,) + tuple(x.shape), dtype=torch.bfloat16, device=x.device)
    _check(_L().nos_layernorm_f32_grid(x.data_ptr(), w.data_ptr(), b.data_ptr(), None, out.data_ptr(), rows, D, eps,
                                       layernorm_wgs(rows), _stream()))
    return out


def bias_gelu_(y: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """In place ``y = GELU(y + b)`` (exact erf) with the HIP epilogue kernel."""
    N = y.shape[-1]
    if N % 4 != 0:
        y.copy_(F.gelu(y + b))
        return y
    _check(_L().nos_bias_gelu_f32(y.data_ptr(), b.data_ptr(), y.numel() // N, N, _stream()))
    return y


def gelu_epilogue(y: torch.Tensor) -> torch.Tensor:
    y.copy_(F.gelu(y))
    return y


def linear(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor]) -> torch.Tensor:
    """``x @ w^T + b`` on the MFMA GEMM (or hipBLASLt where the tuner found it faster)."""
    if not _use_hip(x) or x.dtype != torch.float32:
        return F.linear(x, w, b)
    from .gemm import gemm
    return gemm(x, w, b)


def linear_gelu(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """``GELU(x @ w^T + b)`` with bias and exact GELU fused into the GEMM's store."""
    if not _use_hip(x) or x.dtype != torch.float32:
        return F.gelu(F.linear(x, w, b))
    from .gemm import gemm
    return gemm(x, w, b, gelu=True)


def linear_residual(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, res: torch.Tensor,
                    res2: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``res + x @ w^T + b (+ res2)`` with bias and residual(s) fused into the GEMM's store;
    ``res2`` ([T, N], broadcast over the batch) is YOLOS's per-layer mid position embedding."""
    if not _use_hip(x) or x.dtype != torch.float32:
        y = res + F.linear(x, w, b)
        return y + res2 if res2 is not None else y
    from .gemm import gemm
    return gemm(x, w, b, residual=res, residual2=res2)


def x3_active(t: torch.Tensor) -> bool:
    """True when the model's fp32 products on ``t`` run in the x3 format on the HIP kernels."""
    return t.is_cuda and t.dtype == torch.float32 and get_fp32_matmul() == "x3" and _use_hip(t)


def linear_x3(a3: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor], gelu: bool = False,
              residual: Optional[torch.Tensor] = None, residual2: Optional[torch.Tensor] = None,
              out_x3: bool = False, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``a @ w^T + b`` (GELU) (+ residuals) from the x3 planes of ``a``; the result is fp32, or its x3
    planes when ``out_x3`` (for the next x3 consumer)."""
    if not _use_hip(a3):
        a = (a3[0].double() + a3[1].double() + a3[2].double()).float()
        y = F.linear(a, w, b)
        if gelu:
            y = F.gelu(y)
        if residual is not None:
            y = y + residual
        if residual2 is not None:
            y = y + residual2
        return split3(y) if out_x3 else y
    from .gemm import gemm_x3
    return gemm_x3(a3, w, b, gelu=gelu, residual=residual, residual2=residual2, out_f32=not out_x3, out_x3=out_x3,
                   out=out)


def _head_lib() -> ctypes.CDLL:
    L = _L()
    if not getattr(L, "_nos_head_bound", False):
        vp, i32 = ctypes.c_void_p, ctypes.c_int
        P = ctypes.POINTER
        L.nos_small_linear_f32.argtypes = [i32, P(vp), P(i32), P(vp), P(vp), P(vp), P(i32), P(i32), P(i32), i32, i32,
                                           vp, vp, ctypes.c_float, vp]
        L.nos_patch_planes_f32.argtypes = [vp, vp, i32, i32, i32, i32, i32, i32, i32, vp]
        L.nos_head_last_error.restype = ctypes.c_char_p
        L._nos_head_bound = True
    return L


ACT_NONE, ACT_RELU, ACT_SIGMOID = 0, 1, 2


def small_linear(groups, M: int, K: int, ln: Optional[Tuple[torch.Tensor, torch.Tensor, float]] = None) -> None:
    """Up to two row-aligned fp32 GEMMs in one launch (``csrc/head.hip``): each group is
    ``(x, ldx, w, b, y, ldy, act)`` with ``x``/``y`` device pointers (ints) or tensors whose rows are
    ``ldx``/``ldy`` apart; ``y[m, :n] = act(LN?(x[m, :K]) @ w.T + b)``; ``ln = (weight, bias, eps)``
    normalises x's rows (over K) while staging them. Exact fp32 FMAs on the vector ALUs."""
    L = _head_lib()
    n = len(groups)
    VP, I32 = ctypes.c_void_p * n, ctypes.c_int * n

    def ptr(t):
        return t if isinstance(t, int) else (t.data_ptr() if t is not None else None)
    xs = VP(*[ptr(g[0]) for g in groups])
    ldx = I32(*[g[1] for g in groups])
    ws = VP(*[g[2].data_ptr() for g in groups])
    bs = VP(*[ptr(g[3]) for g in groups])
    ys = VP(*[ptr(g[4]) for g in groups])
    ldy = I32(*[g[5] for g in groups])
    ns = I32(*[g[2].shape[0] for g in groups])
    acts = I32(*[g[6] for g in groups])
    lw, lb, eps = (ln[0].data_ptr(), ln[1].data_ptr(), float(ln[2])) if ln is not None else (None, None, 0.0)
    rc = L.nos_small_linear_f32(n, xs, ldx, ws, bs, ys, ldy, ns, acts, M, K, lw, lb, eps, _stream())
    if rc != 0:
        raise RuntimeError(f"nos small_linear failed: {L.nos_head_last_error().decode()} (rc={rc})")


def detection_heads(det: torch.Tensor, ln_f, cls_layers, box_layers) -> Tuple[torch.Tensor, torch.Tensor]:
    """YOLOS' final LayerNorm + class MLP + box MLP (3 Linear layers each, ReLU between, sigmoid on
    the boxes) on ``det`` ``[M, D]`` (contiguous rows) in three launches: layer 1 of both heads with
    the LayerNorm fused, then layers 2 and 3 of both heads side by side. Returns ``(logits, boxes)``."""
    M, D = det.shape
    c1, c2, c3 = cls_layers
    b1, b2, b3 = box_layers
    hid = c1.weight.shape[0]
    h1 = torch.empty(M, 2 * hid, device=det.device)
    h2 = torch.empty(M, 2 * hid, device=det.device)
    logits = torch.empty(M, c3.weight.shape[0], device=det.device)
    boxes = torch.empty(M, b3.weight.shape[0], device=det.device)
    eb = h1.element_size() * hid
    small_linear([(det, D, c1.weight, c1.bias, h1, 2 * hid, ACT_RELU),
                  (det, D, b1.weight, b1.bias, h1.data_ptr() + eb, 2 * hid, ACT_RELU)],
                 M, D, ln=(ln_f.weight, ln_f.bias, ln_f.eps))
    small_linear([(h1, 2 * hid, c2.weight, c2.bias, h2, 2 * hid, ACT_RELU),
                  (h1.data_ptr() + eb, 2 * hid, b2.weight, b2.bias, h2.data_ptr() + eb, 2 * hid, ACT_RELU)],
                 M, hid)
    small_linear([(h2, 2 * hid, c3.weight, c3.bias, logits, logits.shape[1], ACT_NONE),
                  (h2.data_ptr() + eb, 2 * hid, b3.weight, b3.bias, boxes, boxes.shape[1], ACT_SIGMOID)],
                 M, hid)
    return logits, boxes


def patch_planes(pixels: torch.Tensor, patch: int) -> Optional[torch.Tensor]:
    """x3 planes ``[3, B*gh*gw, C*p*p]`` of the patch matrix straight from the image (im2col and
    split in one kernel); None when the image layout does not allow it (odd patch or width)."""
    B, C, Hh, Ww = pixels.shape
    if patch % 2 or Ww % 2 or not pixels.is_contiguous():
        return None
    gh, gw = Hh // patch, Ww // patch
    out = torch.empty(3, B * gh * gw, C * patch * patch, dtype=torch.bfloat16, device=pixels.device)
    L = _head_lib()
    rc = L.nos_patch_planes_f32(pixels.data_ptr(), out.data_ptr(), B, C, Hh, Ww, patch, gh, gw, _stream())
    if rc != 0:
        raise RuntimeError(f"nos patch_planes failed: {L.nos_head_last_error().decode()} (rc={rc})")
    return out


def patch_embed(pixels: torch.Tensor, w: torch.Tensor, b: torch.Tensor, patch: int,
                pos: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Non-overlapping patch embedding (a stride-``patch`` conv) as one unfold copy + the MFMA GEMM,
    with the bias and the patch position embeddings (``pos``: [P, D]) fused into the store.
    Returns [B, P, D]; written into ``out`` ([B*P, D] contiguous) when given."""
    B, C, Hh, Ww = pixels.shape
    gh, gw = Hh // patch, Ww // patch
    if not _use_hip(pixels) or pixels.dtype != torch.float32:
        y = F.conv2d(pixels, w, b, stride=patch).flatten(2).transpose(1, 2)
        return y + pos if pos is not None else y
    def im2col() -> torch.Tensor:
        return pixels[:, :, :gh * patch, :gw * patch].reshape(B, C, gh, patch, gw, patch) \
            .permute(0, 2, 4, 1, 3, 5).reshape(B * gh * gw, C * patch * patch)
    if x3_active(pixels) and (C * patch * patch) % 32 == 0:
        from .gemm import gemm_x3
        planes = patch_planes(pixels, patch)
        y = gemm_x3(planes if planes is not None else split3(im2col()), w.reshape(w.shape[0], -1), b,
                    residual2=pos, out=out)
        return y.view(B, gh * gw, -1)
    cols = im2col()
    from .gemm import gemm
    y = gemm(cols, w.reshape(w.shape[0], -1), b, residual2=pos, out=out)
    return y.view(B, gh * gw, -1)


def attention_ref(qkv: torch.Tensor, heads: int, head_dim: int, scale: float) -> torch.Tensor:
    B, T, _ = qkv.shape
    q, k, v = qkv.view(B, T, 3, heads, head_dim).permute(2, 0, 3, 1, 4)
    o = F.scaled_dot_product_attention(q, k, v, scale=scale)
    return o.transpose(1, 2).reshape(B, T, heads * head_dim)


def attention_qkv(qkv: torch.Tensor, heads: int, head_dim: int, scale: float) -> torch.Tensor:
    if not _use_hip(qkv) or qkv.dtype != torch.float32 or head_dim != 64:
        return attention_ref(qkv, heads, head_dim, scale)
    qkv = qkv.contiguous()
    B, T, _ = qkv.shape
    out = torch.empty(B, T, heads * head_dim, dtype=qkv.dtype, device=qkv.device)
    if get_fp32_matmul() == "x3":
        cus = slice_cus()
        hb = attention_head_block(cus, heads)
        return attention_x3(split3(qkv), out, heads, head_dim, scale, attention_x3_waves(cus, B, T, hb),
                            head_block=hb)
    return attention_sk(qkv, out, heads, head_dim, scale, attention_waves(slice_cus(), B, T, heads))


def attention_sk(qkv: torch.Tensor, out: torch.Tensor, heads: int, head_dim: int, scale: float,
                 waves: int) -> torch.Tensor:
    """Stream-K launch with an explicit persistent grid of ``waves`` waves; the partial-segment
    workspace comes from the caller's stream-ordered allocator."""
    B, T, _ = qkv.shape
    L = _L()
    ws = torch.empty(L.nos_attention_ws_bytes(waves) // 4, dtype=torch.float32, device=qkv.device)
    _check(L.nos_attention_f32_sk(qkv.data_ptr(), out.data_ptr(), ws.data_ptr(), B, T, heads, head_dim, scale,
                                  waves, _stream()))
    return out


def attention_unsplit(qkv: torch.Tensor, heads: int, head_dim: int, scale: float) -> torch.Tensor:
    """One wave per (query tile, head): no workspace, normalised in-kernel (A/B reference)."""
    B, T, _ = qkv.shape
    out = torch.empty(B, T, heads * head_dim, dtype=qkv.dtype, device=qkv.device)
    _check(_L().nos_attention_f32(qkv.data_ptr(), out.data_ptr(), B, T, heads, head_dim, scale, _stream()))
    return out


def gelu_ref(x: torch.Tensor) -> torch.Tensor:
    return 0.5 * x * (1.0 + torch.erf(x / math.sqrt(2.0)))
