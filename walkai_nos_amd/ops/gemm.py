"""fp32 GEMM with fused epilogues on the hand-written MFMA kernel (``csrc/gemm.hip``).

``gemm(x, w, bias=None, gelu=False, residual=None)`` computes ``x @ w^T (+ bias) (GELU) (+ residual)``
in one kernel. The tile shape (64x64, 128x64, 64x128 or 128x128; stage depth 32 or 64) is chosen per
``(M, N, K, epilogue, slice CUs)``: the first call of a new key outside HIP-graph capture times every
eligible tile on the caller's stream (3 reps each, replayed from a HIP graph so host launch overhead
is excluded) and caches the fastest together with
hipBLASLt (``torch.addmm``) as a candidate, so the kernel is only used where it actually wins on
the slice it runs on. During graph capture an untuned key falls back to a static heuristic (the tile
count that best fills the slice's workgroup slots).
"""
from __future__ import annotations

import ctypes
import threading
from typing import Dict, Optional, Tuple

import torch

from . import kernels as K

EPI_BIAS, EPI_GELU, EPI_RES, EPI_RES2 = 1, 2, 4, 8
#: config -> (BM, BN, BK): workgroup tile and stage depth
TILES = {0: (64, 64, 32), 1: (128, 64, 32), 2: (64, 128, 32), 3: (128, 128, 32),
         4: (64, 64, 64), 5: (128, 64, 64), 6: (64, 128, 64),
         7: (64, 64, 32), 8: (128, 64, 32), 9: (64, 128, 32)}  # 7-9: single-buffered LDS
#: resident workgroups per CU for each config (LDS- or VGPR-limited)
SLOTS_PER_CU = {0: 4, 1: 2, 2: 2, 3: 2, 4: 2, 5: 1, 6: 1, 7: 8, 8: 5, 9: 5}
LIBRARY = -1  # "use hipBLASLt" choice in the tuning cache

_lock = threading.Lock()
_cache: Dict[Tuple[int, int, int, int, int], int] = {}
_bound = False


def _lib() -> ctypes.CDLL:
    global _bound
    L = K._L()
    if not _bound:
        vp, i32 = ctypes.c_void_p, ctypes.c_int
        L.nos_gemm_f32.argtypes = [vp, vp, vp, vp, vp, i32, vp, i32, i32, i32, i32, i32, vp]
        L.nos_gemm_last_error.restype = ctypes.c_char_p
        _bound = True
    return L


def eligible(M: int, N: int, Kd: int) -> list:
    if Kd % 32 or M < 1:
        return []
    return [c for c, (bm, bn, bk) in TILES.items() if N % bn == 0 and Kd % bk == 0]


def heuristic(M: int, N: int, cus: int, cands: list) -> int:
    """Fewest 'rounds' of tiles over the slice's workgroup slots, then the larger tile."""
    best, best_key = cands[0], None
    for c in cands:
        bm, bn, _ = TILES[c]
        tiles = -(-M // bm) * (N // bn)
        slots = SLOTS_PER_CU[c] * cus
        rounds = -(-tiles // slots)
        # time ~ rounds x per-tile work / per-slot rate; bigger tiles run ~15% more efficiently
        est = rounds * bm * bn * (1.0 if bm * bn >= 8192 else 1.15) / (4.0 / SLOTS_PER_CU[c])
        key = (est, -bm * bn)
        if best_key is None or key < best_key:
            best, best_key = c, key
    return best


def _launch(cfg: int, x2: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor], res2: Optional[torch.Tensor],
            out: torch.Tensor, epi: int, r2: Optional[torch.Tensor] = None) -> None:
    M, Kd = x2.shape
    N = w.shape[0]
    rc = _lib().nos_gemm_f32(x2.data_ptr(), w.data_ptr(), bias.data_ptr() if bias is not None else None,
                             res2.data_ptr() if res2 is not None else None,
                             r2.data_ptr() if r2 is not None else None, r2.shape[0] if r2 is not None else 0,
                             out.data_ptr(), M, N, Kd, epi, cfg, torch.cuda.current_stream().cuda_stream)
    if rc != 0:
        raise RuntimeError(f"nos gemm failed: {_lib().nos_gemm_last_error().decode()} (rc={rc})")


def _library(x2, w, bias, res2, out, epi, r2=None) -> None:
    if epi & EPI_RES2:
        _library(x2, w, bias, res2, out, epi & ~EPI_RES2)
        M = out.shape[0]
        out.view(-1, r2.shape[0], out.shape[1]).add_(r2) if M % r2.shape[0] == 0 else out.add_(r2[:M])
        return
    if epi & EPI_RES:
        c = res2 + bias if bias is not None else res2
        torch.addmm(c, x2, w.t(), out=out)
    elif bias is not None and not epi & EPI_GELU:
        torch.addmm(bias, x2, w.t(), out=out)
    elif bias is not None:
        torch.mm(x2, w.t(), out=out)
        K.bias_gelu_(out, bias)
        return
    else:
        torch.mm(x2, w.t(), out=out)
    if epi & EPI_GELU:
        if epi & EPI_RES:
            raise ValueError("GELU with residual is not an epilogue of this model")
        K.gelu_epilogue(out)


def _gpu_time(fn, stream, reps: int = 3) -> float:
    """GPU milliseconds of ``reps`` calls. On a side stream (the slice's CU-masked stream in the
    bench) the calls are captured into a HIP graph and replayed, so host launch overhead is not
    timed; on the legacy default stream (no capture allowed) plain event timing is the fallback."""
    fn()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if stream.cuda_stream != 0:
        stream.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=stream):
            for _ in range(reps):
                fn()
        g.replay()
        st.record(stream)
        g.replay()
        en.record(stream)
        en.synchronize()
        return st.elapsed_time(en)
    st.record(stream)
    for _ in range(reps):
        fn()
    en.record(stream)
    en.synchronize()
    return st.elapsed_time(en)


def _tune(key, cands, x2, w, bias, res2, out, epi, r2=None) -> int:
    stream = torch.cuda.current_stream()
    timings = {}
    for c in cands + [LIBRARY]:
        fn = (lambda c=c: _library(x2, w, bias, res2, out, epi, r2)) if c == LIBRARY else \
            (lambda c=c: _launch(c, x2, w, bias, res2, out, epi, r2))
        timings[c] = _gpu_time(fn, stream)
    best = min(timings, key=timings.get)
    with _lock:
        _cache[key] = best
    return best


def choose(M: int, N: int, Kd: int, epi: int, cus: int) -> Optional[int]:
    with _lock:
        return _cache.get((M, N, Kd, epi, cus))


def gemm(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None, gelu: bool = False,
         residual: Optional[torch.Tensor] = None, tile: Optional[int] = None,
         residual2: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``x @ w^T (+bias) (GELU) (+residual) (+residual2)`` for fp32 CUDA tensors.

    ``residual2`` is ``[R, N]`` (or ``[1, R, N]``) broadcast over the batch by row index modulo R;
    ``out`` (contiguous ``[..., N]`` with ``M`` rows) receives the result in place; ``tile`` forces
    a config."""
    shp = x.shape
    x2 = x.reshape(-1, shp[-1]).contiguous()
    M, Kd = x2.shape
    N = w.shape[0]
    if out is None:
        out2 = torch.empty(M, N, dtype=x.dtype, device=x.device)
    else:
        if not out.is_contiguous() or out.numel() != M * N:
            raise ValueError("gemm: out must be contiguous with M x N elements")
        out2 = out.view(M, N)
    res2 = residual.reshape(M, N).contiguous() if residual is not None else None
    r2 = residual2.reshape(-1, N).contiguous() if residual2 is not None else None
    epi = (EPI_BIAS if bias is not None else 0) | (EPI_GELU if gelu else 0) | (EPI_RES if residual is not None else 0) \
        | (EPI_RES2 if residual2 is not None else 0)
    cands = eligible(M, N, Kd)
    result = out2.view(*shp[:-1], N) if out is None else out
    if tile is not None:
        _launch(tile, x2, w.contiguous(), bias, res2, out2, epi, r2)
        return result
    cus = K.slice_cus()
    key = (M, N, Kd, epi, cus)
    cfg = choose(*key)
    if cfg is None:
        if not cands:
            cfg = LIBRARY
        elif torch.cuda.is_current_stream_capturing():
            cfg = heuristic(M, N, cus, cands)
        else:
            cfg = _tune(key, cands, x2, w.contiguous(), bias, res2, out2, epi, r2)
    if cfg == LIBRARY:
        _library(x2, w, bias, res2, out2, epi, r2)
    else:
        _launch(cfg, x2, w.contiguous(), bias, res2, out2, epi, r2)
    return result


def tuning_table() -> Dict[str, str]:
    with _lock:
        return {f"M{m}_N{n}_K{k}_epi{e}_cus{c}": ("hipblaslt" if v == LIBRARY else "x".join(map(str, TILES[v][:2]))
                                                  + f"/k{TILES[v][2]}" + ("/sb" if v >= 7 else ""))
                for (m, n, k, e, c), v in sorted(_cache.items())}
