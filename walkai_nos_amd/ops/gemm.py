"""fp32 GEMMs with fused epilogues on hand-written MFMA kernels: the x3 GEMM (``csrc/gemm_x3.hip``,
:func:`gemm_x3`, the default model path — fp32-accurate on the bf16 matrix cores) and the
f32-input-MFMA GEMM (``csrc/gemm.hip``, :func:`gemm`).

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
import os
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


# ---- x3: fp32-accurate GEMM on the bf16 matrix cores (csrc/gemm_x3.hip) -------------------------
#: config -> (BM, BN, LDS buffers, pipeline): "r" = register-staged loads one stage ahead,
#: "d" = LDS-DMA (global_load_lds) with nbuf-1 stages in flight, "d8" / "d2" = the same with 8 / 2
#: waves per workgroup
X3_TILES = {0: (64, 64, 2, "r"), 1: (128, 64, 2, "r"), 2: (64, 128, 2, "r"), 3: (128, 128, 2, "r"),
            4: (64, 64, 1, "r"), 5: (128, 64, 1, "r"), 6: (64, 128, 1, "r"),
            7: (64, 64, 3, "d"), 8: (64, 64, 4, "d"), 9: (128, 64, 3, "d"), 10: (64, 128, 3, "d"),
            11: (128, 128, 3, "d"), 12: (64, 64, 2, "d"),
            13: (128, 128, 3, "d8"), 14: (128, 128, 2, "d8"),
            15: (32, 64, 3, "d2"), 16: (32, 64, 2, "d2"), 17: (64, 32, 2, "d2"),
            # 64-deep stages: whole 128-byte row segments per DMA lane group (K % 64 == 0)
            18: (64, 64, 2, "d64"), 19: (64, 64, 3, "d64"), 20: (64, 32, 2, "d64"), 21: (32, 64, 2, "d64"),
            22: (64, 32, 3, "d64"), 23: (128, 64, 2, "d864"), 24: (64, 128, 2, "d864"),
            25: (128, 64, 4, "d"), 26: (64, 128, 4, "d"),
            # v_mfma_f32_16x16x32_bf16 tiles
            27: (64, 64, 2, "m16"), 28: (64, 64, 3, "m16"), 29: (128, 128, 2, "m16w8"), 30: (32, 64, 2, "m16w2"),
            31: (64, 32, 2, "m16w2"),
            # 96/192-wide tiles: 216 tiles at M = 3401 for N = 384 / 1536 (one round on 256 CUs)
            32: (128, 192, 2, "d"), 33: (64, 96, 2, "d2"), 34: (64, 192, 2, "d2"),
            # 8 waves of 64x64 (a third fewer LDS fragment bytes per MFMA than 64x32 waves)
            35: (256, 128, 2, "d8"), 36: (256, 128, 2, "m16w8"), 37: (128, 256, 2, "d8"),
            # persistent stream-of-stages (grid = resident slots of the slice)
            100: (64, 64, 3, "p"), 101: (64, 64, 2, "p"), 102: (128, 128, 3, "p8"), 103: (64, 128, 3, "p"),
            104: (128, 64, 3, "p"), 105: (64, 64, 2, "p64"), 106: (64, 32, 2, "p64"), 107: (128, 64, 2, "p864"),
            108: (128, 64, 4, "p"), 109: (64, 128, 4, "p"), 110: (256, 128, 2, "p8"),
            # 8 waves on 16x16x32, the second half of the workgroup half a stage behind its SIMD
            # partners (gemm_x3t): three LDS buffers, one stage of DMA in flight. Opt-in
            # (NOS_X3_STAGGER=1): measured 1-5% slower than tile 29 (profiles/gemm_stagger_ab_r4.json)
            38: (128, 128, 3, "t16w8")}
#: persistent (stream-of-stages) configs: the grid is the slice's resident workgroup slots
X3_PERSISTENT = frozenset(c for c, t in X3_TILES.items() if t[3].startswith("p"))
#: resident workgroups per CU (LDS- or VGPR-limited)
X3_SLOTS_PER_CU = {0: 2, 1: 1, 2: 1, 3: 1, 4: 5, 5: 3, 6: 3, 7: 2, 8: 1, 9: 1, 10: 1, 11: 1, 12: 3,
                   13: 1, 14: 1, 15: 2, 16: 4, 17: 4,
                   18: 1, 19: 1, 20: 2, 21: 2, 22: 1, 23: 1, 24: 1, 25: 1, 26: 1, 27: 3, 28: 2, 29: 1, 30: 4, 31: 4,
                   32: 1, 33: 2, 34: 1, 35: 1, 36: 1, 37: 1, 38: 1,
                   100: 2, 101: 3, 102: 1, 103: 1, 104: 1, 105: 1, 106: 2, 107: 1, 108: 1, 109: 1, 110: 1}
_x3_cache: Dict[Tuple[int, int, int, int, int, int, int], int] = {}
#: the x3 tuner's timings per key (ms for 3 graph-replayed calls), for tools/model_replay.py --tables
_x3_times: Dict[Tuple[int, int, int, int, int, int, int], Dict[int, float]] = {}
_x3_bound = False


def _lib_x3() -> ctypes.CDLL:
    global _x3_bound
    L = K._L()
    if not _x3_bound:
        vp, i32, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
        L.nos_gemm_x3.argtypes = [vp, sz, vp, sz, vp, vp, vp, i32, vp, vp, sz, i32, i32, i32, i32, i32, vp]
        L.nos_gemm_x3_persistent.argtypes = [vp, sz, vp, sz, vp, vp, vp, i32, vp, vp, sz, i32, i32, i32, i32, i32,
                                             i32, vp]
        L.nos_gemm_x3_last_error.restype = ctypes.c_char_p
        L.nos_gemm_x3_partials.argtypes = [vp, sz, vp, sz, vp, i32, i32, i32, i32, i32, vp]
        L.nos_gemm_x3_set_group.argtypes = [i32]
        L.nos_gemm_x3_f32a.argtypes = [vp, vp, sz, vp, vp, vp, i32, vp, vp, sz, i32, i32, i32, i32, i32, vp]
        L.nos_gemm_x3_streamk_map.argtypes = [i32, i32, i32, i32, i32, vp]
        L.nos_gemm_x3_streamk.argtypes = [vp, sz, vp, sz, vp, i32, i32, i32, i32, i32, vp]
        L.nos_gemm_x3_set_ablate.argtypes = [i32]
        ablate = int(os.environ.get("NOS_X3_ABLATE", "0"))  # timing studies only: results are invalid
        if ablate:
            import logging
            logging.getLogger("nos.gemm").warning("NOS_X3_ABLATE=%d: x3 GEMM operand loads / stores skipped, "
                                                  "results are INVALID (timing study)", ablate)
        L.nos_gemm_x3_set_ablate(ablate)
        g = int(os.environ.get("NOS_X3_GROUP_M", str(X3_GROUP_M)))
        if L.nos_gemm_x3_set_group(g) != 0:
            raise RuntimeError(f"NOS_X3_GROUP_M={g}: {L.nos_gemm_x3_last_error().decode()}")
        _x3_bound = True
    return L


#: tile rows per group of the x3 GEMMs' grouped tile order (1 = row-major); NOS_X3_GROUP_M overrides
X3_GROUP_M = 1


def set_group_m(g: int) -> None:
    """Grouped tile order of the x3 GEMMs: ``g`` tile rows walked per column step (1 = row-major)."""
    L = _lib_x3()
    if L.nos_gemm_x3_set_group(int(g)) != 0:
        raise ValueError(L.nos_gemm_x3_last_error().decode())


def weight_planes(w: torch.Tensor) -> torch.Tensor:
    """x3 planes of a weight, split once and cached ON the weight tensor (its view base, for a view
    such as the patch embedding's reshaped kernel) and re-split when the weight is modified in
    place (its version counter moves). Keying on the tensor object — not its address — keeps a
    freed weight's planes from being served to a new tensor that reuses the memory."""
    owner = w._base if w._base is not None else w
    key = (w.storage_offset(), tuple(w.shape), tuple(w.stride()))
    cache = owner.__dict__.setdefault("_nos_x3", {})
    hit = cache.get(key)
    if hit is not None and hit[0] == w._version:
        return hit[1]
    if w.is_cuda and torch.cuda.is_current_stream_capturing():
        raise RuntimeError("weight_planes: weights must be split before graph capture (run one eager forward)")
    p = K.split3(w.detach().contiguous())
    cache[key] = (w._version, p)
    return p


def x3_eligible(N: int, Kd: int) -> list:
    """Tiles that can run this shape; ``NOS_X3_EXCLUDE`` (comma-separated kind prefixes, e.g.
    ``m16,p``), ``NOS_X3_DROP`` (comma-separated tile ids) and ``NOS_X3_MIN_TILE`` (minimum BM*BN)
    drop tiles from autotuning for A/B runs."""
    if Kd % 32:
        return []
    skip = tuple(x for x in os.environ.get("NOS_X3_EXCLUDE", "").split(",") if x)
    drop = {int(x) for x in os.environ.get("NOS_X3_DROP", "").split(",") if x}
    min_area = int(os.environ.get("NOS_X3_MIN_TILE", "0"))
    stagger = os.environ.get("NOS_X3_STAGGER", "0") == "1"  # the staggered tile: measured slower, opt-in
    return [c for c, (bm, bn, _, kind) in X3_TILES.items()
            if N % bn == 0 and (not kind.endswith("64") or Kd % 64 == 0) and not (skip and kind.startswith(skip))
            and bm * bn >= min_area and c not in drop and (stagger or not kind.startswith("t"))]


#: tiles at least this large (BM*BN) on a partition that shares the GPU with sibling partitions
SHARED_SLICE_MIN_TILE = 8192


def shared_slice_tiles(cands: list, cus: int) -> list:
    """Tiles for a slice smaller than the GPU. Autotuning times each tile alone on its slice, but a
    partition runs beside its siblings and they share every XCD's L2 and the Infinity Cache:
    there a 128-wide tile, which moves half the operand bytes of a 64x64 one, wins although
    the isolated timing calls them even (measured on concurrent partitions: QPX +3%, CPX +2-4%,
    DPX/SPX unchanged; `profiles/kbench_r1_modes_min_tile.txt`). Whole-GPU slices keep every tile."""
    if cus >= K.total_cus() or "NOS_X3_MIN_TILE" in os.environ:
        return cands
    big = [c for c in cands if X3_TILES[c][0] * X3_TILES[c][1] >= SHARED_SLICE_MIN_TILE]
    return big or cands


_TUNED_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "x3_tuned.json")
_tuned: Optional[Dict[str, int]] = None


def tuned_table() -> Dict[str, int]:
    """Tiles measured on CONCURRENT sibling partitions (``tools/contention.py --emit-table``): the
    isolated autotuner cannot see what a slice's neighbours cost it, so where the table has the
    exact (shape, epilogue, outputs, slice size) key its tile wins. ``NOS_X3_TUNED=0`` ignores it,
    ``NOS_X3_TUNED_PATH`` reads another table."""
    global _tuned
    if _tuned is None:
        table: Dict[str, int] = {}
        path = os.environ.get("NOS_X3_TUNED_PATH", _TUNED_PATH)  # another table (A/B runs)
        if os.environ.get("NOS_X3_TUNED", "1") != "0" and os.path.exists(path):
            import json
            with open(path) as f:
                table = {k: int(v["tile"]) for k, v in json.load(f).items() if int(v["tile"]) in X3_TILES}
        _tuned = table
    return _tuned


def x3_heuristic(M: int, N: int, cus: int, cands: list) -> int:
    best, best_key = cands[0], None
    for c in cands:
        bm, bn, _, _ = X3_TILES[c]
        tiles = -(-M // bm) * (N // bn)
        rounds = -(-tiles // (X3_SLOTS_PER_CU[c] * cus))
        key = (rounds * bm * bn / min(X3_SLOTS_PER_CU[c], 2), -bm * bn)
        if best_key is None or key < best_key:
            best, best_key = c, key
    return best


def _launch_x3(cfg, a3, w3, bias, res, r2, out, out3, epi) -> None:
    _, M, Kd = a3.shape
    N = w3.shape[1]
    args = (a3.data_ptr(), a3[0].numel(), w3.data_ptr(), w3[0].numel(),
            bias.data_ptr() if bias is not None else None,
            res.data_ptr() if res is not None else None,
            r2.data_ptr() if r2 is not None else None, r2.shape[0] if r2 is not None else 0,
            out.data_ptr() if out is not None else None,
            out3.data_ptr() if out3 is not None else None, out3[0].numel() if out3 is not None else 0,
            M, N, Kd, epi)
    stream = torch.cuda.current_stream().cuda_stream
    if cfg >= 100:
        grid = max(1, X3_SLOTS_PER_CU[cfg] * K.slice_cus() - int(os.environ.get("NOS_X3_PGRID_SLACK", "0")))
        rc = _lib_x3().nos_gemm_x3_persistent(*args, cfg - 100, grid, stream)
    else:
        rc = _lib_x3().nos_gemm_x3(*args, cfg, stream)
    if rc != 0:
        raise RuntimeError(f"nos gemm_x3 failed: {_lib_x3().nos_gemm_x3_last_error().decode()} (rc={rc})")


def gemm_x3(a3: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None, gelu: bool = False,
            residual: Optional[torch.Tensor] = None, residual2: Optional[torch.Tensor] = None,
            out_f32: bool = True, out_x3: bool = False, out: Optional[torch.Tensor] = None,
            tile: Optional[int] = None):
    """fp32-accurate ``a @ w^T (+bias) (GELU) (+residual) (+residual2)`` from x3 planes.

    ``a3``: ``[3, ..., K]`` bf16 planes of the fp32 activation; ``w``: the fp32 weight ``[N, K]``
    (split once, cached) or its planes ``[3, N, K]``. Returns the fp32 result ``[..., N]`` and/or its
    x3 planes ``[3, ..., N]`` (a tuple when both are requested)."""
    lead = a3.shape[1:-1]
    Kd = a3.shape[-1]
    a3 = a3.reshape(3, -1, Kd)
    if not a3.is_contiguous():
        a3 = a3.contiguous()
    M = a3.shape[1]
    w3 = w if w.dim() == 3 else weight_planes(w)
    N = w3.shape[1]
    dev = a3.device
    o = None
    if out_f32:
        if out is not None:
            if not out.is_contiguous() or out.numel() != M * N:
                raise ValueError("gemm_x3: out must be contiguous with M x N elements")
            o = out.view(M, N)
        else:
            o = torch.empty(M, N, dtype=torch.float32, device=dev)
    o3 = torch.empty(3, M, N, dtype=torch.bfloat16, device=dev) if out_x3 else None
    res = residual.reshape(M, N).contiguous() if residual is not None else None
    r2 = residual2.reshape(-1, N).contiguous() if residual2 is not None else None
    epi = (EPI_BIAS if bias is not None else 0) | (EPI_GELU if gelu else 0) | (EPI_RES if residual is not None else 0) \
        | (EPI_RES2 if residual2 is not None else 0)
    if tile is None:
        cus, pin = K.slice_cus(), K.slice_pin()
        key = (M, N, Kd, epi, int(out_f32) | 2 * int(out_x3), cus, pin)
        with _lock:
            tile = _x3_cache.get(key)
        if tile is None and not pin:  # the contention table was measured on spread (unpinned) slices
            tile = tuned_table().get(f"M{M}_N{N}_K{Kd}_epi{epi}_out{key[4]}_cus{cus}")
            if tile is not None and N % X3_TILES[tile][1] == 0:
                with _lock:
                    _x3_cache[key] = tile
            else:
                tile = None
        if tile is None:
            cands = x3_eligible(N, Kd)
            if not cands:
                raise ValueError(f"gemm_x3: unsupported shape N={N} K={Kd}")
            if not pin:  # a pinned partition owns its XCDs' L2s: tiles are timed as it runs them
                cands = shared_slice_tiles(cands, cus)
            else:
                # pinned launches dispatch 8 / popcount(pin) physical workgroups per logical one (the
                # others exit at once, pin.h): only the persistent kernels keep that to one round
                cands = [c for c in cands if c in X3_PERSISTENT] or cands
            if torch.cuda.is_current_stream_capturing():
                tile = x3_heuristic(M, N, cus, cands)
            else:
                stream = torch.cuda.current_stream()
                times = {c: _gpu_time(lambda c=c: _launch_x3(c, a3, w3, bias, res, r2, o, o3, epi), stream)
                         for c in cands}
                tile = min(times, key=times.get)
                with _lock:
                    _x3_cache[key] = tile
                    _x3_times[key] = times
    _launch_x3(tile, a3, w3, bias, res, r2, o, o3, epi)
    rf = None if o is None else (o.view(*lead, N) if out is None else out)
    r3 = None if o3 is None else o3.view(3, *lead, N)
    if out_f32 and out_x3:
        return rf, r3
    return rf if out_f32 else r3


# ---- fp32 activation operand (csrc/gemm_x3.hip gemm_x3a) ---------------------------------------
#: fp32-A configs -> (BM, BN): 8 waves on 16x16x32, A split into planes in the kernel
X3A_TILES = {0: (128, 128), 1: (256, 128)}


def gemm_x3_f32a(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None, gelu: bool = False,
                 residual: Optional[torch.Tensor] = None, residual2: Optional[torch.Tensor] = None,
                 out_f32: bool = True, out_x3: bool = False, cfg: int = 0):
    """:func:`gemm_x3` with the activation as fp32 rows ``[..., K]`` (4 B per element instead of
    three 2-B planes): the kernel splits it into the same planes in registers, so the result is
    bit-identical to ``gemm_x3(K.split3(x), ...)`` on the 16x16x32 8-wave tile of the same shape."""
    lead = x.shape[:-1]
    Kd = x.shape[-1]
    x2 = x.reshape(-1, Kd)
    if not x2.is_contiguous():
        x2 = x2.contiguous()
    M = x2.shape[0]
    w3 = w if w.dim() == 3 else weight_planes(w)
    N = w3.shape[1]
    o = torch.empty(M, N, dtype=torch.float32, device=x.device) if out_f32 else None
    o3 = torch.empty(3, M, N, dtype=torch.bfloat16, device=x.device) if out_x3 else None
    res = residual.reshape(M, N).contiguous() if residual is not None else None
    r2 = residual2.reshape(-1, N).contiguous() if residual2 is not None else None
    epi = (EPI_BIAS if bias is not None else 0) | (EPI_GELU if gelu else 0) | (EPI_RES if residual is not None else 0) \
        | (EPI_RES2 if residual2 is not None else 0)
    rc = _lib_x3().nos_gemm_x3_f32a(x2.data_ptr(), w3.data_ptr(), w3[0].numel(),
                                    bias.data_ptr() if bias is not None else None,
                                    res.data_ptr() if res is not None else None,
                                    r2.data_ptr() if r2 is not None else None, r2.shape[0] if r2 is not None else 0,
                                    o.data_ptr() if o is not None else None,
                                    o3.data_ptr() if o3 is not None else None, o3[0].numel() if o3 is not None else 0,
                                    M, N, Kd, epi, cfg, torch.cuda.current_stream().cuda_stream)
    if rc != 0:
        raise RuntimeError(f"nos gemm_x3 f32a failed: {_lib_x3().nos_gemm_x3_last_error().decode()} (rc={rc})")
    rf = None if o is None else o.view(*lead, N)
    r3 = None if o3 is None else o3.view(3, *lead, N)
    if out_f32 and out_x3:
        return rf, r3
    return rf if out_f32 else r3


# ---- split-K partials + combine-and-LayerNorm --------------------------------------------------
#: LDS-DMA tiles offered to the split-K partial path (32x32 MFMA and 16x16 MFMA, 4 and 8 waves)
SPLIT_TILES = (7, 9, 10, 11, 12, 13, 14, 18, 23, 24, 29, 32, 35, 36, 38)
SPLIT_COUNTS = (2, 3, 4)
#: smallest slice that times split-K against the fused path: on 32-CU (CPX) slices the isolated
#: timing picks split-K, but with all eight partitions busy the fused path serves 2% more
#: (383.0 vs 375.6 inf/s per GPU; 64-CU request lanes keep split-K: 438.6 vs 430.7,
#: profiles/splitk_slice_ab_r2.json)
SPLITK_MIN_CUS = 64


def gemm_x3_partials(a3: torch.Tensor, w: torch.Tensor, cfg: int, splits: int,
                     out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Split-K partial sums of ``a @ w^T``: ``[splits, M, N]`` fp32, plane s summing the s-th K range
    (``csrc/gemm_x3.hip``, one launch of tiles x splits workgroups, no epilogue). The consumer adds
    the planes (``kernels.splitk_layernorm``): the hand-off is the kernel boundary."""
    Kd = a3.shape[-1]
    a3 = a3.reshape(3, -1, Kd)
    if not a3.is_contiguous():
        a3 = a3.contiguous()
    M = a3.shape[1]
    w3 = w if w.dim() == 3 else weight_planes(w)
    N = w3.shape[1]
    if out is None:
        out = torch.empty(splits, M, N, dtype=torch.float32, device=a3.device)
    rc = _lib_x3().nos_gemm_x3_partials(a3.data_ptr(), a3[0].numel(), w3.data_ptr(), w3[0].numel(), out.data_ptr(),
                                        M, N, Kd, cfg, splits, torch.cuda.current_stream().cuda_stream)
    if rc != 0:
        raise RuntimeError(f"nos gemm_x3 partials failed: {_lib_x3().nos_gemm_x3_last_error().decode()} (rc={rc})")
    return out


# ---- stream-K partials --------------------------------------------------------------------------
#: stream-K configs (csrc/gemm_x3.hip gemm_x3k) -> (BM, BN, K stage depth, resident workgroups per CU)
X3K_TILES = {0: (64, 64, 32, 2), 1: (128, 64, 64, 1), 2: (64, 128, 64, 1), 3: (128, 64, 32, 1), 4: (64, 64, 64, 1),
             5: (128, 128, 32, 1)}


def streamk_map(M: int, N: int, Kd: int, cfg: int, P: int) -> Tuple[int, ...]:
    """The work split of a stream-K launch: ``(P, U, nk, bm, bn, tiles_n, planes)`` (P clamped to
    the unit count; ``planes`` = depth of the partial buffer)."""
    out = (ctypes.c_int * 7)()
    if _lib_x3().nos_gemm_x3_streamk_map(M, N, Kd, cfg, P, out) != 0:
        raise ValueError(_lib_x3().nos_gemm_x3_last_error().decode())
    return tuple(out)


def gemm_x3_streamk(a3: torch.Tensor, w: torch.Tensor, cfg: int, P: int,
                    out: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, Tuple[int, ...]]:
    """Stream-K partial sums of ``a @ w^T`` over ``P`` workgroups: ``([planes, M, N] fp32, map)``;
    plane s of tile t holds its s-th K segment for s < segments(t) (``csrc/streamk.h``), the rest is
    never written. ``kernels.streamk_layernorm`` with the same map is the consumer."""
    Kd = a3.shape[-1]
    a3 = a3.reshape(3, -1, Kd)
    if not a3.is_contiguous():
        a3 = a3.contiguous()
    M = a3.shape[1]
    w3 = w if w.dim() == 3 else weight_planes(w)
    N = w3.shape[1]
    m = streamk_map(M, N, Kd, cfg, P)
    if out is not None and (tuple(out.shape) != (m[6], M, N) or not out.is_contiguous()):
        raise ValueError(f"gemm_x3_streamk: out must be a contiguous [{m[6]}, {M}, {N}] buffer")
    part = out if out is not None else torch.empty(m[6], M, N, dtype=torch.float32, device=a3.device)
    rc = _lib_x3().nos_gemm_x3_streamk(a3.data_ptr(), a3[0].numel(), w3.data_ptr(), w3[0].numel(), part.data_ptr(),
                                       M, N, Kd, cfg, m[0], torch.cuda.current_stream().cuda_stream)
    if rc != 0:
        raise RuntimeError(f"nos gemm_x3 stream-K failed: {_lib_x3().nos_gemm_x3_last_error().decode()} (rc={rc})")
    return part, m


def streamk_candidates(N: int, Kd: int, cus: int) -> list:
    """(config, P) pairs that can run this shape: P = the slice's resident workgroup slots (and,
    for two-slot tiles, one per CU)."""
    out = []
    for c, (bm, bn, bk, slots) in X3K_TILES.items():
        if N % bn or Kd % bk:
            continue
        out += [(c, s * cus) for s in range(slots, 0, -1)]
    return out


def split_candidates(N: int, Kd: int) -> list:
    """(tile, splits) pairs that can run this shape in the partials mode."""
    out = []
    for c in SPLIT_TILES:
        bm, bn, _, kind = X3_TILES[c]
        if kind.startswith("t") and os.environ.get("NOS_X3_STAGGER", "0") != "1":
            continue
        bk = 64 if kind.endswith("64") else 32
        if N % bn or Kd % bk:
            continue
        out += [(c, sp) for sp in SPLIT_COUNTS if Kd // bk >= 2 * sp]
    return out


_fused_cache: Dict[tuple, tuple] = {}
#: the tuner's timings per key (ms for 3 graph-replayed calls), for tools/model_replay.py --tables
_fused_times: Dict[tuple, Dict[tuple, float]] = {}


def linear_residual_ln_x3(a3: torch.Tensor, w: torch.Tensor, b: torch.Tensor, residual: torch.Tensor,
                          residual2: Optional[torch.Tensor] = None, ln=None):
    """``x = a @ w^T + b + residual (+ residual2)`` and, with ``ln = (weight, bias, eps)``, the x3
    planes of LayerNorm(x): the transformer's projection/fc2 step and the LayerNorm after it. Two
    pipelines, picked per (shape, slice) by timing both on the caller's stream: the fused-epilogue
    GEMM + a LayerNorm kernel, or a split-K partial GEMM (more workgroups for the N = 384 shapes)
    + one kernel that adds the partials, bias and residuals and normalises. Returns ``(x, planes)``
    (planes None without ``ln``)."""
    from . import kernels as K
    lead = residual.shape
    N = w.shape[0] if w.dim() == 2 else w.shape[1]
    Kd = a3.shape[-1]
    M = residual.numel() // N
    key = (M, N, Kd, residual2 is not None, ln is not None, K.slice_cus(), K.slice_pin())
    with _lock:
        choice = _fused_cache.get(key)

    def unsplit():
        x = gemm_x3(a3, w, b, residual=residual, residual2=residual2)
        return x, (K.layernorm_x3(x, ln[0], ln[1], ln[2]) if ln is not None else None)

    def split(cfg, sp):
        part = gemm_x3_partials(a3, w, cfg, sp)
        return K.splitk_layernorm(part, b, residual, residual2, ln, lead)

    def streamk(cfg, P):
        part, m = gemm_x3_streamk(a3, w, cfg, P)
        return K.streamk_layernorm(part, m, b, residual, residual2, ln, lead)
    if choice is None:
        if torch.cuda.is_current_stream_capturing() or os.environ.get("NOS_SPLITK", "1") == "0" \
                or K.slice_cus() < SPLITK_MIN_CUS:
            # NOS_SPLITK=0: the fused-epilogue GEMM + LayerNorm only (A/B runs); slices below
            # SPLITK_MIN_CUS have enough tiles per CU already, and there the partial planes' extra
            # write + read costs more than it balances under sibling partitions
            choice = ("unsplit",)
        else:
            stream = torch.cuda.current_stream()
            times = {("unsplit",): _gpu_time(unsplit, stream)}
            for c, sp in split_candidates(N, Kd):
                times[("split", c, sp)] = _gpu_time(lambda c=c, sp=sp: split(c, sp), stream)
            # stream-K partials (gemm_x3k): opt-in — on the model's shapes it is 15-25% slower than
            # the best split-K / unsplit pipeline (profiles/gemm_tuner_r4_streamk.json)
            if os.environ.get("NOS_STREAMK", "0") == "1":
                for c, P in streamk_candidates(N, Kd, K.slice_cus()):
                    times[("streamk", c, P)] = _gpu_time(lambda c=c, P=P: streamk(c, P), stream)
            choice = min(times, key=times.get)
            with _lock:
                _fused_cache[key] = choice
                _fused_times[key] = times
    if choice[0] == "streamk":
        return streamk(choice[1], choice[2])
    return unsplit() if choice[0] == "unsplit" else split(choice[1], choice[2])


def x3_table() -> Dict[str, str]:
    """The x3 tiles picked so far: shape/epilogue/outputs/slice -> ``BMxBN/<kind>`` (tile id)."""
    with _lock:
        return {f"M{m}_N{n}_K{k}_epi{e}_out{o}_cus{c}_pin{p}": "x".join(map(str, X3_TILES[v][:2])) + f"/{X3_TILES[v][3]}"
                + f" ({v})" for (m, n, k, e, o, c, p), v in sorted(_x3_cache.items())}


def x3_timings(top: int = 6) -> Dict[str, Dict[str, float]]:
    """The fastest ``top`` tiles the x3 tuner timed per key: ``BMxBN/<kind> (id)`` -> µs per call."""
    with _lock:
        return {f"M{m}_N{n}_K{k}_epi{e}_out{o}_cus{c}_pin{p}":
                {"x".join(map(str, X3_TILES[t][:2])) + f"/{X3_TILES[t][3]} ({t})": round(ms * 1000 / 3, 2)
                 for t, ms in sorted(v.items(), key=lambda x: x[1])[:top]}
                for (m, n, k, e, o, c, p), v in sorted(_x3_times.items())}


def fused_timings() -> Dict[str, Dict[str, float]]:
    """Every pipeline the projection/fc2 tuner timed, per key: ``/``-joined choice -> µs per call."""
    with _lock:
        return {f"M{m}_N{n}_K{k}_r2{int(r2)}_ln{int(ln)}_cus{c}_pin{p}":
                {"/".join(map(str, ch)): round(t * 1000 / 3, 2) for ch, t in sorted(v.items(), key=lambda x: x[1])}
                for (m, n, k, r2, ln, c, p), v in sorted(_fused_times.items())}


def fused_table() -> Dict[str, str]:
    with _lock:
        return {f"M{m}_N{n}_K{k}_r2{int(r2)}_ln{int(ln)}_cus{c}_pin{p}": "/".join(map(str, v))
                for (m, n, k, r2, ln, c, p), v in sorted(_fused_cache.items())}
