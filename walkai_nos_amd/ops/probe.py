"""Slice probe: achievable FLOP/s per CU and HBM GB/s inside a compute partition or CU-mask slice.

Python side of ``csrc/probe.hip``.  The agent runs :func:`probe_slice` after every partition
commit and publishes the result (annotation ``nos.nebuly.com/status-probe`` + the
``nos_probe_tflops_per_cu`` gauge), so the partitioner and the metrics exporter work with measured
MI355X numbers instead of datasheet ones (BASELINE.json north star).
"""
from __future__ import annotations

import ctypes
from dataclasses import asdict, dataclass
from typing import Dict, List, Optional, Sequence

from .native import load

LIB = "libnos_probe.so"

DTYPES = {"bf16": 0, "bf16_16x16": 1, "fp32": 2, "fp8": 3, "fp8_scaled": 4}
HBM_MODES = {"stride": 0, "slab_nt": 1, "slab": 2, "slab_nt16": 3, "slab_nt4": 4}


class ProbeResult(ctypes.Structure):
    _fields_ = [("ms", ctypes.c_double), ("flops", ctypes.c_double), ("rate", ctypes.c_double),
                ("n_wg", ctypes.c_int32), ("mhz", ctypes.c_double)]


_configured = False


def _lib() -> ctypes.CDLL:
    global _configured
    L = load(LIB)
    if not _configured:
        L.nos_probe_last_error.restype = ctypes.c_char_p
        L.nos_stream_create.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_uint32), ctypes.c_uint32,
                                        ctypes.POINTER(ctypes.c_void_p)]
        L.nos_stream_get_cumask.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]
        L.nos_stream_destroy.argtypes = [ctypes.c_void_p]
        L.nos_probe_mfma.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_int, ctypes.POINTER(ProbeResult)]
        L.nos_probe_hbm.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                    ctypes.POINTER(ProbeResult)]
        L.nos_probe_hbm_mode.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_int, ctypes.POINTER(ProbeResult)]
        L.nos_probe_census.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                       ctypes.POINTER(ctypes.c_uint32)]
        L.nos_probe_cu_count.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
        L.nos_probe_device_count.argtypes = [ctypes.POINTER(ctypes.c_int)]
        _configured = True
    return L


def _check(rc: int) -> None:
    if rc != 0:
        raise RuntimeError(f"nos probe: {_lib().nos_probe_last_error().decode()} (rc={rc})")


def device_count() -> int:
    n = ctypes.c_int(0)
    _check(_lib().nos_probe_device_count(ctypes.byref(n)))
    return n.value


def cu_count(device: int = 0) -> int:
    n = ctypes.c_int(0)
    _check(_lib().nos_probe_cu_count(device, ctypes.byref(n)))
    return n.value


def mask_words(cus: Sequence[int], total_cus: int = 256) -> List[int]:
    words = [0] * ((total_cus + 31) // 32)
    for c in cus:
        if not 0 <= c < total_cus:
            raise ValueError(f"CU {c} out of range 0..{total_cus - 1}")
        words[c // 32] |= 1 << (c % 32)
    return words


class Stream:
    """A HIP stream, optionally restricted to a CU set (``hipExtStreamCreateWithCUMask``)."""

    def __init__(self, device: int = 0, cus: Optional[Sequence[int]] = None, total_cus: Optional[int] = None):
        self.device = device
        self.cus = list(cus) if cus is not None else None
        h = ctypes.c_void_p()
        if self.cus is None:
            _check(_lib().nos_stream_create(device, None, 0, ctypes.byref(h)))
        else:
            tot = total_cus or cu_count(device)
            w = mask_words(self.cus, tot)
            arr = (ctypes.c_uint32 * len(w))(*w)
            _check(_lib().nos_stream_create(device, arr, len(w), ctypes.byref(h)))
        self.handle = h.value

    def cumask(self, n_words: int = 8) -> List[int]:
        arr = (ctypes.c_uint32 * n_words)()
        _check(_lib().nos_stream_get_cumask(self.handle, n_words, arr))
        return list(arr)

    def torch_stream(self):
        import torch
        return torch.cuda.ExternalStream(self.handle, device=torch.device("cuda", self.device))

    def close(self) -> None:
        if self.handle:
            _check(_lib().nos_stream_destroy(self.handle))
            self.handle = None

    def __enter__(self) -> "Stream":
        return self

    def __exit__(self, *a: object) -> None:
        self.close()


@dataclass
class SliceProbe:
    dtype: str
    n_cus: int
    ms: float
    tflops: float
    tflops_per_cu: float
    n_wg: int
    mhz: float = 0.0  # mean shader clock over the loop (s_memtime / s_memrealtime)

    @property
    def pct_of_clock_peak(self) -> float:
        """Achieved rate over the matrix-pipe peak at the measured clock (0 if unknown)."""
        # matrix-pipe FLOP per clock per CU
        # (non-scaled fp8 MFMAs run at the bf16 rate; the block-scaled 32x32x64 form at twice it)
        per_clk = {"bf16": 4096, "bf16_16x16": 4096, "fp32": 256, "fp8": 4096, "fp8_scaled": 8192}.get(self.dtype, 0)
        if not self.mhz or not per_clk:
            return 0.0
        return 100.0 * self.tflops * 1e12 / (per_clk * self.n_cus * self.mhz * 1e6)


def probe_mfma(dtype: str = "bf16", device: int = 0, stream: Optional[Stream] = None, n_cus: Optional[int] = None,
               wg_per_cu: int = 2, iters: int = 4096, reps: int = 5) -> SliceProbe:
    n_cus = n_cus or (len(stream.cus) if stream is not None and stream.cus is not None else cu_count(device))
    n_wg = max(1, n_cus * wg_per_cu)
    r = ProbeResult()
    _check(_lib().nos_probe_mfma(device, stream.handle if stream else None, DTYPES[dtype], n_wg, iters, reps,
                                 ctypes.byref(r)))
    return SliceProbe(dtype, n_cus, r.ms, r.rate, r.rate / n_cus, n_wg, r.mhz)


def probe_hbm(device: int = 0, stream: Optional[Stream] = None, nbytes: int = 1 << 30, n_wg: Optional[int] = None,
              reps: int = 5, mode: str = "slab_nt") -> Dict[str, float]:
    n_cus = len(stream.cus) if stream is not None and stream.cus is not None else cu_count(device)
    r = ProbeResult()
    # default: one slab-copy workgroup per CU, non-temporal (best of the tools/hbm_sweep.py sweep,
    # profiles/hbm_sweep_r2.json: 6.1 TB/s on a 16 GiB copy; more workgroups per CU thrash DRAM pages)
    _check(_lib().nos_probe_hbm_mode(device, stream.handle if stream else None, nbytes, n_wg or n_cus, reps,
                                     HBM_MODES[mode], ctypes.byref(r)))
    return {"ms": r.ms, "gbps": r.rate, "bytes": r.flops, "n_cus": n_cus}


def census(device: int = 0, stream: Optional[Stream] = None, n_wg: int = 2048, spin: int = 2000) -> List[Dict[str, int]]:
    """Placement of each workgroup: CU id / SE id decoded from HW_REG_HW_ID, XCC id."""
    buf = (ctypes.c_uint32 * (2 * n_wg))()
    _check(_lib().nos_probe_census(device, stream.handle if stream else None, n_wg, spin, buf))
    out = []
    for i in range(n_wg):
        hw, xcc = buf[2 * i], buf[2 * i + 1]
        out.append({"wg": i, "cu": (hw >> 8) & 0xF, "sh": (hw >> 12) & 0x1, "se": (hw >> 13) & 0x7,
                    "xcc": xcc & 0xF, "raw_hw_id": hw})
    return out


def distinct_cus(placements: List[Dict[str, int]]) -> int:
    return len({(p["xcc"], p["se"], p["sh"], p["cu"]) for p in placements})


def probe_slice(cus: Optional[Sequence[int]] = None, device: int = 0, dtypes: Sequence[str] = ("bf16", "fp32"),
                iters: int = 2048) -> Dict[str, object]:
    """Probe one slice (None = whole device) and return a JSON-able summary."""
    with Stream(device, cus) as s:
        out: Dict[str, object] = {"n_cus": len(cus) if cus is not None else cu_count(device)}
        for d in dtypes:
            out[d] = asdict(probe_mfma(d, device, s, iters=iters))
        return out
