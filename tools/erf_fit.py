"""Coefficients of the packed erf / GELU in ``csrc/epilogue.h``, and their fp32 accuracy.

erf(z) = z + z*P(z^2) for |z| < 1 (P of degree 5), 1 - exp(-z^2) * R(min(|z|, 4) - 2.5) for
|z| >= 1 (R of degree 7). Both are fitted by iteratively reweighted least squares on the ABSOLUTE
error of erf (an approximation of the minimax fit), then the kernel's operation sequence is
replayed in fp32 (fused multiply-adds rounded once, exp2 rounded to fp32) and compared with fp64.

    python tools/erf_fit.py            # prints the coefficients and the fp32 error report
"""
from __future__ import annotations

import os
import re
from typing import Dict, List, Tuple

import numpy as np

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc", "epilogue.h")


def _erf64(x: np.ndarray) -> np.ndarray:
    from scipy.special import erf
    return erf(x)


def _erfc64(x: np.ndarray) -> np.ndarray:
    from scipy.special import erfc
    return erfc(x)


def _irls(V: np.ndarray, f: np.ndarray, scale: np.ndarray, iters: int = 40) -> np.ndarray:
    w = np.ones(len(f))
    for _ in range(iters):
        W = (scale * w)[:, None]
        c, *_ = np.linalg.lstsq(V * W, f * scale * w, rcond=None)
        e = np.abs(scale * (V @ c - f))
        w = w * (e / e.max()) ** 0.35 + 1e-4
        w /= w.mean()
    return c


def fit(deg_small: int = 5, deg_big: int = 7) -> Tuple[np.ndarray, np.ndarray]:
    z = np.linspace(1e-4, 1, 6000)
    c_small = _irls(np.vander(z * z, deg_small + 1, increasing=True), _erf64(z) / z - 1.0, z)
    z = np.linspace(1.0, 4.0, 6000)
    e2 = np.exp(-z * z)
    c_big = _irls(np.vander(z - 2.5, deg_big + 1, increasing=True), _erfc64(z) / e2, e2)
    return c_small, c_big


def header_coefficients(path: str = HEADER) -> Dict[str, List[float]]:
    """The two Horner chains as written in the header (highest degree first in the source)."""
    src = open(path).read()
    out = {}
    for name, var in (("small", "p"), ("big", "r")):
        first = re.search(rf"nos_f2 {var} = nos_f2s\(([-+0-9.e]+)f\)", src)
        rest = re.findall(rf"{var} = nos_fma2\([ut], {var}, nos_f2s\(([-+0-9.e]+)f\)\)", src)
        coeffs = [float(first.group(1))] + [float(x) for x in rest]
        out[name] = coeffs[::-1]  # lowest degree first
    return out


def _fma(a, b, c):
    return (a.astype(np.float64) * b.astype(np.float64) + np.asarray(c, np.float64)).astype(np.float32)


def _horner(t: np.ndarray, c: List[float]) -> np.ndarray:
    f32 = np.float32
    p = np.full_like(t, f32(c[-1]))
    for k in range(len(c) - 2, -1, -1):
        p = _fma(t, p, f32(c[k]))
    return p


def erf32(z: np.ndarray, small: List[float], big: List[float]) -> np.ndarray:
    """``nos_erf2`` replayed in fp32."""
    f32 = np.float32
    az = np.abs(z).astype(f32)
    u = (az * az).astype(f32)
    a = _fma(az, _horner(u, small), az)
    zc = np.minimum(az, f32(4.0))
    r = _horner((zc - f32(2.5)).astype(f32), big)
    ex = ((zc * zc).astype(f32) * f32(-1.4426950408889634)).astype(f32)
    e = np.exp2(ex.astype(np.float64)).astype(f32)
    b = _fma(-e, r, f32(1.0))
    return np.copysign(np.where(az < f32(1.0), a, b), z).astype(f32)


def gelu32(x: np.ndarray, small: List[float], big: List[float]) -> np.ndarray:
    f32 = np.float32
    hx = (x * f32(0.5)).astype(f32)
    return _fma(hx, erf32((x * f32(0.70710678118654752)).astype(f32), small, big), hx)


def report(small: List[float], big: List[float], n: int = 2_000_001) -> Dict[str, float]:
    f32 = np.float32
    x = np.concatenate([np.linspace(-12, 12, n), np.random.RandomState(0).randn(n // 2) * 3]).astype(f32)
    z = (x * f32(0.70710678118654752)).astype(f32)
    x64 = x.astype(np.float64)
    ref = x64 * 0.5 * (1 + _erf64(x64 / np.sqrt(2)))
    textbook = (x * f32(0.5) * (f32(1.0) + _erf64(z.astype(np.float64)).astype(f32))).astype(f32)
    return {"erf_max_abs_err": float(np.abs(erf32(z, small, big) - _erf64(z.astype(np.float64))).max()),
            "gelu_max_abs_err": float(np.abs(gelu32(x, small, big) - ref).max()),
            "gelu_textbook_fp32_max_abs_err": float(np.abs(textbook - ref).max())}


if __name__ == "__main__":
    cs, cb = fit()
    print("small (lowest degree first):", ", ".join("%.9e" % np.float32(c) for c in cs))
    print("big   (lowest degree first):", ", ".join("%.9e" % np.float32(c) for c in cb))
    hc = header_coefficients()
    print("header:", report(hc["small"], hc["big"]))
