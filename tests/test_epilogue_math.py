"""The packed GELU of the x3 GEMM epilogue (``csrc/epilogue.h``), replayed in fp32 on the CPU with
the coefficients read from the header: erf within 1e-7 and GELU no worse than the textbook fp32
formula with a correctly rounded erf (what torch's exact GELU evaluates). The kernel itself is
checked against fp64 on the GPU (``tests/test_gpu_kernels.py``)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))

import erf_fit  # noqa: E402


def test_header_coefficients_are_the_fitted_ones():
    hc = erf_fit.header_coefficients()
    assert len(hc["small"]) == 6 and len(hc["big"]) == 8
    cs, cb = erf_fit.fit()
    np.testing.assert_allclose(hc["small"], cs, rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(hc["big"], cb, rtol=1e-5, atol=1e-9)


def test_packed_gelu_is_fp32_accurate():
    hc = erf_fit.header_coefficients()
    r = erf_fit.report(hc["small"], hc["big"], n=400_001)
    assert r["erf_max_abs_err"] < 1e-7, r
    assert r["gelu_max_abs_err"] <= r["gelu_textbook_fp32_max_abs_err"] * 1.05, r
