"""Kubernetes resource.Quantity parsing/formatting (subset used by the operator).

Quantities are represented internally as ``int`` milli-units for cpu-like values and
plain integers for everything else is what the scheduler needs; to stay exact we parse
to :class:`fractions.Fraction` and expose helpers for the two common views.
"""
from __future__ import annotations

import functools

import re
from fractions import Fraction
from typing import Union

_SUFFIX = {
    "": Fraction(1),
    "m": Fraction(1, 1000),
    "u": Fraction(1, 10**6),
    "n": Fraction(1, 10**9),
    "k": Fraction(10**3),
    "M": Fraction(10**6),
    "G": Fraction(10**9),
    "T": Fraction(10**12),
    "P": Fraction(10**15),
    "E": Fraction(10**18),
    "Ki": Fraction(2**10),
    "Mi": Fraction(2**20),
    "Gi": Fraction(2**30),
    "Ti": Fraction(2**40),
    "Pi": Fraction(2**50),
    "Ei": Fraction(2**60),
}
_RE = re.compile(r"^([+-]?[0-9.]+(?:[eE][+-]?[0-9]+)?)(Ki|Mi|Gi|Ti|Pi|Ei|m|u|n|k|M|G|T|P|E)?$")

QuantityLike = Union[str, int, float, Fraction]


def parse_quantity(q: QuantityLike) -> Fraction:
    if isinstance(q, Fraction):
        return q
    if isinstance(q, bool):
        raise ValueError(f"invalid quantity {q!r}")
    if isinstance(q, int):
        return Fraction(q)
    if isinstance(q, float):
        return Fraction(q).limit_denominator(10**9)
    return _parse_str(str(q).strip())


@functools.lru_cache(maxsize=4096)
def _parse_str(s: str) -> Fraction:
    """Memoised string parse: a cluster's pods repeat a handful of quantity strings."""
    m = _RE.match(s)
    if not m:
        raise ValueError(f"invalid quantity {s!r}")
    num, suf = m.group(1), m.group(2) or ""
    return Fraction(num) * _SUFFIX[suf]


def quantity_value(q: QuantityLike) -> int:
    """Integer value rounded up (Quantity.Value semantics)."""
    f = parse_quantity(q)
    n = f.numerator // f.denominator
    return n if n == f else n + 1


def quantity_milli(q: QuantityLike) -> int:
    f = parse_quantity(q) * 1000
    n = f.numerator // f.denominator
    return n if n == f else n + 1


def format_quantity(v: Union[int, Fraction]) -> str:
    f = Fraction(v)
    if f.denominator == 1:
        return str(f.numerator)
    milli = f * 1000
    if milli.denominator == 1:
        return f"{milli.numerator}m"
    return str(float(f))
