"""Generic helpers used across the framework.

Behavioural parity with the reference's ``pkg/util/util.go:36-213`` (env helpers,
set/map helpers, ``UnorderedEqual`` multiset compare, ``LocalEndpoint``,
FNV-1a hashing).  ``unordered_equal`` is O(n log n) via canonical sorting instead
of the reference's O(n^2) pairwise scan (util.go:170-198) but has the same
multiset semantics.
"""
from __future__ import annotations

import json
import os
from collections import Counter
from typing import Any, Callable, Dict, Iterable, List, Mapping, TypeVar

T = TypeVar("T")
K = TypeVar("K")
V = TypeVar("V")


def get_env_or_default(name: str, default: str) -> str:
    v = os.environ.get(name)
    return default if v in (None, "") else v


def get_env_or_panic(name: str) -> str:
    v = os.environ.get(name)
    if not v:
        raise RuntimeError(f"environment variable {name} is required but not set")
    return v


def copy_map(m: Mapping[K, V]) -> Dict[K, V]:
    return dict(m)


def get_keys(*maps: Mapping[K, Any]) -> List[K]:
    seen: Dict[K, None] = {}
    for m in maps:
        for k in m:
            seen.setdefault(k, None)
    return list(seen)


def in_slice(x: T, items: Iterable[T]) -> bool:
    return any(x == i for i in items)


def filter_list(items: Iterable[T], keep: Callable[[T], bool]) -> List[T]:
    return [i for i in items if keep(i)]


def _canon(x: Any) -> str:
    """Canonical, order-independent key for deep-equality multiset compare."""
    if hasattr(x, "canonical"):
        return x.canonical()
    if hasattr(x, "__dict__") and not isinstance(x, type):
        return json.dumps(_to_plain(x), sort_keys=True, default=str)
    return json.dumps(_to_plain(x), sort_keys=True, default=str)


def _to_plain(x: Any) -> Any:
    if isinstance(x, dict):
        return {str(k): _to_plain(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_to_plain(v) for v in x]
    if hasattr(x, "_asdict"):
        return _to_plain(x._asdict())
    if hasattr(x, "__dataclass_fields__"):
        return {k: _to_plain(getattr(x, k)) for k in x.__dataclass_fields__}
    return x


def unordered_equal(a: Iterable[Any], b: Iterable[Any]) -> bool:
    """True when ``a`` and ``b`` contain the same elements with the same multiplicities."""
    return Counter(_canon(x) for x in a) == Counter(_canon(x) for x in b)


def local_endpoint(path: str) -> str:
    """unix-socket URL for a local path (reference ``LocalEndpoint``, util.go:201-207)."""
    return "unix://" + os.path.abspath(path)


def hash_fnv32a(s: str) -> int:
    h = 0x811C9DC5
    for byte in s.encode():
        h ^= byte
        h = (h * 0x01000193) & 0xFFFFFFFF
    return h


def clamp(x: int, lo: int, hi: int) -> int:
    return max(lo, min(hi, x))
