"""Known GPU models and their allowed compute-partition geometries.

Reference: ``pkg/gpu/mig/known_configs.go:24-185`` (per-model allowed MIG geometries,
``SetKnownGeometries`` validate-then-replace, ``GetAllowedGeometries``) and
``allowed_geometries.go:25-82`` (YAML/JSON ``[{models: [...], allowedGeometries: [{p: q}]}]``).

MI355X semantics: geometries are **homogeneous per GPU** — one ``amdsmi_set_gpu_compute_partition``
call switches the whole device — so the allowed set is ``{spx:1}``, ``{dpx:2}``, ``{qpx:4}``,
``{cpx:8}`` for every NPS mode that supports that compute mode.  The YAML format is the
reference's, extended with optional ``memoryGB`` / ``computeUnits`` / ``xcds`` per model.
"""
from __future__ import annotations

import copy
import re
import threading
from dataclasses import dataclass, field
from typing import Dict, Iterable, List, Mapping, Optional, Tuple

import yaml

from ..geometry import Geometry
from .profile import COMPUTE_MODES, MEMORY_MODES, is_valid_profile, parse_profile


@dataclass
class GpuModelSpec:
    model: str
    memory_gb: int
    compute_units: int
    xcds: int
    allowed_geometries: List[Geometry] = field(default_factory=list)
    #: bf16 MFMA TFLOP/s per CU a healthy GPU of this model delivers in the probe kernel
    #: (csrc/probe.hip); partitions/slices probing below a fraction of it are withheld (None: no rule)
    probe_bf16_tflops_per_cu: Optional[float] = None

    def geometries_for_nps(self, nps: Optional[str]) -> List[Geometry]:
        if nps is None:
            return [dict(g) for g in self.allowed_geometries]
        return [dict(g) for g in self.allowed_geometries if all(p.endswith("_" + nps) for p in g)]

    def supported_nps(self) -> List[str]:
        out = []
        for g in self.allowed_geometries:
            for p in g:
                n = parse_profile(p).nps
                if n not in out:
                    out.append(n)
        return sorted(out, key=lambda n: MEMORY_MODES[n])


def _homogeneous(modes: Mapping[str, Iterable[str]]) -> List[Geometry]:
    out: List[Geometry] = []
    for nps, cms in modes.items():
        for cm in cms:
            out.append({f"{cm}_{nps}": COMPUTE_MODES[cm]})
    return out


def normalize_model(model: str) -> str:
    """``AMD_Instinct_MI355X`` / ``AMD Instinct MI355X`` / ``mi355x`` -> ``MI355X``."""
    s = re.sub(r"[^A-Za-z0-9]", "", model or "").upper()
    for prefix in ("AMDINSTINCT", "INSTINCT", "AMD"):
        if s.startswith(prefix):
            s = s[len(prefix):]
    return s


# MI355X: 8 XCDs x 32 CUs, 288 GB HBM3E (MI355X_MICROARCH.md "Chip-level parameters"). Probe rate:
# 1576.5 bf16 TFLOP/s over 256 CUs on the box = 6.16 per CU (profiles/operator_gpu_report_r3.json).
# Compute-partition availability per NPS mode: NPS1 allows every mode; NPS2 requires at least two
# partitions; NPS4/NPS8 require at least as many compute partitions as memory partitions.
_DEFAULT_SPECS: Dict[str, GpuModelSpec] = {
    "MI355X": GpuModelSpec("MI355X", 288, 256, 8, _homogeneous({
        "nps1": ["spx", "dpx", "qpx", "cpx"], "nps2": ["dpx", "qpx", "cpx"]}), 6.16),
    "MI350X": GpuModelSpec("MI350X", 288, 256, 8, _homogeneous({
        "nps1": ["spx", "dpx", "qpx", "cpx"], "nps2": ["dpx", "qpx", "cpx"]})),
    "MI325X": GpuModelSpec("MI325X", 256, 304, 8, _homogeneous({
        "nps1": ["spx", "dpx", "qpx", "cpx"], "nps4": ["cpx"]})),
    "MI300X": GpuModelSpec("MI300X", 192, 304, 8, _homogeneous({
        "nps1": ["spx", "dpx", "qpx", "cpx"], "nps4": ["cpx"]})),
}

_lock = threading.Lock()
_known: Dict[str, GpuModelSpec] = copy.deepcopy(_DEFAULT_SPECS)


def validate_geometry(g: Mapping[str, int]) -> None:
    if not g:
        raise ValueError("geometry cannot be empty")
    for p, q in g.items():
        if not is_valid_profile(p):
            raise ValueError(f"invalid compute-partition profile {p!r}")
        if not isinstance(q, int) or q < 1:
            raise ValueError(f"invalid quantity {q!r} for profile {p!r}: must be >= 1")
    if len(g) != 1:
        raise ValueError(f"compute partitions are homogeneous per GPU; geometry {dict(g)} mixes modes")
    (p, q), = g.items()
    if q != parse_profile(p).partitions:
        raise ValueError(f"profile {p!r} always yields {parse_profile(p).partitions} partitions, got {q}")


def validate_specs(specs: Mapping[str, GpuModelSpec]) -> None:
    for name, s in specs.items():
        if not s.allowed_geometries:
            raise ValueError(f"model {name!r} has no allowed geometries")
        for g in s.allowed_geometries:
            validate_geometry(g)
        if s.memory_gb <= 0 or s.compute_units <= 0 or s.xcds <= 0:
            raise ValueError(f"model {name!r}: memoryGB/computeUnits/xcds must be > 0")


_geo_cache: Dict[Tuple[str, Optional[str]], Optional[List[Tuple[Tuple[str, int], ...]]]] = {}


def set_known_geometries(specs: Mapping[str, GpuModelSpec]) -> None:
    """Validate then atomically replace the global table (reference ``SetKnownGeometries``)."""
    validate_specs(specs)
    global _known
    with _lock:
        _known = {normalize_model(k): copy.deepcopy(v) for k, v in specs.items()}
        _geo_cache.clear()


def reset_known_geometries() -> None:
    global _known
    with _lock:
        _known = copy.deepcopy(_DEFAULT_SPECS)
        _geo_cache.clear()


def get_known_geometries() -> Dict[str, GpuModelSpec]:
    with _lock:
        return copy.deepcopy(_known)


def get_model_spec(model: str) -> Optional[GpuModelSpec]:
    with _lock:
        s = _known.get(normalize_model(model))
        return copy.deepcopy(s) if s is not None else None


def get_allowed_geometries(model: str, nps: Optional[str] = None) -> Optional[List[Geometry]]:
    """Allowed geometries of ``model`` under memory mode ``nps`` (fresh dicts; the filtered table
    is memoised per (model, nps) — every planner pass builds a model per GPU from it)."""
    with _lock:
        key = (model, nps)
        if key not in _geo_cache:
            s = _known.get(normalize_model(model))
            _geo_cache[key] = None if s is None else [tuple(g.items()) for g in s.geometries_for_nps(nps)]
        hit = _geo_cache[key]
        return None if hit is None else [dict(g) for g in hit]


def load_known_geometries(data: str) -> Dict[str, GpuModelSpec]:
    """Parse the reference YAML/JSON format (JSON is valid YAML)."""
    doc = yaml.safe_load(data) or []
    if not isinstance(doc, list):
        raise ValueError("known geometries must be a list of {models, allowedGeometries}")
    out: Dict[str, GpuModelSpec] = {}
    for entry in doc:
        models = entry.get("models") or []
        geoms = entry.get("allowedGeometries") or []
        if not models:
            raise ValueError("entry without models")
        for m in models:
            base = _DEFAULT_SPECS.get(normalize_model(m))
            spec = GpuModelSpec(
                model=normalize_model(m),
                memory_gb=int(entry.get("memoryGB", base.memory_gb if base else 0)),
                compute_units=int(entry.get("computeUnits", base.compute_units if base else 0)),
                xcds=int(entry.get("xcds", base.xcds if base else 8)),
                allowed_geometries=[{str(k): int(v) for k, v in g.items()} for g in geoms],
                probe_bf16_tflops_per_cu=(float(entry["probeBf16TflopsPerCu"]) if "probeBf16TflopsPerCu" in entry
                                          else (base.probe_bf16_tflops_per_cu if base else None)),
            )
            out[spec.model] = spec
    validate_specs(out)
    return out


def load_known_geometries_file(path: str) -> Dict[str, GpuModelSpec]:
    with open(path) as f:
        return load_known_geometries(f.read())


def dump_known_geometries(specs: Optional[Mapping[str, GpuModelSpec]] = None) -> str:
    specs = specs if specs is not None else get_known_geometries()
    doc = [{"models": [s.model], "memoryGB": s.memory_gb, "computeUnits": s.compute_units, "xcds": s.xcds,
            "allowedGeometries": s.allowed_geometries,
            **({"probeBf16TflopsPerCu": s.probe_bf16_tflops_per_cu} if s.probe_bf16_tflops_per_cu else {})}
           for s in specs.values()]
    return yaml.safe_dump(doc, sort_keys=False)
