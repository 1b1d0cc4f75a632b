"""MI355X compute-partition (XCP) profiles.

The MIG analogue on CDNA4: one MI355X (8 XCDs x 32 CUs) is exposed as 1/2/4/8 logical GPUs in
SPX/DPX/QPX/CPX compute-partition mode, on top of a node-wide NPS1/2/4/8 memory-partition mode
(``amdsmi.h:422-449``).  Profile names follow the AMD k8s-device-plugin "mixed" resource naming
(``amd.com/cpx_nps1`` ...) and deliberately contain no ``-`` so the reference annotation grammar
(split on ``-``) keeps working.

Unlike MIG's ``SmallerThan`` (not a strict weak order) profiles here have a total
order: fewer XCDs first, then memory mode.
"""
from __future__ import annotations

import re
from dataclasses import dataclass
from functools import total_ordering
from typing import Optional

from ... import constant

#: partitions per GPU for each compute-partition mode (MI355X has 8 XCDs)
COMPUTE_MODES = {"spx": 1, "dpx": 2, "qpx": 4, "cpx": 8}
#: memory partitions per GPU for each NPS mode
MEMORY_MODES = {"nps1": 1, "nps2": 2, "nps4": 4, "nps8": 8}

_PROFILE_RE = re.compile(r"^(spx|dpx|qpx|cpx)_(nps[1248])$")


@total_ordering
@dataclass(frozen=True)
class XcpProfile:
    mode: str
    nps: str

    @property
    def name(self) -> str:
        return f"{self.mode}_{self.nps}"

    @property
    def partitions(self) -> int:
        return COMPUTE_MODES[self.mode]

    @property
    def resource_name(self) -> str:
        return constant.AMD_RESOURCE_PREFIX + self.name

    def fraction(self) -> float:
        return 1.0 / self.partitions

    def xcds(self, gpu_xcds: int = 8) -> int:
        return gpu_xcds // self.partitions

    def cus(self, gpu_cus: int = 256) -> int:
        return gpu_cus // self.partitions

    def memory_gb(self, gpu_memory_gb: int = 288) -> int:
        return gpu_memory_gb // self.partitions

    def __lt__(self, other: "XcpProfile") -> bool:
        return (-self.partitions, self.nps) < (-other.partitions, other.nps)

    def __str__(self) -> str:
        return self.name


def is_valid_profile(name: str) -> bool:
    return bool(_PROFILE_RE.match(name))


def parse_profile(name: str) -> XcpProfile:
    m = _PROFILE_RE.match(name)
    if not m:
        raise ValueError(f"invalid compute-partition profile {name!r}")
    return XcpProfile(m.group(1), m.group(2))


def is_xcp_resource(resource_name: str) -> bool:
    return bool(constant.RESOURCE_XCP_REGEX.match(resource_name))


def extract_profile_name(resource_name: str) -> Optional[str]:
    """``amd.com/cpx_nps1`` -> ``cpx_nps1`` (None for anything else)."""
    m = constant.RESOURCE_XCP_REGEX.match(resource_name)
    return m.group(1) if m else None


def as_resource_name(profile: str) -> str:
    return constant.AMD_RESOURCE_PREFIX + profile


def smaller_than(a: str, b: str) -> bool:
    return parse_profile(a) < parse_profile(b)
