"""CU-mask slice profiles (the MPS analogue on MI355X).

Reference: ``pkg/gpu/slicing/profile.go`` (memory-only profiles ``<N>gb``, resource
``nvidia.com/gpu-<N>gb``, regex at ``:31``) and ``constant.go:22-24`` (``MinSliceMemoryGB=1``,
replica separator ``::``).

A slice here has two dimensions:

* ``<m>gb``          — an HBM budget of *m* GB, compute shared with the other shared slices
  (exactly the reference's MPS semantics: "compute shared equally");
* ``<c>cu.<m>gb``    — *c* dedicated CUs (a disjoint CU mask, multiple of :data:`CU_GRANULARITY`,
  placed as whole XCD- and SE-balanced row groups) plus *m* GB of HBM.

Resource names are ``amd.com/gpu-<profile>``; profiles contain no ``-``.
"""
from __future__ import annotations

import re
from dataclasses import dataclass
from functools import total_ordering
from typing import Optional

from ... import constant

MIN_SLICE_MEMORY_GB = 1
#: CU-mask granularity: one CU on every shader engine of every XCD (8 XCDs x 4 SEs = 32 CUs).
#: Measured on the box (``profiles/census_map_r1.json``): mask row r (bits 8r..8r+7, one CU per
#: XCD) sits on shader engine r mod 4, and workgroups are handed to the SEs of an XCD round-robin
#: whatever their number of enabled CUs, so a slice whose rows cover the SEs unevenly runs at the
#: pace of its thinnest SE (a 48-CU slice = 2/2/1/1 CUs per SE ran like a 32-CU one).
CU_GRANULARITY = 32
#: CUs always left to the shared pool when memory-only slices exist
MIN_SHARED_CUS = 32
#: slices (pods, one process each) per GPU before the hardware scheduler time-slices processes:
#: measured with pods as processes (``profiles/procs_cap_r4.json``), 8 memory-only pods share an
#: SPX MI355X evenly (383 inf/s, per-pod max/min 1.03); a 9th and 10th keep the aggregate but not
#: the shares (1.25, 3.0: some processes are switched out for whole scheduling quanta), and at 12-14
#: the aggregate falls to 292 / 271 (14 mixed dedicated + memory-only pods: 192,
#: ``profiles/dense_r4.json``). The node label ``nos.nebuly.com/max-slices-per-gpu`` overrides it.
MAX_SLICES_PER_GPU = 8
#: memory-only slice counts the planner never leaves on a GPU (it carves two at once past them, or
#: waits). Memory-only pods share every CU and the hardware scheduler deals each process's queues
#: over the MEC pipes in runlist (start) order; a HIP process holds two compute queues, so with one
#: stream queue per pod the pods alternate between two pipes and an odd count splits into two rate
#: classes — ceil(n/2) pods at the slow rate, floor(n/2) at the fast one, by start parity, the same
#: on every run (``profiles/fair_probe_r5.json``: 5 pods 73.4 vs 93.7 inf/s, max/min 1.28; 7 pods
#: 54.1 vs 65.5, 1.21; 8 pods 1.003). Three pods get two queues each instead (Allocate's
#: ``sharedSliceHwQueues`` rule) and share evenly. The GPU's aggregate hardly moves with the pod
#: count (366-413 inf/s at 3-8 pods), so skipping an odd count costs no throughput, only the odd
#: pod's start: it waits for a partner or for one of the running pods to finish.
#: ``GpuPartitionerConfig.sharedSliceSkipCounts`` overrides it.
SKIP_SHARED_COUNTS = (5, 7)
REPLICA_SEPARATOR = "::"

_PROFILE_RE = re.compile(r"^(?:(\d+)cu\.)?(\d+)gb$")


@total_ordering
@dataclass(frozen=True)
class SliceProfile:
    memory_gb: int
    cus: int = 0  # 0 => shared compute

    @property
    def name(self) -> str:
        return f"{self.cus}cu.{self.memory_gb}gb" if self.cus else f"{self.memory_gb}gb"

    @property
    def resource_name(self) -> str:
        return constant.RESOURCE_SLICE_PREFIX + self.name

    @property
    def dedicated(self) -> bool:
        return self.cus > 0

    def __lt__(self, other: "SliceProfile") -> bool:
        return (self.memory_gb, self.cus) < (other.memory_gb, other.cus)

    def __str__(self) -> str:
        return self.name


def parse_profile(name: str) -> SliceProfile:
    m = _PROFILE_RE.match(name)
    if not m:
        raise ValueError(f"invalid slice profile {name!r}")
    return SliceProfile(int(m.group(2)), int(m.group(1) or 0))


def is_valid_profile(name: str) -> bool:
    return bool(_PROFILE_RE.match(name))


def new_profile(memory_gb: int, cus: int = 0) -> str:
    return SliceProfile(memory_gb, cus).name


def is_slice_resource(resource_name: str) -> bool:
    return bool(constant.RESOURCE_SLICE_REGEX.match(resource_name))


def extract_profile_name(resource_name: str) -> Optional[str]:
    m = constant.RESOURCE_SLICE_REGEX.match(resource_name)
    return m.group(1) if m else None


def as_resource_name(profile: str) -> str:
    return constant.RESOURCE_SLICE_PREFIX + profile


def extract_gpu_id(device_id: str) -> str:
    """Strip the replica suffix: ``<uuid>::<n>`` -> ``<uuid>`` (reference ``util.go:51-57``)."""
    return device_id.split(REPLICA_SEPARATOR, 1)[0]
