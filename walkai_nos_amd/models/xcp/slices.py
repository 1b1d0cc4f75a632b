"""Sliced MI355X GPUs: mixed per-GPU geometries on one GPU, the MIG-style half of compute partitioning.

A MIG A100 hosts a *mixed* geometry at once (``4g.20gb + 2g.10gb + 1g.5gb``, ref
``pkg/gpu/mig/known_configs.go:41-90``) and changes its free instances around used ones without a
drain (ref ``internal/controllers/migagent/actuator.go:225-229``).  MI355X compute partitions
cannot: SPX/DPX/QPX/CPX are homogeneous per GPU and a flip destroys every partition
(:mod:`.known_configs`).  A **sliced GPU** gets both properties back on MI355X:

* the GPU stays in hardware **SPX** mode (NPS1), and its 256 CUs are carved into CU-mask *slices*
  of the compute-partition sizes — ``spx_nps1`` = 8 row groups, ``dpx_nps1`` = 4, ``qpx_nps1`` = 2,
  ``cpx_nps1`` = 1, a row group being 32 CUs, one on every shader engine of every XCD
  (:mod:`..slicing.cumask`) — with 1/8 of the HBM (36 GB) per group as the slice's budget;
* any mix whose groups add up to at most 8 is a valid geometry (``dpx + 2 qpx``,
  ``dpx + 4 cpx``, ``qpx + 6 cpx`` ...): CU masks place anywhere, so there is no placement
  constraint and no fragmentation beyond the group count;
* a pod asks for the same resource either way (``amd.com/cpx_nps1`` = 1/8 of an MI355X), and a
  slice is served by the nos partition device plugin with ``HSA_CU_MASK`` + the HBM limiter, the
  way the CU-mask slice plugin serves ``amd.com/gpu-<c>cu.<m>gb``;
* re-carving the free slices of a GPU is a configuration change only — no amd-smi call, no
  outage, used slices keep running — so the planner backfills small pods next to big ones.

Isolation is weaker than a hardware partition: slices share the XCDs' L2 and the HBM channels, and
the HBM budget is enforced by the cooperative interposer.  A node opts in with the label
``nos.nebuly.com/xcp-layout=slices`` (every GPU sliced) or ``=auto`` (the planner chooses per GPU:
a hardware mode for homogeneous demand, slices otherwise); ``partitions`` (the default) keeps
hardware partitions only, for pods that need them.

The same :func:`recarve` drives the agent (what to delete and create) and the device plugin (which
free slices to withhold while a re-carve is pending), so the two never disagree.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable, Dict, Iterable, List, Mapping, Optional, Sequence, Set, Tuple

from ..geometry import Geometry
from ..partitioned import PartitionedGPU
from ..slicing.cumask import GROUP_ROWS, Slice
from .profile import is_valid_profile, parse_profile

#: row groups of one MI355X (32 CUs each: 4 per XCD, one per shader engine)
GROUPS = 8
#: separator of a slice's device id: ``<gpu bdf>::x<serial>`` (the BDF resolves to the GPU)
SLICE_SEP = "::x"
#: the hardware mode a sliced GPU runs in, and the profile of its single whole-GPU slice
SLICED_MODE = "spx"
SLICE_NPS = "nps1"

LAYOUT_PARTITIONS = "partitions"
LAYOUT_SLICES = "slices"
LAYOUT_AUTO = "auto"
LAYOUTS = (LAYOUT_PARTITIONS, LAYOUT_SLICES, LAYOUT_AUTO)


def groups_of(profile: str) -> int:
    """Row groups a slice of ``profile`` occupies (``cpx_nps1`` -> 1, ``spx_nps1`` -> 8)."""
    return GROUPS // parse_profile(profile).partitions


def is_slice_profile(profile: str) -> bool:
    return is_valid_profile(profile) and parse_profile(profile).nps == SLICE_NPS


def geometry_groups(g: Mapping[str, int]) -> int:
    return sum(groups_of(p) * q for p, q in g.items() if q > 0)


def all_slice_geometries() -> List[Geometry]:
    """Every full carve-up of a GPU (the mixed analogue of a MIG model's allowed-geometry list)."""
    out: List[Geometry] = [{"spx_nps1": 1}]
    for d in range(2, -1, -1):
        for q in range((GROUPS - 4 * d) // 2, -1, -1):
            c = GROUPS - 4 * d - 2 * q
            g = {p: n for p, n in (("dpx_nps1", d), ("qpx_nps1", q), ("cpx_nps1", c)) if n}
            out.append(g)
    return out


@dataclass
class SlicedGPU(PartitionedGPU):
    """A GPU in SPX mode carved into CU-mask slices (module docstring). ``used``/``free`` count
    slices per profile, like a partitioned GPU; any geometry within :data:`GROUPS` is allowed, and
    free slices may be re-carved at any time."""
    capacity: int = GROUPS

    sliced = True

    def clone(self) -> "SlicedGPU":
        return SlicedGPU(self.model, self.index, [dict(g) for g in self.allowed_geometries], dict(self.used),
                         dict(self.free), dict(self.target) if self.target else None, self.target_sliced,
                         self.degraded, self.capacity)

    # -- capacity ----------------------------------------------------------------------------
    def used_groups(self) -> int:
        return geometry_groups(self.used)

    def free_groups(self) -> int:
        return geometry_groups(self.free)

    def spare_groups(self) -> int:
        """Groups carved into no slice."""
        return self.capacity - self.used_groups() - self.free_groups()

    def room(self) -> int:
        """Groups a new slice may take: everything not in use (free slices can be re-carved)."""
        return self.capacity - self.used_groups()

    def fits(self, profile: str) -> bool:
        return is_slice_profile(profile) and groups_of(profile) <= self.room()

    # -- geometry -----------------------------------------------------------------------------
    def allows_geometry(self, g: Mapping[str, int]) -> bool:
        return all(is_slice_profile(p) and q >= 0 for p, q in g.items()) and geometry_groups(g) <= self.capacity

    def can_apply_geometry(self, g: Mapping[str, int]) -> Tuple[bool, str]:
        if not self.allows_geometry(g):
            return False, f"geometry {dict(g)} does not fit a sliced {self.model} ({self.capacity} groups)"
        for p, q in self.used.items():
            if g.get(p, 0) < q:
                return False, "cannot apply geometry: cannot delete slices being used"
        return True, ""

    def init_geometry(self) -> None:
        self.apply_geometry({f"{SLICED_MODE}_{SLICE_NPS}": 1})

    def claim(self, profile: str) -> None:
        """Reserve one slice of ``profile`` for a pod: a free one if there is one, else carved from
        spare groups and, when those are short, from other free slices (smallest first)."""
        if self.target is not None:
            raise ValueError(f"GPU {self.index} is draining towards {self.target}")
        if not self.fits(profile):
            raise ValueError(f"GPU {self.index}: no room for {profile} ({self.room()} groups not in use)")
        if self.free.get(profile, 0) <= 0:
            need = groups_of(profile) - self.spare_groups()
            for p in sorted(self.free, key=lambda x: (groups_of(x), x)):
                while need > 0 and self.free.get(p, 0) > 0 and p != profile:
                    self.free[p] -= 1
                    need -= groups_of(p)
            self.free = {p: q for p, q in self.free.items() if q > 0}
            self.free[profile] = self.free.get(profile, 0) + 1
        self.add_pod({profile: 1})
        self.free = {p: q for p, q in self.free.items() if q > 0}

    def fill(self, profile: str = "cpx_nps1") -> None:
        """Carve the spare groups into slices of ``profile`` (advertised, so the scheduler can place
        small pods without waiting for the planner)."""
        n = self.spare_groups() // groups_of(profile)
        if n > 0:
            self.free[profile] = self.free.get(profile, 0) + n

    def update_geometry_for(self, required: Mapping[str, int], weight: Optional[Callable[[str], float]] = None) -> bool:
        """Carve the room (free slices re-carved, used kept) to provide ``required``: bigger slices
        first, then the free slices already carved that still fit, then cpx from the rest."""
        want = {p: q for p, q in required.items() if q > 0 and is_slice_profile(p)}
        if not want or self.target is not None:
            return False
        room = self.room()
        new_free: Dict[str, int] = {}
        provided = 0.0
        for p in sorted(want, key=lambda x: (-groups_of(x), x)):
            need = max(0, want[p] - self.free.get(p, 0))
            have = min(self.free.get(p, 0), want[p])
            n = min(have + need, room // groups_of(p))
            if n <= 0:
                continue
            new_free[p] = n
            room -= n * groups_of(p)
            provided += max(0, n - self.free.get(p, 0)) * (1.0 if weight is None else weight(p))
        if provided <= 0:
            return False
        for p, q in sorted(self.free.items(), key=lambda x: (-groups_of(x[0]), x[0])):
            extra = max(0, q - new_free.get(p, 0))
            k = min(extra, room // groups_of(p))
            if k > 0:
                new_free[p] = new_free.get(p, 0) + k
                room -= k * groups_of(p)
        if room > 0:
            new_free["cpx_nps1"] = new_free.get("cpx_nps1", 0) + room
        self.free = new_free
        return True


def new_sliced_gpu(model: str, index: int, used: Optional[Mapping[str, int]] = None,
                   free: Optional[Mapping[str, int]] = None) -> SlicedGPU:
    return SlicedGPU(model, index, all_slice_geometries(), dict(used or {}), dict(free or {}))


# -- node-side slice layout (agent + plugin) ---------------------------------------------------
def slice_groups(s: Slice) -> List[int]:
    return sorted({r // GROUP_ROWS for r in s.rows})


def serial_of(slice_id: str) -> int:
    try:
        return int(slice_id.rsplit(SLICE_SEP, 1)[1])
    except (IndexError, ValueError):
        return -1


@dataclass
class Recarve:
    """One GPU's slice change: slices kept (used ones always), free slices deleted, profiles of
    the slices to create, and whether the whole spec fits now (else the GPU is draining for it)."""
    keep: List[Slice] = field(default_factory=list)
    delete: List[Slice] = field(default_factory=list)
    create: List[str] = field(default_factory=list)
    achievable: bool = True
    blocked: List[str] = field(default_factory=list)

    def is_empty(self) -> bool:
        return not self.delete and not self.create


def recarve(slices: Sequence[Slice], used_ids: Set[str], want: Mapping[str, int],
            capacity: int = GROUPS) -> Recarve:
    """Deterministic slice diff: per profile keep the used slices, then the free ones with the
    lowest serials, up to the spec's count; delete the other free slices; create the missing ones.
    ``achievable``: the kept slices plus the new ones fit in ``capacity`` groups (a spec that asks
    for more than the slices in use leave room for is a drain target: only its deletions apply)."""
    out = Recarve()
    by_prof: Dict[str, List[Slice]] = {}
    for s in slices:
        by_prof.setdefault(s.profile, []).append(s)
    for p, ss in sorted(by_prof.items()):
        ss = sorted(ss, key=lambda s: (s.id not in used_ids, serial_of(s.id), s.id))
        n = max(0, want.get(p, 0))
        for k, s in enumerate(ss):
            if k < n or s.id in used_ids:
                out.keep.append(s)
                if k >= n:
                    out.blocked.append(f"slice {s.id} ({p}) is in use")
            else:
                out.delete.append(s)
    for p, q in sorted(want.items()):
        missing = q - sum(1 for s in out.keep if s.profile == p)
        out.create.extend([p] * max(0, missing))
    used_groups = sum(groups_of(s.profile) for s in out.keep)
    out.achievable = not out.blocked and used_groups + sum(groups_of(p) for p in out.create) <= capacity
    return out


def place_slices(existing: Sequence[Slice], profiles: Sequence[str], gpu_id: str, vram_bytes: int,
                 capacity: int = GROUPS, next_serial: int = 0) -> List[Slice]:
    """New slices next to ``existing`` (never moved): largest first, each on a block of groups
    aligned to its size when one is free (buddy placement, so whole-partition-shaped holes stay
    whole), preferring blocks inside the most-used larger block; else contiguous; else any free
    groups.  Raises ValueError when the groups do not suffice."""
    taken: Set[int] = {g for s in existing for g in slice_groups(s)}
    # serials only grow: a device id kubelet has seen is never reused for another slice
    serial = max(next_serial, 1 + max([serial_of(s.id) for s in existing] or [-1]))
    out: List[Slice] = []
    for p in sorted(profiles, key=lambda x: (-groups_of(x), x)):
        n = groups_of(p)
        free = [g for g in range(capacity) if g not in taken]
        if len(free) < n:
            raise ValueError(f"cannot place a {p} slice: {n} groups needed, {len(free)} free")
        pick: Optional[List[int]] = None
        best: Optional[Tuple[int, ...]] = None
        for start in range(0, capacity - n + 1, n):
            block = list(range(start, start + n))
            if any(g in taken for g in block):
                continue
            # buddy best fit: the block whose smallest enclosing blocks are the most used, so the
            # free space of the emptier halves / quarters stays whole for the bigger slices
            key = []
            size = 2 * n
            while size <= capacity:
                pstart = (start // size) * size
                key.append(-sum(1 for g in range(pstart, pstart + size) if g in taken))
                size *= 2
            key.append(start)
            if best is None or tuple(key) < best:
                best, pick = tuple(key), block
        if pick is None:
            run: List[int] = []
            for g in free:
                run = run + [g] if run and g == run[-1] + 1 else [g]
                if len(run) == n:
                    pick = run
                    break
        pick = pick or free[:n]
        taken.update(pick)
        rows = [GROUP_ROWS * g + i for g in pick for i in range(GROUP_ROWS)]
        out.append(Slice(f"{gpu_id}{SLICE_SEP}{serial}", p, rows, vram_bytes // capacity * n))
        serial += 1
    return out


def apply_recarve(slices: Sequence[Slice], rc: Recarve, gpu_id: str, vram_bytes: int,
                  capacity: int = GROUPS) -> List[Slice]:
    """The GPU's slices after ``rc``: deletions always, creations only when achievable."""
    kept = list(rc.keep)
    if rc.achievable and rc.create:
        nxt = 1 + max([serial_of(s.id) for s in list(slices) + list(rc.delete)] or [-1])
        kept += place_slices(kept, rc.create, gpu_id, vram_bytes, capacity, nxt)
    return sorted(kept, key=lambda s: (serial_of(s.id), s.id))


def parse_gpu_set(value: Optional[str]) -> Set[int]:
    """``"0,2"`` -> {0, 2} (the sliced-GPU annotations); junk entries are ignored."""
    out: Set[int] = set()
    for x in (value or "").split(","):
        x = x.strip()
        if x.isdigit():
            out.add(int(x))
    return out


def format_gpu_set(gpus: Iterable[int]) -> str:
    return ",".join(str(g) for g in sorted(set(gpus)))


def spec_by_gpu(spec: Iterable) -> Dict[int, Dict[str, int]]:
    out: Dict[int, Dict[str, int]] = {}
    for a in spec:
        d = out.setdefault(a.index, {})
        d[a.profile] = d.get(a.profile, 0) + a.quantity
    return {g: {p: q for p, q in d.items() if q > 0} for g, d in out.items()}
