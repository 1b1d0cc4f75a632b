"""CU-mask placement for slices on an MI355X in SPX mode.

Measured on the box (``profiles/gpu_report_r1_first.json``, census of CU-masked streams):

* queue CU-mask bit ``i`` lands on XCD ``i mod 8`` — mask bits 0..31 enable 4 CUs on *every* XCD;
* an XCD whose mask bits are all zero is **not** disabled: a mask of bits {0, 8, 16, ...} (all on
  XCD 0) still ran on all 256 CUs.

* mask row ``r`` (bits ``[8r, 8r+8)``, one CU on each XCD) sits on shader engine ``r mod 4`` of
  every XCD (``profiles/census_map_r1.json``), and each XCD hands workgroups to its 4 SEs
  round-robin, so a slice must also own the same number of CUs on every SE.

So the unit of allocation is a **row group**: 4 consecutive rows ``[4g, 4g+4)`` = 32 mask bits = one
CU on every SE of every XCD; a 256-CU MI355X has 8 groups.  A ``<c>cu`` slice owns ``c/32`` groups
(contiguous when possible).  Memory-only (shared) slices run on the rows no dedicated slice owns.
Rows of slices in use are never moved.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

from .profile import parse_profile

XCDS = 8
ROW_CUS = 8          # mask bits per row (one CU per XCD)
GROUP_ROWS = 4       # rows per allocation group (one CU per SE per XCD)


@dataclass
class Slice:
    """One slice of one GPU as recorded in the slice configuration."""
    id: str                 # device id advertised to kubelet, e.g. "0000:a4:00.0::s3"
    profile: str            # "<c>cu.<m>gb" or "<m>gb"
    rows: List[int] = field(default_factory=list)
    hbm_bytes: int = 0

    @property
    def cus(self) -> List[int]:
        return [8 * r + x for r in sorted(self.rows) for x in range(XCDS)]

    def to_dict(self) -> Dict[str, object]:
        return {"id": self.id, "profile": self.profile, "rows": sorted(self.rows), "hbmBytes": self.hbm_bytes}

    @staticmethod
    def from_dict(d: Dict[str, object]) -> "Slice":
        return Slice(str(d["id"]), str(d["profile"]), [int(x) for x in d.get("rows", [])], int(d.get("hbmBytes", 0)))


def rows_total(cu_count: int) -> int:
    return cu_count // ROW_CUS


def allocate_rows(n_rows: int, taken: Iterable[int], total_rows: int) -> Optional[List[int]]:
    """Whole free row groups for ``n_rows`` rows (a multiple of :data:`GROUP_ROWS`): a contiguous
    run of groups first-fit, else any free groups; None if there are not enough free groups."""
    taken_set = set(taken)
    n_groups = -(-n_rows // GROUP_ROWS)
    free = [g for g in range(total_rows // GROUP_ROWS)
            if not any(GROUP_ROWS * g + i in taken_set for i in range(GROUP_ROWS))]
    if len(free) < n_groups:
        return None
    pick: Optional[List[int]] = None
    run: List[int] = []
    for g in free:
        if run and g != run[-1] + 1:
            run = []
        run.append(g)
        if len(run) == n_groups:
            pick = run
            break
    pick = pick or free[:n_groups]
    return [GROUP_ROWS * g + i for g in pick for i in range(GROUP_ROWS)][:n_rows]


def place(existing: Sequence[Slice], wanted: Sequence[Tuple[str, str]], cu_count: int) -> List[Slice]:
    """Place new slices ``[(id, profile)]`` next to ``existing`` ones (whose rows are kept).
    Raises ValueError when the dedicated CUs do not fit."""
    total = rows_total(cu_count)
    taken = [r for s in existing for r in s.rows]
    out: List[Slice] = []
    # largest first limits fragmentation
    for sid, prof in sorted(wanted, key=lambda w: -parse_profile(w[1]).cus):
        p = parse_profile(prof)
        need = p.cus // ROW_CUS
        rows: List[int] = []
        if need:
            got = allocate_rows(need, taken, total)
            if got is None:
                raise ValueError(f"cannot place slice {prof}: {need} rows needed, "
                                 f"{total - len(set(taken))} free")
            rows = got
            taken.extend(rows)
        out.append(Slice(sid, prof, rows, p.memory_gb * 10**9))
    return out


def shared_rows(slices: Sequence[Slice], cu_count: int) -> List[int]:
    owned = {r for s in slices for r in s.rows}
    return [r for r in range(rows_total(cu_count)) if r not in owned]


def cus_of(s: Slice, all_slices: Sequence[Slice], cu_count: int) -> List[int]:
    """CUs a slice may run on: its own rows, or the shared pool for memory-only slices."""
    if s.rows:
        return s.cus
    return [8 * r + x for r in shared_rows(all_slices, cu_count) for x in range(XCDS)]


def hsa_cu_mask(cus: Iterable[int], device: int = 0) -> str:
    """``HSA_CU_MASK`` value: ``<device>:<ranges>`` (e.g. ``0:0-31,64-95``)."""
    cs = sorted(set(cus))
    if not cs:
        return f"{device}:"
    ranges = []
    start = prev = cs[0]
    for c in cs[1:]:
        if c == prev + 1:
            prev = c
            continue
        ranges.append(f"{start}-{prev}" if prev != start else f"{start}")
        start = prev = c
    ranges.append(f"{start}-{prev}" if prev != start else f"{start}")
    return f"{device}:" + ",".join(ranges)


def mask_hex(cus: Iterable[int], cu_count: int = 256) -> str:
    """32-bit-word hex bitmap (word 0 first), the format of ``hipExtStreamCreateWithCUMask``."""
    words = [0] * ((cu_count + 31) // 32)
    for c in cus:
        words[c // 32] |= 1 << (c % 32)
    return ",".join(f"{w:08x}" for w in words)
