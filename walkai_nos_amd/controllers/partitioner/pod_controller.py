"""Partitioner pod controller (reference ``internal/controllers/gpupartitioner/mig_controller.go:37-213``).

Per Pod event: consider the pod only if it is Pending, unbound and ``PodScheduled=False`` with
reason ``Unschedulable`` (B.8); read the partition profiles it requests; list the nodes opted in
with ``nos.nebuly.com/gpu-partitioning=<kind>``; if every requested profile is already *free*
somewhere do nothing; otherwise re-plan and write the new spec annotations with a fresh plan ID.

Deliberate changes vs the reference:

* Q1 — the "already present" check looks at **free** capacity; the reference also counts used
  devices, so a pod never triggers repartitioning once every device of its profile is in use;
* Q11 — planning is **batched**: all currently pending pods of the same kind are planned together
  after the batch window (``batchWindowTimeoutSeconds`` / ``batchWindowIdleSeconds``), and nodes
  are **scored** (profiles provided, then fewest GPUs whose geometry changes, then name) instead of
  "first node that can change wins";
* Q14 — when no node can help, the pod is requeued with back-off instead of waiting for an
  unrelated event.
"""
from __future__ import annotations

import collections

import logging
import time
from dataclasses import dataclass
from typing import Any, Callable, Dict, List, Mapping, Optional, Tuple, Union

from ...api import v1alpha1 as api
from ...kube import objects as ko
from ...kube.errors import NotFound
from ...kube.runtime import Request, Result
from ...models import annotation as ann
from ...models.defaults import ModelDefaults
from ...models.partitioned import PartitionedNode
from ...models.slicing import gpu as slicing_gpu
from ...models.slicing.gpu import SlicingNode
from ...models.xcp import node as xcp_node
from ...partitioning.planner import Partitioner, build_node_partitioning, new_plan_id
from ...utils import pod as podutil
from ...utils.metrics import REGISTRY
from .lifetimes import LifetimeTracker

log = logging.getLogger("nos.partitioner")

NodeModel = Union[PartitionedNode, SlicingNode]

POLICIES = ("fifo", "batch", "simulate", "pack")


_REQ_CACHE: Dict[Tuple[str, str], Dict[str, int]] = {}


def requested_profiles(kind: str, pod: Dict[str, Any]) -> Dict[str, int]:
    """Profiles a pod requests. Container requests are immutable once a pod exists, so the result
    is memoised per pod UID (the planner re-reads every pending pod on every reconcile)."""
    uid = pod.get("metadata", {}).get("uid")
    key = (kind, uid) if uid else None
    if key is not None:
        hit = _REQ_CACHE.get(key)
        if hit is not None:
            return dict(hit)
    out = xcp_node.get_requested_profiles(pod) if kind == api.PARTITIONING_KIND_XCP \
        else slicing_gpu.get_requested_profiles(pod)
    if key is not None:
        if len(_REQ_CACHE) > 100_000:
            _REQ_CACHE.clear()
        _REQ_CACHE[key] = dict(out)
    return out


def new_node_model(kind: str, node: Dict[str, Any], scoring: str = "fraction",
                   defaults: Optional[ModelDefaults] = None) -> NodeModel:
    """The node's model under the planner's ``defaults`` (layout of unlabeled xcp nodes, memory-only
    counts skipped on cumask GPUs); none given: the library defaults."""
    if kind == api.PARTITIONING_KIND_XCP:
        return xcp_node.new_node(node, scoring, defaults)
    return slicing_gpu.new_node(node, defaults)


def _changed_gpus(before: NodeModel, after: NodeModel) -> int:
    return sum(1 for a, b in zip(before.gpus, after.gpus) if a.geometry() != b.geometry())


def plan_cluster(models: Mapping[str, NodeModel], required: Mapping[str, int]) -> Dict[str, NodeModel]:
    """Greedy over nodes with a score: provided profiles desc, GPUs changed asc, node name asc."""
    remaining = {p: q for p, q in required.items() if q > 0}
    current = dict(models)
    changed: Dict[str, NodeModel] = {}
    while remaining:
        best: Optional[Tuple[Tuple[float, int, str], str, NodeModel]] = None
        for name, m in sorted(current.items()):
            cand = m.clone()
            before_free = m.free()
            if not cand.update_geometry_for(remaining):
                continue
            after_free = cand.free()
            w = getattr(cand, "weight", None)
            provided = sum(min(max(0, after_free.get(p, 0) - before_free.get(p, 0)), q) * (1.0 if w is None else w(p))
                           for p, q in remaining.items())
            if provided <= 0:
                continue
            score = (-provided, _changed_gpus(m, cand), name)
            if best is None or score < best[0]:
                best = (score, name, cand)
        if best is None:
            break
        _, name, cand = best
        before_free = current[name].free()
        current[name] = cand
        changed[name] = cand
        after_free = cand.free()
        for p in list(remaining):
            remaining[p] -= max(0, after_free.get(p, 0) - before_free.get(p, 0))
            if remaining[p] <= 0:
                del remaining[p]
    return changed


def plan_cluster_fifo(models: Mapping[str, NodeModel], pending: List[Dict[str, int]],
                      incoming: Optional[Mapping[str, int]] = None) -> Dict[str, NodeModel]:
    """Head-of-line planning: walk the pending pods in arrival order.  A pod that fits existing free
    capacity *reserves* it in the model (so a later flip cannot destroy it); capacity that in-flight
    plans will provide (``incoming``) is consumed next; otherwise the best node is re-planned for
    exactly that pod (fewest GPUs changed, then name) and the partitions the new geometry creates
    are offered to the pods behind it.  Fair to the oldest request, and a freshly split GPU is
    filled from the queue instead of being split again."""
    current = {n: m.clone() for n, m in models.items()}
    changed: Dict[str, NodeModel] = {}
    extra = {p: q for p, q in (incoming or {}).items() if q > 0}
    hopeless = set()  # profiles no node can provide in this pass (capacity only shrinks within a pass)
    # pods still to walk per request: a memory-only slice count the model skips (SKIP_SHARED_COUNTS)
    # is passed by carving for this pod and the next one with the same request at once
    behind = collections.Counter(tuple(sorted(r.items())) for r in pending)
    for req in pending:
        behind[tuple(sorted(req.items()))] -= 1
        placed = False
        for name in sorted(current):
            try:
                current[name].add_pod(req)
                placed = True
                break
            except ValueError:
                continue
        if not placed and all(extra.get(p, 0) >= q for p, q in req.items()):
            for p, q in req.items():
                extra[p] -= q
            placed = True
        if placed:
            continue
        key = tuple(sorted(req.items()))
        if key in hopeless:
            continue
        best: Optional[Tuple[Tuple[int, str], str, NodeModel]] = None
        wants = [req] + ([{p: 2 * q for p, q in req.items()}] if behind[key] > 0 else [])
        for name, m in sorted(current.items()):
            for want in wants:
                cand = m.clone()
                if not cand.update_geometry_for(want):
                    continue
                try:
                    cand.add_pod(req)
                except ValueError:
                    continue
                break
            else:
                continue
            score = (_changed_gpus(m, cand), name)
            if best is None or score < best[0]:
                best = (score, name, cand)
        if best is None:
            hopeless.add(key)
            continue  # this pod cannot be helped now; later pods may still be
        _, name, cand = best
        current[name] = cand
        changed[name] = cand
    return changed


@dataclass
class PackParams:
    """Knobs of the flip-aware ``pack`` policy (``GpuPartitionerConfig.packing``)."""
    min_fill: float = 0.5           # flip an idle GPU only if the queue fills >= this fraction of it
    starve_after: float = 600.0     # seconds: older pods win an idle GPU regardless of min_fill
    drain_after: float = 7200.0     # seconds: a pod waiting this long makes a busy GPU drain for it
    drain_backlog: float = 2.0      # ... if its profile's queue would fill at least this many GPUs
    spx_reserve: bool = True        # keep idle SPX GPUs for recent whole-GPU demand (multi-GPU)
    reserve_decay: float = 0.5      # EMA decay of the whole-GPU demand estimate per planning pass
    drain_gain: float = 0.3         # drain a busy GPU whose used fraction is this much below the
    drain_gain_after: float = 180.0  # ... fill a profile waiting this long would give it (0 = off)
    reserve_break_fill: float = 2.0  # a queue filling this many GPUs takes a reserved idle SPX GPU
    min_stint: float = 120.0        # seconds: a GPU keeps a mode at least this long before it may be
                                    # drained for another (refilled from its own queue meanwhile)
    replan_every: float = 10.0      # seconds: an unchanged cluster is re-planned at most this often (0 = always)
    unserved_after: float = 300.0   # seconds (x GPUs of the cluster): a profile no GPU serves (none in its mode, none draining
                                    # to it) whose oldest pod waited this long gets a GPU drained for
                                    # it regardless of gain (0 = off) — the fairness that makes a
                                    # single GPU cycle through the modes its pods ask for
    slice_reserve_after: float = 900.0  # seconds: sliced GPUs (xcp-layout slices/auto) — the oldest pod that
                                    # fits on no sliced GPU this long drains one for itself (0 = never)
    slice_reserve_lifetimes: float = 3.75  # ... once the planner has seen pods finish (lifetimes.py): this
                                    # many median pod run times instead (0 = keep the constant)
    slice_reserve_backlog: float = 3.0  # ... stretched by backlog / this (GPUs of waiting work per sliced GPU; 0 = fixed)
    slice_reserve_stretch: float = 4.0  # ... at most this many times (load 1.2 on 2 / 8 GPUs: 98.4 / 99.5% at 4, 88.3 / 97.2 at 2)
    slice_reserve_hold: bool = True  # a reservation holds until a pod of its profile is placed ...
    slice_reserve_hold_max_gpus: int = 2  # ... on clusters of at most this many sliced GPUs (0 = any size): holding
                                    # always gains under a point at load 1.0 on 4-8 GPUs but at load 1.2 every
                                    # GPU ends up held for some profile (4 / 8 GPUs 85 / 83% vs 95 / 97% at 2)
    slice_free_drain: bool = True   # the oldest waiting pod reserves a GPU whose unused room no waiting pod fits,
    slice_free_drain_after: float = 0.5  # ... once it waited this many median pod run times per other sliced GPU
    slice_free_drain_cap: float = 0.75  # ... but at most this many (0 = no cap)
    slice_strand_weight: float = 1.0  # drain victim on a multi-GPU node: its slices in use of profiles pods wait
                                    # for count as idle this many times over the drain (kube-scheduler sees as
                                    # many fewer free slices of them on the node while the drain withholds them)
    slice_whole_overtake: float = 960.0  # seconds: a whole-GPU slice left free goes to the next whole-GPU pod
                                    # unless the oldest waiting pod is this much older (0 = strict FIFO)
    slice_whole_overtake_lifetimes: float = 4.0  # ... this many median pod run times once learned (0 = constant)
    slice_fill: bool = True         # carve a sliced GPU's leftover groups into cpx slices


def _mode_of(gpu: Any) -> Optional[str]:
    if getattr(gpu, "sliced", False):
        return "sliced"  # a layout, not a hardware mode: planned per pod (sliced.py)
    geo = gpu.geometry()
    return next(iter(geo)) if len(geo) == 1 else None


def _nps_of(profile: str) -> Optional[str]:
    return profile.split("_", 1)[1] if "_" in profile else None


def _plan_memory_partitions(current: Dict[str, NodeModel], changed: Dict[str, NodeModel], demand: Dict[str, float],
                            oldest: Dict[str, float], unserved: List[Tuple[Dict[str, int], float]],
                            params: "PackParams", mode_age: Optional[Callable[[str, int], float]],
                            total_gpus: int, frac: Callable[[str], float]) -> None:
    """Node-wide memory-partition (NPS) switches for the pack policy.

    A profile of another NPS than a node's (``cpx_nps2`` on an NPS1 node) needs the whole node
    re-partitioned: the memory mode is node-wide, and the agent changes it only when every GPU is
    idle. For an NPS no node has (or is switching to): an **idle** node — every GPU idle, each past
    ``min_stint`` — is switched when the waiting demand fills ``min_fill`` of a GPU or a pod has
    waited ``starve_after`` (the smallest such node: the fewest GPUs re-partitioned); failing that,
    once a pod has waited ``unserved_after`` x the cluster's GPUs, the least-used node is
    **drained** for it (every GPU's spec changes now, the partition plugin withholds them all).
    The switched node's GPUs take the waiting profiles' modes (most demand first, one GPU per
    started GPU of demand) and the rest the fewest-partition geometry of the new NPS. Profiles of an NPS that
    no node serves leave ``demand`` here: the per-GPU rules can only flip modes within a node's NPS."""
    from ...models.xcp.node import new_gpu
    nps_now = {n: getattr(m, "memory_partition", None) for n, m in current.items()}
    nps_next = {n: getattr(m, "memory_target", None) for n, m in current.items()}
    for target in sorted({_nps_of(p) for p in demand} - {None}):
        profs = sorted((p for p in demand if _nps_of(p) == target), key=lambda p: (-demand[p], p))
        if any(nps_now[n] in (None, target) or nps_next[n] == target for n in current):
            continue  # a node has (or is switching to) this NPS: the per-GPU rules serve it
        need = sum(demand[p] for p in profs)
        waited = max(oldest.get(p, 0.0) for p in profs)

        def past_stint(n: str) -> bool:
            return mode_age is None or params.min_stint <= 0 or \
                all(mode_age(n, g.index) >= params.min_stint for g in current[n].gpus)

        def layout(m: NodeModel) -> List[Dict[str, int]]:
            """Per GPU: a waiting profile's mode (one GPU per started GPU of its demand), then the
            fewest-partition geometry the model allows in the new NPS (SPX needs NPS1)."""
            left = {p: demand[p] for p in profs}
            out = []
            for g in m.gpus:
                p = next((q for q in profs if left[q] > 1e-9), None)
                if p is None:
                    probe = new_gpu(g.model, g.index, target)
                    probe.init_geometry()
                    out.append(probe.geometry())
                    continue
                out.append({p: round(1.0 / frac(p)) if frac(p) > 0 else 1})
                left[p] -= 1.0
            return out
        idle_nodes = [n for n in sorted(current) if current[n].gpus and nps_next[n] is None and past_stint(n)
                      and all(g.is_idle() and g.target is None for g in current[n].gpus)]
        chosen = None
        if idle_nodes and (need + 1e-9 >= params.min_fill or waited >= params.starve_after):
            chosen = min(idle_nodes, key=lambda n: (len(current[n].gpus), n))
            m = current[chosen]
            try:
                new = [new_gpu(g.model, g.index, target) for g in m.gpus]
                for g, geo in zip(new, layout(m)):
                    g.apply_geometry(geo)
            except ValueError:
                chosen = None
            else:
                m.gpus = new
                for i, (req, _) in enumerate(list(unserved)):
                    if len(req) == 1 and next(iter(req)) in profs:
                        try:
                            m.add_pod(req)
                        except (ValueError, AttributeError):
                            continue
        elif params.unserved_after > 0 and waited >= params.unserved_after * max(1, total_gpus):
            cands = [n for n in sorted(current) if current[n].gpus and nps_next[n] is None and past_stint(n)
                     and all(g.target is None for g in current[n].gpus)]
            if cands:
                used = {n: sum(sum(g.used.values()) * frac(p) for g in current[n].gpus for p in g.used)
                        for n in cands}
                chosen = min(cands, key=lambda n: (used[n], n))
                for g, geo in zip(current[chosen].gpus, layout(current[chosen])):
                    g.target = geo
        if chosen is not None:
            current[chosen].memory_target = target
            nps_next[chosen] = target
            changed[chosen] = current[chosen]
        for p in profs:
            demand.pop(p, None)


def plan_cluster_pack(models: Mapping[str, NodeModel], pending: List[Tuple[Dict[str, int], float]],
                      incoming: Optional[Mapping[str, int]] = None, params: Optional[PackParams] = None,
                      spx_demand: float = 0.0,
                      mode_age: Optional[Callable[[str, int], float]] = None,
                      last_served: Optional[Mapping[str, float]] = None,
                      pods_of: Optional[Callable[[str, int], List[Tuple[int, float]]]] = None,
                      life: Any = None) -> Dict[str, NodeModel]:
    """Flip-aware packing for homogeneous compute partitions (the MI355X replacement of the
    reference's "first node that can change wins").

    A mode flip destroys every partition of a GPU and costs seconds of outage (amd-smi switch plus
    device-plugin re-registration), so the policy flips as little as possible and only idle GPUs:

    1. pending pods (oldest first) take existing free partitions — split GPUs are filled first
       because every free partition of the current layout is consumed before any flip — then the
       capacity in-flight plans will provide;
    2. the remaining demand is summed per profile in GPU fractions, each profile remembering its
       oldest waiting pod;
    3. each **idle** GPU (no partition in use; busy GPUs are never touched) is given to the profile
       with the largest demand, but only when the queue fills at least ``min_fill`` of it, or that
       profile's oldest pod has waited ``starve_after`` (so nothing starves): otherwise it keeps
       its mode (hysteresis — an idle GPU left as it is costs nothing, a flip costs an outage);
    4. on multi-GPU nodes idle SPX GPUs are kept as a reserve sized from the recent whole-GPU demand
       (``spx_demand``, an EMA in GPUs), unless a starving pod needs them or a profile's queue
       would fill ``reserve_break_fill`` GPUs (an idle GPU held against a whole GPU of waiting work
       serves nothing; the EMA lags behind whole-GPU pods that have already left);
    5. a profile whose oldest pod has waited ``drain_after``, and whose queue would fill
       ``drain_backlog`` GPUs (a drain idles partitions, so it must buy a full GPU of work), or whose
       oldest pod has waited ``drain_gain_after`` and whose queue would fill a GPU at least
       ``drain_gain`` more than the pods now holding one (a single-GPU node otherwise serves one
       profile for as long as its pods keep arriving), with no idle GPU to take gets one busy
       GPU **drained** for it: the least-used GPU in another mode that has held its mode for at
       least ``min_stint`` (``mode_age``; a GPU just flipped first serves — and refills — its own
       queue) gets the new spec now, is no longer offered to new pods (``PartitionedGPU.target``;
       the nos partition device plugin reports every partition of a GPU being re-partitioned
       Unhealthy, so neither kube-scheduler nor kubelet can place a pod there), and the agent flips
       it when its last pod leaves.  Without this a single GPU that never goes idle would starve
       every other profile forever;
    6. **fairness**: a profile that no GPU serves — none in its mode, none draining towards it — and
       whose oldest pod has waited ``unserved_after`` x (GPUs in the cluster) gets a GPU drained for
       it without the gain
       condition (still the least-used GPU past ``min_stint``).  On a multi-GPU node the GPUs settle
       into modes that match the demand and this rarely fires; on a single GPU it is what makes the
       GPU cycle through the modes its queue asks for, each mode serving (and refilling) for at
       least ``min_stint``.

    ``pending`` = [(requested profiles, age in seconds)], oldest first; ``mode_age(node, gpu)`` =
    seconds since that GPU's mode last changed (None: unknown, treated as old)."""
    params = params or PackParams()
    current = {n: m.clone() for n, m in models.items()}
    changed: Dict[str, NodeModel] = {}
    extra = {p: q for p, q in (incoming or {}).items() if q > 0}
    unserved: List[Tuple[Dict[str, int], float]] = []
    names = sorted(current)

    def best_free(m: NodeModel) -> Dict[str, int]:
        """Most free partitions of each profile on one offered (non-draining) GPU of the node: a
        single-GPU request can only fit where this covers it (the screen that keeps the pass from
        trying — and failing — every GPU of every node for every pending pod at cluster scale)."""
        out: Dict[str, int] = {}
        for g in m.gpus:
            if g.target is None:
                for prof, q in g.free.items():
                    if q > out.get(prof, 0):
                        out[prof] = q
        return out
    free_of = {n: best_free(current[n]) for n in names}
    placed_on: Dict[Tuple[str, int], float] = {}   # (node, GPU) -> oldest pod given a free partition there
    for req, age in pending:
        placed = False
        for name in names:
            bf = free_of[name]
            if any(bf.get(prof, 0) < q for prof, q in req.items()):
                continue
            before = [dict(g.used) for g in current[name].gpus]
            try:
                current[name].add_pod(req)
                free_of[name] = best_free(current[name])
                placed = True
                for g, b in zip(current[name].gpus, before):
                    if g.used != b:
                        placed_on[(name, g.index)] = max(age, placed_on.get((name, g.index), 0.0))
                break
            except ValueError:
                continue
        if not placed and all(extra.get(p, 0) >= q for p, q in req.items()):
            for p, q in req.items():
                extra[p] -= q
            placed = True
        if not placed:
            unserved.append((req, age))
    if not unserved or not current:
        return changed
    if any(getattr(m, "layout", "partitions") != "partitions" for m in current.values()):
        from .sliced import plan_sliced
        plan_sliced(current, models, changed, unserved, params, mode_age, pods_of, life, placed_on)
        if not unserved:
            return changed
    # the homogeneous rules below only touch GPUs of nodes laid out as hardware partitions
    hw_nodes = {n for n, m in current.items() if getattr(m, "layout", "partitions") == "partitions"}
    first = next(iter(current.values()))
    w = getattr(first, "weight", None)
    frac = (lambda p: w(p)) if w is not None else (lambda p: 1.0)
    demand: Dict[str, float] = {}
    oldest: Dict[str, float] = {}
    for req, age in unserved:
        if len(req) != 1:
            continue  # a pod asking for two different profiles cannot be helped by one flip
        (p, q), = req.items()
        demand[p] = demand.get(p, 0.0) + q * frac(p)
        oldest[p] = max(oldest.get(p, 0.0), age)
    total_gpus = sum(len(m.gpus) for m in current.values())
    _plan_memory_partitions(current, changed, demand, oldest, unserved, params, mode_age, total_gpus, frac)
    idle = [(name, g) for name in sorted(hw_nodes) for g in current[name].gpus
            if g.is_idle() and g.target is None]
    spx_gpus = [(n, g) for n in sorted(hw_nodes) for g in current[n].gpus if (_mode_of(g) or "").startswith("spx")]
    reserve = min(len(spx_gpus), int(round(spx_demand))) if (params.spx_reserve and total_gpus > 1) else 0
    # idle GPUs whose mode nobody is waiting for go first; SPX GPUs last (they are the reserve)
    idle.sort(key=lambda ng: (bool(ng[1].degraded), (_mode_of(ng[1]) or "").startswith("spx"), ng[0], ng[1].index))
    spx_kept = sum(1 for n, g in spx_gpus if not g.is_idle())
    for name, g in idle:
        if not demand:
            break
        cur = _mode_of(g)
        best: Optional[Tuple[Tuple[int, float, float], str]] = None
        for p, d in demand.items():
            if p == cur or d <= 0:
                continue
            starving = oldest.get(p, 0.0) >= params.starve_after
            fill = min(d, 1.0)
            if fill + 1e-9 < params.min_fill and not starving:
                continue
            # starving profiles: the longest wait first (FIFO across profiles); otherwise the fullest
            key = (1, oldest.get(p, 0.0), fill) if starving else (0, fill, oldest.get(p, 0.0))
            if best is None or key > best[0]:
                best = (key, p)
        if best is None:
            continue
        (starving, _, _), p = best
        if (cur is not None and cur.startswith("spx") and spx_kept < reserve and not starving
                and demand[p] + 1e-9 < params.reserve_break_fill):
            spx_kept += 1
            continue  # keep this idle SPX GPU for the whole-GPU demand
        trial = g.clone()
        if not trial.update_geometry_for({p: 10**6}) or _mode_of(trial) != p:
            continue
        g.used, g.free = trial.used, trial.free
        changed[name] = current[name]
        # the new partitions serve the waiting pods of that profile
        placed_any = True
        while placed_any and demand.get(p, 0) > 0:
            placed_any = False
            for i, (req, age) in enumerate(unserved):
                if set(req) == {p}:
                    try:
                        g.add_pod(req)
                    except ValueError:
                        break
                    demand[p] -= sum(q * frac(p) for q in req.values())
                    unserved.pop(i)
                    placed_any = True
                    break
        if demand.get(p, 0) <= 1e-9:
            demand.pop(p, None)
    # 5. drain a busy GPU for a profile that has waited too long (backlog rule), or whose waiting
    #    demand would use the GPU much better than the few pods holding it now (gain rule)
    draining_to = {next(iter(g.target)) for m in current.values() for g in m.gpus if g.target}
    served = {_mode_of(g) for m in current.values() for g in m.gpus} | draining_to
    used_of = (lambda g: g.used_fraction(lambda q: round(1.0 / frac(q)))) if w is not None else \
        (lambda g: float(sum(g.used.values())))
    # round robin: the profile served least recently (no GPU in its mode for longest) drains first,
    # then the oldest waiting pod — oldest-first alone lets the profiles with the longest queues
    # take turn after turn while a shorter queue's pods keep waiting
    order = sorted(demand, key=lambda q: ((last_served or {}).get(q, float("-inf")), -oldest.get(q, 0.0)))
    for p in order:
        if p in draining_to:
            continue
        backlog = demand[p] >= params.drain_backlog - 1e-9 and oldest.get(p, 0.0) >= params.drain_after
        gain_ok = params.drain_gain_after > 0 and oldest.get(p, 0.0) >= params.drain_gain_after
        # the fairness wait scales with the node count of GPUs: the more GPUs, the sooner one goes
        # idle on its own and is handed to the waiting profile by rule 3 — a drain is the last resort
        starved = params.unserved_after > 0 and p not in served and \
            oldest.get(p, 0.0) >= params.unserved_after * max(1, total_gpus)
        if not backlog and not gain_ok and not starved:
            continue
        fill = min(demand[p], 1.0)
        cands = [(used_of(g), name, g) for name in sorted(hw_nodes) for g in current[name].gpus
                 if g.target is None and not g.is_idle() and _mode_of(g) != p
                 and (mode_age is None or params.min_stint <= 0 or mode_age(name, g.index) >= params.min_stint)]
        if not backlog:
            # a candidate qualifies through the gain rule, or through fairness — which weighs
            # waiting work: a GPU keeps serving its own profile while that queue holds more
            # GPU-seconds of waiting (demand x oldest wait) than the starved one does; turn-by-turn
            # alternation would give a whole-GPU queue one pod per cycle and a 1/8 queue eight,
            # whatever their demand
            pressure = lambda q: demand.get(q, 0.0) * oldest.get(q, 0.0)  # noqa: E731
            gain_fits = lambda c: gain_ok and w is not None and fill - c[0] >= params.drain_gain - 1e-9  # noqa: E731
            fair_fits = lambda c: starved and pressure(_mode_of(c[2])) <= pressure(p)  # noqa: E731
            cands = [c for c in cands if gain_fits(c) or fair_fits(c)]

        if not cands:
            continue
        _, name, g = min(cands, key=lambda c: (c[0], c[1], c[2].index))
        trial = g.clone()
        trial.used = {}
        trial.free = {}
        if not trial.update_geometry_for({p: 10**6}) or _mode_of(trial) != p:
            continue
        g.target = trial.geometry()
        changed[name] = current[name]
        draining_to.add(p)
        served.add(p)
    return changed


def simulate_schedule(models: Mapping[str, NodeModel], pending: List[Dict[str, int]]) -> Tuple[int, float]:
    """Pods (and GPU fraction) a first-fit scheduler would place, in arrival order, on ``models``."""
    sim = {n: m.clone() for n, m in models.items()}
    pods, frac = 0, 0.0
    for req in pending:
        for name in sorted(sim):
            try:
                sim[name].add_pod(req)
            except ValueError:
                continue
            pods += 1
            w = getattr(sim[name], "weight", None)
            frac += sum(q * (w(p) if w is not None else 1.0) for p, q in req.items())
            break
    return pods, frac


def materialize(orig: NodeModel, planned: NodeModel) -> NodeModel:
    """The planned geometry on the original occupancy (planners leave their own tentative
    reservations in the models they return; a simulation must start from real usage)."""
    out = orig.clone()
    for g_out, g_plan in zip(out.gpus, planned.gpus):
        geo = g_plan.geometry()
        g_out.free = {p: q - g_out.used.get(p, 0) for p, q in geo.items() if q - g_out.used.get(p, 0) > 0}
    return out


def planned_state(models: Mapping[str, NodeModel], changed: Mapping[str, NodeModel]) -> Dict[str, NodeModel]:
    return {n: (materialize(m, changed[n]) if n in changed else m) for n, m in models.items()}


def plan_cluster_simulate(models: Mapping[str, NodeModel], pending: List[Dict[str, int]],
                          incoming: Optional[Mapping[str, int]] = None) -> Dict[str, NodeModel]:
    """Scheduler-simulation planner (reference docs ``dynamic-gpu-partitioning/configuration.md:6-40``:
    "choose the partitioning that schedules the highest number of pending pods").

    Candidate plans: FIFO head-of-line, the whole-batch search, and FIFO over the queue re-ordered
    smallest-first and largest-first. Each candidate's resulting cluster is scheduled by a first-fit
    simulation of the pending queue; the winner schedules the most pods, then the most GPU fraction,
    then changes the fewest GPUs."""
    total: Dict[str, int] = {}
    for req in pending:
        for p, q in req.items():
            total[p] = total.get(p, 0) + q

    def size(req: Dict[str, int]) -> float:
        m = next(iter(models.values()), None)
        w = getattr(m, "weight", None) if m is not None else None
        return sum(q * (w(p) if w is not None else 1.0) for p, q in req.items())

    candidates = [plan_cluster_fifo(models, pending, incoming), plan_cluster(models, total),
                  plan_cluster_fifo(models, sorted(pending, key=size), incoming),
                  plan_cluster_fifo(models, sorted(pending, key=size, reverse=True), incoming)]
    best: Optional[Tuple[Tuple[int, float, int], Dict[str, NodeModel]]] = None
    for changed in candidates:
        final = planned_state(models, changed)
        pods, frac = simulate_schedule(final, pending)
        churn = sum(_changed_gpus(models[n], c) for n, c in changed.items())
        key = (-pods, -frac, churn)
        if best is None or key < best[0]:
            best = (key, changed)
    return best[1] if best is not None else {}


class PodController:
    def __init__(self, client: Any, kind: str = api.PARTITIONING_KIND_XCP, partitioner: Optional[Partitioner] = None,
                 clock: Callable[[], float] = time.time, batch_timeout: float = 0.0, batch_idle: float = 0.0,
                 retry_after: float = 5.0, scoring: str = "fraction", policy: str = "fifo",
                 pack: Optional[PackParams] = None, defaults: Optional[ModelDefaults] = None):
        self.client = client
        self.kind = kind
        self.scoring = scoring
        #: this planner's model defaults (``GpuPartitionerConfig`` through ``ModelDefaults.from_config``)
        self.defaults = defaults or ModelDefaults()
        if policy not in POLICIES:
            raise ValueError(f"unknown planning policy {policy!r}")
        self.policy = policy
        self.pack = pack or PackParams()
        self._first_seen: Dict[str, float] = {}   # pending pod uid -> first time the planner saw it
        self._mode_since: Dict[Tuple[str, int], Tuple[Optional[str], float]] = {}  # (node, gpu) -> (mode, since)
        self._last_served: Dict[str, float] = {}  # profile -> last time a GPU was in its mode
        self.spx_demand = 0.0                     # EMA of whole-GPU demand (GPUs), pack policy
        self.lifetimes = LifetimeTracker()        # run times of finished pods (sliced-GPU drains)
        self.partitioner = partitioner or Partitioner(client)
        self.clock = clock
        self.batch_timeout = batch_timeout
        self.batch_idle = batch_idle
        self.retry_after = retry_after
        self._window_start: Optional[float] = None
        self._window_last: Optional[float] = None
        self.plans_written = 0
        self._explained: Dict[str, str] = {}     # pending pod uid -> the wait reason already recorded
        # (API revision, {request: result}) of read-only reconciles: see reconcile()
        self._idle: Tuple[Optional[int], Dict[Request, Result]] = (None, {})

    # -- helpers -------------------------------------------------------------------------
    def should_consider(self, pod: Dict[str, Any]) -> bool:
        # a pod nos-scheduler holds back for its quota would not run on a new partition either
        return podutil.is_pending(pod) and not podutil.is_scheduled(pod) and podutil.is_unschedulable(pod) \
            and not podutil.is_blocked_by_quota(pod)

    def list_nodes(self) -> List[Dict[str, Any]]:
        return self.client.list("Node", label_selector=f"{api.LABEL_GPU_PARTITIONING}={self.kind}", copy=False)

    def pending_pods(self) -> List[Dict[str, int]]:
        """Per-pod requested profiles of the unschedulable pods, highest priority then oldest first."""
        pods = [p for p in self.client.list("Pod", field_selector="status.phase=Pending", copy=False)
                if self.should_consider(p)]
        pods.sort(key=lambda p: (-podutil.priority(p), p["metadata"].get("creationTimestamp", ""), ko.name(p)))
        out = []
        for p in pods:
            r = requested_profiles(self.kind, p)
            if r:
                out.append(r)
        return out

    def pending_with_age(self) -> List[Tuple[Dict[str, int], float]]:
        """(requested profiles, seconds since the planner first saw the pod), highest priority
        then oldest first (the ``pack`` policy's input)."""
        pods = [p for p in self.client.list("Pod", field_selector="status.phase=Pending", copy=False)
                if self.should_consider(p)]
        pods.sort(key=lambda p: (-podutil.priority(p), p["metadata"].get("creationTimestamp", ""), ko.name(p)))
        now = self.clock()
        seen: Dict[str, float] = {}
        out = []
        for p in pods:
            r = requested_profiles(self.kind, p)
            if not r:
                continue
            uid = p["metadata"].get("uid") or ko.name(p)
            t = self._first_seen.get(uid, now)
            seen[uid] = t
            out.append((r, now - t))
        self._first_seen = seen
        return out

    def pending_requests(self) -> Dict[str, int]:
        out: Dict[str, int] = {}
        for p in self.client.list("Pod", field_selector="status.phase=Pending", copy=False):
            if not self.should_consider(p):
                continue
            for k, v in requested_profiles(self.kind, p).items():
                out[k] = out.get(k, 0) + v
        return out

    def _explain_waits(self, models: Mapping[str, NodeModel]) -> None:
        """CU-mask nodes: record once, as a Normal event on the pod, why a pending pod gets no
        slice although a GPU has room for it — every GPU holds its slice cap
        (``nos.nebuly.com/max-slices-per-gpu``), or the memory-only slice would make a count the
        planner skips (``sharedSliceSkipCounts``: it waits for a second such pod or for a running one
        to finish)."""
        from ...models.slicing.profile import parse_profile
        pods = [p for p in self.client.list("Pod", field_selector="status.phase=Pending", copy=False)
                if self.should_consider(p)]
        live = {p["metadata"].get("uid") or "/".join(ko.key(p)) for p in pods}
        self._explained = {k: v for k, v in self._explained.items() if k in live}
        gpus = [g for m in models.values() for g in m.gpus]
        for p in pods:
            uid = p["metadata"].get("uid") or "/".join(ko.key(p))
            req = requested_profiles(self.kind, p)
            if uid in self._explained or len(req) != 1:
                continue
            (prof, q), = req.items()
            if any(g.free.get(prof, 0) >= q for g in gpus):
                continue   # a free slice waits for it: the scheduler binds it
            reason = message = None
            shared = not parse_profile(prof).dedicated
            fits_unskipped = []
            for g in gpus:
                c = g.clone()
                c.skip_shared = ()
                fits_unskipped.append(c.can_create(prof, q))
            if shared and any(fits_unskipped) and not any(g.can_create(prof, q) for g in gpus):
                n = min(g.shared_count() + q for g, ok in zip(gpus, fits_unskipped) if ok)
                reason, message = "SharedSliceCountSkipped", (
                    f"no memory-only slice carved for {prof}: {n} memory-only pods on one GPU split into two rate "
                    "classes by start order (sharedSliceSkipCounts); waiting for a second such pod or for a "
                    "running one to finish")
            elif gpus and all(g.slice_count() >= g.max_slices for g in gpus) and \
                    any(g.spare_memory_gb() >= parse_profile(prof).memory_gb * q for g in gpus):
                reason, message = "SliceCapReached", (
                    f"every GPU holds its {gpus[0].max_slices} slices (one pod process each; past eight the hardware "
                    "scheduler time-slices processes): label nos.nebuly.com/max-slices-per-gpu to allow more")
            if reason is None:
                continue
            self._explained[uid] = reason
            self._event(p, reason, message)

    def _event(self, pod: Dict[str, Any], reason: str, message: str) -> None:
        try:
            self.client.create({
                "apiVersion": "v1", "kind": "Event",
                "metadata": {"generateName": f"{ko.name(pod)}.", "namespace": ko.namespace(pod)},
                "involvedObject": {"apiVersion": "v1", "kind": "Pod", "name": ko.name(pod),
                                   "namespace": ko.namespace(pod), "uid": pod["metadata"].get("uid", "")},
                "reason": reason, "message": message, "type": "Normal",
                "source": {"component": "nos-gpu-partitioner"}})
        except Exception as e:  # noqa: BLE001 - an event is a courtesy
            log.debug("event for %s not recorded: %s", ko.name(pod), e)

    def _explain_reservations(self, models: Mapping[str, NodeModel], changed: Mapping[str, NodeModel]) -> None:
        """Sliced GPUs: when a pass starts draining a GPU for a pod (a reservation: the spec asks for
        the slices in use plus one that does not fit yet), record it once as a Normal event on the
        oldest pending pod of that profile, with what still runs there — the pod is waiting for that
        GPU to empty, and no new pod is placed on it meanwhile."""
        from ...models.xcp.slices import groups_of
        pods = [p for p in self.client.list("Pod", field_selector="status.phase=Pending", copy=False)
                if self.should_consider(p)]
        pods.sort(key=lambda p: (-podutil.priority(p), p["metadata"].get("creationTimestamp", ""), ko.name(p)))
        live = {p["metadata"].get("uid") or "/".join(ko.key(p)) for p in pods}
        self._explained = {k: v for k, v in self._explained.items() if k in live}
        for name, m in sorted(changed.items()):
            before = {g.index: g for g in getattr(models.get(name), "gpus", [])}
            for g in m.gpus:
                if not getattr(g, "sliced", False) or g.target is None or not g.target_sliced:
                    continue
                old = before.get(g.index)
                if old is not None and old.target == g.target:
                    continue   # a drain already in force
                extra = [x for x, n in g.target.items() if n > g.used.get(x, 0)]
                if not extra:
                    continue
                prof = max(extra, key=lambda x: (groups_of(x), x))
                for p in pods:
                    uid = p["metadata"].get("uid") or "/".join(ko.key(p))
                    if uid in self._explained or set(requested_profiles(self.kind, p)) != {prof}:
                        continue
                    running = sum(n for n in g.used.values() if n > 0)
                    self._explained[uid] = "SlicedGPUReserved"
                    self._event(p, "SlicedGPUReserved",
                                f"GPU {g.index} of node {name} is draining for this pod's {prof} slice: {running} "
                                "pods still run on it, and no new pod is placed there until the slice fits")
                    break

    def _models(self, nodes: List[Dict[str, Any]]) -> Dict[str, NodeModel]:
        out: Dict[str, NodeModel] = {}
        for n in nodes:
            try:
                out[ko.name(n)] = new_node_model(self.kind, n, self.scoring, self.defaults)
            except ValueError as e:
                log.warning("skipping node %s: %s", ko.name(n), e)
        return out

    @staticmethod
    def in_flight(node: Dict[str, Any]) -> bool:
        """A plan was written but the agent has not reported it yet (spec plan != status plan).
        The reference re-plans such nodes on every pod event, rewriting the spec
        with a new plan ID each time; here they are left alone until the agent reports."""
        a = ko.annotations(node)
        spec = a.get(api.ANNOTATION_PARTITIONING_PLAN)
        return bool(spec) and spec != a.get(api.ANNOTATION_REPORTED_PARTITIONING_PLAN)

    def incoming_free(self, node: Dict[str, Any]) -> Dict[str, int]:
        """Capacity an in-flight plan will provide: spec quantities minus what is used now."""
        status, spec = ann.parse_node_annotations(ko.annotations(node))
        used: Dict[Tuple[int, str], int] = {}
        for s in status:
            if s.is_used():
                used[(s.index, s.profile)] = used.get((s.index, s.profile), 0) + s.quantity
        out: Dict[str, int] = {}
        for s in spec:
            q = s.quantity - used.get((s.index, s.profile), 0)
            if q > 0:
                out[s.profile] = out.get(s.profile, 0) + q
        return out

    @staticmethod
    def free_somewhere(models: Mapping[str, NodeModel], requested: Mapping[str, int]) -> bool:
        for p, q in requested.items():
            if sum(m.free().get(p, 0) for m in models.values()) < q:
                return False
        return True

    def _served(self, models: Mapping[str, NodeModel], now: float) -> Dict[str, float]:
        """Last time each profile had a GPU in its mode (the round robin of the drain rules)."""
        for m in models.values():
            for g in getattr(m, "gpus", []):
                mode = _mode_of(g)
                if mode is not None:
                    self._last_served[mode] = now
        return dict(self._last_served)

    def _mode_ages(self, models: Mapping[str, NodeModel], now: float) -> Callable[[str, int], float]:
        """Track when each GPU's reported mode last changed (first sight counts as long ago)."""
        for name, m in models.items():
            for g in getattr(m, "gpus", []):
                mode = _mode_of(g)
                prev = self._mode_since.get((name, g.index))
                if prev is None:
                    self._mode_since[(name, g.index)] = (mode, float("-inf"))
                elif prev[0] != mode:
                    self._mode_since[(name, g.index)] = (mode, now)
        return lambda name, idx: now - self._mode_since.get((name, idx), (None, float("-inf")))[1]

    def _gpu_pods(self, nodes: List[Dict[str, Any]], now: float) -> Callable[[str, int], List[Tuple]]:
        """(groups, seconds run, declared bound) of the pods on each GPU: the agents' ``status-pods``
        annotation names them, their ``startTime`` dates them, ``spec.activeDeadlineSeconds`` bounds
        them (None when not declared); feeds the lifetime model as pods finish."""
        import json

        from ...models.xcp.slices import groups_of
        from .lifetimes import declared_bound
        names = {ko.name(n) for n in nodes}
        # running AND terminal pods: a pod that finished is a run time for the lifetime model (with
        # its own finishedAt), however briefly it ran between two passes
        pods = [p for p in self.client.list("Pod", field_selector="status.phase!=Pending", copy=False)
                if ko.pod_node_name(p) in names]
        groups: Dict[str, int] = {}
        bounds: Dict[str, Optional[float]] = {}
        mine = []
        for p in pods:
            r = requested_profiles(self.kind, p)
            if r:
                mine.append(p)
                if ko.pod_phase(p) == "Running":
                    k = "/".join(ko.key(p))
                    groups[k] = sum(groups_of(x) * q for x, q in r.items())
                    bounds[k] = declared_bound(p)
        ages = self.lifetimes.update(mine, now)
        by: Dict[Tuple[str, int], List[Tuple]] = {}
        for n in nodes:
            try:
                doc = json.loads(ko.annotations(n).get(api.ANNOTATION_GPU_PODS_STATUS) or "{}")
            except ValueError:
                continue
            for g, keys in doc.items():
                if str(g).isdigit():
                    by[(ko.name(n), int(g))] = [(groups[k], ages[k], bounds.get(k)) for k in keys
                                                if k in ages and k in groups]
        return lambda name, idx: by.get((name, idx), [])

    def _update_spx_demand(self, nodes: List[Dict[str, Any]], pending: List[Tuple[Dict[str, int], float]]) -> None:
        """EMA of whole-GPU demand: SPX partitions in use plus SPX pods waiting."""
        used = 0
        for n in nodes:
            status, _ = ann.parse_node_annotations(ko.annotations(n))
            used += sum(s.quantity for s in status if s.is_used() and s.profile.startswith("spx"))
        waiting = sum(q for req, _ in pending for p, q in req.items() if p.startswith("spx"))
        d = self.pack.reserve_decay
        self.spx_demand = d * self.spx_demand + (1 - d) * (used + waiting)

    # -- watch mapping ------------------------------------------------------------------
    @property
    def plan_key(self) -> Request:
        return Request(f"plan-{self.kind}", "")

    def map_pod(self, pod: Dict[str, Any]) -> List[Request]:
        """Every relevant pod event enqueues the same key, so a burst of pending pods is planned
        in one pass (the queue de-duplicates) instead of one full re-plan per pod."""
        if self.should_consider(pod) and requested_profiles(self.kind, pod):
            return [self.plan_key]
        return []

    # -- reconcile ----------------------------------------------------------------------
    def reconcile(self, req: Request) -> Result:
        """Plan for ``req``. A pass that wrote nothing is remembered with the API revision it read:
        while the revision is unchanged (no pod, node or annotation changed) the same request would
        plan on identical inputs and reach the same answer, so the requeues of a waiting plan key
        return that answer without re-planning. Only with a client that exposes ``revision`` (the
        in-memory API server) and without a batch window (whose deadline depends on the clock). The
        ``pack`` policy's starve/stint/drain rules depend on how long pods have waited and GPUs have
        held their mode, so its memo also keys on the clock in ``PackParams.replan_every`` buckets:
        an unchanged cluster is re-planned at most that often (thresholds are acted on at most one
        bucket late)."""
        rev = getattr(self.client, "revision", None) if self.batch_timeout <= 0 else None
        if rev is not None and self.policy == "pack":
            rev = (rev, int(self.clock() // max(1e-9, self.pack.replan_every))) if self.pack.replan_every > 0 else None
        if rev is not None:
            seen, results = self._idle
            if seen == rev and req in results:
                return results[req]
        res = self._reconcile(req)
        if rev is not None:
            after = getattr(self.client, "revision", None)
            if isinstance(rev, tuple):
                after = (after, rev[1])
            if after == rev:
                seen, results = self._idle
                if seen != rev:
                    results = {}
                    self._idle = (rev, results)
                results[req] = res
        return res

    def _reconcile(self, req: Request) -> Result:
        pending: Optional[List[Dict[str, int]]] = None
        if req == self.plan_key:
            pending = self.pending_pods()
            if not pending:
                return Result()
            requested = pending[0]
        else:
            try:
                pod = self.client.get("Pod", req.name, req.namespace)
            except NotFound:
                return Result()
            if not self.should_consider(pod):
                return Result()
            requested = requested_profiles(self.kind, pod)
            if not requested:
                return Result()
        now = self.clock()
        if self.batch_timeout > 0:
            if self._window_start is None:
                self._window_start = now
            self._window_last = now if self._window_last is None else self._window_last
            deadline = min(self._window_start + self.batch_timeout, self._window_last + max(self.batch_idle, 1e-9))
            if now < deadline:
                self._window_last = now
                return Result(requeue_after=deadline - now)
            self._window_start = self._window_last = None
        t0 = time.perf_counter()
        nodes = self.list_nodes()
        flying = [n for n in nodes if self.in_flight(n)]
        settled = [n for n in nodes if not self.in_flight(n)]
        models = self._models(settled)
        # free capacity = settled nodes' free partitions + what in-flight plans will provide
        free_total: Dict[str, int] = {}
        for m in models.values():
            for p, q in m.free().items():
                free_total[p] = free_total.get(p, 0) + q
        for n in flying:
            for p, q in self.incoming_free(n).items():
                free_total[p] = free_total.get(p, 0) + q
        if req != self.plan_key and all(free_total.get(p, 0) >= q for p, q in requested.items()):
            log.debug("pod %s/%s: requested profiles free (or incoming), nothing to do", req.namespace, req.name)
            if flying:
                return Result(requeue_after=self.retry_after)
            return Result()
        if self.policy == "pack":
            incoming = {}
            for n in flying:
                for p, q in self.incoming_free(n).items():
                    incoming[p] = incoming.get(p, 0) + q
            pend = self.pending_with_age()
            self._update_spx_demand(nodes, pend)
            pods_of = self._gpu_pods(nodes, now) \
                if any(getattr(m, "layout", "partitions") != "partitions" for m in models.values()) else None
            changed = plan_cluster_pack(models, pend or [(requested, 0.0)], incoming, self.pack, self.spx_demand,
                                        self._mode_ages(models, now), self._served(models, now),
                                        pods_of, self.lifetimes.model)
            need = requested
        elif self.policy in ("fifo", "simulate"):
            incoming: Dict[str, int] = {}
            for n in flying:
                for p, q in self.incoming_free(n).items():
                    incoming[p] = incoming.get(p, 0) + q
            planner = plan_cluster_fifo if self.policy == "fifo" else plan_cluster_simulate
            if pending is None:
                pending = self.pending_pods()
            changed = planner(models, pending or [requested], incoming)
            need = requested
        else:
            pending = self.pending_requests() or requested
            need = {p: q - free_total.get(p, 0) for p, q in pending.items() if q - free_total.get(p, 0) > 0}
            if not need:
                return Result()
            changed = plan_cluster(models, need)
        REGISTRY.phase_seconds.labels(phase="plan").observe(time.perf_counter() - t0)
        if self.kind == api.PARTITIONING_KIND_CUMASK and req == self.plan_key and not changed:
            self._explain_waits(models)   # a pass that could carve nothing: say why, once per pod
        if not changed:
            log.debug("%s: no node can provide %s now", req.name, need)
            return Result(requeue_after=self.retry_after)
        if self.kind == api.PARTITIONING_KIND_XCP and any(getattr(m, "sliced", False) for c in changed.values()
                                                          for m in c.gpus):
            self._explain_reservations(models, changed)
        by_name = {ko.name(n): n for n in nodes}
        for name, model in changed.items():
            plan_id = new_plan_id(self.clock)
            self.partitioner.apply_partitioning(by_name[name], plan_id,
                                                build_node_partitioning(model, getattr(model, "memory_target", None)))
            REGISTRY.repartitions.labels(node=name, kind=self.kind).inc()
            self.plans_written += 1
        return Result(requeue_after=self.retry_after) if req == self.plan_key else Result()
