"""The ``pack`` policy's planning of sliced GPUs (SPX + CU-mask slices, ``models/xcp/slices.py``).

A sliced GPU changes its free slices without a drain or an amd-smi call, the way a MIG GPU
changes free instances (ref ``internal/controllers/migagent/actuator.go:225-229``), so it is
planned per *pod* rather than per mode:

1. **layout** (``xcp-layout`` label): on a ``slices`` node every idle hardware-partitioned GPU is
   turned into a sliced one (one flip to SPX, then never again); on an ``auto`` node an idle GPU
   whose waiting demand is one non-SPX profile filling at least a whole GPU gets that hardware mode
   (isolation for free when the demand is homogeneous), any other idle GPU is sliced, and a busy
   hardware GPU that blocks a pod waiting ``slice_reserve_after`` drains towards slices;
2. **backfill**: waiting pods, oldest first, are given a slice on the sliced GPU with the least room
   that still fits them (best fit keeps the big holes for big pods), re-carving free slices of
   other profiles as needed;
3. **reservation**: the oldest pod that fits nowhere, once it has waited ``slice_reserve_after``,
   drains the sliced GPU with the fewest groups in use for itself — its spec becomes the slices in
   use plus the pod's slice, which does not fit yet, so the partition plugin withholds every slice
   of that GPU (no new pod lands there) until enough of its pods have left; every pass recomputes
   it from what is in use, and the pod is placed as soon as it fits.  Without it a whole-GPU pod
   would wait behind an endless stream of smaller ones.  A drain withholds the GPU's slices in use
   too, and kube-scheduler still counts their pods' requests, so on a node of several GPUs it sees
   that many fewer free slices of those profiles elsewhere: a GPU only pods of the waiting pod's own
   profile fill is never reserved (nothing to gain), and the victim's hidden slices of profiles pods
   wait for count in its drain cost;
4. **fill**: the groups left over are carved into ``cpx_nps1`` slices, so small pods are scheduled
   without waiting for a planning pass.

Measured (``tools/planner_sweep.py``, ``profiles/planner_sweep_r4_slices.json``) against the
homogeneous pack planner on the same churn.
"""
from __future__ import annotations

from typing import Any, Callable, Dict, List, Mapping, Optional, Tuple

from ...models.xcp.slices import LAYOUT_AUTO, LAYOUT_PARTITIONS, SLICE_NPS, groups_of, is_slice_profile, new_sliced_gpu

Pending = List[Tuple[Dict[str, int], float]]


def _single(req: Mapping[str, int]) -> Optional[Tuple[str, int]]:
    if len(req) != 1:
        return None
    (p, q), = req.items()
    return (p, q) if q > 0 else None


def _spec(g: Any) -> Tuple[Dict[str, int], bool]:
    return dict(g.spec_geometry()), bool(g.spec_sliced())


def _hardware_gpu(g: Any, profile: str) -> Any:
    """An idle GPU re-modelled as a hardware partition of ``profile`` (every partition free)."""
    from ...models.xcp.node import new_gpu
    h = new_gpu(g.model, g.index, profile.split("_", 1)[1])
    h.apply_geometry({profile: round(8 / groups_of(profile))})
    return h


def plan_sliced(current: Dict[str, Any], original: Mapping[str, Any], changed: Dict[str, Any], unserved: Pending,
                params: Any, mode_age: Optional[Callable[[str, int], float]] = None,
                pods_of: Optional[Callable[[str, int], List[Tuple[int, float]]]] = None, life: Any = None,
                placed_on: Optional[Mapping[Tuple[str, int], float]] = None) -> None:
    """Layout choice, backfill, reservation and fill for the sliced GPUs of ``current`` (module
    docstring); places the pods it can (removing them from ``unserved``) and records the nodes
    whose spec changed in ``changed``. ``placed_on``: (node, GPU) -> age of the oldest pending pod
    the caller already gave a free slice there in this pass."""
    before = {n: [_spec(g) for g in m.gpus] for n, m in original.items()}

    def past_stint(name: str, idx: int) -> bool:
        return mode_age is None or params.min_stint <= 0 or mode_age(name, idx) >= params.min_stint

    # 1. layout
    demand: Dict[str, float] = {}
    for req, _ in unserved:
        s = _single(req)
        if s is not None:
            demand[s[0]] = demand.get(s[0], 0.0) + s[1] * groups_of(s[0]) / 8.0
    for name, m in sorted(current.items()):
        layout = getattr(m, "layout", LAYOUT_PARTITIONS)
        if layout == LAYOUT_PARTITIONS or (m.memory_partition or SLICE_NPS) != SLICE_NPS:
            continue
        for i, g in enumerate(m.gpus):
            if g.target is not None or not g.is_idle() or not past_stint(name, g.index):
                continue
            homogeneous = None
            if layout == LAYOUT_AUTO and len(demand) == 1:
                (p, d), = demand.items()
                if d >= 1.0 - 1e-9 and is_slice_profile(p) and groups_of(p) < 8:
                    homogeneous = p
            if homogeneous is not None:
                if g.sliced or g.geometry() != {homogeneous: round(8 / groups_of(homogeneous))}:
                    m.gpus[i] = _hardware_gpu(g, homogeneous)
            elif not g.sliced:
                m.gpus[i] = new_sliced_gpu(g.model, g.index)
    sliced = [(name, g) for name, m in sorted(current.items()) for g in m.gpus if g.sliced]
    # a reservation is recomputed every pass from the slices in use (the original model)
    used_now = {(name, g.index): dict(g.used) for name, m in original.items() for g in m.gpus}
    for _, g in sliced:
        if g.target is not None and g.target_sliced:
            g.target = None
    # thresholds: seconds until the planner has seen pods finish, then multiples of their median
    # run time (a cluster whose pods run for hours is not judged by a bench's minutes)
    learned = life is not None and life.ready()
    median = life.median() if learned else None
    reserve_after = params.slice_reserve_after
    overtake = params.slice_whole_overtake
    if learned and params.slice_reserve_lifetimes > 0:
        reserve_after = params.slice_reserve_lifetimes * median
    if learned and params.slice_whole_overtake_lifetimes > 0:
        overtake = params.slice_whole_overtake_lifetimes * median
    # under overload the reservation threshold stretches with the backlog (GPUs of waiting work per
    # sliced GPU): every drain idles groups, and when the queue is long anyway, draining for
    # whole-GPU pods less often serves more and shortens the waits behind them
    backlog = sum(groups_of(s[0]) * s[1] / 8.0 for s in (_single(r) for r, _ in unserved)
                  if s is not None and is_slice_profile(s[0])) / max(1, len(sliced))
    if params.slice_reserve_backlog > 0:
        reserve_after *= min(params.slice_reserve_stretch, max(1.0, backlog / params.slice_reserve_backlog))
    aged = learned and pods_of is not None
    waiting_profiles = {s[0] for s in (_single(r) for r, _ in unserved) if s is not None}
    sliced_on: Dict[str, List[Any]] = {}
    for name, g in sliced:
        sliced_on.setdefault(name, []).append(g)

    def drain_key(name: str, g: Any, need: int) -> float:
        """How much a drain of ``g`` for ``need`` groups idles: the expected idle group-seconds
        until its running pods free the room (their ages against the observed run times,
        ``lifetimes.drain_cost``), plus, on a node of several GPUs, ``slice_strand_weight`` x the
        groups in use of profiles pods wait for x the expected wait; else the groups in use."""
        if not aged:
            return float(g.used_groups())
        from .lifetimes import drain_cost
        cost, wait = drain_cost(pods_of(name, g.index), g.capacity, need, life, used=g.used_groups())
        if params.slice_strand_weight > 0 and len(sliced_on.get(name, ())) > 1:
            # the drain withholds its slices in use, and kube-scheduler stops seeing as many free
            # slices of their profiles on the node's other GPUs: groups of profiles pods wait for
            strand = sum(groups_of(p) * n for p, n in used_now.get((name, g.index), {}).items()
                         if n > 0 and p in waiting_profiles)
            cost += params.slice_strand_weight * strand * wait
        return cost

    # reservations in force: a sliced GPU whose spec asks for its slices in use plus one that does
    # not fit yet is draining for the biggest such slice, and keeps draining for a pod of that
    # profile until one is placed (re-deciding every pass against a threshold that moves with the
    # backlog let reservations lapse, and small pods refilled the GPU in between: the drain never
    # ended, and the groups its pods freed idled all along)
    held: Dict[Tuple[str, int], str] = {}
    if params.slice_reserve_hold and (params.slice_reserve_hold_max_gpus <= 0
                                      or len(sliced) <= params.slice_reserve_hold_max_gpus):
        for name, m in original.items():
            for og in m.gpus:
                if getattr(og, "sliced", False) and og.target is not None and og.target_sliced:
                    extra = [x for x, n in og.target.items() if n > og.used.get(x, 0) and is_slice_profile(x)]
                    if extra:
                        held[(name, og.index)] = max(extra, key=lambda x: (groups_of(x), x))
    by_key = {(name, g.index): g for name, g in sliced}
    name_of = {id(g): name for name, g in sliced}

    def futile(name: str, g: Any, p: str, q: int) -> bool:
        """A drain of ``g`` for one slice of ``p`` that only its own ``p`` pods block: the slices of
        ``p`` in use leave no room for another even once every other pod has left (a whole-GPU pod
        reserving a GPU another whole-GPU pod runs on). Such a drain idles nothing while they run
        and gains nothing when one ends (its free slice is what the pod needs, and kube-scheduler
        binds the oldest pod of ``p`` to it anyway), but the plugin withholds those slices in use,
        and kube-scheduler, which counts their requests against a node allocatable without them,
        stops seeing the free ``p`` slices of the node's other GPUs for as long as it lasts. A pod
        of several slices does need the drain: one freed slice would go to a one-slice pod."""
        return q == 1 and groups_of(p) * (used_now.get((name, g.index), {}).get(p, 0) + 1) > g.capacity

    def reserve(name: str, g: Any, p: str, q: int) -> None:
        """Drain ``g`` for ``q`` slices of ``p``: its spec becomes the slices in use plus those."""
        want = {k: v for k, v in used_now.get((name, g.index), {}).items() if v > 0}
        want[p] = want.get(p, 0) + q
        g.used = {k: v for k, v in used_now.get((name, g.index), {}).items() if v > 0}
        g.free = {}
        g.target, g.target_sliced = want, True

    def place(g: Any, p: str, q: int, age: Optional[float] = None) -> None:
        for _ in range(q):
            g.claim(p)
        key = (name_of[id(g)], g.index)
        claimed[key] = max(claimed.get(key, 0.0), float("inf") if age is None else age)

    # GPUs that took a pod in this pass -> the oldest such pod's wait: a free slice the caller gave
    # a pending pod, or a backfill below. A drain withholds the GPU and strands those pods, so only
    # an overdue reservation of a pod older than all of them may take such a GPU
    claimed: Dict[Tuple[str, int], float] = dict(placed_on or {})
    # 2a. whole-GPU runs: a sliced GPU a whole-GPU pod just left (its one free slice is the whole
    # GPU) goes to the next waiting whole-GPU pod unless the oldest waiting pod is more than
    # ``overtake`` older. Handing it to smaller pods instead means draining it again for the next
    # whole-GPU pod, and every such drain idles most of the GPU for a good part of a pod lifetime
    if overtake > 0 and unserved:
        oldest = max(age for _, age in unserved)
        for name, g in sliced:
            free = [(p, n) for p, n in g.free.items() if n > 0]
            if g.target is not None or not g.is_idle() or len(free) != 1 or free[0][1] != 1 \
                    or groups_of(free[0][0]) != g.capacity:
                continue
            nxt = next(((req, age) for req, age in unserved if _single(req) == (free[0][0], 1)), None)
            if nxt is not None and nxt[1] >= oldest - overtake:
                place(g, free[0][0], 1, nxt[1])
                unserved.remove(nxt)
    # 2b./3. backfill and reservation, oldest first
    reserved = False
    waiting: Pending = []   # pods that fit nowhere and reserved nothing, oldest first
    for req, age in list(unserved):
        s = _single(req)
        if s is None or not is_slice_profile(s[0]):
            continue
        p, q = s
        need = q * groups_of(p)
        if need > 8:
            continue
        cands = [(bool(g.degraded), g.room(), name, g.index, g) for name, g in sliced
                 if g.target is None and g.room() >= need]
        if cands:
            place(min(cands, key=lambda c: c[:4])[-1], p, q, age)
            unserved.remove((req, age))
            continue
        hk = next((k for k in sorted(held) if held[k] == p and claimed.get(k, -1.0) < age and by_key.get(k) is not None
                   and by_key[k].target is None and not futile(k[0], by_key[k], p, q)), None)
        if hk is not None:
            reserve(hk[0], by_key[hk], p, q)
            continue
        if reserved or params.slice_reserve_after <= 0 or age < reserve_after:
            waiting.append((req, age))
            continue
        victims = [(bool(g.degraded), drain_key(name, g, need), name, g.index, g) for name, g in sliced
                   if g.target is None and claimed.get((name, g.index), -1.0) < age and not futile(name, g, p, q)]
        if not victims and any(g.target is None for _, g in sliced):
            waiting.append((req, age))
            continue  # every sliced GPU just took an older pod: reconsider on the next pass
        if not victims:
            # an auto node's busy hardware GPU in another mode drains towards slices for the pod
            hw = [(sum(g.used.values()), name, g.index, g) for name, m in sorted(current.items())
                  if getattr(m, "layout", LAYOUT_PARTITIONS) == LAYOUT_AUTO
                  for g in m.gpus if not g.sliced and g.target is None and not g.is_idle()
                  and past_stint(name, g.index)]
            if hw:
                _, name, _, g = min(hw, key=lambda c: c[:3])
                g.target, g.target_sliced = {p: q}, True
                reserved = True
            continue
        *_, g = min(victims, key=lambda c: c[:4])
        reserve(name_of[id(g)], g, p, q)
        reserved = True
    # 3b. a free drain: after the backfill every pod that still waits is bigger than the unused room
    # of every GPU not draining, so that room idles whatever the planner does; the oldest waiting
    # pod reserves the GPU with the most of it. Where reservations are held (clusters of at most
    # ``slice_reserve_hold_max_gpus`` sliced GPUs) it is held like any other until a pod of its
    # profile is placed — a smaller pod that arrives meanwhile waits; with more GPUs it is re-decided
    # every pass and lapses once a smaller pod arrives that the room fits. Measured (8 seeds x 200
    # quanta, load 1.0): letting free drains lapse on 1-2 GPUs too cost 1.5 points of allocation on
    # two GPUs (95.3 -> 93.9%) and raised the worst p99 wait (7.0 -> 8.8 lifetimes)
    if params.slice_free_drain:
        draining = {max((x for x, n in g.target.items() if n > g.used.get(x, 0)), key=groups_of, default=None)
                    for _, g in sliced if g.target is not None}
        # with more GPUs one empties on its own sooner: the wait before a free drain scales with them
        per = params.slice_free_drain_after * max(0, len(sliced) - 1)
        if params.slice_free_drain_cap > 0:
            per = min(per, params.slice_free_drain_cap)
        free_after = per * (median if learned else 240.0)
        for req, age in waiting:
            p, q = _single(req)
            if p in draining or age < free_after:
                continue          # one GPU at a time drains for a profile: the others keep serving
            need = q * groups_of(p)
            idle = [(-g.room(), g.used_groups(), name, g.index, g) for name, g in sliced
                    if g.target is None and (name, g.index) not in claimed and 0 < g.room() < need]
            if not idle:
                break
            g = min(idle, key=lambda c: c[:4])[-1]
            reserve(name_of[id(g)], g, p, q)
            draining.add(p)
    # 4. fill
    if params.slice_fill:
        for _, g in sliced:
            if g.target is None:
                g.fill()
    for name, m in current.items():
        if name in before and [_spec(g) for g in m.gpus] != before[name]:
            changed[name] = m

