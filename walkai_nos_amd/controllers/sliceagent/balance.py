"""Uneven memory-only slices after departures: reported with a Node event and a metric.

Memory-only slices share every CU, and the command processor deals each process's compute queues
over the hardware pipes in creation order: at 5 or 7 running pods on one GPU they split into two
rate classes by start parity (``models/slicing/profile.py`` ``SKIP_SHARED_COUNTS``,
``profiles/fair_probe_r5.json``). The planner never *starts* a GPU's 5th or 7th memory-only pod,
and the start gate (``deviceplugin/startgate.py``) orders the starts it lets through — but a
departure from 6 or 8 leaves 5 or 7 running, in two classes, until the next start makes the count
even again (``tests/test_gpu_native.py`` churn test: 3 of 8 replaced, max/min 1.028 once refilled).
Nothing on the node can move a running process's queues, so that state is reported, not hidden:
per GPU, the gauge ``nos_shared_slices_uneven`` is 1 while the count of memory-only slices in use is
one of the skipped counts, and each transition into it records a ``SharedSlicesUneven`` Warning
event on the Node (back to even: a ``SharedSlicesEven`` Normal event). The slice agent's reporter
runs the check on every report (``refresh_interval``), and hands every memory-only slice whose pod
left to ``on_release`` — the start gate's ``forget``, so a container that left (or never reached the
GPU) holds no later start back.
"""
from __future__ import annotations

import logging
from typing import Any, Callable, Dict, Iterable, Optional

from ...models.slicing.profile import SKIP_SHARED_COUNTS, parse_profile

log = logging.getLogger("nos.sliceagent.balance")

_gauge = None


def _metric():
    global _gauge
    if _gauge is None:
        from prometheus_client import Gauge

        from ...utils.metrics import REGISTRY
        _gauge = Gauge("nos_shared_slices_uneven",
                       "1 while a GPU runs a count of memory-only slice pods that splits them into two rate classes",
                       ["node", "gpu"], registry=REGISTRY.registry)
    return _gauge


def shared_in_use(slices: Dict[int, Iterable[Any]], used_ids: set) -> Dict[int, int]:
    """Per GPU, the memory-only slices (no dedicated CUs) whose device kubelet has allocated."""
    out: Dict[int, int] = {}
    for g, ss in slices.items():
        out[g] = sum(1 for s in ss if s.id in used_ids and not parse_profile(s.profile).dedicated)
    return out


class SharedBalance:
    """Watches the memory-only slice counts of one node's GPUs (module docstring)."""

    def __init__(self, node: str, load_slices: Callable[[], Dict[int, Iterable[Any]]],
                 used_ids: Callable[[], set], event: Optional[Callable[[str, str, str], None]] = None,
                 skip_counts: Iterable[int] = SKIP_SHARED_COUNTS, on_release: Optional[Callable[[str], None]] = None):
        self.node = node
        self.load_slices = load_slices
        self.used_ids = used_ids
        self.event = event
        self.skip = frozenset(int(n) for n in skip_counts)
        self.on_release = on_release
        self.uneven: Dict[int, int] = {}   # GPU -> the uneven count it was last seen at
        self.in_use: set = set()           # memory-only slice ids in use at the last check

    def check(self) -> Dict[int, int]:
        """Update the gauge and record transitions; returns GPU -> uneven count now."""
        slices, used = self.load_slices(), self.used_ids()
        shared_now = {s.id for ss in slices.values() for s in ss if s.id in used and not parse_profile(s.profile).dedicated}
        if self.on_release is not None:
            for sid in sorted(self.in_use - shared_now):
                self.on_release(sid)
        self.in_use = shared_now
        counts = shared_in_use(slices, used)
        now = {g: n for g, n in counts.items() if n in self.skip}
        g_ = _metric()
        for g in counts:
            g_.labels(node=self.node, gpu=str(g)).set(1 if g in now else 0)
        for g, n in sorted(now.items()):
            if self.uneven.get(g) != n:
                self._emit("SharedSlicesUneven", "Warning",
                           f"GPU {g} runs {n} memory-only slice pods: an odd count from 5 splits them into two "
                           f"rate classes by start order until the next start or stop makes it even")
        for g in sorted(set(self.uneven) - set(now)):
            self._emit("SharedSlicesEven", "Normal",
                       f"GPU {g} runs {counts.get(g, 0)} memory-only slice pods: the compute share is even again")
        self.uneven = now
        return now

    def _emit(self, reason: str, kind: str, message: str) -> None:
        log.info("%s: %s", reason, message)
        if self.event is None:
            return
        try:
            self.event(reason, kind, message)
        except Exception as e:  # noqa: BLE001 - the metric carries it; the event is a courtesy
            log.warning("event %s not recorded: %s", reason, e)


def node_event(client: Any, node: str) -> Callable[[str, str, str], None]:
    """Records an event on the Node (``source.component`` nos-sliceagent)."""
    def f(reason: str, kind: str, message: str) -> None:
        client.create({
            "apiVersion": "v1", "kind": "Event",
            "metadata": {"generateName": f"{node}.", "namespace": "default"},
            "involvedObject": {"apiVersion": "v1", "kind": "Node", "name": node},
            "reason": reason, "message": message, "type": kind,
            "source": {"component": "nos-sliceagent", "host": node}})
    return f
