"""Uneven memory-only slice counts after departures: a Node event and a gauge
(controllers/sliceagent/balance.py; VERDICT r5 #2, the churn case)."""
from __future__ import annotations

from walkai_nos_amd.controllers.sliceagent.balance import SharedBalance, node_event, shared_in_use
from walkai_nos_amd.models.slicing.cumask import Slice
from walkai_nos_amd.utils.metrics import REGISTRY


def _slices(n_shared: int, n_dedicated: int = 0, gpu: int = 0):
    ss = [Slice(f"0000:a4:00.0::s{i}", "16gb") for i in range(n_shared)]
    ss += [Slice(f"0000:a4:00.0::d{i}", "32cu.24gb", rows=[i]) for i in range(n_dedicated)]
    return {gpu: ss}


def _gauge(node: str, gpu: int) -> float:
    return REGISTRY.registry.get_sample_value("nos_shared_slices_uneven", {"node": node, "gpu": str(gpu)})


def test_counts_only_memory_only_slices_in_use():
    s = _slices(8, 2)
    used = {x.id for x in s[0][:5]} | {s[0][-1].id}
    assert shared_in_use(s, used) == {0: 5}


def test_departures_to_an_odd_count_are_reported_once_and_cleared_when_even():
    slices = _slices(8, 1)
    ids = [x.id for x in slices[0][:8]]
    used = set(ids)
    events = []
    b = SharedBalance("n1", lambda: slices, lambda: used, lambda r, k, m: events.append((r, k, m)))
    assert b.check() == {}                          # 8 running: even, nothing to say
    assert _gauge("n1", 0) == 0
    used -= set(ids[:3])                            # 3 of 8 leave: 5 run, two rate classes
    assert b.check() == {0: 5}
    assert _gauge("n1", 0) == 1
    assert [(r, k) for r, k, _ in events] == [("SharedSlicesUneven", "Warning")]
    assert "5 memory-only" in events[0][2]
    b.check()                                       # still 5: no second event
    assert len(events) == 1
    used.add(ids[0])                                # a start makes it 6
    assert b.check() == {}
    assert _gauge("n1", 0) == 0
    assert [r for r, _, _ in events] == ["SharedSlicesUneven", "SharedSlicesEven"]
    used -= {ids[3], ids[4]}                        # 6 - 2 = 4: even, nothing new
    assert len(used) == 4 and b.check() == {} and len(events) == 2
    used |= {ids[1], ids[2], ids[3]}                # 4 + 3 = 7: uneven at a new count
    assert b.check() == {0: 7}
    assert events[-1][0] == "SharedSlicesUneven" and "7 memory-only" in events[-1][2]


def test_skip_counts_follow_the_configuration():
    slices = _slices(8)
    used = {x.id for x in slices[0][:6]}
    b = SharedBalance("n2", lambda: slices, lambda: used, None, skip_counts=[6])
    assert b.check() == {0: 6}


def test_node_event_shape_and_reporter_wiring():
    created = []

    class Client:
        def create(self, obj):
            created.append(obj)

    node_event(Client(), "n3")("SharedSlicesUneven", "Warning", "msg")
    ev = created[0]
    assert ev["kind"] == "Event" and ev["involvedObject"] == {"apiVersion": "v1", "kind": "Node", "name": "n3"}
    assert ev["reason"] == "SharedSlicesUneven" and ev["type"] == "Warning"

    # the slice agent's reporter runs the check after every report
    from walkai_nos_amd.controllers.sliceagent.agent import setup_slice_agent
    from walkai_nos_amd.kube.memory import InMemoryAPIServer
    from walkai_nos_amd.kube.runtime import Manager

    class Store:
        def load(self):
            return {}

    class SC:
        def used_ids(self):
            return set()

    mgr = Manager(InMemoryAPIServer())
    _, reporter, _ = setup_slice_agent(mgr, "n3", SC(), Store())
    assert reporter.observers == [reporter.balance.check]
    assert reporter.balance.check() == {}


def test_released_slices_are_forgotten_by_the_start_gate():
    # a memory-only pod that left no longer holds the next start on its GPU back
    from walkai_nos_amd.deviceplugin.startgate import StartGate

    slices = _slices(3)
    ids = [x.id for x in slices[0]]
    used = set(ids)
    gate = StartGate(ready=lambda sid: False, timeout=20.0, clock=lambda: 0.0, sleep=lambda s: None)
    gate.enter(0, [ids[2]])                         # ids[2] let through last, never ready
    b = SharedBalance("n4", lambda: slices, lambda: used, None, on_release=gate.forget)
    b.check()
    assert gate._last[0][0] == ids[2]
    used.discard(ids[2])                            # its pod left
    b.check()
    assert 0 not in gate._last                      # the next start on GPU 0 does not wait for it
