"""In-memory API server and controller runtime semantics (the envtest substitute)."""
import threading

import pytest

from walkai_nos_amd.kube import objects as ko
from walkai_nos_amd.kube.errors import AlreadyExists, Conflict, NotFound
from walkai_nos_amd.kube.memory import InMemoryAPIServer, create_merge_patch, merge_patch
from walkai_nos_amd.kube.quantity import format_quantity, parse_quantity, quantity_milli, quantity_value
from walkai_nos_amd.kube.runtime import (FuncPredicate, Manager, Request, Result, SimClock, Watch, WorkQueue,
                                         run_until_idle)


def test_crud_resource_version_and_conflict():
    a = InMemoryAPIServer()
    n = a.create(ko.new_node("n1", {"x": "1"}))
    assert n["metadata"]["resourceVersion"] == "1" and n["metadata"]["uid"]
    with pytest.raises(AlreadyExists):
        a.create(ko.new_node("n1"))
    stale = a.get("Node", "n1")
    a.patch("Node", "n1", {"metadata": {"labels": {"y": "2"}}})
    stale["metadata"]["labels"]["z"] = "3"
    with pytest.raises(Conflict):
        a.update(stale)
    fresh = a.get("Node", "n1")
    fresh["metadata"]["labels"]["z"] = "3"
    out = a.update(fresh)
    assert out["metadata"]["labels"] == {"x": "1", "y": "2", "z": "3"}
    a.delete("Node", "n1")
    with pytest.raises(NotFound):
        a.get("Node", "n1")


def test_noop_patch_does_not_bump_or_emit():
    a = InMemoryAPIServer()
    a.create(ko.new_node("n"))
    events = []
    a.watch("Node", lambda e, o, old: events.append(e), replay=False)
    a.patch("Node", "n", {"metadata": {"annotations": {"k": "v"}}})
    rv = a.get("Node", "n")["metadata"]["resourceVersion"]
    a.patch("Node", "n", {"metadata": {"annotations": {"k": "v"}}})
    assert a.get("Node", "n")["metadata"]["resourceVersion"] == rv
    assert events == ["MODIFIED"]


def test_merge_patch_rfc7386():
    assert merge_patch({"a": {"b": 1, "c": 2}}, {"a": {"b": None, "d": 3}}) == {"a": {"c": 2, "d": 3}}
    orig = {"metadata": {"annotations": {"a": "1", "b": "2"}}}
    mod = {"metadata": {"annotations": {"b": "3", "c": "4"}}}
    p = create_merge_patch(orig, mod)
    assert p == {"metadata": {"annotations": {"a": None, "b": "3", "c": "4"}}}
    assert merge_patch(orig, p) == mod


def test_selectors_and_namespaces():
    a = InMemoryAPIServer()
    a.create(ko.new_pod("p1", "ns1", labels_={"app": "x"}, node_name="n1"))
    a.create(ko.new_pod("p2", "ns2", labels_={"app": "y"}, node_name="n2"))
    a.create(ko.new_pod("p3", "ns1", labels_={"app": "x"}, node_name="n2", phase="Running"))
    assert [ko.name(p) for p in a.list("Pod", label_selector="app=x")] == ["p1", "p3"]
    assert [ko.name(p) for p in a.list("Pod", namespace="ns2")] == ["p2"]
    assert sorted(ko.name(p) for p in a.list("Pod", field_selector="spec.nodeName=n2")) == ["p2", "p3"]
    assert [ko.name(p) for p in a.list("Pod", field_selector="status.phase=Running")] == ["p3"]
    assert [ko.name(p) for p in a.list("Pod", label_selector="app!=x")] == ["p2"]
    assert sorted(ko.name(p) for p in a.list("Pod", label_selector="app")) == ["p1", "p2", "p3"]


def test_bind_subresource():
    a = InMemoryAPIServer()
    a.create(ko.new_pod("p", "default"))
    a.bind("p", "default", "node-a")
    p = a.get("Pod", "p", "default")
    assert p["spec"]["nodeName"] == "node-a"
    assert ko.get_condition(p, "PodScheduled")["status"] == "True"
    with pytest.raises(Conflict):
        a.bind("p", "default", "node-b")


def test_quantities():
    assert quantity_value("16Gi") == 16 * 2**30
    assert quantity_milli("500m") == 500 and quantity_milli("2") == 2000
    assert quantity_value("1") == 1 and quantity_value("1.5") == 2
    assert parse_quantity("1k") == 1000
    assert format_quantity(3) == "3"
    with pytest.raises(ValueError):
        parse_quantity("abc")


def test_workqueue_dedup_delay_and_backoff():
    clock = SimClock(0)
    q = WorkQueue(clock)
    r = Request("a")
    q.add(r)
    q.add(r)
    assert len(q) == 1
    got = q.get_nowait()
    assert got == r
    q.add(r)  # added while processing -> dirty, re-queued on done
    assert q.get_nowait() is None
    q.done(r)
    assert q.get_nowait() == r
    q.done(r)
    q.add_after(r, 5)
    assert q.get_nowait() is None
    clock.advance(5)
    assert q.get_nowait() == r
    q.done(r)
    q.add_rate_limited(r)
    q.add_rate_limited(r)
    assert q.next_due() == pytest.approx(5 + 0.005)  # first failure waits the base delay, the second 2x
    q.forget(r)


def test_controller_predicates_requeue_and_errors():
    clock = SimClock(100)
    a = InMemoryAPIServer(clock=clock)
    calls = []

    def reconcile(req):
        calls.append((clock(), req.name))
        if len(calls) == 1:
            raise RuntimeError("transient")
        if len(calls) == 2:
            return Result(requeue_after=10)
        return Result()

    m = Manager(a, clock=clock)
    only_x = FuncPredicate(create=lambda o: ko.name(o).startswith("x"),
                           update=lambda o, n: ko.name(n).startswith("x"))
    m.new_controller("c", reconcile, [Watch("Node", [only_x])])
    a.create(ko.new_node("x1"))
    a.create(ko.new_node("y1"))
    run_until_idle([m], clock, horizon=60)
    names = [n for _, n in calls]
    assert names == ["x1", "x1", "x1"]  # error -> back-off retry -> requeue_after -> done
    assert calls[2][0] - calls[1][0] == pytest.approx(10)


def test_threaded_manager_runs_workers():
    a = InMemoryAPIServer()
    seen = []
    done = threading.Event()

    def reconcile(req):
        seen.append(req.name)
        if len(seen) >= 3:
            done.set()
        return Result()

    m = Manager(a)
    m.new_controller("c", reconcile, [Watch("Node")], max_concurrent_reconciles=2)
    m.start()
    try:
        for i in range(3):
            a.create(ko.new_node(f"n{i}"))
        assert done.wait(5)
    finally:
        m.stop()
    assert sorted(seen) == ["n0", "n1", "n2"]
    assert m.healthy() and m.ready()
