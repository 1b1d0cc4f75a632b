"""The start gate (``deviceplugin/startgate.py``): memory-only slice containers of one GPU start one
after another through the slice plugin's ``PreStartContainer``."""
from __future__ import annotations

import threading
import time

from walkai_nos_amd.deviceplugin.startgate import StartGate, kfd_compute_queues, kfd_slice_ready, pids_with_slice


class FakeClock:
    def __init__(self):
        self.t = 0.0

    def __call__(self):
        return self.t

    def sleep(self, dt):
        self.t += dt


def test_each_start_waits_for_the_previous_containers_queues():
    clk = FakeClock()
    ready_at = {"s0": 3.0, "s1": 5.0}
    g = StartGate(ready=lambda s: clk.t >= ready_at.get(s, 1e9), timeout=20.0, poll=0.5, clock=clk, sleep=clk.sleep)
    assert g.enter(0, ["s0"]) == 0.0                      # the first passes at once
    assert g.enter(0, ["s1"]) == 3.0                      # s0's queues at t = 3
    assert g.enter(1, ["t0"]) == 0.0                      # another GPU: its own queue
    assert g.enter(0, ["s2"]) == 2.0                      # s1 ready at t = 5
    assert [s for _, s in g.order] == ["s0", "s1", "t0", "s2"] and g.timeouts == 0


def test_a_container_that_never_opens_the_gpu_holds_the_next_at_most_the_timeout():
    clk = FakeClock()
    g = StartGate(ready=lambda s: False, timeout=10.0, poll=1.0, clock=clk, sleep=clk.sleep)
    g.enter(0, ["dead"])
    assert g.enter(0, ["next"]) == 10.0 and g.timeouts == 1
    # a start long after the previous one (churn) does not wait at all
    clk.t += 600.0
    assert g.enter(0, ["later"]) == 0.0


def test_concurrent_starts_are_serialised_in_arrival_order():
    """Eight containers ask at once (kubelet starts a Deployment's pods concurrently); each becomes
    ready 50 ms after it was let through: the gate lets them through one at a time."""
    let = {}
    lock = threading.Lock()

    def ready(s):
        return s in let and time.monotonic() - let[s] >= 0.05

    g = StartGate(ready=ready, timeout=5.0, poll=0.005)
    orig = g.enter

    def enter(gpu, ids):
        w = orig(gpu, ids)
        with lock:
            let[ids[0]] = time.monotonic()
        return w

    threads = [threading.Thread(target=enter, args=(0, [f"s{i}"])) for i in range(8)]
    t0 = time.monotonic()
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    assert len(g.order) == 8 and g.timeouts == 0
    times = sorted(let.values())
    assert all(b - a >= 0.045 for a, b in zip(times, times[1:])), times
    assert time.monotonic() - t0 < 3.0


def test_kfd_probe_reads_compute_queues_and_slice_env(tmp_path):
    proc, kfd = tmp_path / "proc", tmp_path / "kfd"
    for pid, ids, queues in ((101, "bdf::s0", ["0", "0", "1"]), (102, "bdf::s1,bdf::s2", ["0", "1"]), (103, None, [])):
        (proc / str(pid)).mkdir(parents=True)
        env = b"PATH=/bin\0" + (f"NOS_SLICE_IDS={ids}".encode() + b"\0" if ids else b"")
        (proc / str(pid) / "environ").write_bytes(env)
        for i, t in enumerate(queues):
            q = kfd / str(pid) / "queues" / str(i)
            q.mkdir(parents=True)
            (q / "type").write_text(t + "\n")
    (proc / "self").mkdir()
    assert pids_with_slice("bdf::s0", str(proc)) == [101]
    assert pids_with_slice("bdf::s2", str(proc)) == [102]
    assert pids_with_slice("bdf::s9", str(proc)) == []
    assert kfd_compute_queues(101, str(kfd)) == 2 and kfd_compute_queues(102, str(kfd)) == 1
    assert kfd_slice_ready("bdf::s0", proc=str(proc), kfd=str(kfd))
    assert not kfd_slice_ready("bdf::s1", proc=str(proc), kfd=str(kfd))      # one compute queue so far
    assert kfd_slice_ready("bdf::s1", min_queues=1, proc=str(proc), kfd=str(kfd))


def test_slice_plugin_asks_for_prestart_and_gates_only_memory_only_slices():
    from walkai_nos_amd.device.protos import dp
    from walkai_nos_amd.device.slicing_client import MemorySliceStore
    from walkai_nos_amd.deviceplugin.server import SliceDevicePlugin
    from walkai_nos_amd.models.slicing.cumask import place
    slices = place([], [("bdf::m0", "16gb"), ("bdf::m1", "16gb"), ("bdf::d0", "32cu.36gb")], 256)
    store = MemorySliceStore()
    store.save({0: slices})
    seen = []
    gate = StartGate(ready=lambda s: True, timeout=1.0)
    gate.enter = lambda gpu, ids, bdf=None: seen.append((gpu, list(ids), bdf)) or 0.0
    shared = SliceDevicePlugin("amd.com/gpu-16gb", store, {0: "/dev/dri/renderD128"}, socket_dir="/tmp",
                               start_gate=gate)
    assert shared.GetDevicePluginOptions(None, None).pre_start_required
    assert not SliceDevicePlugin("amd.com/gpu-16gb", store, {}, socket_dir="/tmp").options().pre_start_required
    shared.PreStartContainer(dp.PreStartContainerRequest(devicesIDs=["bdf::m1"]), None)
    ded = SliceDevicePlugin("amd.com/gpu-32cu.36gb", store, {}, socket_dir="/tmp", start_gate=gate)
    ded.PreStartContainer(dp.PreStartContainerRequest(devicesIDs=["bdf::d0"]), None)
    assert seen == [(0, ["bdf::m1"], "bdf")]


def test_slice_agent_config_validates_the_gate():
    import pytest

    from walkai_nos_amd.api.config import GpuAgentConfig
    assert GpuAgentConfig().sharedSliceStartGateSeconds == 20.0
    with pytest.raises(ValueError):
        GpuAgentConfig(sharedSliceStartGateSeconds=45).validate()


def test_kfd_probe_without_a_shared_pid_namespace(tmp_path):
    """The agent's PIDs are not the KFD's (a PID namespace of its own): the previous container's
    process is the one on its GPU that reached its queues since it was let through."""
    from walkai_nos_amd.deviceplugin.startgate import KfdProbe, kfd_gpu_id
    kfd, topo, proc = tmp_path / "kfd", tmp_path / "topo", tmp_path / "proc"
    proc.mkdir()
    for node, (gid, loc) in enumerate((("0", 0), ("17010", (0x65 << 8)), ("9999", (0x75 << 8)))):
        d = topo / str(node)
        d.mkdir(parents=True)
        (d / "gpu_id").write_text(gid + "\n")
        (d / "properties").write_text(f"cpu_cores_count 0\nlocation_id {loc}\ndomain 0\n")
    assert kfd_gpu_id("0000:65:00.0", str(topo)) == "17010" and kfd_gpu_id("0000:99:00.0", str(topo)) is None

    def add(pid, gid, types):
        for i, t in enumerate(types):
            q = kfd / str(pid) / "queues" / str(i)
            q.mkdir(parents=True)
            (q / "type").write_text(t)
            (q / "gpuid").write_text(gid)
    add(500, "17010", ["0", "0", "1"])           # an older pod, ready
    p = KfdProbe(proc=str(proc), kfd=str(kfd), topology=str(topo))
    bdf = "0000:65:00.0"
    snap = p.snapshot(bdf)
    assert snap == {500}
    assert not p.ready("bdf::s1", bdf, snap)
    add(777, "9999", ["0", "0"])                 # another GPU's process: not ours
    assert not p.ready("bdf::s1", bdf, snap)
    add(600, "17010", ["0"])                     # ours, one queue so far
    assert not p.ready("bdf::s1", bdf, snap)
    add(601, "17010", ["0", "0"])
    assert p.ready("bdf::s1", bdf, snap)
