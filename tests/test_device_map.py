"""Physical-GPU <-> logical-partition map, re-enumeration after flips, the busy check, the
journal/start-up reconciliation and the agent's GPU-context hygiene.

These pin the MI355X partition semantics the reference gets for free from NVML re-initialising
around every call (ref pkg/gpu/nvml/client.go:46-57): after SPX -> CPX every GPU is eight logical
devices with new ids, and nothing may resolve against the old layout.
"""
import json
import os
import subprocess
import sys

import pytest

from walkai_nos_amd.api import v1alpha1 as api
from walkai_nos_amd.controllers.agent.actuator import Actuator
from walkai_nos_amd.controllers.agent.reporter import Reporter
from walkai_nos_amd.controllers.agent.shared import SharedState
from walkai_nos_amd.device.amdsmi import FakeAmdSmi
from walkai_nos_amd.device.partition_client import PartitionClient
from walkai_nos_amd.device.podresources import StaticResourceClient
from walkai_nos_amd.device.topology import ProcInfo, build_device_map
from walkai_nos_amd.kube import objects as ko
from walkai_nos_amd.kube.memory import InMemoryAPIServer
from walkai_nos_amd.kube.runtime import Request
from walkai_nos_amd.models.errors import GpuError
from walkai_nos_amd.parallel.barrier import LocalBarrier

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_cpx_flip_reenumerates_eight_logical_devices_per_gpu():
    smi = FakeAmdSmi(n_gpus=8)
    m0 = smi.device_map()
    assert len(m0.devices) == 8 and [g.index for g in m0.gpus] == list(range(8))
    old_ids = [d.device_id for d in m0.devices]
    for g in range(8):
        smi.set_compute_partition(g, "CPX")
    m = smi.device_map()
    assert m.generation > m0.generation
    assert len(m.devices) == 64 and len(m.hip_ids()) == 64 and m.hip_ids() == list(range(64))
    for g in range(8):
        parts = m.partitions_of(g)
        assert [d.partition_index for d in parts] == list(range(8))
        assert all(d.bdf == m.gpus[g].bdf and d.cu_count == 32 for d in parts)
        assert m.gpus[g].cu_count == 256 and m.gpus[g].vram_bytes == 288 * 10**9
    # every id form resolves to (gpu, partition); partition ids of the SPX layout are gone except
    # partition 0 (the GPU itself), whose physical GPU is unchanged
    for d in m.devices:
        for a in d.aliases():
            r = smi.resolve(a)
            assert (r.gpu_index, r.partition_index) == (d.gpu_index, d.partition_index)
    assert smi.resolve(f"{m.gpus[3].bdf}::s7").gpu_index == 3  # CU-mask slice id on a GPU
    new_ids = {d.device_id for d in m.devices}
    assert set(old_ids) <= new_ids  # partition 0 keeps the GPU's UUID
    with pytest.raises(GpuError) as e:
        smi.resolve("GPU-fake-0000-cpx9")
    assert e.value.is_not_found()
    # back to SPX: the CPX partition ids stop resolving
    cpx_ids = [d.device_id for d in m.partitions_of(5)[1:]]
    smi.set_compute_partition(5, "SPX")
    smi.miss_rescan_interval = 0.0
    for i in cpx_ids:
        with pytest.raises(GpuError):
            smi.resolve(i)
    assert len(smi.device_map().devices) == 57


def test_partition_client_reports_cpx_per_partition_devices():
    smi = FakeAmdSmi(n_gpus=2)
    alloc = lambda: [(f"amd.com/{d.compute_mode.lower()}_{d.memory_mode.lower()}", d.device_id)  # noqa: E731
                     for d in smi.logical_devices()]
    pc = PartitionClient(StaticResourceClient(lambda: [], alloc), smi)
    pc.set_profile(1, "cpx_nps1")
    assert pc.current_profiles() == {0: "spx_nps1", 1: "cpx_nps1"}
    devs = pc.get_partition_devices()
    by_gpu = devs.group_by_gpu_index()
    assert len(by_gpu[1]) == 8 and len(by_gpu[0]) == 1


def test_build_device_map_groups_processors_by_bdf_and_partition_id():
    # processors listed out of order, partition id only in the KFD location bits for one GPU
    procs = [ProcInfo(0, "u-b1", "0000:15:00.0", bdf_id=(1 << 28), hip_id=3),
             ProcInfo(1, "u-a0", "0000:05:00.0", partition_id=0, hip_id=0),
             ProcInfo(2, "u-b0", "0000:15:00.0", bdf_id=0, hip_id=2),
             ProcInfo(3, "u-a1", "0000:05:00.0", partition_id=1, hip_id=1)]
    m = build_device_map(procs, lambda p: "dpx", lambda p: "nps1")
    assert [(d.gpu_index, d.partition_index, d.uuid) for d in m.devices] == \
        [(0, 0, "u-a0"), (0, 1, "u-a1"), (1, 0, "u-b0"), (1, 1, "u-b1")]
    assert m.modes() == {0: "dpx_nps1", 1: "dpx_nps1"}
    assert m.resolve("0000:15:00.0").uuid == "u-b0"


class Env:
    def __init__(self, n_gpus=2, barrier=None):
        self.api = InMemoryAPIServer()
        self.api.create(ko.new_node("node-a"))
        self.smi = FakeAmdSmi(n_gpus=n_gpus)
        self.used = []
        self.pc = PartitionClient(StaticResourceClient(lambda: list(self.used), self.alloc), self.smi)
        self.shared = SharedState()
        self.sizes = []

        def factory(n):
            self.sizes.append(n)
            return barrier if barrier is not None else LocalBarrier(n)
        self.actuator = Actuator(self.api, self.pc, self.shared, "node-a", barrier_factory=factory)
        self.reporter = Reporter(self.api, self.pc, self.shared, refresh_interval=10)

    def alloc(self):
        return [(f"amd.com/{d.compute_mode.lower()}_{d.memory_mode.lower()}", d.device_id)
                for d in self.smi.logical_devices()]

    def spec(self, anns):
        self.api.patch("Node", "node-a", {"metadata": {"annotations": anns}})

    def annotations(self):
        return ko.annotations(self.api.get("Node", "node-a"))


def test_commit_barrier_spans_every_logical_device_of_the_node():
    e = Env(n_gpus=8)
    spec = {f"nos.nebuly.com/spec-gpu-{g}-cpx_nps1": "8" for g in range(8)}
    spec[api.ANNOTATION_PARTITIONING_PLAN] = "7"
    e.spec(spec)
    e.reporter.reconcile(Request("node-a"))
    e.actuator.reconcile(Request("node-a"))
    assert e.sizes == [64] and len(e.actuator.last_votes) == 64 and all(e.actuator.last_votes)
    e.reporter.reconcile(Request("node-a"))
    a = e.annotations()
    assert all(a[f"nos.nebuly.com/status-gpu-{g}-cpx_nps1-free"] == "8" for g in range(8))
    assert api.ANNOTATION_INFLIGHT_PLAN not in a  # journal cleared after the commit


def test_flip_is_refused_while_a_process_holds_the_gpu():
    e = Env(n_gpus=2)
    e.smi.set_processes(0, 1, partition=0)  # e.g. a pod outside kubelet's accounting
    e.spec({"nos.nebuly.com/spec-gpu-0-cpx_nps1": "8", "nos.nebuly.com/spec-gpu-1-cpx_nps1": "8",
            api.ANNOTATION_PARTITIONING_PLAN: "1"})
    e.reporter.reconcile(Request("node-a"))
    with pytest.raises(GpuError) as err:
        e.actuator.reconcile(Request("node-a"))
    assert err.value.code == GpuError.BUSY
    # GPU 1 was idle and got flipped; GPU 0 was never touched
    assert e.smi.get_compute_partition(0) == "SPX" and e.smi.get_compute_partition(1) == "CPX"
    assert [c for c in e.smi.set_calls if c[1] == 0] == []
    e.smi.set_processes(0, 0)
    e.reporter.reconcile(Request("node-a"))
    e.actuator.reconcile(Request("node-a"))  # retried once the GPU is idle
    assert e.smi.get_compute_partition(0) == "CPX"


def test_actuator_stops_gpu_helpers_before_flipping():
    e = Env(n_gpus=1)
    p = subprocess.Popen([sys.executable, "-c", "import time; time.sleep(60)"])
    e.shared.helpers.add(p)
    e.spec({"nos.nebuly.com/spec-gpu-0-cpx_nps1": "8", api.ANNOTATION_PARTITIONING_PLAN: "1"})
    e.reporter.reconcile(Request("node-a"))
    e.actuator.reconcile(Request("node-a"))
    assert p.poll() is not None and e.smi.get_compute_partition(0) == "CPX"


def test_no_helper_starts_while_a_flip_holds_the_gate():
    import threading
    import time
    from walkai_nos_amd.parallel.spawned import HelperRegistry
    reg = HelperRegistry()
    started = []

    def spawn():
        p = reg.spawn([sys.executable, "-c", "pass"], timeout=10.0)
        started.append(time.monotonic())
        p.wait()
    with reg.held():
        t = threading.Thread(target=spawn)
        t.start()
        time.sleep(0.3)
        assert not started  # held back while the flip runs
        released = time.monotonic()
    t.join(10)
    assert started and started[0] >= released
    with reg.held():
        with pytest.raises(TimeoutError):
            reg.spawn([sys.executable, "-c", "pass"], timeout=0.1)


def test_actuator_holds_helpers_back_during_the_switch():
    e = Env(n_gpus=1)
    seen = []
    real = e.smi.set_compute_partition

    def switch(gpu, mode):
        seen.append(e.shared.helpers._held)
        return real(gpu, mode)
    e.smi.set_compute_partition = switch
    e.spec({"nos.nebuly.com/spec-gpu-0-cpx_nps1": "8", api.ANNOTATION_PARTITIONING_PLAN: "1"})
    e.reporter.reconcile(Request("node-a"))
    e.actuator.reconcile(Request("node-a"))
    assert seen == [1] and e.shared.helpers._held == 0


def test_veto_from_a_missing_partition_rolls_back():
    e = Env(n_gpus=2)

    def verify(g, p):
        return False  # e.g. a partition that did not come up
    e.actuator.verify = verify
    e.spec({"nos.nebuly.com/spec-gpu-1-qpx_nps1": "4", api.ANNOTATION_PARTITIONING_PLAN: "3"})
    e.reporter.reconcile(Request("node-a"))
    with pytest.raises(GpuError):
        e.actuator.reconcile(Request("node-a"))
    assert e.smi.get_compute_partition(1) == "SPX"
    assert e.actuator.last_votes.count(False) == 4  # the four partitions of the flipped GPU
    assert e.shared.last_commit == "failed"


def test_startup_rolls_forward_a_plan_journalled_before_a_crash():
    e = Env(n_gpus=2)
    # the previous agent journalled plan 9 (both GPUs -> CPX), flipped GPU 0 and died
    e.spec({"nos.nebuly.com/spec-gpu-0-cpx_nps1": "8", "nos.nebuly.com/spec-gpu-1-cpx_nps1": "8",
            api.ANNOTATION_PARTITIONING_PLAN: "9",
            api.ANNOTATION_INFLIGHT_PLAN: json.dumps({"plan": "9", "from": {"0": "spx_nps1", "1": "spx_nps1"},
                                                      "to": {"0": "cpx_nps1", "1": "cpx_nps1"}})})
    e.smi.set_compute_partition(0, "CPX")
    out = e.actuator.startup()
    assert out["action"] == "roll-forward" and out["modes"] == {0: "cpx_nps1", 1: "spx_nps1"}
    assert out["modes_after"] == {0: "cpx_nps1", 1: "cpx_nps1"}
    assert api.ANNOTATION_INFLIGHT_PLAN not in e.annotations()
    # a superseded journal: the current spec wins
    e2 = Env(n_gpus=1)
    e2.spec({"nos.nebuly.com/spec-gpu-0-dpx_nps1": "2", api.ANNOTATION_PARTITIONING_PLAN: "11",
             api.ANNOTATION_INFLIGHT_PLAN: json.dumps({"plan": "10", "to": {"0": "cpx_nps1"}})})
    out = e2.actuator.startup()
    assert out["action"] == "superseded" and out["modes_after"] == {0: "dpx_nps1"}
    # nothing in flight: nothing to do
    assert e2.actuator.startup()["action"] == "none"


def test_spawned_barrier_helper_votes_and_checks_device_count():
    from walkai_nos_amd.parallel.spawned import SpawnedNodeBarrier
    b = SpawnedNodeBarrier(3, backend="local")
    assert b.vote_all([True, True, True]) and b.last["sum"] == 3
    assert not b.vote_all([True, False, True])
    assert not b.vote_all([True, True])  # wrong participant count is a veto


def test_agent_process_never_loads_hip_through_a_full_commit():
    from walkai_nos_amd.testing.hygiene import run_agent_cycle
    r = run_agent_cycle()
    assert r["commit"] == "ok" and r["devices"] == 9
    assert set(r["probe"]["slices"]) == {f"gpu0.p{k}" for k in range(8)} | {"gpu1.p0"}
    assert not r["hip_loaded"] and not r["torch"] and not r["kfd_open"]


def test_local_barrier_timeout_closes_the_generation():
    import threading
    b = LocalBarrier(2, timeout=0.05)
    assert b.vote(True) is False           # nobody else came: this round is closed as False
    late = []
    t = threading.Thread(target=lambda: late.append(LocalBarrier.vote(b, True)))
    b.timeout = 5.0
    t.start()
    assert b.vote(True) is True            # a fresh round, not completed by the stale vote
    t.join()
    assert late == [True]


def test_veto_when_a_gpu_drops_out_of_the_map_after_the_switch():
    """a flip after which a GPU is missing from the re-enumerated map has no device to
    carry its veto, and the GPUs behind it are renumbered: the commit must still be vetoed and the
    rollback must address the surviving GPUs by BDF, not by (shifted) index."""
    e = Env(n_gpus=3)
    real = e.smi._set_compute_partition

    def switch_and_lose(proc, mode):
        real(proc, mode)
        g = e.smi._gpu_of(proc)
        if g.index == 1 and mode == "CPX":
            e.smi._gpus.remove(g)          # GPU 1 did not come back from the mode change
    e.smi._set_compute_partition = switch_and_lose
    e.spec({"nos.nebuly.com/spec-gpu-0-dpx_nps1": "2", "nos.nebuly.com/spec-gpu-1-cpx_nps1": "8",
            api.ANNOTATION_PARTITIONING_PLAN: "5"})
    e.reporter.reconcile(Request("node-a"))
    with pytest.raises(GpuError):
        e.actuator.reconcile(Request("node-a"))
    votes = e.actuator.last_votes
    assert votes and not any(votes)
    assert e.shared.last_commit == "failed"
    m = e.smi.device_map()
    assert [g.bdf for g in m.gpus] == ["0000:05:00.0", "0000:25:00.0"]
    # GPU 0 rolled back to SPX; the old GPU 2 (now index 1) was never flipped
    assert e.smi.get_compute_partition(0) == "SPX" and e.smi.get_compute_partition(1) == "SPX"
    assert sorted(e.smi.set_calls) == [("compute", 0, "DPX"), ("compute", 0, "SPX"), ("compute", 1, "CPX")]


def test_native_helper_vetoes_a_device_count_mismatch():
    """The native commit-barrier helper (csrc/gpuhelper.cpp) vetoes when the HIP devices it sees
    differ from the device map — more votes than the map has, or (on this CPU host) no device at
    all — and still prints its one JSON line with the phase timings."""
    from walkai_nos_amd.ops import native
    from walkai_nos_amd.parallel.spawned import NATIVE_HELPER, SpawnedNodeBarrier, run_helper
    if not native.available(NATIVE_HELPER):
        pytest.skip("native helper not built")
    res = run_helper(["barrier", "--votes", "1,1,1", "--expect", "2"], 60.0, program=native.lib_path(NATIVE_HELPER))
    assert res["native"] is True and res["n"] == 3 and res["sum"] == 0 and "error" in res
    assert set(res) >= {"hip_init_ms", "comm_init_ms", "allreduce_ms", "destroy_ms", "total_ms"}
    b = SpawnedNodeBarrier(2, backend="rccl", native=True)
    assert not b.vote_all([True, True, True])          # more votes than the map's devices
    assert b.last.get("error") and b.last["wall_ms"] > 0
    if not native.gpu_present():
        assert not b.vote_all([True, True])            # no GPU here: the helper sees 0 != 2
