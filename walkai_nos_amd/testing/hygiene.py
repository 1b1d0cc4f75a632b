"""Process-hygiene harness for the node agents: drive one agent cycle in a fresh interpreter and
report whether the *agent* process loaded HIP, imported torch or opened ``/dev/kfd`` (it must
not: the GPU work runs in spawned helpers, ``cmd/gpuhelper.py``).  Used by the CPU test
(fake amd-smi, local barrier) and the GPU test (native amd-smi, RCCL barrier, HIP probe)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

AGENT_SCRIPT = r"""
import json, sys
sys.path.insert(0, %(root)r)
from walkai_nos_amd.api import v1alpha1 as api
from walkai_nos_amd.controllers.agent.probe import ProbeRunner, device_map_targets, spawned_round
from walkai_nos_amd.controllers.agent.setup import setup_partition_agent
from walkai_nos_amd.device.amdsmi import new_backend
from walkai_nos_amd.device.partition_client import PartitionClient
from walkai_nos_amd.device.podresources import StaticResourceClient
from walkai_nos_amd.kube import objects as ko
from walkai_nos_amd.kube.memory import InMemoryAPIServer
from walkai_nos_amd.kube.runtime import Manager, Request
from walkai_nos_amd.parallel.spawned import HelperRegistry, SpawnedNodeBarrier

smi = new_backend(%(backend)r, n_gpus=2)
api_ = InMemoryAPIServer()
api_.create(ko.new_node("n"))
alloc = lambda: [(f"amd.com/{d.compute_mode.lower()}_{d.memory_mode.lower()}", d.device_id) for d in smi.logical_devices()]
pc = PartitionClient(StaticResourceClient(lambda: [], alloc), smi)
helpers = HelperRegistry()
mgr = Manager(api_)
probe = lambda sh: ProbeRunner(sh, "n", targets=device_map_targets(smi), asynchronous=False,
                               round_fn=spawned_round(sh.helpers, backend=%(probe_backend)r)).annotations
shared, reporter, actuator = setup_partition_agent(
    mgr, "n", pc, barrier_factory=lambda k: SpawnedNodeBarrier(k, backend=%(barrier_backend)r, registry=helpers),
    probe=probe, helpers=helpers)
reporter.reconcile(Request("n"))
target = %(target)r
if target:
    from walkai_nos_amd.models.xcp.profile import parse_profile
    api_.patch("Node", "n", {"metadata": {"annotations": {"nos.nebuly.com/spec-gpu-0-" + target:
                                                          str(parse_profile(target).partitions),
                                                          api.ANNOTATION_PARTITIONING_PLAN: "1"}}})
    actuator.reconcile(Request("n"))
reporter.reconcile(Request("n"))
direct = None
if %(direct_barrier)r:
    n = len(smi.logical_devices())
    b = SpawnedNodeBarrier(n, backend=%(barrier_backend)r, registry=helpers)
    direct = {"ok": b.vote_all([True] * n), "info": b.last, "veto": b.vote_all([False] + [True] * (n - 1))}
maps = open("/proc/self/maps").read()
fds = []
import os
for fd in os.listdir("/proc/self/fd"):
    try:
        fds.append(os.readlink("/proc/self/fd/" + fd))
    except OSError:
        pass
print(json.dumps({"hip_loaded": "libamdhip64" in maps, "torch": "torch" in sys.modules,
                  "kfd_open": any(f == "/dev/kfd" for f in fds), "commit": shared.last_commit,
                  "probe": json.loads(ko.annotations(api_.get("Node", "n")).get(api.ANNOTATION_PROBE_RESULT, "{}")),
                  "devices": len(smi.logical_devices()), "direct_barrier": direct,
                  "map": smi.device_map().describe()}))
"""


def run_agent_cycle(backend="fake", barrier_backend="local", probe_backend="fake", target="cpx_nps1",
                    direct_barrier=False):
    """Run one partition-agent cycle (report, optional apply of ``target`` on GPU 0, report with
    probe-on-commit, optional direct commit-barrier votes) in a fresh interpreter and return what
    it saw of itself: whether HIP/torch got loaded or /dev/kfd opened in the *agent* process."""
    code = AGENT_SCRIPT % {"root": ROOT, "backend": backend, "barrier_backend": barrier_backend,
                           "probe_backend": probe_backend, "target": target, "direct_barrier": direct_barrier}
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    return json.loads(p.stdout.strip().splitlines()[-1])
