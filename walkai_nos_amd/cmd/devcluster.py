"""nos-devcluster: the real control plane as OS processes on one machine, no Kubernetes needed.

Starts the in-memory API server behind its REST facade (``kube/apiserver.py``) and writes a
kubeconfig; creates fake MI355X nodes; runs ``nos-gpupartitioner`` and one ``nos-partitionagent``
per node (fake amd-smi inside each agent; ``--kind cumask``: ``nos-sliceagent``) as separate
processes against that kubeconfig; and plays
the parts a cluster would — one kubelet per node (``testing/kubelet.py``: plugin registration,
ListAndWatch, admission through the plugin's ``Allocate``, PodResources) and kube-scheduler
(``sim.cluster.KubeScheduler``: allocatable minus requests). With ``--quota`` it also runs
``nos-operator`` and ``nos-scheduler`` (Elastic Resource Quotas; pods opt in with
``schedulerName: nos-scheduler``). The reference's equivalent developer loop is a kind cluster
(``hack/kind/cluster.yaml``) with the operator deployed into it.

    nos-devcluster --nodes 2 --gpus 1 --demo        # submit sample pods and print what happens
    nos-devcluster --nodes 1 --gpus 8               # then create pods through the kubeconfig it prints

Pods are plain ``v1.Pod`` objects requesting ``amd.com/<mode>_<nps>``; a pod finishes when its
``nos.nebuly.com/dev-runtime-seconds`` annotation has elapsed after it started (default: runs
until deleted).
"""
from __future__ import annotations

import argparse
import logging
import os
import subprocess
import sys
import tempfile
import time
from types import SimpleNamespace
from typing import Any, Callable, Dict, List, Optional

from .. import constant
from ..api import v1alpha1 as api
from ..api.config import GpuAgentConfig, GpuPartitionerConfig, MigAgentConfig, dump_config
from ..kube import objects as ko
from ..kube.apiserver import APIFacade
from ..kube.rest import from_kubeconfig
from ..sim.cluster import KubeScheduler
from ..testing.kubelet import FakeKubelet

log = logging.getLogger("nos.devcluster")
RUNTIME_ANNOTATION = "nos.nebuly.com/dev-runtime-seconds"
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def node_labels(gpus: int, model: str = "MI355X", kind: str = api.PARTITIONING_KIND_XCP,
                layout: Optional[str] = "partitions") -> Dict[str, str]:
    """Labels of a fake MI355X node; ``layout`` None leaves ``nos.nebuly.com/xcp-layout`` off (the
    partitioner's ``defaultXcpLayout`` applies)."""
    out = {api.LABEL_GPU_PARTITIONING: kind,
           constant.LABEL_AMD_GPU_PRODUCT: f"AMD_Instinct_{model}", constant.LABEL_AMD_GPU_COUNT: str(gpus),
           constant.LABEL_AMD_GPU_VRAM: "288G", constant.LABEL_AMD_GPU_CU_COUNT: "256"}
    if kind == api.PARTITIONING_KIND_XCP and layout is not None:   # explicit (the default is slices)
        out[api.LABEL_XCP_LAYOUT] = layout
    return out


def fast_partitioner_config(**packing: float) -> GpuPartitionerConfig:
    """Second-scale planner timings (the defaults are minutes: production pod lifetimes)."""
    p = {"minStintSeconds": 0, "unservedAfterSeconds": 1, "drainGainAfterSeconds": 1, "replanEverySeconds": 0.2}
    p.update(packing)
    return GpuPartitionerConfig(healthProbeBindAddress="0", metricsBindAddress="0", batchWindowTimeoutSeconds=1.0,
                                batchWindowIdleSeconds=0.3, planningPolicy="pack", packing=p)


class DevCluster:
    def __init__(self, root: str, nodes: int = 1, gpus: int = 1,
                 partitioner: Optional[GpuPartitionerConfig] = None, report_interval: float = 1.0,
                 bookmark_every: float = 5.0, amd_smi_backend: str = "fake", quota: bool = False,
                 kind: str = api.PARTITIONING_KIND_XCP, layout: Optional[str] = "partitions"):
        self.root = root
        self.n_nodes, self.gpus = nodes, gpus
        self.partitioner_cfg = partitioner or fast_partitioner_config()
        self.report_interval = report_interval
        self.amd_smi_backend = amd_smi_backend   # native: the agents drive this machine's real GPUs
        self.quota = quota                       # also run nos-operator and nos-scheduler (Elastic Resource Quotas)
        self.kind = kind                         # xcp: partition agents; cumask: CU-mask slice agents
        self.xcp_layout = layout                 # xcp nodes' nos.nebuly.com/xcp-layout
        self.facade = APIFacade(bookmark_every=bookmark_every)
        self.procs: Dict[str, subprocess.Popen] = {}
        self._argv: Dict[str, Any] = {}
        self.logs: Dict[str, str] = {}
        self.kubelets: Dict[str, FakeKubelet] = {}
        self.client: Any = None
        self.scheduler: Optional[KubeScheduler] = None
        self.kubeconfig = ""
        self.started: Dict[tuple, float] = {}

    # -- lifecycle -----------------------------------------------------------------------
    def start(self) -> "DevCluster":
        self.facade.start()
        self.kubeconfig = self.facade.write_kubeconfig(os.path.join(self.root, "kubeconfig"))
        self.client = from_kubeconfig(self.kubeconfig)
        names = [f"node-{i}" for i in range(self.n_nodes)]
        for n in names:
            self.client.create(ko.new_node(n, node_labels(self.gpus, kind=self.kind, layout=self.xcp_layout)))
            self.kubelets[n] = FakeKubelet(os.path.join(self.root, n), self.client, n)
        self._spawn("gpupartitioner", "walkai_nos_amd.cmd.gpupartitioner", self.partitioner_cfg,
                    "GpuPartitionerConfig", {})
        for n in names:
            k = self.kubelets[n]
            common = dict(healthProbeBindAddress="0", metricsBindAddress="0",
                          reportConfigIntervalSeconds=self.report_interval, amdSmiBackend=self.amd_smi_backend,
                          fakeGpus=self.gpus, podResourcesSocket=k.podres_socket, commitBarrier="none",
                          probeOnCommit=False, devicePluginDir=k.dir,
                          fakeStateFile=os.path.join(k.root, "fake-amdsmi.json"))
            if self.kind == api.PARTITIONING_KIND_CUMASK:
                self._spawn(f"sliceagent-{n}", "walkai_nos_amd.cmd.sliceagent", GpuAgentConfig(**common),
                            "GpuAgentConfig", {constant.ENV_NODE_NAME: n})
            else:
                self._spawn(f"partitionagent-{n}", "walkai_nos_amd.cmd.partitionagent",
                            MigAgentConfig(devicePlugin="nos", sliceStateFile=os.path.join(k.root, "xcp-slices.json"),
                                           **common), "MigAgentConfig", {constant.ENV_NODE_NAME: n})
        if self.quota:
            quiet = ["--metrics-bind-address", "0", "--health-probe-bind-address", "0", "--leader-elect", "false"]
            self._spawn("nos-operator", "walkai_nos_amd.cmd.nosoperator", None, "", {}, quiet)
            self._spawn("nos-scheduler", "walkai_nos_amd.cmd.nosscheduler", None, "", {}, quiet)
        self.scheduler = KubeScheduler(self.client, {n: SimpleNamespace(name=n) for n in names},
                                       on_bind=self._on_bind)
        return self

    def restart(self, name: str) -> None:
        """Stop a component process and start it again with the same configuration (crash /
        upgrade scenarios: the agent's start-up reconciliation, the partitioner's re-planning)."""
        p = self.procs[name]
        p.terminate()
        try:
            p.wait(timeout=10)
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
        argv, env = self._argv[name]
        with open(self.logs[name], "a") as out:
            self.procs[name] = subprocess.Popen(argv, stdout=out, stderr=subprocess.STDOUT, env=env, cwd=self.root)

    def _spawn(self, name: str, module: str, cfg: Any, kind: str, env: Dict[str, str],
               extra: Optional[List[str]] = None) -> None:
        argv = [sys.executable, "-m", module, "--kubeconfig", self.kubeconfig] + list(extra or [])
        if cfg is not None:
            path = os.path.join(self.root, f"{name}.yaml")
            with open(path, "w") as f:
                f.write(dump_config(cfg, kind))
            argv += ["--config", path]
        self.logs[name] = os.path.join(self.root, f"{name}.log")
        e = dict(os.environ, PYTHONPATH=REPO + os.pathsep + os.environ.get("PYTHONPATH", ""), **env)
        self._argv[name] = (argv, e)
        with open(self.logs[name], "w") as out:
            self.procs[name] = subprocess.Popen(argv, stdout=out, stderr=subprocess.STDOUT, env=e, cwd=self.root)

    def stop(self) -> None:
        for p in self.procs.values():
            if p.poll() is None:
                p.terminate()
        for p in self.procs.values():
            try:
                p.wait(timeout=10)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        for k in self.kubelets.values():
            k.stop()
        if self.client is not None:
            self.client.close()
        self.facade.stop()

    def _on_bind(self, pod: Dict[str, Any], node: str) -> None:
        if self.kubelets[node].admit(pod, node) is not None:
            self.started[(ko.namespace(pod), ko.name(pod))] = time.time()

    # -- loop ----------------------------------------------------------------------------
    def tail(self, n: int = 30) -> str:
        out = []
        for name, path in self.logs.items():
            with open(path) as f:
                out.append(f"--- {name}\n" + "".join(f.readlines()[-n:]))
        return "\n".join(out)

    def step(self) -> None:
        for name, p in self.procs.items():
            if p.poll() is not None:
                raise RuntimeError(f"{name} exited with {p.returncode}\n{self.tail()}")
        for k in self.kubelets.values():
            k.sync()
        self.scheduler.reconcile(KubeScheduler.KEY)
        self._kubelet_pods()
        now = time.time()
        for (ns, name), t0 in list(self.started.items()):
            try:
                pod = self.client.get("Pod", name, ns)
            except Exception:  # noqa: BLE001 - deleted by the user
                self.started.pop((ns, name), None)
                continue
            rt = ko.annotations(pod).get(RUNTIME_ANNOTATION)
            if rt is not None and now - t0 >= float(rt):
                self.started.pop((ns, name), None)
                self.kubelets[ko.pod_node_name(pod)].finish(ns, name)

    def _kubelet_pods(self) -> None:
        """What each kubelet sees of its pods: pods another scheduler (nos-scheduler) bound here are
        admitted; devices of pods deleted (finished, evicted, preempted) are released."""
        pods = {(ko.namespace(p), ko.name(p)): p for p in self.client.list("Pod")}
        for node, k in self.kubelets.items():
            for key in [key for key in k.used if key not in pods]:
                with k.lock:
                    k.used.pop(key, None)
                self.started.pop(key, None)
            for key, p in pods.items():
                if ko.pod_node_name(p) == node and ko.pod_phase(p) == "Pending" and key not in k.used:
                    self._on_bind(p, node)

    def run_until(self, cond: Callable[[], bool], timeout: float, what: str, period: float = 0.2) -> None:
        deadline = time.time() + timeout
        while time.time() < deadline:
            self.step()
            if cond():
                return
            time.sleep(period)
        raise TimeoutError(f"timed out waiting for {what}\n{self.tail()}")

    # -- views ---------------------------------------------------------------------------
    def allocatable(self, node: str, profile: str) -> int:
        return int(ko.node_allocatable(self.client.get("Node", node)).get(f"amd.com/{profile}", "0"))

    def phase(self, name: str, namespace: str = "default") -> str:
        return ko.pod_phase(self.client.get("Pod", name, namespace))

    def submit(self, name: str, profile: str, runtime_s: Optional[float] = None, namespace: str = "default",
               scheduler_name: str = "default-scheduler"):
        """A pod requesting one ``amd.com/<profile>`` (``cpx_nps1``, ``gpu-64cu.72gb``, ...)."""
        pod = ko.new_pod(name, namespace, requests={f"amd.com/{profile}": 1}, scheduler_name=scheduler_name)
        if runtime_s is not None:
            pod["metadata"]["annotations"][RUNTIME_ANNOTATION] = str(runtime_s)
        return self.client.create(pod)

    def layout(self) -> Dict[str, Dict[str, str]]:
        out = {}
        for n in self.kubelets:
            anns = ko.annotations(self.client.get("Node", n))
            out[n] = {k.split("/", 1)[1]: v for k, v in sorted(anns.items())
                      if k.startswith((api.ANNOTATION_GPU_SPEC_PREFIX, api.ANNOTATION_GPU_STATUS_PREFIX))}
        return out


def _demo(c: DevCluster) -> None:
    print("demo: eight 1/8-GPU pods (20 s each), then a whole-GPU pod (10 s)", flush=True)
    for i in range(8):
        c.submit(f"cpx-{i}", "cpx_nps1", runtime_s=20)
    c.run_until(lambda: all(c.phase(f"cpx-{i}") == "Running" for i in range(8)), 120, "the 1/8 pods")
    print("all eight 1/8 pods run:", c.layout(), flush=True)
    c.submit("whole", "spx_nps1", runtime_s=10)
    c.run_until(lambda: c.phase("whole") == "Running", 180, "the whole-GPU pod")
    node = ko.pod_node_name(c.client.get("Pod", "whole", "default"))
    print(f"the whole-GPU pod runs on {node} (a one-node cluster drains its GPU first):", c.layout(), flush=True)
    c.run_until(lambda: not c.started, 60, "the pods to finish")
    print("every pod finished:", c.layout(), flush=True)


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser(description="nos control plane as local processes (no Kubernetes)")
    ap.add_argument("--nodes", type=int, default=1)
    ap.add_argument("--gpus", type=int, default=1, help="fake MI355X GPUs per node")
    ap.add_argument("--dir", default="", help="working directory (kubeconfig, configs, logs); default: a temp dir")
    ap.add_argument("--demo", action="store_true", help="submit sample pods, print the layouts, exit")
    ap.add_argument("--quota", action="store_true", help="also run nos-operator and nos-scheduler")
    ap.add_argument("--kind", default=api.PARTITIONING_KIND_XCP, choices=api.PARTITIONING_KINDS,
                    help="xcp: compute partitions (partition agents); cumask: CU-mask slices (slice agents)")
    ap.add_argument("--layout", default="partitions", choices=("partitions", "slices", "auto", "default"),
                    help="xcp nodes' nos.nebuly.com/xcp-layout label (default: no label, the partitioner's "
                         "defaultXcpLayout); the demo shows the flips of hardware partitions")
    ap.add_argument("--log-level", default="info")
    a = ap.parse_args(argv)
    logging.basicConfig(level=getattr(logging, a.log_level.upper(), logging.INFO))
    root = a.dir or tempfile.mkdtemp(prefix="nos-devcluster-")
    os.makedirs(root, exist_ok=True)
    c = DevCluster(root, nodes=a.nodes, gpus=a.gpus, quota=a.quota, kind=a.kind,
                   layout=None if a.layout == "default" else a.layout).start()
    print(f"nos dev cluster: {a.nodes} node(s) x {a.gpus} GPU(s); KUBECONFIG={c.kubeconfig}; logs in {root}",
          flush=True)
    try:
        if a.kind == api.PARTITIONING_KIND_XCP:
            c.run_until(lambda: all(c.allocatable(n, "spx_nps1") == a.gpus for n in c.kubelets), 60,
                        "the partition agents to report")
        if a.demo and a.kind == api.PARTITIONING_KIND_XCP:
            _demo(c)
            return 0
        last = None
        while True:
            c.step()
            lay = c.layout()
            if lay != last:
                print(lay, flush=True)
                last = lay
            time.sleep(0.5)
    except KeyboardInterrupt:
        return 0
    finally:
        c.stop()


if __name__ == "__main__":
    sys.exit(main())
