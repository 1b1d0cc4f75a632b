"""Partition agent (the mig-agent; reference ``cmd/migagent/migagent.go:56-199``).

Per-node DaemonSet: reads ``NODE_NAME``; builds the kubelet PodResources client (its error is
fatal here), one amd-smi session and the partition client; at startup checks that the
node has at least one compute-partition-capable GPU and runs the start-up reconciliation
(:meth:`Actuator.startup`: a plan journalled but not committed before a crash is rolled forward);
then runs the reporter and the actuator sharing a :class:`SharedState`.

Compute partitions are served by the agent's own nos partition device plugin (``devicePlugin:
nos``, default): a GPU the partitioner drains has every partition reported Unhealthy, so no new pod
lands on it, and a flip is pushed to kubelet through ListAndWatch instead of restarting a plugin
pod (``devicePlugin: amd`` keeps the AMD k8s-device-plugin + restart path, without drains).

The agent process never initialises HIP: the RCCL commit barrier (one communicator over every
logical device of the re-enumerated node, 64 in CPX on 8 GPUs) and the probe-on-commit kernels run
in spawned helper processes (``cmd/gpuhelper.py``) that exit before the next flip.
"""
from __future__ import annotations

import logging
import os
import sys

from .. import constant
from ..api.config import MigAgentConfig, load_config_file
from ..controllers.agent.setup import setup_partition_agent
from ..device.amdsmi import new_backend
from ..device.deviceplugin_client import DevicePluginClient
from ..device.partition_client import PartitionClient
from ..device.podresources import PodResourcesClient
from ..kube.runtime import Watch
from ..utils.predicates import AnnotationsChanged, ExcludeDelete, MatchingName
from ..utils.util import get_env_or_panic
from .common import (apply_manager_flags, base_parser, make_client, make_manager, run_until_signal,
                     serve_endpoints, setup_logging)

log = logging.getLogger("nos.partitionagent")


def node_barrier_factory(registry, backend: str = "xgmi"):
    """Commit barrier per commit: a spawned helper voting over ``n`` logical devices (the actuator
    passes one vote per device of the re-enumerated map)."""
    from ..parallel.spawned import SpawnedNodeBarrier
    return lambda n: SpawnedNodeBarrier(n, backend=backend, registry=registry)


def nos_partition_plugin(client, node: str, smi, resources, cfg, slice_store=None, degraded=None):
    """The nos partition device plugin of this node: its view (device map, the node's spec/status
    annotations, kubelet's allocated ids, the CU-mask slices of sliced GPUs), one gRPC plugin per
    ``amd.com/<mode>_<nps>`` resource, and the hook the actuator calls after a flip."""
    from ..deviceplugin.partitions import AllocatablePublisher, PartitionPluginHook, PartitionState, \
        partition_plugin_manager
    from ..kube import objects as ko

    def used_ids():
        return {d.device_id for d in resources.get_used_devices()}
    state = PartitionState(smi.device_map, lambda: ko.annotations(client.get("Node", node)), used_ids,
                           slices=slice_store.load if slice_store is not None else None, degraded=degraded)
    plugins = partition_plugin_manager(state, socket_dir=cfg.devicePluginDir,
                                       kubelet_socket=os.path.join(cfg.devicePluginDir, "kubelet.sock"),
                                       shim_path=cfg.hbmLimitShimPath,
                                       shim_present=lambda: os.path.exists(cfg.hbmLimitShimPath))
    publisher = AllocatablePublisher(client, node) if cfg.publishAllocatable else None
    return PartitionPluginHook(plugins, state, publisher), plugins


def main(argv=None) -> int:
    args = base_parser("nos partition agent").parse_args(argv)
    setup_logging(args.log_level)
    cfg = load_config_file(args.config, "MigAgentConfig") if args.config else MigAgentConfig()
    apply_manager_flags(cfg, args)
    node = get_env_or_panic(constant.ENV_NODE_NAME)
    client = make_client(args.kubeconfig, cached=("Node",))
    smi = new_backend(cfg.amdSmiBackend, n_gpus=cfg.fakeGpus, state_file=cfg.fakeStateFile)
    gpus = smi.list_gpus()
    if not gpus:
        log.error("no AMD GPU found on node %s", node)
        return 1
    resources = PodResourcesClient(cfg.podResourcesSocket)
    pc = PartitionClient(resources, smi)
    mgr = make_manager(client, cfg, "partitionagent")
    plugins = None
    slice_store = None
    runner: dict = {}   # the probe runner, once built (the plugin withholds what it finds degraded)
    if cfg.devicePlugin == "nos":
        from ..device.slicing_client import FileSliceStore
        slice_store = FileSliceStore(cfg.sliceStateFile)  # sliced GPUs (xcp-layout slices/auto)
        dp, plugins = nos_partition_plugin(client, node, smi, resources, cfg, slice_store,
                                           degraded=lambda: runner["r"].degraded() if "r" in runner else {})
        mgr.new_controller("nos-partition-plugin", dp.reconcile,
                           [Watch("Node", [ExcludeDelete(), MatchingName(node), AnnotationsChanged()])])
    else:
        dp = DevicePluginClient(client, cfg.devicePluginLabel, cfg.devicePluginNamespace or None)
    from ..parallel.spawned import HelperRegistry, native_helper
    if cfg.commitBarrier == "xgmi" and native_helper() is None:
        # fail before the first flip, not after it: a barrier that cannot start is a veto, and a
        # node whose every commit is vetoed rolls every flip back
        log.error("commitBarrier xgmi needs the native nos-gpuhelper (make native); not found")
        return 1
    helpers = HelperRegistry()
    bf = node_barrier_factory(helpers, cfg.commitBarrier) if cfg.commitBarrier != "none" else None
    probe = None
    if cfg.probeOnCommit:
        from ..controllers.agent.probe import ProbeRunner, device_map_targets
        from ..models.xcp.known_configs import get_model_spec
        spec = get_model_spec(gpus[0].model)

        def probe(shared):
            runner["r"] = ProbeRunner(shared, node, targets=device_map_targets(
                smi, slice_store.load if slice_store is not None else None),
                used=lambda: {d.device_id for d in resources.get_used_devices()},
                expected_per_cu=spec.probe_bf16_tflops_per_cu if spec else None,
                healthy_fraction=cfg.probeHealthyFraction)
            return runner["r"].annotations
    _, _, actuator = setup_partition_agent(mgr, node, pc, device_plugin=dp, barrier_factory=bf,
                                           refresh_interval=cfg.reportConfigIntervalSeconds, probe=probe,
                                           helpers=helpers, slice_store=slice_store)
    log.info("device map: %s", smi.device_map().describe())
    log.info("start-up reconciliation: %s", actuator.startup())
    from ..exporters.gpu_metrics import GpuMetricsPoller
    GpuMetricsPoller(smi, node).register(mgr)
    from ..controllers.hbmguard import HbmGuard, node_pods_by_uid, pod_event, pod_evictor, shared_memory_partitions
    # sliced GPUs' slices (HBM budget and CU mask), and hardware partitions sharing one memory pool
    # (CPX on NPS1: HBM only, their CUs are hardware-isolated)
    HbmGuard(smi, slice_store.load if slice_store is not None else dict, node,
             pods_by_device=resources.get_used_devices_by_pod, pods_by_uid=node_pods_by_uid(client, node),
             evict=pod_evictor(client, node), action=cfg.hbmGuard, slack_bytes=cfg.hbmGuardSlackBytes,
             partitions=lambda: shared_memory_partitions(smi.device_map()), cu_action=cfg.cuGuard,
             cu_strikes=cfg.cuGuardStrikes, cu_count=smi.device_map().gpus[0].cu_count or 256,
             event=pod_event(client, node)).register(mgr, cfg.hbmGuardIntervalSeconds)
    serve_endpoints(mgr, cfg)
    stop = None
    if plugins is not None:
        import threading
        from ..deviceplugin.server import run_forever
        stop = threading.Event()
        threading.Thread(target=run_forever, args=(plugins, 2.0, stop), name="nos-partition-plugins",
                         daemon=True).start()
    return run_until_signal(mgr, stop) if stop is not None else run_until_signal(mgr)


if __name__ == "__main__":
    sys.exit(main())
