"""CU-mask slice agent (the gpu-agent; reference ``cmd/gpuagent/gpuagent.go:54-152``).

Refuses to run on a GPU that is not in SPX mode (the reference refuses MIG-enabled GPUs): CU
masks are applied within one logical device.  Runs the slice reporter/actuator and the nos device
plugin manager for the node's slices.
"""
from __future__ import annotations

import logging
import os
import sys
import threading

from .. import constant
from ..api.config import GpuAgentConfig, load_config_file
from ..controllers.sliceagent.agent import setup_slice_agent
from ..device.amdsmi import new_backend
from ..device.podresources import PodResourcesClient
from ..device.slicing_client import ConfigMapSliceStore, SlicingClient
from ..deviceplugin.server import PluginManager, render_nodes_from_sysfs, run_forever
from ..utils.util import get_env_or_panic
from .common import (apply_manager_flags, base_parser, make_client, make_manager, run_until_signal,
                     serve_endpoints, setup_logging)

log = logging.getLogger("nos.sliceagent")


def any_partitioned_gpu(smi) -> bool:
    return any(smi.get_compute_partition(g.index) != "SPX" for g in smi.list_gpus())


def main(argv=None) -> int:
    args = base_parser("nos CU-mask slice agent").parse_args(argv)
    setup_logging(args.log_level)
    cfg = load_config_file(args.config, "GpuAgentConfig") if args.config else GpuAgentConfig()
    apply_manager_flags(cfg, args)
    node = get_env_or_panic(constant.ENV_NODE_NAME)
    client = make_client(args.kubeconfig, cached=("Node", "ConfigMap"))
    smi = new_backend(cfg.amdSmiBackend, n_gpus=cfg.fakeGpus, state_file=cfg.fakeStateFile)
    if any_partitioned_gpu(smi):
        log.error("CU-mask slicing needs every GPU in SPX mode; use the partition agent on this node")
        return 1
    gpus = smi.list_gpus()
    store = ConfigMapSliceStore(client, node)
    sc = SlicingClient(PodResourcesClient(cfg.podResourcesSocket), smi)
    mgr = make_manager(client, cfg, "sliceagent")
    # render nodes and slice health come from the device map (a slice whose GPU left the map is
    # Unhealthy); the sysfs listing is only the fallback for a map without render minors
    from ..deviceplugin.startgate import StartGate
    gate = StartGate(timeout=cfg.sharedSliceStartGateSeconds) if cfg.sharedSliceStartGateSeconds > 0 else None
    plugins = PluginManager(store, render_nodes_from_sysfs(), socket_dir=cfg.devicePluginDir,
                            kubelet_socket=os.path.join(cfg.devicePluginDir, "kubelet.sock"),
                            cu_count=gpus[0].cu_count or 256, shim_path=cfg.hbmLimitShimPath, device_map=smi.device_map,
                            shared_hw_queues=cfg.sharedSliceHwQueues, start_gate=gate)

    class Notify:
        def restart(self, node_name, timeout=60):
            plugins.sync()

    cu_count = gpus[0].cu_count or 256
    probe = None
    if cfg.probeOnCommit:
        from ..controllers.agent.probe import ProbeRunner
        from ..controllers.sliceagent.agent import slice_probe_targets
        probe = lambda shared: ProbeRunner(shared, node, targets=slice_probe_targets(store, cu_count)).annotations  # noqa: E731
    setup_slice_agent(mgr, node, sc, store, device_plugin=Notify(), refresh_interval=cfg.reportConfigIntervalSeconds,
                      cu_count=cu_count, memory_gb=int(gpus[0].vram_bytes // 10**9) or 288, probe=probe,
                      on_release=gate.forget if gate is not None else None)
    stop = threading.Event()
    threading.Thread(target=run_forever, args=(plugins, 2.0, stop), daemon=True).start()
    from ..exporters.gpu_metrics import GpuMetricsPoller
    GpuMetricsPoller(smi, node).register(mgr)
    from ..controllers.hbmguard import HbmGuard, node_pods_by_uid, pod_event, pod_evictor
    HbmGuard(smi, store.load, node, pods_by_device=sc.resources.get_used_devices_by_pod,
             pods_by_uid=node_pods_by_uid(client, node), evict=pod_evictor(client, node), action=cfg.hbmGuard,
             slack_bytes=cfg.hbmGuardSlackBytes, cu_action=cfg.cuGuard, cu_strikes=cfg.cuGuardStrikes,
             cu_count=cu_count, event=pod_event(client, node)).register(mgr, cfg.hbmGuardIntervalSeconds)
    serve_endpoints(mgr, cfg)
    return run_until_signal(mgr, stop)


if __name__ == "__main__":
    sys.exit(main())
