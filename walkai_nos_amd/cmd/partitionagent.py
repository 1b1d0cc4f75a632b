"""Partition agent (the mig-agent; reference ``cmd/migagent/migagent.go:56-199``).

Per-node DaemonSet: reads ``NODE_NAME``; builds the kubelet PodResources client (its error is
fatal here), one amd-smi session and the partition client; at startup checks that the
node has at least one compute-partition-capable GPU and runs the start-up reconciliation
(:meth:`Actuator.startup`: a plan journalled but not committed before a crash is rolled forward);
then runs the reporter and the actuator sharing a :class:`SharedState`.

The agent process never initialises HIP: the RCCL commit barrier (one communicator over every
logical device of the re-enumerated node, 64 in CPX on 8 GPUs) and the probe-on-commit kernels run
in spawned helper processes (``cmd/gpuhelper.py``) that exit before the next flip.
"""
from __future__ import annotations

import logging
import sys

from .. import constant
from ..api.config import MigAgentConfig, load_config_file
from ..controllers.agent.setup import setup_partition_agent
from ..device.amdsmi import new_backend
from ..device.deviceplugin_client import DevicePluginClient
from ..device.partition_client import PartitionClient
from ..device.podresources import PodResourcesClient
from ..utils.util import get_env_or_panic
from .common import base_parser, make_client, make_manager, run_until_signal, serve_endpoints, setup_logging

log = logging.getLogger("nos.partitionagent")


def node_barrier_factory(registry, backend: str = "rccl"):
    """Commit barrier per commit: a spawned helper voting over ``n`` logical devices (the actuator
    passes one vote per device of the re-enumerated map)."""
    from ..parallel.spawned import SpawnedNodeBarrier
    return lambda n: SpawnedNodeBarrier(n, backend=backend, registry=registry)


def main(argv=None) -> int:
    args = base_parser("nos partition agent").parse_args(argv)
    setup_logging(args.log_level)
    cfg = load_config_file(args.config, "MigAgentConfig") if args.config else MigAgentConfig()
    node = get_env_or_panic(constant.ENV_NODE_NAME)
    client = make_client(args.kubeconfig, cached=("Node",))
    smi = new_backend(cfg.amdSmiBackend)
    gpus = smi.list_gpus()
    if not gpus:
        log.error("no AMD GPU found on node %s", node)
        return 1
    resources = PodResourcesClient(cfg.podResourcesSocket)
    pc = PartitionClient(resources, smi)
    dp = DevicePluginClient(client, cfg.devicePluginLabel, cfg.devicePluginNamespace or None)
    mgr = make_manager(client, cfg, "partitionagent")
    from ..parallel.spawned import HelperRegistry
    helpers = HelperRegistry()
    bf = node_barrier_factory(helpers) if cfg.commitBarrier == "rccl" else None
    probe = None
    if cfg.probeOnCommit:
        from ..controllers.agent.probe import ProbeRunner, device_map_targets
        probe = lambda shared: ProbeRunner(shared, node, targets=device_map_targets(smi)).annotations  # noqa: E731
    _, _, actuator = setup_partition_agent(mgr, node, pc, device_plugin=dp, barrier_factory=bf,
                                           refresh_interval=cfg.reportConfigIntervalSeconds, probe=probe,
                                           helpers=helpers)
    log.info("device map: %s", smi.device_map().describe())
    log.info("start-up reconciliation: %s", actuator.startup())
    from ..exporters.gpu_metrics import GpuMetricsPoller
    GpuMetricsPoller(smi, node).register(mgr)
    serve_endpoints(mgr, cfg)
    return run_until_signal(mgr)


if __name__ == "__main__":
    sys.exit(main())
