"""nos-scheduler with the CapacityScheduling plugin (docs ``elastic-resource-quota/configuration.md``).

``--config`` takes a ``CapacitySchedulingArgs`` file (``nvidiaGpuResourceMemoryGB`` /
``amdGpuResourceMemoryGB``); pods opt in with ``schedulerName: nos-scheduler``.
"""
from __future__ import annotations

import sys

from ..api.config import CapacitySchedulingArgs, GpuPartitionerConfig, load_config_file
from ..quota.gpu_memory import GpuMemoryCalculator
from ..quota.scheduler import setup_nos_scheduler
from .common import (apply_manager_flags, base_parser, make_client, make_manager, run_until_signal,
                     serve_endpoints, setup_logging)


def main(argv=None) -> int:
    ap = base_parser("nos scheduler")
    args = ap.parse_args(argv)
    setup_logging(args.log_level)
    sargs = load_config_file(args.config, "CapacitySchedulingArgs") if args.config else CapacitySchedulingArgs()
    client = make_client(args.kubeconfig)
    mcfg = GpuPartitionerConfig()
    mcfg.leaderElection.leaderElect = True
    mcfg.leaderElection.resourceName = "nos-scheduler.nebuly.com"
    apply_manager_flags(mcfg, args)
    mgr = make_manager(client, mcfg, "nos-scheduler")
    setup_nos_scheduler(mgr, GpuMemoryCalculator(sargs.nvidiaGpuResourceMemoryGB))
    serve_endpoints(mgr, mcfg)
    return run_until_signal(mgr)


if __name__ == "__main__":
    sys.exit(main())
