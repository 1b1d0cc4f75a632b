"""nos-operator: (Composite)ElasticQuota status and pod capacity labels."""
from __future__ import annotations

import os
import sys

from ..api.config import CapacitySchedulingArgs, GpuPartitionerConfig, load_config_file
from ..quota.gpu_memory import GpuMemoryCalculator
from ..quota.operator import setup_quota_operator
from .common import (apply_manager_flags, base_parser, make_client, make_manager, run_until_signal,
                     serve_endpoints, setup_logging)


def main(argv=None) -> int:
    args = base_parser("nos operator").parse_args(argv)
    setup_logging(args.log_level)
    sargs = load_config_file(args.config, "CapacitySchedulingArgs") if args.config else CapacitySchedulingArgs()
    if not args.config and os.environ.get("NOS_GPU_MEMORY_GB"):
        sargs.nvidiaGpuResourceMemoryGB = int(os.environ["NOS_GPU_MEMORY_GB"])
        sargs.validate()
    client = make_client(args.kubeconfig)
    mcfg = GpuPartitionerConfig()
    mcfg.leaderElection.leaderElect = True
    mcfg.leaderElection.resourceName = "nos-operator.nebuly.com"
    apply_manager_flags(mcfg, args)
    mgr = make_manager(client, mcfg, "nos-operator")
    setup_quota_operator(mgr, GpuMemoryCalculator(sargs.nvidiaGpuResourceMemoryGB))
    serve_endpoints(mgr, mcfg)
    return run_until_signal(mgr)


if __name__ == "__main__":
    sys.exit(main())
