"""gpupartitioner: control-plane partitioner (reference ``cmd/gpupartitioner/gpupartitioner.go:49-132``).

Loads ``GpuPartitionerConfig`` (validated), optionally the known-geometries YAML (validated, then
installed globally), registers the node initialiser and the pod controllers for both partitioning
kinds, serves health/metrics and runs with leader election.
"""
from __future__ import annotations

import logging
import sys

from ..api.config import GpuPartitionerConfig, load_config_file
from ..controllers.partitioner.setup import setup_partitioner
from ..models.defaults import ModelDefaults
from ..models.xcp.known_configs import load_known_geometries_file, set_known_geometries
from .common import (apply_manager_flags, base_parser, make_client, make_manager, run_until_signal,
                     serve_endpoints, setup_logging)

log = logging.getLogger("nos.gpupartitioner")


def main(argv=None) -> int:
    args = base_parser("nos GPU partitioner").parse_args(argv)
    setup_logging(args.log_level)
    cfg = load_config_file(args.config, "GpuPartitionerConfig") if args.config else GpuPartitionerConfig()
    apply_manager_flags(cfg, args)
    if cfg.knownMigGeometriesFile:
        set_known_geometries(load_known_geometries_file(cfg.knownMigGeometriesFile))
        log.info("loaded known geometries from %s", cfg.knownMigGeometriesFile)
    client = make_client(args.kubeconfig)
    mgr = make_manager(client, cfg, "gpupartitioner")
    defaults = ModelDefaults.from_config(cfg)
    if defaults.xcp_layout != "partitions":
        # upgrade note (docs/upgrade.md): unlabeled xcp nodes follow defaultXcpLayout
        log.warning("xcp nodes without the nos.nebuly.com/xcp-layout label are planned as %r "
                    "(defaultXcpLayout); label a node xcp-layout=partitions to keep hardware partitions",
                    defaults.xcp_layout)
    setup_partitioner(mgr, batch_timeout=cfg.batchWindowTimeoutSeconds, batch_idle=cfg.batchWindowIdleSeconds,
                      scoring=cfg.scoring, policy=cfg.planningPolicy, pack=cfg.pack_params(), defaults=defaults)
    serve_endpoints(mgr, cfg)
    return run_until_signal(mgr)


if __name__ == "__main__":
    sys.exit(main())
