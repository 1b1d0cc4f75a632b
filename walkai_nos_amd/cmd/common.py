"""Shared plumbing for the component entry points: flags, logging, API client, health/metrics
servers, leader election (reference ``cmd/*/*.go`` manager setup)."""
from __future__ import annotations

import argparse
import logging
import os
import signal
import sys
import threading
from typing import Any, Optional

from ..api.config import ManagerConfig
from ..kube.leader import LeaderElector
from ..kube.runtime import Manager
from ..utils.metrics import REGISTRY, check_route, metrics_route, serve


def base_parser(description: str) -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(description=description)
    ap.add_argument("--config", default="", help="ComponentConfig file (config.nos.nebuly.com/v1alpha1)")
    ap.add_argument("--kubeconfig", default=os.environ.get("KUBECONFIG", ""), help="kubeconfig (default: in-cluster)")
    ap.add_argument("--log-level", "--zap-log-level", dest="log_level", default="info")
    # controller-runtime's manager flags; when given they override the config file ("0" disables a server)
    ap.add_argument("--metrics-bind-address", dest="metrics_bind_address", default=None)
    ap.add_argument("--health-probe-bind-address", dest="health_probe_bind_address", default=None)
    ap.add_argument("--leader-elect", dest="leader_elect", default=None, choices=("true", "false"))
    return ap


def apply_manager_flags(cfg: ManagerConfig, args: argparse.Namespace) -> ManagerConfig:
    """Command-line manager flags over the component's config (the reference's binaries take the same
    three flags, ``cmd/*/*.go``)."""
    if getattr(args, "metrics_bind_address", None) is not None:
        cfg.metricsBindAddress = args.metrics_bind_address
    if getattr(args, "health_probe_bind_address", None) is not None:
        cfg.healthProbeBindAddress = args.health_probe_bind_address
    if getattr(args, "leader_elect", None) is not None:
        cfg.leaderElection.leaderElect = args.leader_elect == "true"
    cfg.validate()
    return cfg


def setup_logging(level: str) -> None:
    lvl = {"debug": logging.DEBUG, "info": logging.INFO, "error": logging.ERROR}.get(level.lower(), logging.INFO)
    logging.basicConfig(level=lvl, stream=sys.stderr,
                        format='{"ts":"%(asctime)s","level":"%(levelname)s","logger":"%(name)s","msg":"%(message)s"}')


def make_client(kubeconfig: str = "", cached: Any = True) -> Any:
    """REST client for the cluster; reconcilers read through an informer cache, like
    controller-runtime's manager client.  ``cached``: True (the default kinds), a tuple of kinds
    (node agents cache only Nodes), or False (periodic exporters list on demand)."""
    from ..kube.cache import DEFAULT_CACHED, CachedClient
    from ..kube.rest import RESTClient, from_kubeconfig
    rest = from_kubeconfig(kubeconfig) if kubeconfig else RESTClient.in_cluster()
    if not cached:
        return rest
    return CachedClient(rest, DEFAULT_CACHED if cached is True else tuple(cached))


def make_manager(client: Any, cfg: ManagerConfig, component: str) -> Manager:
    le = None
    if cfg.leaderElection.leaderElect:
        c = cfg.leaderElection
        le = LeaderElector(client, c.resourceName, c.resourceNamespace, lease_duration=c.leaseDurationSeconds,
                           renew_deadline=c.renewDeadlineSeconds, retry_period=c.retryPeriodSeconds,
                           release_on_cancel=c.leaderElectionReleaseOnCancel)
    mgr = Manager(client, leader_election=le)
    return mgr


def serve_endpoints(mgr: Manager, cfg: ManagerConfig) -> None:
    if cfg.healthProbeBindAddress and cfg.healthProbeBindAddress != "0":
        serve(cfg.healthProbeBindAddress, {"/healthz": check_route(mgr.healthy), "/readyz": check_route(mgr.ready)})
    if cfg.metricsBindAddress and cfg.metricsBindAddress != "0":
        serve(cfg.metricsBindAddress, {"/metrics": metrics_route(REGISTRY)})


def run_until_signal(mgr: Manager, extra_stop: Optional[threading.Event] = None) -> int:
    stop = extra_stop or threading.Event()
    signal.signal(signal.SIGTERM, lambda *_: stop.set())
    signal.signal(signal.SIGINT, lambda *_: stop.set())
    mgr.start()
    stop.wait()
    mgr.stop()
    return 0
