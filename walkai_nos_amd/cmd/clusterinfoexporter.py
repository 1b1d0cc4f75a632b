"""cluster-info exporter (reference ``cmd/clusterinfoexporter/clusterinfoexporter.go:37-133``).

Flags ``--endpoint``, ``--interval`` (default 1m; <= 0 means 1m), ``--http-timeout`` (10s),
``--api-token``; sends one snapshot immediately, then every interval.  Deployed as a Deployment,
not a DaemonSet (every node POSTed the same cluster-wide snapshot).
"""
from __future__ import annotations

import argparse
import os
import logging
import sys
import threading

from ..exporters.clusterinfo import Collector, Exporter
from .common import make_client, setup_logging

log = logging.getLogger("nos.clusterinfoexporter")


def parse_duration(s: str) -> float:
    s = s.strip()
    units = {"ms": 1e-3, "s": 1.0, "m": 60.0, "h": 3600.0}
    for u in ("ms", "s", "m", "h"):
        if s.endswith(u):
            return float(s[: -len(u)]) * units[u]
    return float(s)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="nos cluster-info exporter")
    ap.add_argument("--endpoint", required=True)
    ap.add_argument("--interval", default="1m")
    ap.add_argument("--http-timeout", default="10s")
    ap.add_argument("--api-token", default=os.environ.get("NOS_API_TOKEN", ""))
    ap.add_argument("--kubeconfig", default="")
    ap.add_argument("--log-level", default="info")
    args = ap.parse_args(argv)
    setup_logging(args.log_level)
    interval = parse_duration(args.interval)
    if interval <= 0:
        interval = 60.0
    ex = Exporter(Collector(make_client(args.kubeconfig, cached=False)), args.endpoint, args.api_token,
                  parse_duration(args.http_timeout))
    stop = threading.Event()
    while not stop.is_set():
        try:
            ex.send_snapshot()
        except Exception as e:  # noqa: BLE001 - keep exporting
            log.error("unable to send snapshot: %s", e)
        stop.wait(interval)
    return 0


if __name__ == "__main__":
    sys.exit(main())
