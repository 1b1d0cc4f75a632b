"""Telemetry exporter job (reference ``cmd/metricsexporter/metricsexporter.go:33-91``): always exits 0."""
from __future__ import annotations

import argparse
import sys

from ..exporters.telemetry import run


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="nos install telemetry")
    ap.add_argument("--metrics-file", required=True)
    ap.add_argument("--metrics-endpoint", required=True)
    args = ap.parse_args(argv)
    return run(args.metrics_file, args.metrics_endpoint)


if __name__ == "__main__":
    sys.exit(main())
