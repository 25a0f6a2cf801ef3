"""One-shot telemetry exporter (``cmd/metricsexporter/metricsexporter.go:33-91``):
reads the metrics YAML written by the install hook and POSTs it as JSON.
Opt-in: with no endpoint the document is printed (a local JSON dump), and a
failure never fails the install (exit 0, as the reference).

python -m nos_amd.cmd.metricsexporter --metrics-file metrics.yaml [--metrics-endpoint URL]
"""
from __future__ import annotations

import argparse
import json
import logging
from pathlib import Path

import yaml

log = logging.getLogger("nos_amd.cmd.metricsexporter")


def schema(doc: dict) -> dict:
    """``metrics.Metrics`` (``cmd/metricsexporter/metrics/metrics.go:24-42``)."""
    comps = doc.get("components") or {}
    return {"installationUUID": doc.get("installationUUID", ""),
            "nodes": [{"name": n.get("name", ""), "capacity": n.get("capacity") or {}, "labels": n.get("labels") or {},
                       "nodeInfo": n.get("nodeInfo") or {}} for n in doc.get("nodes") or []],
            "chartValues": doc.get("chartValues"),
            "components": {"nosGpuPartitioner": bool(comps.get("nosGpuPartitioner")),
                           "nosScheduler": bool(comps.get("nosScheduler")),
                           "nosOperator": bool(comps.get("nosOperator"))}}


def collect_nodes(api) -> list[dict]:
    """Node facts for the document (what the Helm hook gathers)."""
    out = []
    for n in api.list("Node"):
        out.append({"name": n["metadata"]["name"], "capacity": (n.get("status") or {}).get("capacity") or {},
                    "labels": {k: v for k, v in (n["metadata"].get("labels") or {}).items()
                               if k.startswith(("amd.com/", "nos.nebuly.com/"))},
                    "nodeInfo": (n.get("status") or {}).get("nodeInfo") or {}})
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--metrics-file", default="")
    ap.add_argument("--metrics-endpoint", default="")
    ap.add_argument("--log-level", default="info")
    args = ap.parse_args(argv)
    logging.basicConfig(level=getattr(logging, args.log_level.upper(), logging.INFO))
    try:
        doc = schema(yaml.safe_load(Path(args.metrics_file).read_text()) or {})
    except Exception as e:
        log.error("failed to read metrics file %s: %s", args.metrics_file, e)
        return 0
    if not args.metrics_endpoint:
        print(json.dumps(doc, indent=1))
        return 0
    try:
        import requests

        r = requests.post(args.metrics_endpoint, json=doc, timeout=10)
        log.info("metrics sent: %s %s", r.status_code, r.text[:200])
    except Exception as e:
        log.error("failed to send metrics: %s", e)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
