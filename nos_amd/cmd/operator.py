"""nos-amd operator (``cmd/operator/operator.go:50-126``): the ElasticQuota
and CompositeElasticQuota reconcilers + their validating webhooks.

python -m nos_amd.cmd.operator --config operator_config.yaml [--api-server URL]
"""
from __future__ import annotations

import logging

from . import common

log = logging.getLogger("nos_amd.cmd.operator")


def build(api, cfg):
    from ..controllers.elasticquota import CompositeElasticQuotaReconciler, ElasticQuotaReconciler

    mgr = common.manager_for(api, "nos-operator", cfg)
    mgr.add(ElasticQuotaReconciler(api, cfg.amd_gpu_resource_memory_gb).controller())
    mgr.add(CompositeElasticQuotaReconciler(api, cfg.amd_gpu_resource_memory_gb).controller())
    return mgr


def main(argv=None) -> int:
    ap = common.parser(__doc__.splitlines()[0])
    ap.add_argument("--webhook-port", type=int, default=0, help="serve the validating webhooks (0: off)")
    ap.add_argument("--webhook-cert-dir", default="", help="dir with tls.crt/tls.key")
    args = ap.parse_args(argv)
    cfg = common.load_config(args.config, "OperatorConfig")
    common.apply_overrides(cfg, args)
    api = common.connect(args)
    mgr = build(api, cfg)
    port = args.webhook_port  # in-cluster: cfg.webhook.port (9443) behind the ValidatingWebhookConfiguration
    if port:
        from ..api.webhook_server import WebhookServer

        WebhookServer(api, port=port, cert_dir=args.webhook_cert_dir or None).start()
        log.info("webhooks on :%d", port)
    common.serve_health(cfg.health.health_probe_bind_address, mgr.healthz, mgr.readyz)
    common.serve_metrics(cfg.metrics.bind_address)
    mgr.start()
    log.info("operator started")
    return common.run_until_signal(mgr.stop, mgr.lost_leadership)


if __name__ == "__main__":
    raise SystemExit(main())
