"""Device-plugin configuration watcher (the NVIDIA ``config-manager`` sidecar
role).

The cumask partitioner writes ``<node>-<planId>`` into the device-plugin
ConfigMap and points the node label ``nos.nebuly.com/device-plugin.config``
at it (``mps/partitioner.go:61-111``).  This controller follows that label:
when it (or the referenced ConfigMap entry) changes it loads the entry into
the plugin, which re-advertises its slices without a restart.
"""
from __future__ import annotations

import logging

from ..api import constants as C
from ..kube import objects as ko
from ..partitioning.strategies import DevicePluginConfigRef
from ..runtime.manager import Controller, Request, Result
from ..runtime.predicates import ExcludeDelete, MatchingName
from .plugin import NosAmdDevicePlugin

log = logging.getLogger("nos_amd.deviceplugin.config")


class ConfigWatcher:
    def __init__(self, api, node_name: str, plugin: NosAmdDevicePlugin, cm_ref: DevicePluginConfigRef | None = None):
        self.api, self.node_name, self.plugin = api, node_name, plugin
        self.cm_ref = cm_ref or DevicePluginConfigRef()
        self.loads = 0

    def reconcile(self, req: Request | None) -> Result:
        node = self.api.try_get("Node", self.node_name)
        if node is None or self.plugin.mode not in (C.PARTITIONING_CUMASK, C.PARTITIONING_HYBRID):
            return Result()
        key = ko.labels(node).get(C.LABEL_DEVICE_PLUGIN_CONFIG)
        if not key:
            return Result()
        cmap = self.api.try_get("ConfigMap", self.cm_ref.name, self.cm_ref.namespace)
        data = (cmap or {}).get("data") or {}
        if key not in data:
            log.info("node %s: config %s not (yet) in ConfigMap %s/%s", self.node_name, key, self.cm_ref.namespace,
                     self.cm_ref.name)
            return Result(requeue_after=1.0)
        if key == self.plugin.config_key and self.plugin.config is not None:
            return Result()
        self.plugin.set_config(key, data[key])
        self.loads += 1
        log.info("node %s: device plugin loaded config %s", self.node_name, key)
        return Result()

    def _map_cm(self, cm: dict) -> list[Request]:
        if ko.name(cm) == self.cm_ref.name and ko.namespace(cm) == self.cm_ref.namespace:
            return [Request(self.node_name, "")]
        return []

    def controller(self) -> Controller:
        return (Controller(f"dp-config-{self.node_name}", self)
                .for_kind("Node", ExcludeDelete(), MatchingName(self.node_name))
                .watches("ConfigMap", self._map_cm, ExcludeDelete(), namespace=self.cm_ref.namespace))
