"""Device-plugin restart after a repartition (``pkg/gpu/client.go:51-135``).

When the partition agent switches a GPU's compute/memory mode, the device
plugin of that node must re-enumerate.  The plugin's own amd-smi session
only sees the new partitions after it re-enumerates (``nos_smi_rescan``,
which the deployed plugin runs every ``rescanSeconds``); restarting it is the
immediate, reference-compatible path: delete the plugin pod on this node
(label ``app=nos-amd-device-plugin``) and wait until its replacement is
Running (5 s poll, 1 min timeout).
"""
from __future__ import annotations

import logging
import time

from ..api import constants as C
from ..kube import objects as ko

log = logging.getLogger("nos_amd.agents.dpclient")


class DevicePluginClient:
    def __init__(self, api, node_name: str, namespace: str = "nos-system",
                 label: tuple[str, str] = C.DEFAULT_DEVICE_PLUGIN_DS_LABEL, poll_s: float = 5.0,
                 timeout_s: float = 60.0):
        self.api, self.node_name, self.namespace = api, node_name, namespace
        self.selector = f"{label[0]}={label[1]}"
        self.poll_s, self.timeout_s = poll_s, timeout_s

    def _pods(self) -> list[dict]:
        return self.api.list("Pod", self.namespace, label_selector=self.selector,
                             field_selector=f"{C.POD_NODE_NAME_KEY}={self.node_name}")

    def restart(self) -> None:
        old = {ko.uid(p) for p in self._pods()}
        for p in self._pods():
            self.api.delete("Pod", ko.name(p), ko.namespace(p))
        self.wait_until_running(exclude=old)

    def wait_until_running(self, exclude: set[str] = frozenset()) -> None:
        deadline = time.monotonic() + self.timeout_s
        while time.monotonic() < deadline:
            for p in self._pods():
                if ko.uid(p) not in exclude and ko.pod_phase(p) == ko.RUNNING:
                    return
            time.sleep(self.poll_s)
        raise TimeoutError(f"device plugin pod on {self.node_name} not Running after {self.timeout_s}s")

    # the partition actuator calls refresh() on its device plugins after a switch
    def refresh(self) -> None:
        try:
            self.restart()
        except Exception as e:
            log.error("device plugin restart on %s failed: %s", self.node_name, e)
