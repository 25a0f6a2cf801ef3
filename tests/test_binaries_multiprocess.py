"""The nos-amd binaries as separate processes over the wire (the reference's
kind-cluster flow): API server, operator, scheduler, gpupartitioner, a
simulated cumask node (kubelet + device plugin + PodResources socket) and the
gpuagent reading it over gRPC.  A pending ``amd.com/gpu-10gb`` pod must be
planned, realised by the device plugin, handshaken by the gpuagent and end
Running with a CU mask."""
from __future__ import annotations

import os
import socket
import subprocess
import sys
import time
from pathlib import Path

import pytest
import yaml

from nos_amd.api import constants as C
from nos_amd.api import v1alpha1
from nos_amd.kube import factory as kf
from nos_amd.kube import objects as ko
from nos_amd.kube.client import KubeClient

REPO = Path(__file__).resolve().parent.parent


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _wait(pred, timeout: float, procs=()) -> bool:
    end = time.time() + timeout
    while time.time() < end:
        for p in procs:
            if p.poll() is not None:
                raise RuntimeError(f"process {p.args} exited with {p.returncode}")
        try:
            if pred():
                return True
        except Exception:
            pass
        time.sleep(0.2)
    return False


@pytest.mark.timeout(120)
def test_cumask_flow_across_processes(tmp_path):
    port = _free_port()
    url = f"http://127.0.0.1:{port}"
    env = dict(os.environ, PYTHONPATH=str(REPO), NODE_NAME="node-0")
    common = ["--api-server", url, "--health-probe-bind-address", "0", "--metrics-bind-address", "0"]
    gp_cfg = tmp_path / "gp.yaml"
    gp_cfg.write_text(yaml.safe_dump({"kind": "GpuPartitionerConfig", "batchWindowTimeoutSeconds": 2,
                                      "batchWindowIdleSeconds": 0.5, "devicePluginDelaySeconds": 0.2}))
    ga_cfg = tmp_path / "ga.yaml"
    ga_cfg.write_text(yaml.safe_dump({"kind": "GpuAgentConfig", "reportConfigIntervalSeconds": 1,
                                      "probeEnabled": False}))
    sock = tmp_path / "kubelet.sock"
    cmds = [
        ["nos_amd.cmd.apiserver", "--port", str(port)],
        ["nos_amd.cmd.operator", *common],
        ["nos_amd.cmd.scheduler", *common],
        ["nos_amd.cmd.gpupartitioner", "--config", str(gp_cfg), *common],
        ["nos_amd.cmd.simnode", "--name", "node-0", "--kind", "cumask", "--gpus", "2",
         "--podresources-socket", str(sock), *common],
        ["nos_amd.cmd.gpuagent", "--config", str(ga_cfg), "--fake-gpus", "2",
         "--podresources-socket", str(sock), *common],
    ]
    procs: list[subprocess.Popen] = []
    logs = []
    try:
        for i, c in enumerate(cmds):
            log = open(tmp_path / f"p{i}.log", "w")
            logs.append(log)
            procs.append(subprocess.Popen([sys.executable, "-m", *c], env=env, stdout=log, stderr=subprocess.STDOUT))
            if i == 0:
                assert _wait(lambda: KubeClient(url).list("Namespace") is not None, 30, procs)
            if i == 4:
                assert _wait(sock.exists, 30, procs)
        api = KubeClient(url)
        assert _wait(lambda: ko.labels(api.get("Node", "node-0")).get(C.LABEL_AMD_COUNT) == "2", 30, procs)
        c = kf.build_container("main").with_cpu_milli_request(100).with_requests({"amd.com/gpu-10gb": 1}) \
            .with_limits({"amd.com/gpu-10gb": 1}).get()
        api.create(kf.build_pod("default", "yolos").with_container(c).with_scheduler_name("nos-scheduler")
                   .with_phase(ko.PENDING).get())
        assert _wait(lambda: ko.pod_phase(api.get("Pod", "yolos", "default")) == ko.RUNNING, 60, procs), \
            (tmp_path / "p3.log").read_text()[-3000:]
        ann = ko.annotations(api.get("Node", "node-0"))
        assert ann.get("nos.nebuly.com/spec-gpu-0-10gb") == "1"
        # the gpuagent process saw the slice through PodResources gRPC and closed the plan handshake
        assert _wait(lambda: ko.annotations(api.get("Node", "node-0")).get(C.ANNOTATION_REPORTED_PARTITIONING_PLAN)
                     == ann[C.ANNOTATION_PARTITIONING_PLAN], 30, procs)
        assert _wait(lambda: ko.annotations(api.get("Node", "node-0")).get(
            "nos.nebuly.com/status-gpu-0-10gb-used") == "1", 30, procs)
        # the operator labels quota usage: no quota here, but webhooks are enforced by the API server
        api.create(kf.build_namespace("team").get())
        api.create(v1alpha1.build_eq("team", "q").with_min({"cpu": "1"}).get())
        with pytest.raises(Exception):
            api.create(v1alpha1.build_eq("team", "q2").with_min({"cpu": "1"}).get())
    finally:
        for p in reversed(procs):
            p.terminate()
        for p in reversed(procs):
            try:
                p.wait(timeout=10)
            except subprocess.TimeoutExpired:
                p.kill()
        for log in logs:
            log.close()


@pytest.mark.timeout(90)
def test_partition_agent_binary_reports_over_the_wire(tmp_path):
    """The partition agent as its own process (NODE_NAME, --fake-gpus, PodResources
    over gRPC from a simulated node): it labels the node with the amd-smi GPU
    facts and publishes the partition status annotations the gpupartitioner
    plans from."""
    port = _free_port()
    url = f"http://127.0.0.1:{port}"
    env = dict(os.environ, PYTHONPATH=str(REPO), NODE_NAME="node-p")
    common = ["--api-server", url, "--health-probe-bind-address", "0", "--metrics-bind-address", "0"]
    pa_cfg = tmp_path / "pa.yaml"
    pa_cfg.write_text(yaml.safe_dump({"kind": "PartitionAgentConfig", "reportConfigIntervalSeconds": 1}))
    sock = tmp_path / "kubelet.sock"
    cmds = [
        ["nos_amd.cmd.apiserver", "--port", str(port)],
        ["nos_amd.cmd.simnode", "--name", "node-p", "--kind", "partition", "--gpus", "2",
         "--podresources-socket", str(sock), *common],
        ["nos_amd.cmd.partagent", "--config", str(pa_cfg), "--fake-gpus", "2", "--no-device-plugin-restart",
         "--podresources-socket", str(sock), *common],
    ]
    procs: list[subprocess.Popen] = []
    logs = []
    try:
        for i, c in enumerate(cmds):
            log = open(tmp_path / f"p{i}.log", "w")
            logs.append(log)
            procs.append(subprocess.Popen([sys.executable, "-m", *c], env=env, stdout=log, stderr=subprocess.STDOUT))
            if i == 0:
                assert _wait(lambda: KubeClient(url).list("Namespace") is not None, 30, procs)
            if i == 1:
                assert _wait(sock.exists, 30, procs)
        api = KubeClient(url)

        def reported():
            n = api.get("Node", "node-p")
            ann = ko.annotations(n)
            return (ko.labels(n).get(C.LABEL_AMD_COUNT) == "2"
                    and any(k.startswith("nos.nebuly.com/status-gpu-0-") for k in ann)
                    and any(k.startswith("nos.nebuly.com/status-gpu-1-") for k in ann))
        assert _wait(reported, 40, procs), (tmp_path / "p2.log").read_text()[-3000:]
    finally:
        for p in reversed(procs):
            p.terminate()
        for p in reversed(procs):
            try:
                p.wait(timeout=10)
            except subprocess.TimeoutExpired:
                p.kill()
        for log in logs:
            log.close()
