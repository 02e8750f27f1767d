"""Per-node-pool drivers: ``AMDGPUDriver`` objects with ``driver.useDriverCRD``
(api/driver_cr.py, controller/manifests.py state_driver_pools)."""

import os
import time

from amdgpu_operator.api.clusterpolicy import REFERENCE_SET_FLAGS, deep_merge, parse_set_flags
from amdgpu_operator.api.driver_cr import amdgpu_driver
from amdgpu_operator.controller.reconciler import CP_API
from amdgpu_operator.helm import render as H
from amdgpu_operator.helm.crd import crd_yaml
from amdgpu_operator.testing.simcluster import NodeSpec, SimCluster

REF = parse_set_flags(REFERENCE_SET_FLAGS)


def test_driver_crd_file_is_generated_from_spec():
    with open(os.path.join(H.CHART_DIR, "crds", "amd.com_amdgpudrivers.yaml")) as f:
        assert f.read() == crd_yaml("driver"), "run python -m amdgpu_operator.helm.crd driver > .../amd.com_amdgpudrivers.yaml"


def _wait(pred, timeout=30.0):
    deadline = time.time() + timeout
    while time.time() < deadline:
        if pred():
            return True
        time.sleep(0.05)
    return False


def test_driver_pools_deploy_per_selector_and_report_conflicts(tmp_path):
    c = SimCluster(str(tmp_path / "c"), [NodeSpec("gpu-a", 1), NodeSpec("gpu-b", 1), NodeSpec("gpu-c", 1)],
                   fake_gpu=True).start()
    try:
        for node, pool in (("gpu-a", "canary"), ("gpu-b", "main"), ("gpu-c", "main")):
            c.client.patch("v1", "Node", node, {"metadata": {"labels": {"pool": pool}}})
        c.client.create(amdgpu_driver("canary", {"nodeSelector": {"pool": "canary"}, "driverVersion": "6.14.0"}))
        c.client.create(amdgpu_driver("main", {"nodeSelector": {"pool": "main"}}))
        c.install_operator(deep_merge(REF, {"driver": {"useDriverCRD": True}}))
        c.wait_ready(60, {"gpu-a": 1, "gpu-b": 1, "gpu-c": 1})
        pods = {p["spec"]["nodeName"]: p for p in c.pods(c.namespace)
                if p["metadata"]["name"].startswith("amd-driver-daemonset-")}
        assert pods["gpu-a"]["metadata"]["name"].startswith("amd-driver-daemonset-canary-")
        assert pods["gpu-b"]["metadata"]["name"].startswith("amd-driver-daemonset-main-")
        env = {e["name"]: e.get("value") for e in pods["gpu-a"]["spec"]["containers"][0]["env"]}
        assert env["AMDGPU_DRIVER_VERSION"] == "6.14.0"
        assert "amd-driver-daemonset" not in {d["metadata"]["name"] for d in c.client.list("apps/v1", "DaemonSet")}
        assert _wait(lambda: (c.client.get(CP_API, "AMDGPUDriver", "main").get("status") or {}).get("state") == "ready")
        st = c.client.get(CP_API, "AMDGPUDriver", "main")["status"]
        assert st["nodes"] == ["gpu-b", "gpu-c"] and st["nodeCount"] == 2
        # a catch-all pool overlaps both: every object touching a contested node reports it
        c.client.create(amdgpu_driver("everything", {}))
        assert _wait(lambda: (c.client.get(CP_API, "AMDGPUDriver", "everything").get("status") or {}).get(
            "state") == "error")
        assert "more than one AMDGPUDriver" in c.client.get(CP_API, "AMDGPUDriver", "main")["status"]["message"]
        assert _wait(lambda: (c.policy().get("status") or {}).get("state") == "notReady")
        c.client.delete(CP_API, "AMDGPUDriver", "everything")
        assert _wait(lambda: (c.policy().get("status") or {}).get("state") == "ready")
        # deleting a pool removes its DaemonSet (owner reference)
        c.client.delete(CP_API, "AMDGPUDriver", "canary")
        assert _wait(lambda: "amd-driver-daemonset-canary" not in {
            d["metadata"]["name"] for d in c.client.list("apps/v1", "DaemonSet")})
    finally:
        c.stop()
