"""Sandbox workloads (VM passthrough): vfio-manager binding on a fake PCI
tree, the sandbox device plugin over the kubelet gRPC contract, operand
selection by amd.com/gpu.workload.config, and a simulated cluster with a
container node next to a vm-passthrough node."""

import os
import threading
import time

import pytest

from amdgpu_operator.api.clusterpolicy import (REFERENCE_SET_FLAGS, ClusterPolicySpec, cluster_policy, deep_merge,
                                               parse_set_flags)
from amdgpu_operator.controller.manifests import STATE_BUILDERS
from amdgpu_operator.controller.nodes import desired_labels
from amdgpu_operator.controller.reconciler import ClusterPolicyReconciler
from amdgpu_operator.deviceplugin import api
from amdgpu_operator.deviceplugin.server import PluginConfig
from amdgpu_operator.kube import resources as R
from amdgpu_operator.kube.client import LocalClient
from amdgpu_operator.kube.fakeapi import FakeApiServer
from amdgpu_operator.sandbox import WORKLOAD_CONFIG_LABEL
from amdgpu_operator.sandbox import vfio as VF
from amdgpu_operator.sandbox.plugin import SandboxPluginManager, kubevirt_env, resource_name
from amdgpu_operator.testing import fakesys
from amdgpu_operator.testing.fakekubelet import FakeKubelet

GPU_LABEL = {"feature.node.kubernetes.io/pci-1200_1002.present": "true"}
SANDBOX = {"sandboxWorkloads": {"enabled": True}}


@pytest.fixture
def tree(tmp_path):
    root = str(tmp_path / "host")
    fakesys.build_node(root, 4)
    return root, fakesys.FakePciKernel(root)


def test_bind_all_moves_whole_groups_to_vfio(tree):
    root, k = tree
    gpus = k.gpus()
    assert len(gpus) == 4 and all(g.driver == "amdgpu" and g.iommu_group for g in gpus)
    # a second function in the first GPU's group must follow it; a bridge must not
    grp = gpus[0].iommu_group
    for bdf, cls in (("0000:99:00.1", "0x040300"), ("0000:98:00.0", "0x060400")):
        fakesys._w(f"{root}/sys/bus/pci/devices/{bdf}/vendor", "0x1002\n")
        fakesys._w(f"{root}/sys/bus/pci/devices/{bdf}/class", f"{cls}\n")
        fakesys._link(f"../../../../bus/pci/devices/{bdf}", f"{root}/sys/kernel/iommu_groups/{grp}/devices/{bdf}")
        fakesys._link(f"../../../../kernel/iommu_groups/{grp}", f"{root}/sys/bus/pci/devices/{bdf}/iommu_group")
    res = VF.bind_all(k)
    assert k.modprobes == ["vfio-pci"]  # loaded on first use
    assert all(r.changed and r.driver == VF.VFIO_DRIVER for r in res)
    first = next(r for r in res if r.group == grp)
    assert "0000:99:00.1" in first.functions and "0000:98:00.0" not in first.functions
    assert k.function("0000:99:00.1").driver == "vfio-pci" and k.function("0000:98:00.0").driver is None
    with open(f"{root}/sys/bus/pci/devices/{gpus[1].bdf}/driver_override") as f:
        assert f.read().strip() == "vfio-pci"  # pinned: a rescan cannot hand it back to amdgpu
    ok, msg, detail = VF.check_bound(k)
    assert ok and "4 GPU(s)" in msg and all(d["vfio_dev"] for d in detail)
    assert not any(r.changed for r in VF.bind_all(k))  # idempotent
    back = VF.unbind_all(k)
    assert all(r.driver == "amdgpu" for r in back)
    assert not os.path.exists(k.vfio_dev(grp)) and not VF.check_bound(k)[0]


def test_bind_waits_for_gpu_users_then_fails(tree):
    _, k = tree
    k.set_busy([4242])
    t0 = time.monotonic()
    with pytest.raises(VF.VfioError, match="4242"):
        VF.bind_all(k, timeout=0.2)
    assert time.monotonic() - t0 >= 0.2
    assert all(g.driver == "amdgpu" for g in k.gpus())  # nothing pulled from under the user
    threading.Timer(0.1, k.set_busy, ([],)).start()
    assert len(VF.bind_all(k, timeout=5.0)) == 4


def test_group_viability_query(tree, monkeypatch):
    _, k = tree
    VF.bind_all(k)
    grp = k.gpus()[0].iommu_group
    assert VF.group_viable(k.vfio_dev(grp)) is None  # a regular file in the test tree: not asked
    assert VF.VFIO_GROUP_GET_STATUS == 0x3B67
    monkeypatch.setattr(VF, "group_viable", lambda path: not path.endswith("/" + grp))
    ok, msg, _ = VF.check_bound(k)
    assert not ok and "not viable" in msg and f"group {grp}" in msg


def test_no_iommu_group_is_an_error(tmp_path):
    root = str(tmp_path / "h")
    fakesys.build_node(root, 1)
    k = fakesys.FakePciKernel(root)
    os.unlink(f"{root}/sys/bus/pci/devices/{k.gpus()[0].bdf}/iommu_group")
    with pytest.raises(VF.VfioError, match="IOMMU"):
        VF.bind_all(k)


def test_sandbox_plugin_registers_and_allocates_vfio_groups(tree, tmp_path):
    _, k = tree
    VF.bind_all(k)
    sock_dir = str(tmp_path / "dp")
    kubelet = FakeKubelet(sock_dir)
    kubelet.start()
    cfg = PluginConfig(socket_dir=sock_dir, health_poll_ms=50, watch_interval_s=0.05)
    mgr = SandboxPluginManager(cfg, k)
    mgr.start()
    try:
        res = resource_name(fakesys.MI355X_DEVICE_ID)
        assert res == "amd.com/MI355X" and list(mgr.servers) == [res]
        assert kubelet.wait_registered(res, min_devices=4)
        assert kubelet.allocatable(res) == 4
        ids, c = kubelet.allocate(res, 2)
        bdfs = c.envs[kubevirt_env(res)].split(",")
        assert sorted(bdfs) == sorted(ids) and kubevirt_env(res) == "PCI_RESOURCE_AMD_COM_MI355X"
        paths = [d.host_path for d in c.devices]
        groups = {k.function(b).iommu_group for b in bdfs}
        assert paths[0] == "/dev/vfio/vfio" and sorted(paths[1:]) == sorted(f"/dev/vfio/{g}" for g in groups)
        assert "/dev/kfd" not in paths  # a VM gets the PCI function, not the container compute path
        # the host hands one GPU back to amdgpu: it turns Unhealthy
        bdf = k.gpus()[0].bdf
        k.set_override(bdf, "")
        k.unbind(bdf)
        k.probe(bdf)
        deadline = time.time() + 5
        while time.time() < deadline and kubelet.allocatable(res) != 3:
            time.sleep(0.02)
        assert kubelet.allocatable(res) == 3
    finally:
        mgr.stop()
        kubelet.stop()


def test_workload_config_selects_operands():
    spec = ClusterPolicySpec.model_validate(SANDBOX)
    vm = {"metadata": {"name": "n", "labels": {**GPU_LABEL, WORKLOAD_CONFIG_LABEL: "vm-passthrough"}}}
    p = desired_labels(vm, spec)
    deploy = sorted(k for k, v in p.items() if k.startswith("amd.com/gpu.deploy.") and v == "true")
    assert deploy == ["amd.com/gpu.deploy.sandbox-device-plugin", "amd.com/gpu.deploy.sandbox-validator",
                      "amd.com/gpu.deploy.vfio-manager"]
    ctr = {"metadata": {"name": "c", "labels": dict(GPU_LABEL)}}
    p = desired_labels(ctr, spec)  # default workload: container
    assert p["amd.com/gpu.deploy.driver"] == "true" and "amd.com/gpu.deploy.vfio-manager" not in p
    # without sandbox mode the workload label means nothing
    p = desired_labels(vm, ClusterPolicySpec())
    assert p["amd.com/gpu.deploy.driver"] == "true" and "amd.com/gpu.deploy.vfio-manager" not in p
    # switching a validated container node to vm-passthrough drops its validation
    was = {"metadata": {"name": "s", "labels": {**GPU_LABEL, WORKLOAD_CONFIG_LABEL: "vm-passthrough",
                                                "amd.com/gpu.deploy.driver": "true", "amd.com/gpu.validated": "true"}}}
    p = desired_labels(was, spec)
    assert p["amd.com/gpu.deploy.driver"] is None and p["amd.com/gpu.validated"] is None
    # an unknown value falls back to the default workload
    odd = {"metadata": {"name": "o", "labels": {**GPU_LABEL, WORKLOAD_CONFIG_LABEL: "vm-vgpu"}}}
    assert desired_labels(odd, spec)["amd.com/gpu.deploy.driver"] == "true"


def test_sandbox_states_off_by_default():
    c = LocalClient(FakeApiServer())
    c.create(R.new("v1", "Namespace", "gpu-operator-resources"))
    c.create(R.new("v1", "Node", "gpu-a", labels=GPU_LABEL))
    c.create(cluster_policy(spec=parse_set_flags(REFERENCE_SET_FLAGS)))
    res = ClusterPolicyReconciler(c, "gpu-operator-resources").reconcile()
    states = {r.name: r for r in res.states}
    for s in ("state-vfio-manager", "state-sandbox-validation", "state-sandbox-device-plugin"):
        assert not states[s].enabled
    names = {d["metadata"]["name"] for d in c.list("apps/v1", "DaemonSet", "gpu-operator-resources")}
    assert not names & {"amd-vfio-manager", "amd-sandbox-validator", "amd-sandbox-device-plugin-daemonset"}
    spec = ClusterPolicySpec.model_validate(SANDBOX)
    for s in ("state-vfio-manager", "state-sandbox-validation", "state-sandbox-device-plugin"):
        ds = [o for o in STATE_BUILDERS[s](spec, "ns", []) if o["kind"] == "DaemonSet"][0]
        sel = ds["spec"]["template"]["spec"]["nodeSelector"]
        assert list(sel) == [f"amd.com/gpu.deploy.{s.replace('state-', '').replace('-validation', '-validator')}"]


def test_sim_container_and_passthrough_nodes(tmp_path):
    """One container node and one vm-passthrough node under one ClusterPolicy:
    amd.com/gpu on the first, amd.com/MI355X (vfio) on the second; switching
    the second back returns its GPUs to amdgpu and amd.com/gpu."""
    from amdgpu_operator.testing.simcluster import NodeSpec, SimCluster

    c = SimCluster(str(tmp_path / "c"), [NodeSpec("ctr-0", 2), NodeSpec("vm-0", 2)], fake_gpu=True).start()
    try:
        c.client.patch("v1", "Node", "vm-0", {"metadata": {"labels": {WORKLOAD_CONFIG_LABEL: "vm-passthrough"}}})
        c.install_operator(deep_merge(parse_set_flags(REFERENCE_SET_FLAGS), SANDBOX))
        c.wait_ready(60, {"ctr-0": 2, "vm-0": {"amd.com/MI355X": 2}})
        vm = c.nodes["vm-0"]
        k = vm.env.extra["pci_backend"]
        assert all(g.driver == "vfio-pci" for g in k.gpus())
        assert all(g.driver == "amdgpu" for g in c.nodes["ctr-0"].env.extra["pci_backend"].gpus())
        pods = {p["metadata"]["name"].rsplit("-", 1)[0] for p in c.pods() if p["spec"].get("nodeName") == "vm-0"}
        assert "amd-vfio-manager" in pods and "amd-driver-daemonset" not in pods
        alloc = c.client.get("v1", "Node", "vm-0")["status"]["allocatable"]
        assert int(alloc.get("amd.com/gpu", "0")) == 0
        from amdgpu_operator.cli.verify import verify

        rep = verify(c.client, c.namespace, 2)  # the reference's checks pass on a mixed cluster
        assert rep.ok, rep.table()
        assert "vm-passthrough amd.com/<product>=2" in next(x.detail for x in rep.checks if x.name == "allocatable[vm-0]")
        # back to containers: GPUs return to amdgpu, the container path validates the node again
        c.client.patch("v1", "Node", "vm-0", {"metadata": {"labels": {WORKLOAD_CONFIG_LABEL: "container"}}})
        deadline = time.time() + 60
        while time.time() < deadline and not all(g.driver == "amdgpu" for g in k.gpus()):
            time.sleep(0.05)
        assert all(g.driver == "amdgpu" for g in k.gpus())
        c.wait_ready(60, {"ctr-0": 2, "vm-0": 2})
    finally:
        c.stop()


def test_device_plugin_api_constants():
    assert api.VERSION == "v1beta1"
