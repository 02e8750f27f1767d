"""Partition manager on a fake MI355X node (partition/manager.py): the
device must be idle - GPU pods gone, the node's own amd-smi/KFD clients
(device plugin, metrics exporter, validator) paused - before amd-smi may
change a partition, and a memory-partition (NPS) change goes through the
driver container's amdgpu reload."""

import os
import threading
import time

import pytest

from amdgpu_operator.driver import manager as DM
from amdgpu_operator.kube import resources as R
from amdgpu_operator.kube.client import LocalClient
from amdgpu_operator.kube.fakeapi import FakeApiServer
from amdgpu_operator.nodeenv import NodeEnv
from amdgpu_operator.partition import manager as PM
from amdgpu_operator.testing import fakesys

NS = "gpu-operator-resources"
PROFILES = {"all-spx": {"compute": "SPX", "memory": "NPS1"}, "all-cpx": {"compute": "CPX", "memory": "NPS2"},
            "all-qpx": {"compute": "QPX", "memory": "NPS1"}}
DEFAULT = PM.Profile("SPX", "NPS1")


def _pod(name, app=None, gpu=False):
    ctr = {"name": "c", "image": "x"}
    if gpu:
        ctr["resources"] = {"limits": {"amd.com/gpu": "1"}}
    return {"apiVersion": "v1", "kind": "Pod",
            "metadata": {"name": name, "namespace": NS, "labels": {"app": app} if app else {}},
            "spec": {"nodeName": "n1", "containers": [ctr]}}


@pytest.fixture
def node(tmp_path):
    root = str(tmp_path / "host")
    fakesys.build_node(root, 2)
    c = LocalClient(FakeApiServer())
    c.create(R.new("v1", "Namespace", NS))
    n = R.new("v1", "Node", "n1")
    n["metadata"]["labels"] = {PM._deploy_label(o): "true" for o in PM.PAUSE_OPERANDS}
    c.create(n)
    env = NodeEnv("n1", c, host_root=root, validations_dir=str(tmp_path / "val"), namespace=NS, poll_s=0.01)
    env.extra["kmod"] = fakesys.SimModule(root)
    for app in ("amd-device-plugin-daemonset", "amd-metrics-exporter", "amd-operator-validator"):
        c.create(_pod(f"{app}-x", app))
    c.create(_pod("workload", gpu=True))
    return env


class NodeAgents:
    """What the DaemonSet controller + kubelet + driver container do on the
    node meanwhile: a paused operand's pod goes (and its KFD handle with it,
    unless ``lingering``), and the driver container serves reload requests."""

    def __init__(self, env, lingering=()):
        self.env, self.lingering = env, set(lingering)
        self.stop = threading.Event()
        self.procs = os.path.join(env.sysfs_root(), "sys/class/kfd/kfd/proc")
        os.makedirs(self.procs, exist_ok=True)
        self.pids = {"amd-device-plugin-daemonset": "701", "amd-metrics-exporter": "702"}
        for pid in self.pids.values():
            os.makedirs(os.path.join(self.procs, pid))
        self.threads = [threading.Thread(target=self._ds, daemon=True),
                        threading.Thread(target=DM.serve_reload_requests, args=(env, self.stop, {}), daemon=True)]

    def _ds(self):
        c = self.env.client
        while not self.stop.wait(0.01):
            labels = c.get("v1", "Node", "n1")["metadata"].get("labels") or {}
            for op in PM.PAUSE_OPERANDS:
                if labels.get(PM._deploy_label(op)) != PM.PAUSED:
                    continue
                app = PM._app(op)
                for p in c.list("v1", "Pod", NS, label_selector=f"app={app}"):
                    c.delete("v1", "Pod", p["metadata"]["name"], NS)
                pid = self.pids.get(app)
                if pid and app not in self.lingering and os.path.isdir(os.path.join(self.procs, pid)):
                    os.rmdir(os.path.join(self.procs, pid))

    def __enter__(self):
        for th in self.threads:
            th.start()
        return self

    def __exit__(self, *exc):
        self.stop.set()
        for th in self.threads:
            th.join(5)


def _label(env, key):
    return (env.client.get("v1", "Node", "n1")["metadata"].get("labels") or {}).get(key)


def _modes(env):
    from amdgpu_operator.discovery import topology

    return {(g.compute_partition, g.memory_partition) for g in topology.enumerate_gpus(env.sysfs_root())}


def test_mi355x_profiles_only():
    PM.Profile("CPX", "NPS2").validate()
    PM.Profile("QPX", "NPS1").validate()
    for bad in (("TPX", "NPS1"), ("CPX", "NPS4"), ("QPX", "NPS8"), ("SPX", "NPS2")):
        with pytest.raises(ValueError):
            PM.Profile(*bad).validate()


def test_busy_backend_refuses_while_kfd_users_exist(node):
    be = PM.SysfsBackend(node.host_root, PM.sysfs_partition_rebuilder(node.host_root, 2))
    os.makedirs(os.path.join(node.host_root, "sys/class/kfd/kfd/proc/999"))
    with pytest.raises(PM.PartitionBusy):
        be.apply(0, PM.Profile("QPX", "NPS1"))
    os.rmdir(os.path.join(node.host_root, "sys/class/kfd/kfd/proc/999"))
    be.apply(0, PM.Profile("QPX", "NPS1"))
    assert _modes(node) == {("QPX", "NPS1")}


def test_lingering_exporter_refuses_the_change_and_restores_the_node(node):
    be = PM.SysfsBackend(node.host_root, PM.sysfs_partition_rebuilder(node.host_root, 2))
    node.client.patch("v1", "Node", "n1", {"metadata": {"labels": {"amd.com/gpu.partition-config": "all-qpx"}}})
    with NodeAgents(node, lingering={"amd-metrics-exporter"}):
        res = PM.reconcile_node(node, be, PROFILES, DEFAULT, timeout=1.0)
    assert not res["changed"] and "702" in res["error"]
    assert _label(node, PM.STATE_LABEL) == "failed" and _modes(node) == {("SPX", "NPS1")}
    assert all(_label(node, PM._deploy_label(o)) == "true" for o in PM.PAUSE_OPERANDS)  # operands back


def test_compute_change_after_the_clients_stopped(node):
    be = PM.SysfsBackend(node.host_root, PM.sysfs_partition_rebuilder(node.host_root, 2))
    node.client.patch("v1", "Node", "n1", {"metadata": {"labels": {"amd.com/gpu.partition-config": "all-qpx"}}})
    with NodeAgents(node):
        res = PM.reconcile_node(node, be, PROFILES, DEFAULT, timeout=10.0)
    assert res["changed"] and not res["driver_reloaded"], res
    assert set(res["paused"]) == set(PM.PAUSE_OPERANDS) and res["evicted"] == [f"{NS}/workload"]
    assert _modes(node) == {("QPX", "NPS1")} and _label(node, PM.APPLIED_LABEL) == "all-qpx"
    assert all(_label(node, PM._deploy_label(o)) == "true" for o in PM.PAUSE_OPERANDS)
    assert node.extra["kmod"].log == []  # no reload for a compute-only change


def test_memory_partition_change_goes_through_the_driver_reload(node):
    be = PM.SysfsBackend(node.host_root, PM.sysfs_partition_rebuilder(node.host_root, 2))
    DM.install(node, timeout=5)
    node.client.patch("v1", "Node", "n1", {"metadata": {"labels": {"amd.com/gpu.partition-config": "all-cpx"}}})
    t0 = time.time()
    with NodeAgents(node):
        res = PM.reconcile_node(node, be, PROFILES, DEFAULT, timeout=10.0)
    assert res["changed"] and res["driver_reloaded"], res
    assert _modes(node) == {("CPX", "NPS2")}
    kmod = node.extra["kmod"]
    assert kmod.log[:2] == ["unload", "partition CPX/NPS2"]  # the new NPS mode came with the module load
    from amdgpu_operator.validator.validate import read_ready

    assert read_ready(node, "driver")["time"] >= t0 and read_ready(node, "driver")["gpus"] == 16
    assert not os.path.exists(node.validation_file(PM.RELOAD_REQUEST))


def test_memory_change_without_a_driver_container_fails_cleanly(node):
    be = PM.SysfsBackend(node.host_root, PM.sysfs_partition_rebuilder(node.host_root, 2))
    node.client.patch("v1", "Node", "n1", {"metadata": {"labels": {"amd.com/gpu.partition-config": "all-cpx"}}})
    agents = NodeAgents(node)
    agents.threads = agents.threads[:1]  # no driver container on the node
    with agents:
        res = PM.reconcile_node(node, be, PROFILES, DEFAULT, timeout=0.5)
    assert not res["changed"] and "did not reload" in res["error"]
    assert _label(node, PM.STATE_LABEL) == "failed"
    assert all(_label(node, PM._deploy_label(o)) == "true" for o in PM.PAUSE_OPERANDS)


def test_apply_waits_for_a_driver_health_amd_smi_poll(node):
    """amd-driver-health is not paused for a change (it watches the driver
    through the reload) and opens amd-smi every minute.  A poll under way
    when the change starts makes the device BUSY; the change holds further
    polls off (.smi-hold) and applies once the running one has ended."""
    from amdgpu_operator.utils import smihold

    be = PM.SysfsBackend(node.host_root, PM.sysfs_partition_rebuilder(node.host_root, 2),
                         validations_dir=node.validations_dir)
    node.client.patch("v1", "Node", "n1", {"metadata": {"labels": {"amd.com/gpu.partition-config": "all-qpx"}}})
    in_poll, ended = threading.Event(), []

    def poll():  # driver/manager.py publish_smi: one slow amd-smi session
        with smihold.client(node.validations_dir) as allowed:
            assert allowed
            in_poll.set()
            time.sleep(0.4)
            ended.append(time.monotonic())

    th = threading.Thread(target=poll)
    th.start()
    in_poll.wait(5)
    with pytest.raises(PM.PartitionBusy, match="amd-smi clients"):  # the race the hold-off prevents
        be.apply(0, PM.Profile("QPX", "NPS1"))
    applied = []
    real_apply = be.apply
    be.apply = lambda p, prof: (applied.append(time.monotonic()), real_apply(p, prof))[1]
    skipped = []

    def later_polls():  # polls that start during the change are skipped, not raced
        while not ended:
            time.sleep(0.01)
        with smihold.client(node.validations_dir) as allowed:
            skipped.append(not allowed)

    th2 = threading.Thread(target=later_polls)
    th2.start()
    with NodeAgents(node):
        res = PM.reconcile_node(node, be, PROFILES, DEFAULT, timeout=10.0)
    th.join()
    th2.join()
    assert res["changed"], res
    assert applied and ended and min(applied) >= ended[0]  # applied only after the poll let go
    assert skipped == [True]
    assert _modes(node) == {("QPX", "NPS1")} and not smihold.held(node.validations_dir)


def test_publish_smi_skips_its_poll_while_held(node):
    from amdgpu_operator.utils import smihold

    node.extra["_smi_published"] = ("ok: earlier", 0.0)
    smihold.hold(node.validations_dir, "partition test")
    assert DM.publish_smi(node, True, refresh_s=0.0) == "ok: earlier"  # no amd-smi session opened
    smihold.release(node.validations_dir)


def test_failed_unload_during_a_reload_restores_driver_ready(node, monkeypatch):
    """a reload whose unload fails (amdgpu still in use) must not
    leave the node's operands gated on a driver-ready that never comes: the
    module is still live, so driver-ready is written again at once (and the
    loss marker leaves the recovery to the health monitor otherwise)."""
    from amdgpu_operator.validator.validate import read_ready

    DM.install(node, timeout=5)
    kmod = node.extra["kmod"]

    def busy_unload(env=None, timeout=0.0):
        raise RuntimeError("rmmod: amdgpu in use")

    monkeypatch.setattr(kmod, "unload", busy_unload)
    t0 = time.time()
    with pytest.raises(RuntimeError, match="in use"):
        DM.reload_module(node, {}, "memory partition NPS2")
    ready = read_ready(node, "driver")
    assert ready and ready["time"] >= t0 and ready.get("recovered")
    assert not os.path.exists(node.validation_file(DM.LOST_MARKER))  # claimed by the recovery


def _dra_pod(name, claim, with_ref=True):
    ctr = {"name": "c", "image": "x", "resources": {"claims": [{"name": "g"}]} if with_ref else {}}
    return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": NS},
            "spec": {"nodeName": "n1", "resourceClaims": [{"name": "g", "resourceClaimName": claim}],
                     "containers": [ctr]}}


def _alloc_claim(c, name, driver):
    claim = c.create({"apiVersion": "resource.k8s.io/v1beta1", "kind": "ResourceClaim",
                      "metadata": {"name": name, "namespace": NS},
                      "spec": {"devices": {"requests": [{"name": "g", "deviceClassName": driver}]}}})
    claim["status"] = {"allocation": {"devices": {"results": [
        {"request": "g", "driver": driver, "pool": "n1", "device": "gpu-0"}]}}}
    c.update_status(claim)


def test_dra_claim_holders_are_gpu_pods(node):
    """with the DRA driver the node's GPUs are held through
    ResourceClaims, not amd.com/gpu limits.  A partition change evicts (and
    waits for) those pods too; a pod whose claim another DRA driver (a NIC's)
    allocated, or that names no claim in any container, stays."""
    from amdgpu_operator.wellknown import uses_gpu

    c = node.client
    _alloc_claim(c, "gpu-claim", "gpu.amd.com")
    _alloc_claim(c, "nic-claim", "rdma.example.com")
    c.create(_dra_pod("dra-gpu", "gpu-claim"))
    c.create(_dra_pod("dra-nic", "nic-claim"))
    c.create(_dra_pod("dra-unreferenced", "gpu-claim", with_ref=False))
    c.create(_dra_pod("dra-pending", "not-yet"))  # its claim is not there yet: counts (safe side)
    assert uses_gpu(c.get("v1", "Pod", "dra-gpu", NS)) and uses_gpu(c.get("v1", "Pod", "dra-nic", NS))  # no lookup
    evicted = PM.evict_gpu_pods(node)
    assert sorted(evicted) == sorted(f"{NS}/{n}" for n in ("workload", "dra-gpu", "dra-pending")), evicted
    left = {p["metadata"]["name"] for p in c.list("v1", "Pod", NS)}
    assert {"dra-nic", "dra-unreferenced"} <= left and not {"dra-gpu", "workload"} & left
    assert PM.wait_gpu_pods_gone(node, 1.0)


def test_driver_upgrade_drains_dra_claim_holders():
    """The driver upgrade's drain lists a gpu.amd.com claim holder as a GPU
    pod (an amdgpu unload would find the module busy under it)."""
    from amdgpu_operator.controller import upgrade as U

    c = LocalClient(FakeApiServer())
    c.create(R.new("v1", "Namespace", NS))
    c.create(R.new("v1", "Node", "n1"))
    _alloc_claim(c, "gpu-claim", "gpu.amd.com")
    _alloc_claim(c, "nic-claim", "rdma.example.com")
    c.create(_dra_pod("dra-gpu", "gpu-claim"))
    c.create(_dra_pod("dra-nic", "nic-claim"))
    c.create(_pod("plugin-pod", gpu=True))
    ctl = U.DriverUpgradeController(c, NS)
    assert sorted(p["metadata"]["name"] for p in ctl._gpu_pods("n1")) == ["dra-gpu", "plugin-pod"]
