"""Cluster-wide driver upgrade (controller/upgrade.py): a driver spec change on
a running cluster walks the GPU nodes through cordon -> GPU-pod eviction ->
driver pod restart -> revalidation -> uncordon, at most
``maxParallelUpgrades`` nodes at a time (SURVEY.md §5.3 recovery tier)."""

import os
import time

import pytest

from amdgpu_operator.api.clusterpolicy import REFERENCE_SET_FLAGS, ClusterPolicySpec, deep_merge, parse_set_flags
from amdgpu_operator.controller import manifests as M
from amdgpu_operator.controller import upgrade as U
from amdgpu_operator.kube import resources as R
from amdgpu_operator.kube.client import LocalClient
from amdgpu_operator.kube.fakeapi import FakeApiServer
from amdgpu_operator.testing.simcluster import NodeSpec, SimCluster
from amdgpu_operator.validator.validate import VALIDATED_LABEL

REF = parse_set_flags(REFERENCE_SET_FLAGS)


def test_driver_daemonset_is_ondelete_with_spec_hash():
    spec = ClusterPolicySpec.model_validate(REF)
    ds = [o for o in M.state_driver(spec, "ns", None) if o["kind"] == "DaemonSet"][0]
    assert ds["spec"]["updateStrategy"] == {"type": "OnDelete"}
    assert ds["spec"]["template"]["metadata"]["labels"][U.HASH_LABEL] == U.driver_spec_hash(spec)
    other = ClusterPolicySpec.model_validate(deep_merge(REF, {"driver": {"driverVersion": "6.14.0"}}))
    assert U.driver_spec_hash(other) != U.driver_spec_hash(spec)
    manual = ClusterPolicySpec.model_validate(deep_merge(REF, {"driver": {"upgradePolicy": {"autoUpgrade": False}}}))
    ds = [o for o in M.state_driver(manual, "ns", None) if o["kind"] == "DaemonSet"][0]
    assert ds["spec"]["updateStrategy"]["type"] == "RollingUpdate"


class _Clock:
    def __init__(self):
        self.t = 1000.0

    def __call__(self):
        return self.t


def _unit_cluster(policy: dict):
    """Fake API with one driver node, its outdated driver pod and a GPU pod
    that stays Terminating after deletion (graceful deletion modelled)."""
    api = FakeApiServer()
    api.graceful_pod_deletion = True
    c = LocalClient(api)
    c.create(R.new("v1", "Namespace", "gpu-operator-resources"))
    deploy = M.DEPLOY_LABEL.format(M.OPERAND_LABELS["driver"])
    c.create({"apiVersion": "v1", "kind": "Node", "metadata": {"name": "n1", "labels": {deploy: "true"}}})
    c.create({"apiVersion": "v1", "kind": "Pod",
              "metadata": {"name": "drv-old", "namespace": "gpu-operator-resources",
                           "labels": {"app": U.DRIVER_DS, U.HASH_LABEL: "old"}},
              "spec": {"nodeName": "n1", "containers": [{"name": "amd-driver-ctr"}]}})
    c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "train", "namespace": "default"},
              "spec": {"nodeName": "n1", "terminationGracePeriodSeconds": 60,
                       "containers": [{"name": "c", "resources": {"limits": {"amd.com/gpu": "1"}}}]}})
    spec = ClusterPolicySpec.model_validate(deep_merge(REF, {"driver": {"upgradePolicy": policy}}))
    return c, spec


def _node(c):
    n = c.get("v1", "Node", "n1")
    return (n["metadata"].get("labels") or {}).get(U.STATE_LABEL), n


def test_drain_waits_for_terminating_pods_and_retry_uncordons(tmp_path):
    c, spec = _unit_cluster({"drainEnabled": True, "drainTimeoutSeconds": 10, "podDeletionForce": False})
    clock = _Clock()
    ctl = U.DriverUpgradeController(c, "gpu-operator-resources", clock=clock)
    ctl.step(spec)
    st, n = _node(c)
    # evicted, but the pod is still Terminating (holds /dev/kfd): no driver restart yet
    assert st == U.POD_DELETION and n["spec"]["unschedulable"] is True
    assert n["metadata"]["annotations"][U.CORDONED_ANN] == "true"
    assert c.get("v1", "Pod", "train", "default")["metadata"]["deletionTimestamp"]
    assert c.get("v1", "Pod", "drv-old", "gpu-operator-resources")
    clock.t += 5
    ctl.step(spec)
    assert _node(c)[0] == U.POD_DELETION
    clock.t += 6  # past drainTimeoutSeconds, no force: the attempt fails, node stays cordoned
    ctl.step(spec)
    st, n = _node(c)
    assert st == U.FAILED and n["spec"]["unschedulable"] is True
    # the pod finally terminates; after the back-off the node is retried
    c.delete("v1", "Pod", "train", "default", grace_period_seconds=0)
    clock.t += 11
    ctl.step(spec)
    st, n = _node(c)
    # the retry finds the node cordoned by the first attempt and keeps that record
    assert st == U.VALIDATION and n["metadata"]["annotations"][U.CORDONED_ANN] == "true"
    assert c.get("v1", "Pod", "drv-old", "gpu-operator-resources")["metadata"]["deletionTimestamp"]
    c.delete("v1", "Pod", "drv-old", "gpu-operator-resources", grace_period_seconds=0)
    desired = U.driver_spec_hash(spec)
    c.create({"apiVersion": "v1", "kind": "Pod",
              "metadata": {"name": "drv-new", "namespace": "gpu-operator-resources",
                           "labels": {"app": U.DRIVER_DS, U.HASH_LABEL: desired}},
              "spec": {"nodeName": "n1", "containers": [{"name": "amd-driver-ctr"}]},
              "status": {"conditions": [{"type": "Ready", "status": "True"}]}})
    p = c.get("v1", "Pod", "drv-new", "gpu-operator-resources")
    p["status"] = {"conditions": [{"type": "Ready", "status": "True"}]}
    c.update_status(p)
    c.patch("v1", "Node", "n1", {"metadata": {"labels": {VALIDATED_LABEL: "true"}}})
    ctl.step(spec)
    assert _node(c)[0] == U.VALIDATION  # the driver pod has not reported the new module yet
    c.patch("v1", "Node", "n1", {"metadata": {"annotations": {U.LOADED_HASH_ANN: desired}}})
    ctl.step(spec)
    st, n = _node(c)
    # the new module is live: only now is the validator restarted, and a
    # validation from before (here: the label set above) no longer counts
    assert st == U.VALIDATION and VALIDATED_LABEL not in (n["metadata"].get("labels") or {})
    assert n["metadata"]["annotations"][U.VALIDATOR_RESTART_ANN] == p["metadata"]["uid"]
    ctl.step(spec)
    assert _node(c)[0] == U.VALIDATION  # waiting for the fresh validator
    c.patch("v1", "Node", "n1", {"metadata": {"labels": {VALIDATED_LABEL: "true"}}})  # it validated
    ctl.step(spec)
    st, n = _node(c)
    assert st == U.DONE and n["spec"]["unschedulable"] is False
    assert U.CORDONED_ANN not in n["metadata"]["annotations"] and U.VALIDATOR_RESTART_ANN not in n["metadata"]["annotations"]


def test_user_cordon_survives_a_failed_and_retried_upgrade():
    c, spec = _unit_cluster({"drainEnabled": False, "drainTimeoutSeconds": 5, "podDeletionForce": False})
    c.patch("v1", "Node", "n1", {"spec": {"unschedulable": True}})  # cordoned by the admin
    clock = _Clock()
    ctl = U.DriverUpgradeController(c, "gpu-operator-resources", clock=clock)
    ctl.step(spec)
    assert _node(c)[1]["metadata"]["annotations"][U.CORDONED_ANN] == "false"
    clock.t += 6
    ctl.step(spec)
    assert _node(c)[0] == U.FAILED
    clock.t += 6
    ctl.step(spec)
    st, n = _node(c)
    assert st == U.POD_DELETION and n["metadata"]["annotations"][U.CORDONED_ANN] == "false"


def test_force_deletes_terminating_pods_after_the_timeout():
    c, spec = _unit_cluster({"drainEnabled": True, "drainTimeoutSeconds": 5, "podDeletionForce": True})
    clock = _Clock()
    ctl = U.DriverUpgradeController(c, "gpu-operator-resources", clock=clock)
    ctl.step(spec)
    assert _node(c)[0] == U.POD_DELETION
    clock.t += 6
    ctl.step(spec)
    assert _node(c)[0] == U.VALIDATION
    assert not [p for p in c.list("v1", "Pod", "default")]


@pytest.mark.slow
def test_rolling_driver_upgrade_one_node_at_a_time(tmp_path):
    nodes = [NodeSpec(f"gpu-{i}", 2) for i in range(3)]
    # deleted pods stay Terminating for 0.3 s, as on a real API server
    c = SimCluster(str(tmp_path / "c"), nodes, fake_gpu=True, termination_s=0.3).start()
    try:
        c.install_operator(deep_merge(REF, {"driver": {"upgradePolicy": {"maxParallelUpgrades": 1}}}))
        c.wait_ready(60, {n.name: 2 for n in nodes})
        old_hash = U.driver_spec_hash(ClusterPolicySpec.model_validate(c.policy()["spec"]))
        # a GPU workload on gpu-1: evicted before its driver is replaced
        c.client.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "trainer", "namespace": "default"},
                         "spec": {"nodeName": "gpu-1", "containers": [{"name": "main", "image": "x", "command": ["true"],
                                                                       "resources": {"limits": {"amd.com/gpu": "1"}}}]}})
        trainer_gone, restart_at = [None], {n.name: None for n in nodes}

        def record(etype, obj):
            if obj.get("kind") == "Pod" and obj["metadata"]["name"] == "trainer" and etype == "DELETED":
                trainer_gone[0] = time.monotonic()
            if obj.get("kind") == "Node" and (obj["metadata"].get("labels") or {}).get(U.STATE_LABEL) == U.POD_RESTART:
                restart_at[obj["metadata"]["name"]] = restart_at[obj["metadata"]["name"]] or time.monotonic()

        c.api.hooks.append(record)
        cp = c.policy()
        cp["spec"]["driver"]["driverVersion"] = "6.14.0"
        c.client.update(cp)
        new_hash = U.driver_spec_hash(ClusterPolicySpec.model_validate(cp["spec"]))
        assert new_hash != old_hash
        max_active, seen = 0, set()
        deadline = time.time() + 90
        while time.time() < deadline:
            states = {n["metadata"]["name"]: (n["metadata"].get("labels") or {}).get(U.STATE_LABEL, "")
                      for n in c.client.list("v1", "Node")}
            seen |= set(states.values())
            max_active = max(max_active, sum(1 for s in states.values() if s in U.ACTIVE))
            if all(s == U.DONE for s in states.values()):
                break
            time.sleep(0.02)
        assert all(s == U.DONE for s in states.values()), states
        assert max_active == 1
        assert U.VALIDATION in seen  # cordon + eviction + restart can finish within one pass
        pods = [p for p in c.client.list("v1", "Pod", c.namespace) if p["metadata"]["name"].startswith(U.DRIVER_DS)]
        assert len(pods) == 3 and all(p["metadata"]["labels"][U.HASH_LABEL] == new_hash for p in pods)
        for n in c.client.list("v1", "Node"):
            assert not (n.get("spec") or {}).get("unschedulable")
            deadline = time.time() + 30
            while (n["metadata"].get("labels") or {}).get(VALIDATED_LABEL) != "true" and time.time() < deadline:
                time.sleep(0.05)
                n = c.client.get("v1", "Node", n["metadata"]["name"])
            assert n["metadata"]["labels"][VALIDATED_LABEL] == "true"
        assert not [p for p in c.client.list("v1", "Pod", "default") if p["metadata"]["name"] == "trainer"]
        # every node now runs the new module: the old one was unloaded first
        for name, node in c.nodes.items():
            with open(os.path.join(node.env.sysfs_root(), "sys/module/amdgpu/version")) as f:
                assert f.read().strip() == "6.14.0"
            kl = node.env.extra["kmod"].log
            assert kl[-2:] == ["unload", "install 6.14.0"], kl
            ann = c.client.get("v1", "Node", name)["metadata"]["annotations"]
            assert ann[U.LOADED_VERSION_ANN] == "6.14.0" and ann[U.LOADED_HASH_ANN] == new_hash
        # the GPU workload was gone (not merely Terminating) before gpu-1's driver pod restarted
        assert trainer_gone[0] is not None and restart_at["gpu-1"] is not None
        assert trainer_gone[0] <= restart_at["gpu-1"]
        deadline = time.time() + 10  # the status write follows the last node transition
        while c.policy()["status"]["driverUpgrade"]["nodes"] != {U.DONE: 3} and time.time() < deadline:
            time.sleep(0.05)
        assert c.policy()["status"]["driverUpgrade"]["nodes"] == {U.DONE: 3}
        assert 'amd_gpu_operator_driver_upgrade_nodes{state="upgrade-done"} 3' in c.reconciler.metrics.render()
    finally:
        c.stop()


def test_no_upgrade_labels_on_a_fresh_install(tmp_path):
    c = SimCluster(str(tmp_path / "c"), [NodeSpec("gpu-0", 1)], fake_gpu=True).start()
    try:
        c.install_operator(REF)
        c.wait_ready(60, {"gpu-0": 1})
        labels = c.client.get("v1", "Node", "gpu-0")["metadata"].get("labels") or {}
        assert U.STATE_LABEL not in labels
        assert "driverUpgrade" not in (c.policy().get("status") or {})
    finally:
        c.stop()
