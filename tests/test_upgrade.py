"""Cluster-wide driver upgrade (controller/upgrade.py): a driver spec change on
a running cluster walks the GPU nodes through cordon -> GPU-pod eviction ->
driver pod restart -> revalidation -> uncordon, at most
``maxParallelUpgrades`` nodes at a time (SURVEY.md §5.3 recovery tier)."""

import time

import pytest

from amdgpu_operator.api.clusterpolicy import REFERENCE_SET_FLAGS, ClusterPolicySpec, deep_merge, parse_set_flags
from amdgpu_operator.controller import manifests as M
from amdgpu_operator.controller import upgrade as U
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


@pytest.mark.slow
def test_rolling_driver_upgrade_one_node_at_a_time(tmp_path):
    nodes = [NodeSpec(f"gpu-{i}", 2) for i in range(3)]
    c = SimCluster(str(tmp_path / "c"), nodes, fake_gpu=True).start()
    try:
        c.install_operator(deep_merge(REF, {"driver": {"upgradePolicy": {"maxParallelUpgrades": 1}}}))
        c.wait_ready(60, {n.name: 2 for n in nodes})
        old_hash = U.driver_spec_hash(ClusterPolicySpec.model_validate(c.policy()["spec"]))
        # a GPU workload on gpu-1: evicted before its driver is replaced
        c.client.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "trainer", "namespace": "default"},
                         "spec": {"nodeName": "gpu-1", "containers": [{"name": "main", "image": "x", "command": ["true"],
                                                                       "resources": {"limits": {"amd.com/gpu": "1"}}}]}})
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
