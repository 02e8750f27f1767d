"""The RBAC we ship, enforced: the simulated API server authorizes every
request of the operator and of each operand process against the ClusterRoles
the chart and the operator create (kube/rbac.py), as kube-apiserver would.
A verb missing from a role is a 403 here, not a surprise on a real cluster
(/root/reference/README.md:101-111: `helm install --wait` must finish)."""

import pytest

from amdgpu_operator.api.clusterpolicy import REFERENCE_SET_FLAGS, parse_set_flags
from amdgpu_operator.kube import rbac
from amdgpu_operator.kube.fakeapi import FakeApiServer
from amdgpu_operator.testing.simcluster import NodeSpec, SimCluster


def test_rule_matching():
    api = FakeApiServer()
    api.create({"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRole", "metadata": {"name": "r"},
                "rules": [{"apiGroups": [""], "resources": ["nodes", "pods/status"], "verbs": ["get", "patch"]},
                          {"apiGroups": ["apps"], "resources": ["*"], "verbs": ["list"]},
                          {"apiGroups": [""], "resources": ["configmaps"], "verbs": ["get"], "resourceNames": ["c"]}]})
    api.create({"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRoleBinding", "metadata": {"name": "b"},
                "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "ClusterRole", "name": "r"},
                "subjects": [{"kind": "ServiceAccount", "name": "sa", "namespace": "ns"}]})
    a = rbac.Authorizer(api)
    u = "system:serviceaccount:ns:sa"
    assert a.allowed(u, "get", "", "nodes", None, "n1") and a.allowed(u, "patch", "", "pods/status", "ns", "p")
    assert not a.allowed(u, "update", "", "nodes", None, "n1") and not a.allowed(u, "patch", "", "pods", "ns", "p")
    assert a.allowed(u, "list", "apps", "daemonsets", "ns", None) and not a.allowed(u, "get", "apps", "daemonsets", "ns", "d")
    assert a.allowed(u, "get", "", "configmaps", "ns", "c") and not a.allowed(u, "get", "", "configmaps", "ns", "other")
    assert not a.allowed("system:serviceaccount:ns:other", "get", "", "nodes", None, "n1")
    assert rbac.verb_of("GET", None, True) == "watch" and rbac.verb_of("GET", "x", False) == "get"


@pytest.mark.parametrize("flags", [
    [],
    ["draDriver.enabled=true", "devicePlugin.enabled=false", "driver.rdma.enabled=true", "migManager.enabled=true"],
], ids=["reference", "dra-rdma-partition"])
def test_bring_up_needs_no_permission_we_do_not_grant(tmp_path, flags):
    c = SimCluster(str(tmp_path / "c"), [NodeSpec("gpu-1", 2)], fake_gpu=True, process_containers=True,
                   rbac=True).start()
    try:
        c.install_operator(parse_set_flags(REFERENCE_SET_FLAGS + flags))
        c.wait_ready(90, {"gpu-1": 2} if not flags else None)
        assert not c._http.denied, c._http.denied
    finally:
        c.stop()
