"""The user-facing manifests under deploy/examples: every object passes the
apiserver validation the simulated cluster enforces (kube/validation.py), and
the pod examples run to completion on a simulated MI355X node - through the
device plugin, or through the DRA driver (a ResourceClaimTemplate the
resourceclaim controller turns into a per-pod claim; one claim shared by two
pods, prepared once and unprepared after the last)."""

import os
import time

import pytest
import yaml

from amdgpu_operator.api.clusterpolicy import REFERENCE_SET_FLAGS, parse_set_flags
from amdgpu_operator.kube.validation import validate

EX = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "deploy", "examples")
RV1B1 = "resource.k8s.io/v1beta1"


def _docs(name):
    with open(os.path.join(EX, name)) as f:
        return [d for d in yaml.safe_load_all(f) if d]


def test_every_example_is_valid():
    names = sorted(n for n in os.listdir(EX) if n.endswith(".yaml"))
    assert len(names) >= 4
    for n in names:
        for d in _docs(n):
            assert not validate(d), (n, d["kind"], validate(d))


def test_validation_rejects_broken_claims_and_claim_references():
    bad_claim = {"apiVersion": RV1B1, "kind": "ResourceClaim", "metadata": {"name": "c", "namespace": "d"},
                 "spec": {"devices": {"requests": [{"name": "gpus", "count": 0, "deviceClassName": "gpu.amd.com"},
                                                   {"name": "gpus", "allocationMode": "Some"}],
                                      "constraints": [{"requests": ["nope"], "matchAttribute": "numaNode"}]}}}
    errs = " | ".join(validate(bad_claim))
    for want in ("count 0", "duplicate", "deviceClassName: required", "allocationMode 'Some'",
                 "'nope' is not a request", "fully qualified"):
        assert want in errs, (want, errs)
    pod = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "p", "namespace": "d"},
           "spec": {"resourceClaims": [{"name": "g", "resourceClaimName": "a", "resourceClaimTemplateName": "b"},
                                       {"name": "h"}],
                    "containers": [{"name": "c", "image": "i", "resources": {"claims": [{"name": "x"}]}}]}}
    errs = " | ".join(validate(pod))
    assert errs.count("exactly one of resourceClaimName") == 2 and "not in spec.resourceClaims" in errs


def _create_all(c, docs, ns="default"):
    for d in docs:
        d.setdefault("metadata", {}).setdefault("namespace", ns)
        c.client.create(d)


def _phase(c, name, ns="default"):
    return ((c.client.get("v1", "Pod", name, ns).get("status") or {}).get("phase"))


def _wait(pred, timeout=30.0):
    deadline = time.monotonic() + timeout
    while time.monotonic() < deadline:
        if pred():
            return True
        time.sleep(0.02)
    return pred()


@pytest.fixture
def short_tmp():
    import shutil
    import tempfile

    d = tempfile.mkdtemp(prefix="ex", dir="/tmp")
    yield __import__("pathlib").Path(d)
    shutil.rmtree(d, ignore_errors=True)


def test_device_plugin_pod_example_runs(short_tmp):
    from amdgpu_operator.testing.simcluster import NodeSpec, SimCluster

    c = SimCluster(str(short_tmp / "c"), [NodeSpec("gpu-1", 8)], fake_gpu=True).start()
    try:
        c.install_operator(parse_set_flags(REFERENCE_SET_FLAGS))
        c.wait_ready(60, {"gpu-1": 8})
        docs = _docs("gpu-pod.yaml")
        docs[0]["spec"]["nodeName"] = "gpu-1"  # no scheduler for amd.com/gpu pods in the simulation
        _create_all(c, docs)
        assert _wait(lambda: _phase(c, "amd-gpu-check") in ("Succeeded", "Failed")), _phase(c, "amd-gpu-check")
        assert _phase(c, "amd-gpu-check") == "Succeeded"
    finally:
        c.stop()


def test_dra_examples_run(short_tmp):
    from amdgpu_operator.discovery import topology
    from amdgpu_operator.testing.simcluster import NodeSpec, SimCluster

    c = SimCluster(str(short_tmp / "c"), [NodeSpec("gpu-1", 8)], fake_gpu=True).start()
    try:
        c.install_operator(parse_set_flags(REFERENCE_SET_FLAGS + ["draDriver.enabled=true",
                                                                  "devicePlugin.enabled=false"]))
        c.wait_ready(60, {})
        env = c.nodes["gpu-1"].env
        gpus = {f"gpu-{g.index}": g for g in topology.enumerate_gpus(env.sysfs_root())}

        # a ResourceClaimTemplate: the pod gets its own claim, owned by it
        _create_all(c, _docs("dra-gpu-claim-template.yaml"))
        assert _wait(lambda: _phase(c, "dra-gemm") in ("Succeeded", "Failed")), _phase(c, "dra-gemm")
        pod = c.client.get("v1", "Pod", "dra-gemm", "default")
        assert pod["status"]["phase"] == "Succeeded", pod["status"]
        assert pod["spec"]["nodeName"] == "gpu-1"
        (st,) = pod["status"]["resourceClaimStatuses"]
        claim = c.client.get(RV1B1, "ResourceClaim", st["resourceClaimName"], "default")
        assert st["name"] == "gpus" and claim["metadata"]["name"].startswith("dra-gemm-gpus-")
        assert claim["metadata"]["ownerReferences"][0]["uid"] == pod["metadata"]["uid"]
        res = claim["status"]["allocation"]["devices"]["results"]
        assert len(res) == 2 and len({gpus[r["device"]].numa_node for r in res}) == 1
        c.client.delete("v1", "Pod", "dra-gemm", "default")
        assert _wait(lambda: not c.client.list(RV1B1, "ResourceClaim"))  # garbage-collected with the pod

        # one claim, two pods: the same GPU, prepared once, unprepared after the last pod
        _create_all(c, _docs("dra-shared-claim.yaml"))
        assert _wait(lambda: {_phase(c, "shared-a"), _phase(c, "shared-b")} <= {"Succeeded", "Failed"})
        assert _phase(c, "shared-a") == _phase(c, "shared-b") == "Succeeded"
        claim = c.client.get(RV1B1, "ResourceClaim", "shared-mi355x", "default")
        assert len(claim["status"]["allocation"]["devices"]["results"]) == 1
        cdi = os.path.join(env.cdi_dir, f"gpu.amd.com-claim_{claim['metadata']['uid']}.json")
        assert _wait(lambda: not os.path.exists(cdi), 10)  # both pods done: unprepared
        c.client.delete(RV1B1, "ResourceClaim", "shared-mi355x", "default")
    finally:
        c.stop()


@pytest.mark.parametrize("dra", [False, True], ids=["device-plugin", "dra"])
def test_verify_run_pod(short_tmp, dra):
    """``amdgpu-operator verify --run-pod``: per GPU node one 1-GPU pod (an
    amd.com/gpu limit, or a ResourceClaim with the DRA driver) must succeed;
    it leaves no pod or claim behind.  The pod runs the ClusterPolicy's
    validator image - here from a mirror registry (``validator.repository``),
    with a pull secret - and, with the DRA driver, claims from the policy's
    own DeviceClass (``draDriver.deviceClass``)."""
    from amdgpu_operator.cli.verify import verify
    from amdgpu_operator.testing.simcluster import NodeSpec, SimCluster

    flags = REFERENCE_SET_FLAGS + ["validator.repository=mirror.example.com/gpu", "validator.version=7.2.0-r5"]
    flags += ["draDriver.enabled=true", "devicePlugin.enabled=false", "draDriver.deviceClass=mi355x.example.com"] \
        if dra else []
    values = parse_set_flags(flags)
    values["validator"]["imagePullSecrets"] = ["mirror-creds"]
    c = SimCluster(str(short_tmp / "c"), [NodeSpec("gpu-1", 4), NodeSpec("gpu-2", 2)], fake_gpu=True).start()
    seen = []
    c.api.hooks.append(lambda etype, obj: seen.append(obj) if etype == "ADDED"
                       and obj.get("kind") in ("Pod", "ResourceClaim")
                       and obj["metadata"].get("name", "").startswith("amd-gpu-verify-") else None)
    try:
        c.install_operator(values)
        c.wait_ready(60, {} if dra else {"gpu-1": 4, "gpu-2": 2})
        rep = verify(c.client, c.namespace, run_pods=True, pod_timeout=30)
        pods = [x for x in rep.checks if x.name.startswith("gpu-pod[")]
        assert rep.ok and len(pods) == 2, rep.table()
        assert all(("dra claim" if dra else "amd.com/gpu=1") in x.detail for x in pods), rep.table()
        assert not [p for p in c.client.list("v1", "Pod", c.namespace)
                    if p["metadata"]["name"].startswith("amd-gpu-verify-")
                    and not p["metadata"].get("deletionTimestamp")]
        assert not c.client.list(RV1B1, "ResourceClaim")
        created = [o for o in seen if o["kind"] == "Pod"]
        assert len(created) == 2
        for pod in created:
            ctr = pod["spec"]["containers"][0]
            assert ctr["image"] == "mirror.example.com/gpu/amd-operator-validator:7.2.0-r5"
            assert pod["spec"]["imagePullSecrets"] == [{"name": "mirror-creds"}]
        if dra:
            assert all(o["spec"]["devices"]["requests"][0]["deviceClassName"] == "mi355x.example.com"
                       for o in seen if o["kind"] == "ResourceClaim")
    finally:
        c.stop()


def test_a_bare_image_name_does_not_pull(short_tmp):
    """A real kubelet pulls ``amd-operator-validator`` from Docker Hub and the
    pod ends in ImagePullBackOff; the simulated kubelet's registry holds only
    the chart's and the ClusterPolicy's images, so it does the same - and
    ``verify --run-pod --pod-image <bare>`` fails, naming the pull error."""
    from amdgpu_operator.cli.verify import verify
    from amdgpu_operator.testing.simcluster import NodeSpec, SimCluster

    c = SimCluster(str(short_tmp / "c"), [NodeSpec("gpu-1", 1)], fake_gpu=True).start()
    try:
        c.install_operator(parse_set_flags(REFERENCE_SET_FLAGS))
        c.wait_ready(60, {"gpu-1": 1})
        rep = verify(c.client, c.namespace, run_pods=True, pod_image="amd-operator-validator", pod_timeout=2)
        (pod,) = [x for x in rep.checks if x.name.startswith("gpu-pod[")]
        assert not pod.ok and "Pending" in pod.detail and "ImagePull" in pod.detail, pod.detail
        docs = _docs("gpu-pod.yaml")
        docs[0]["spec"]["nodeName"] = "gpu-1"
        docs[0]["spec"]["containers"][0]["image"] = "amd-operator-validator"
        _create_all(c, docs)
        def reason():
            st = c.client.get("v1", "Pod", "amd-gpu-check", "default").get("status") or {}
            return (((st.get("containerStatuses") or [{}])[0].get("state") or {}).get("waiting") or {}).get("reason")

        assert _wait(lambda: reason() == "ImagePullBackOff"), reason()
        assert _phase(c, "amd-gpu-check") == "Pending"
        # every pod the product itself created pulled: the operands and the validator's pods ran
        assert all(p["status"]["phase"] in ("Running", "Succeeded") for p in c.client.list("v1", "Pod", c.namespace))
    finally:
        c.stop()
