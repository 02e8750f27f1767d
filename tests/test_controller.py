"""ClusterPolicy reconciler: states, node labels, drift, disable/enable,
invalid specs, multiple policies, CRD cleanup."""

import pytest

from amdgpu_operator.api.clusterpolicy import (REFERENCE_SET_FLAGS, ClusterPolicySpec, cluster_policy,
                                               parse_set_flags, spec_from_values)
from amdgpu_operator.controller.manifests import STATE_BUILDERS
from amdgpu_operator.controller.nodes import NFD_SCANNED_ANN, desired_labels, is_gpu_node
from amdgpu_operator.controller.reconciler import CP_API, ClusterPolicyReconciler, cleanup_crd
from amdgpu_operator.helm.crd import crd
from amdgpu_operator.kube import resources as R
from amdgpu_operator.kube.client import LocalClient, NotFound
from amdgpu_operator.kube.fakeapi import FakeApiServer

NS = "gpu-operator-resources"
GPU_LABEL = {"feature.node.kubernetes.io/pci-1200_1002.present": "true"}


@pytest.fixture
def env():
    c = LocalClient(FakeApiServer())
    c.create(R.new("v1", "Namespace", NS))
    c.create(R.new("v1", "Node", "gpu-a", labels=GPU_LABEL))
    c.create(R.new("v1", "Node", "cpu-a"))
    return c, ClusterPolicyReconciler(c, NS)


def ds_names(c):
    return sorted(d["metadata"]["name"] for d in c.list("apps/v1", "DaemonSet", NS))


def mark_all_ds_ready(c, desired=1):
    for ds in c.list("apps/v1", "DaemonSet", NS):
        ds["status"] = {"desiredNumberScheduled": desired, "numberReady": desired, "updatedNumberScheduled": desired,
                        "observedGeneration": ds["metadata"]["generation"]}
        c.update_status(ds)


def test_reference_install_creates_expected_operands(env):
    c, rec = env
    c.create(cluster_policy(spec=spec_from_values(parse_set_flags(REFERENCE_SET_FLAGS))))
    res = rec.reconcile()
    assert res.state == "notReady" and res.gpu_nodes == 1
    assert ds_names(c) == ["amd-container-toolkit-daemonset", "amd-device-plugin-daemonset", "amd-driver-daemonset",
                           "amd-metrics-exporter", "amd-node-status-exporter", "amd-operator-validator",
                           "gpu-feature-discovery", "node-feature-discovery-worker"]
    # migManager.enabled=false -> no partition manager (README.md:109)
    assert "amd-partition-manager" not in ds_names(c)
    labels = c.get("v1", "Node", "gpu-a")["metadata"]["labels"]
    assert labels["amd.com/gpu.present"] == "true"
    assert labels["amd.com/gpu.deploy.driver"] == "true"
    assert "amd.com/gpu.deploy.partition-manager" not in labels
    assert "amd.com/gpu.present" not in c.get("v1", "Node", "cpu-a")["metadata"]["labels"] if c.get(
        "v1", "Node", "cpu-a")["metadata"].get("labels") else True
    drv = c.get("apps/v1", "DaemonSet", "amd-driver-daemonset", NS)
    ctrs = [x["name"] for x in drv["spec"]["template"]["spec"]["containers"]]
    assert ctrs == ["amd-driver-ctr", "amd-driver-health"]  # 2/2 like README.md:138-139
    assert drv["spec"]["template"]["spec"]["nodeSelector"] == {"amd.com/gpu.deploy.driver": "true"}


def test_ready_requires_daemonsets_and_validated_nodes(env):
    c, rec = env
    c.create(cluster_policy())
    rec.reconcile()
    mark_all_ds_ready(c)
    assert rec.reconcile().state == "notReady"  # node not validated yet
    c.patch("v1", "Node", "gpu-a", {"metadata": {"labels": {"amd.com/gpu.validated": "true"}}})
    res = rec.reconcile()
    assert res.state == "ready"
    st = c.get(CP_API, "ClusterPolicy", "cluster-policy")["status"]
    assert st["state"] == "ready" and st["timeToReadySeconds"] >= 0
    assert R.condition(c.get(CP_API, "ClusterPolicy", "cluster-policy"), "Ready")["status"] == "True"


def test_reconcile_is_idempotent_and_reverts_drift(env):
    c, rec = env
    c.create(cluster_policy())
    rec.reconcile()
    assert sum(s.changed for s in rec.reconcile().states) == 0
    c.patch("apps/v1", "DaemonSet", "amd-device-plugin-daemonset",
            {"spec": {"template": {"spec": {"nodeSelector": {"x": "y"}}}}}, NS)
    res = rec.reconcile()
    assert sum(s.changed for s in res.states) == 1
    ds = c.get("apps/v1", "DaemonSet", "amd-device-plugin-daemonset", NS)
    assert ds["spec"]["template"]["spec"]["nodeSelector"] == {"amd.com/gpu.deploy.device-plugin": "true"}
    c.delete("apps/v1", "DaemonSet", "gpu-feature-discovery", NS)
    rec.reconcile()
    assert "gpu-feature-discovery" in ds_names(c)


def test_disable_operand_removes_objects_and_labels(env):
    c, rec = env
    c.create(cluster_policy())
    rec.reconcile()
    cp = c.get(CP_API, "ClusterPolicy", "cluster-policy")
    cp["spec"]["gfd"]["enabled"] = False
    cp["spec"]["migManager"]["enabled"] = True
    c.update(cp)
    res = rec.reconcile()
    assert "gpu-feature-discovery" not in ds_names(c)
    assert "amd-partition-manager" in ds_names(c)
    labels = c.get("v1", "Node", "gpu-a")["metadata"]["labels"]
    assert "amd.com/gpu.deploy.gpu-feature-discovery" not in labels
    assert labels["amd.com/gpu.deploy.partition-manager"] == "true"
    assert {s.name: s.enabled for s in res.states}["state-gpu-feature-discovery"] is False


def test_user_opt_out_label_is_sticky(env):
    c, rec = env
    c.patch("v1", "Node", "gpu-a", {"metadata": {"labels": {"amd.com/gpu.deploy.driver": "false"}}})
    c.create(cluster_policy())
    rec.reconcile()
    assert c.get("v1", "Node", "gpu-a")["metadata"]["labels"]["amd.com/gpu.deploy.driver"] == "false"


def test_node_losing_gpu_is_unlabelled(env):
    c, rec = env
    c.create(cluster_policy())
    rec.reconcile()
    c.patch("v1", "Node", "gpu-a", {"metadata": {"labels": {k: None for k in GPU_LABEL}}})
    rec.reconcile()
    labels = c.get("v1", "Node", "gpu-a")["metadata"]["labels"]
    assert not any(k.startswith("amd.com/gpu.") for k in labels)


def test_invalid_spec_sets_error(env):
    c, rec = env
    bad = cluster_policy()
    bad["spec"]["driver"]["enabeld"] = True
    c.create(bad)
    res = rec.reconcile()
    assert res.state == "error"
    st = c.get(CP_API, "ClusterPolicy", "cluster-policy")["status"]
    assert st["state"] == "error" and R.condition({"status": st}, "Error")["status"] == "True"
    assert c.list("apps/v1", "DaemonSet", NS) == []


def test_second_policy_is_ignored(env):
    c, rec = env
    c.create(cluster_policy("first"))
    c.create(cluster_policy("second"))
    rec.reconcile()
    assert c.get(CP_API, "ClusterPolicy", "second")["status"]["state"] == "ignored"


def test_zero_gpu_cluster_converges(env):
    c, rec = env
    c.delete("v1", "Node", "gpu-a")
    c.create(cluster_policy())
    rec.reconcile()
    mark_all_ds_ready(c, desired=0)
    for ds in c.list("apps/v1", "DaemonSet", NS):
        if ds["metadata"]["name"].startswith("node-feature"):
            ds["status"] = {"desiredNumberScheduled": 1, "numberReady": 1, "updatedNumberScheduled": 1,
                            "observedGeneration": 1}
            c.update_status(ds)
    # the NFD pod is Ready but the node shows no scan yet (a Node read older
    # than the DaemonSet status): zero GPU nodes is not yet an answer
    res = rec.reconcile()
    assert res.state == "notReady"
    assert "0/1 nodes labelled" in next(r.detail for r in res.states if r.name == "state-node-feature-discovery")
    c.patch("v1", "Node", "cpu-a", {"metadata": {"annotations": {NFD_SCANNED_ANN: "true"}}})
    assert rec.reconcile().state == "ready"


def test_owner_references_make_operands_garbage_collected(env):
    c, rec = env
    c.create(cluster_policy())
    rec.reconcile()
    c.delete(CP_API, "ClusterPolicy", "cluster-policy")
    assert c.list("apps/v1", "DaemonSet", NS) == []


def test_cleanup_crd(env):
    c, rec = env
    c.create(crd())
    c.create(cluster_policy())
    assert cleanup_crd(c) is True
    assert c.list(CP_API, "ClusterPolicy") == []
    with pytest.raises(NotFound):
        c.get("apiextensions.k8s.io/v1", "CustomResourceDefinition", "clusterpolicies.amd.com")
    assert cleanup_crd(c) is False


def test_every_state_builder_yields_valid_objects():
    spec = ClusterPolicySpec.model_validate({"migManager": {"enabled": True},
                                             "dcgmExporter": {"serviceMonitor": {"enabled": True}}})
    owner = [{"uid": "u", "kind": "ClusterPolicy", "name": "cp", "apiVersion": CP_API}]
    for name, fn in STATE_BUILDERS.items():
        for o in fn(spec, NS, owner):
            R.rtype_of(o)  # registered kind
            assert o["metadata"]["name"]
            if o["kind"] == "DaemonSet":
                t = o["spec"]["template"]
                assert t["metadata"]["labels"]["app"] == o["metadata"]["name"]
                assert all(ct["command"] in (["amdgpu-operator"], ["amdgpu-nfd"]) for ct in t["spec"]["containers"])


def test_node_detection_rules():
    assert is_gpu_node({"metadata": {"labels": {"feature.node.kubernetes.io/pci-1002.present": "true"}}})
    assert is_gpu_node({"metadata": {}, "status": {"capacity": {"amd.com/gpu": "8"}}})
    assert not is_gpu_node({"metadata": {"labels": {"feature.node.kubernetes.io/pci-10de.present": "true"}}})
    patch = desired_labels({"metadata": {"labels": GPU_LABEL}}, ClusterPolicySpec())
    assert patch["amd.com/gpu.present"] == "true"


def test_operator_metrics_endpoint(env):
    import urllib.request

    from amdgpu_operator.cli.main import _health_server

    c, rec = env
    c.create(cluster_policy())
    rec.reconcile()
    mark_all_ds_ready(c)
    c.patch("v1", "Node", "gpu-a", {"metadata": {"labels": {"amd.com/gpu.validated": "true"}}})
    assert rec.reconcile().state == "ready"
    srv = _health_server(0, rec.metrics)
    try:
        port = srv.server_address[1]
        text = urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=5).read().decode()
        assert urllib.request.urlopen(f"http://127.0.0.1:{port}/healthz", timeout=5).read() == b"ok\n"
    finally:
        srv.shutdown()
    samples = dict(line.rsplit(" ", 1) for line in text.splitlines() if line and not line.startswith("#"))
    assert samples["amd_gpu_operator_reconcile_total"] == "2"
    assert samples["amd_gpu_operator_reconcile_duration_seconds_count"] == "2"
    assert samples['amd_gpu_operator_reconcile_duration_seconds_bucket{le="+Inf"}'] == "2"
    assert samples["amd_gpu_operator_policy_ready"] == "1"
    assert float(samples["amd_gpu_operator_time_to_ready_seconds"]) >= 0
    assert 'amd_gpu_operator_state_ready_seconds{state="state-driver"}' in samples


def test_psa_labels_operand_namespace(env):
    c, rec = env
    c.create(cluster_policy(spec={"psa": {"enabled": True}}))
    rec.reconcile()
    labels = c.get("v1", "Namespace", NS)["metadata"]["labels"]
    assert labels["pod-security.kubernetes.io/enforce"] == "privileged"
    assert labels["pod-security.kubernetes.io/warn"] == "privileged"


def test_toolkit_set_as_default_runtime():
    from amdgpu_operator.toolkit.install import dropin_config

    txt = dropin_config("amd", "/usr/local/amd/amdgpu-oci-hook", "/var/run/cdi", set_as_default=True)
    assert 'default_runtime_name = "amd"' in txt
    assert "default_runtime_name" not in dropin_config("amd", "/h", "/var/run/cdi")


def test_every_mount_has_a_volume_and_probing_containers_see_host_dev():
    """Operands read the host through NodeEnv.host_root=/host: the N1 probe
    needs /host/sys AND /host/dev (sys/module/amdgpu, /dev/kfd, render
    nodes), so every container that probes the driver mounts both."""
    from amdgpu_operator.api.clusterpolicy import REFERENCE_SET_FLAGS, ClusterPolicySpec, parse_set_flags
    from amdgpu_operator.controller import manifests as M

    spec = ClusterPolicySpec.model_validate(parse_set_flags(REFERENCE_SET_FLAGS))
    probing = (["validate", "driver"], ["validate", "gpu"], ["driver", "install"], ["driver", "monitor"],
               ["driver", "prepare-upgrade"])
    seen = 0
    for state, builder in M.STATE_BUILDERS.items():
        for o in builder(spec, "ns", None):
            if o["kind"] != "DaemonSet":
                continue
            pod = o["spec"]["template"]["spec"]
            vols = {v["name"]: v for v in pod["volumes"]}
            for c in pod.get("initContainers", []) + pod["containers"]:
                mounts = {m["name"]: m["mountPath"] for m in c.get("volumeMounts", [])}
                assert set(mounts) <= set(vols), (o["metadata"]["name"], c["name"], set(mounts) - set(vols))
                args = c.get("args") or []
                gate = {e["name"]: e.get("value") for e in c.get("env") or []}.get("VALIDATION_GATE", "")
                if any(args[:2] == p for p in probing) or "driver" in gate.split(","):
                    seen += 1
                    paths = set(mounts.values())
                    assert "/host/sys" in paths and ("/host/dev" in paths or "/host" in paths), (c["name"], paths)
                    if "host-dev" in mounts:
                        assert vols["host-dev"]["hostPath"]["path"] == "/dev"
    assert seen >= 5


def test_image_pull_secrets_and_validation_pod_image():
    """<operand>.imagePullSecrets reach the pods; the plugin-validation pods the
    validator creates run the validator's configured image, not a bare name."""
    from amdgpu_operator.api.clusterpolicy import ClusterPolicySpec
    from amdgpu_operator.controller import manifests as M

    spec = ClusterPolicySpec.model_validate({
        "validator": {"repository": "registry.example/amd", "version": "1.2.3", "imagePullSecrets": ["regcred"]},
        "nfd": {"imagePullSecrets": ["nfdcred"]}})
    ds = [o for o in M.state_validator(spec, "ns", None) if o["kind"] == "DaemonSet"][0]
    pod = ds["spec"]["template"]["spec"]
    assert pod["imagePullSecrets"] == [{"name": "regcred"}]
    env = {e["name"]: e.get("value") for e in (pod["initContainers"] or pod["containers"])[0]["env"]}
    assert env["VALIDATOR_IMAGE"] == "registry.example/amd/amd-operator-validator:1.2.3"
    assert env["VALIDATOR_IMAGE_PULL_SECRETS"] == "regcred"
    nfd = [o for o in M.state_nfd(spec, "ns", None) if o["kind"] == "DaemonSet"][0]
    assert nfd["spec"]["template"]["spec"]["imagePullSecrets"] == [{"name": "nfdcred"}]
    drv = [o for o in M.state_driver(spec, "ns", None) if o["kind"] == "DaemonSet"][0]
    assert "imagePullSecrets" not in drv["spec"]["template"]["spec"]


def test_plugin_validation_pods_use_the_validator_image(tmp_path):
    import threading
    import time

    from amdgpu_operator.kube import resources as R
    from amdgpu_operator.kube.client import LocalClient
    from amdgpu_operator.kube.fakeapi import FakeApiServer
    from amdgpu_operator.nodeenv import NodeEnv
    from amdgpu_operator.testing import fakesys
    from amdgpu_operator.validator import validate as V

    root = str(tmp_path / "host")
    fakesys.build_node(root, 1)
    c = LocalClient(FakeApiServer())
    c.create(R.new("v1", "Namespace", "gpu-operator-resources"))
    node = R.new("v1", "Node", "n1")
    node["status"] = {"allocatable": {"amd.com/gpu": "1"}}
    c.create(node)
    env = NodeEnv("n1", c, host_root=root, validations_dir=str(tmp_path / "val"), poll_s=0.01)
    env.extra["validator_image"] = {"image": "reg/amd-operator-validator:9", "pull_policy": "Always",
                                    "pull_secrets": ["s1"]}
    seen = []

    def kubelet():  # completes the pod like a kubelet would
        deadline = time.time() + 5
        while time.time() < deadline:
            for p in c.list("v1", "Pod", "gpu-operator-resources"):
                seen.append(p["spec"])
                p["status"] = {"phase": "Succeeded"}
                c.update_status(p)
                return
            time.sleep(0.01)

    th = threading.Thread(target=kubelet)
    th.start()
    os_ready = V.validate_plugin(env, timeout=5)
    th.join()
    assert os_ready["ok"] and seen
    ctr = seen[0]["containers"][0]
    assert ctr["image"] == "reg/amd-operator-validator:9" and ctr["imagePullPolicy"] == "Always"
    assert seen[0]["imagePullSecrets"] == [{"name": "s1"}]
    assert os_ready["allocatable_source"] == "node-status"
    # a config file renamed the (time-sliced) resource: Node.status shows
    # only amd.com/gpu.shared replicas; one pod for the node's one GPU
    node = c.get("v1", "Node", "n1")
    node["status"] = {"allocatable": {"amd.com/gpu.shared": "4"}}
    c.update_status(node)
    seen.clear()
    th = threading.Thread(target=kubelet)
    th.start()
    rep = V.validate_plugin(env, timeout=5)
    th.join()
    assert rep["resources"] == {"amd.com/gpu.shared": 1} and rep["pods"] == 1
    assert seen[0]["containers"][0]["resources"]["limits"] == {"amd.com/gpu.shared": "1"}


def _driver_ds(spec):
    from amdgpu_operator.controller import manifests as M

    return [o for o in M.state_driver(spec, "ns", None) if o["kind"] == "DaemonSet"][0]


def test_driver_image_and_package_mirror_are_separate():
    """driver.repository is the image registry like every operand's; the
    package mirror is driver.packageRepository (round 2 conflated the two and
    rendered the image as "/amd-driver:<version>")."""
    spec = ClusterPolicySpec.model_validate({"driver": {"packageRepository": "http://mirror.local"}})
    ctr = _driver_ds(spec)["spec"]["template"]["spec"]["containers"][0]
    assert ctr["image"] == "registry.local/amd-gpu-operator/amd-driver:0.1.0"
    env = {e["name"]: e.get("value") for e in ctr["env"]}
    assert env["AMDGPU_REPO_BASE"] == "http://mirror.local"


def test_dkms_driver_mounts_host_headers_read_only():
    pod = _driver_ds(ClusterPolicySpec())["spec"]["template"]["spec"]
    mounts = {m["name"]: m for m in pod["containers"][0]["volumeMounts"]}
    assert mounts["host-usr-src"]["mountPath"] == "/host/usr/src" and mounts["host-usr-src"]["readOnly"]
    assert {"name": "host-usr-src", "hostPath": {"path": "/usr/src", "type": "DirectoryOrCreate"}} in pod["volumes"]
    # the firmware is staged under /run/amd, a hostPath at the same path (install.sh stage_firmware)
    assert mounts["run-amd"]["mountPath"] == "/run/amd"
    pre = _driver_ds(ClusterPolicySpec.model_validate({"driver": {"usePrecompiled": True}}))["spec"]["template"]["spec"]
    assert "host-usr-src" not in {v["name"] for v in pre["volumes"]}


def _kernel_node(c, name, kernel):
    labels = {**GPU_LABEL, **({"feature.node.kubernetes.io/kernel-version.full": kernel} if kernel else {})}
    c.create(R.new("v1", "Node", name, labels=labels))


def test_precompiled_driver_runs_one_daemonset_per_kernel(env):
    from amdgpu_operator.controller.manifests import KERNEL_LABEL

    c, rec = env
    c.patch("v1", "Node", "gpu-a", {"metadata": {"labels": {KERNEL_LABEL: "6.8.0-45-generic"}}})
    _kernel_node(c, "gpu-b", "6.8.0-45-generic")
    _kernel_node(c, "gpu-c", "5.15.0-119-generic")
    c.create(cluster_policy(spec={"driver": {"usePrecompiled": True, "driverVersion": "6.12.12",
                                             "repository": "registry.example/amd"}}))
    rec.reconcile()
    drv = {d["metadata"]["name"]: d for d in c.list("apps/v1", "DaemonSet", NS) if "driver" in d["metadata"]["name"]}
    assert sorted(drv) == ["amd-driver-daemonset-5-15-0-119-generic", "amd-driver-daemonset-6-8-0-45-generic"]
    d = drv["amd-driver-daemonset-6-8-0-45-generic"]["spec"]["template"]["spec"]
    assert d["containers"][0]["image"] == "registry.example/amd/amd-driver:6.12.12-6.8.0-45-generic"
    assert d["nodeSelector"] == {"amd.com/gpu.deploy.driver": "true", KERNEL_LABEL: "6.8.0-45-generic"}
    env_ = {e["name"]: e.get("value") for e in d["containers"][0]["env"]}
    assert env_["AMDGPU_USE_PRECOMPILED"] == "true"
    # the node reboots into a new kernel: its DaemonSet follows, the unused one goes
    c.patch("v1", "Node", "gpu-c", {"metadata": {"labels": {KERNEL_LABEL: "6.8.0-45-generic"}}})
    rec.reconcile()
    assert [n for n in ds_names(c) if "driver" in n] == ["amd-driver-daemonset-6-8-0-45-generic"]
    # back to DKMS: the policy-wide DaemonSet, no per-kernel ones
    cp = c.list(CP_API, "ClusterPolicy")[0]
    cp["spec"]["driver"]["usePrecompiled"] = False
    c.update(cp)
    rec.reconcile()
    assert [n for n in ds_names(c) if "driver" in n] == ["amd-driver-daemonset"]


def test_precompiled_waits_for_the_kernel_label(env):
    c, rec = env  # gpu-a has no kernel-version label yet (NFD has not run)
    c.create(cluster_policy(spec={"driver": {"usePrecompiled": True}}))
    res = rec.reconcile()
    drv = next(r for r in res.states if r.name == "state-driver")
    assert not drv.ready and "no kernel-version label yet on ['gpu-a']" in drv.detail
    assert not [n for n in ds_names(c) if "driver" in n]


def test_kernel_suffix_is_a_dns_label():
    from amdgpu_operator.controller.manifests import kernel_suffix

    assert kernel_suffix("6.8.0-45-generic") == "6-8-0-45-generic"
    long = kernel_suffix("5.14.0-427.13.1.el9_4.x86_64+debug.with.a.very.long.local.suffix")
    assert len(long) <= 40 and long.replace("-", "").isalnum() and not long.startswith("-")


def test_node_labelled_by_nfd_during_a_pass_gets_its_gpu_labels_in_that_pass():
    """NFD labels the node while the first pass is still creating objects: the
    pass puts the GPU-node labels on at its next state (a Node event sets
    _nodes_changed), instead of leaving them to the next pass."""
    c = LocalClient(FakeApiServer())
    c.create(R.new("v1", "Namespace", NS))
    c.create(R.new("v1", "Node", "gpu-b"))  # not yet labelled by NFD
    rec = ClusterPolicyReconciler(c, NS)
    c.create(cluster_policy(spec=spec_from_values(parse_set_flags(REFERENCE_SET_FLAGS))))
    builders = dict(STATE_BUILDERS)

    def nfd_then_label(spec, ns, owner):
        objs = builders["state-node-feature-discovery"](spec, ns, owner)
        c.patch("v1", "Node", "gpu-b", {"metadata": {"labels": GPU_LABEL}})  # the NFD worker, mid-pass
        rec._nodes_changed = True  # what the operator's Node watch does
        return objs

    STATE_BUILDERS["state-node-feature-discovery"] = nfd_then_label
    try:
        res = rec.reconcile()
    finally:
        STATE_BUILDERS.update(builders)
    assert res.gpu_nodes == 1
    labels = c.get("v1", "Node", "gpu-b")["metadata"]["labels"]
    assert labels["amd.com/gpu.present"] == "true" and labels["amd.com/gpu.deploy.driver"] == "true"


def test_an_event_that_waited_through_a_long_pass_starts_the_next_at_once():
    """Debounce: an event right behind a pass waits out the window (echoes of
    the pass's own writes coalesce); an event that came in during a long pass
    has waited already and the next pass starts at once."""
    import queue
    import threading
    import time

    rec = ClusterPolicyReconciler(None, NS)
    events: queue.Queue = queue.Queue()
    starts, stop = [], threading.Event()

    class Res:
        state = "notReady"

    def fake_reconcile():
        starts.append(time.monotonic())
        if len(starts) == 1:
            time.sleep(0.3)
            events.put(("Node", time.monotonic() - 0.25))  # came in 0.25 s ago, mid-pass
        elif len(starts) == 2:
            events.put(("DaemonSet", time.monotonic() + 0.0))  # right behind this pass: an echo
        else:
            stop.set()
        return Res()

    rec.reconcile = fake_reconcile
    events.put(("start", time.monotonic()))
    t = threading.Thread(target=rec._loop, args=(stop, events, 30.0, 0.2, None))
    t.start()
    t.join(5)
    assert len(starts) == 3
    assert starts[1] - starts[0] < 0.3 + 0.1  # no debounce wait after the long pass
    assert starts[2] - starts[1] >= 0.19  # the echo waited out the window


def test_states_apply_validator_early_and_report_in_order(env):
    """A pass applies the validator's objects right after the driver's (its
    pod starts the bring-up's longest chain) and reports the states in the
    ClusterPolicy's order."""
    from amdgpu_operator.api.clusterpolicy import STATES
    from amdgpu_operator.controller.reconciler import APPLY_ORDER

    c, rec = env
    order = [s for s, _ in APPLY_ORDER]
    assert order[:4] == ["pre-requisites", "state-node-feature-discovery", "state-driver", "state-operator-validation"]
    assert sorted(order) == sorted(s for s, _ in STATES)
    created = []
    orig = c.create

    def record(obj):
        if obj.get("kind") == "DaemonSet":
            created.append(obj["metadata"]["name"])
        return orig(obj)

    c.create = record
    c.create(cluster_policy(spec=spec_from_values(parse_set_flags(REFERENCE_SET_FLAGS))))
    res = rec.reconcile()
    assert [r.name for r in res.states] == [s for s, _ in STATES]
    assert created.index("amd-operator-validator") < created.index("amd-container-toolkit-daemonset")
    assert created.index("amd-driver-daemonset") < created.index("amd-operator-validator")
