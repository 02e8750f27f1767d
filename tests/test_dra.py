"""DRA driver ``gpu.amd.com`` (dra/): ResourceSlice content, kubelet
registration, NodePrepareResources / NodeUnprepareResources with CDI specs
and a checkpoint, the structured-parameters allocator of the simulated
scheduler, and the wire codec against google.protobuf."""

import json
import os

import grpc
import pytest

from amdgpu_operator.dra import api
from amdgpu_operator.dra.driver import DraDriver, device_class, resource_slice
from amdgpu_operator.discovery import topology as T
from amdgpu_operator.kube import resources as R
from amdgpu_operator.kube.client import LocalClient
from amdgpu_operator.kube.fakeapi import FakeApiServer
from amdgpu_operator.nodeenv import NodeEnv
from amdgpu_operator.testing import fakedra, fakesys

RV1B1 = "resource.k8s.io/v1beta1"


def _claim(name, count=1, selectors=(), constraints=(), mode=None, ns="default"):
    req = {"name": "gpus", "deviceClassName": api.DRIVER_NAME, "count": count,
           "selectors": [{"cel": {"expression": e}} for e in selectors]}
    if mode:
        req["allocationMode"] = mode
        req.pop("count")
    return {"apiVersion": RV1B1, "kind": "ResourceClaim", "metadata": {"name": name, "namespace": ns},
            "spec": {"devices": {"requests": [req], "constraints": list(constraints)}}}


@pytest.fixture
def short_tmp():
    """unix socket paths are limited to 107 bytes; xdist's tmp_path can exceed it"""
    import shutil
    import tempfile

    d = tempfile.mkdtemp(prefix="dra", dir="/tmp")
    yield __import__("pathlib").Path(d)
    shutil.rmtree(d, ignore_errors=True)


@pytest.fixture
def node(short_tmp):
    tmp_path = short_tmp
    root = str(tmp_path / "host")
    fakesys.build_node(root, 8)
    c = LocalClient(FakeApiServer())
    c.create(R.new("v1", "Node", "n1"))
    c.create(device_class())
    env = NodeEnv("n1", c, host_root=root, validations_dir=str(tmp_path / "val"), poll_s=0.01,
                  device_plugin_dir=str(tmp_path / "kubelet" / "device-plugins"), cdi_dir=str(tmp_path / "cdi"))
    drv = DraDriver(env)
    drv.publish()
    drv.serve()
    yield env, drv, str(tmp_path / "kubelet")
    drv.stop()


def test_slice_lists_every_device_with_its_attributes(tmp_path):
    root = str(tmp_path / "cpx")
    fakesys.build_node(root, 2, compute_partition="CPX")
    gpus = T.enumerate_gpus(root)
    s = resource_slice("n1", gpus, "uid-1", "6.12.12")
    devs = s["spec"]["devices"]
    assert s["spec"]["driver"] == "gpu.amd.com" and s["spec"]["pool"] == {"name": "n1", "generation": 1,
                                                                           "resourceSliceCount": 1}
    assert [d["name"] for d in devs] == [f"gpu-{i}" for i in range(16)]
    a = devs[9]["basic"]["attributes"]
    assert a["productName"] == {"string": "AMD-Instinct-MI355X"} and a["architecture"] == {"string": "gfx950"}
    assert a["computePartition"] == {"string": "CPX"} and a["physicalIndex"] == {"int": 1}
    assert a["partitionIndex"] == {"int": 1} and a["driverVersion"] == {"version": "6.12.12"}
    assert devs[9]["basic"]["capacity"]["computeUnits"] == {"value": str(gpus[9].cu_count)}
    assert s["metadata"]["ownerReferences"][0]["kind"] == "Node"


def test_register_allocate_prepare_unprepare(node):
    env, drv, kdir = node
    k = fakedra.FakeDraKubelet(kdir)
    assert k.discover() == {api.DRIVER_NAME: drv.endpoint} and drv.registered.is_set()
    c = env.client
    # 2 GPUs on one NUMA node with at least 200 GiB each
    claim = c.create(_claim("job", 2, selectors=['device.capacity["gpu.amd.com"].memory.compareTo(quantity("200Gi")) >= 0',
                                                 'device.attributes["gpu.amd.com"].productName == "AMD-Instinct-MI355X"'],
                            constraints=[{"matchAttribute": "gpu.amd.com/numaNode"}]))
    claim = fakedra.allocate(c, claim, "n1")
    res = claim["status"]["allocation"]["devices"]["results"]
    assert len(res) == 2 and {r["pool"] for r in res} == {"n1"}
    gpus = {f"gpu-{g.index}": g for g in T.enumerate_gpus(env.sysfs_root())}
    assert len({gpus[r["device"]].numa_node for r in res}) == 1
    out = k.prepare(api.DRIVER_NAME, [claim])[claim["metadata"]["uid"]]
    assert not out.error and [d.device_name for d in out.devices] == [r["device"] for r in res]
    uid = claim["metadata"]["uid"]
    assert out.devices[0].cdi_device_ids == [f"gpu.amd.com/claim={uid}-{res[0]['device']}"]
    with open(drv.cdi_path(uid)) as f:
        spec = json.load(f)
    assert spec["kind"] == "gpu.amd.com/claim" and spec["containerEdits"]["deviceNodes"][0]["path"] == "/dev/kfd"
    assert [d["containerEdits"]["deviceNodes"][0]["path"] for d in spec["devices"]] == \
        [gpus[r["device"]].render_node for r in res]
    # idempotent, and a restarted driver answers from its checkpoint
    assert k.prepare(api.DRIVER_NAME, [claim])[uid].devices[0].device_name == res[0]["device"]
    drv2 = DraDriver(env)
    assert drv2.prepared[uid]["devices"] == drv.prepared[uid]["devices"]
    # a second claim gets other devices; a claim asking for too many fails to allocate
    other = fakedra.allocate(c, c.create(_claim("job2", 6)), "n1")
    assert not ({r["device"] for r in res} & {r["device"] for r in other["status"]["allocation"]["devices"]["results"]})
    with pytest.raises(ValueError, match="no fitting set"):
        fakedra.allocate(c, c.create(_claim("job3", 1)), "n1")
    assert not k.unprepare(api.DRIVER_NAME, [claim])[uid].error
    assert not os.path.exists(drv.cdi_path(uid)) and uid not in drv.prepared
    assert not k.unprepare(api.DRIVER_NAME, [claim])[uid].error  # again: still fine


def test_prepare_errors_name_the_claim(node):
    env, drv, kdir = node
    k = fakedra.FakeDraKubelet(kdir)
    k.discover()
    c = env.client
    claim = c.create(_claim("a", 1))
    unalloc = k.prepare(api.DRIVER_NAME, [claim])[claim["metadata"]["uid"]]
    assert "no gpu.amd.com device allocated on n1" in unalloc.error
    fake = dict(claim, metadata=dict(claim["metadata"], uid="not-the-uid"))
    assert "kubelet asked for not-the-uid" in k.prepare(api.DRIVER_NAME, [fake])["not-the-uid"].error
    gone = dict(claim, metadata=dict(claim["metadata"], name="gone"))
    assert "not found" in k.prepare(api.DRIVER_NAME, [gone])[claim["metadata"]["uid"]].error


def test_allocation_modes_and_selectors(node):
    env, _, _ = node
    c = env.client
    every = fakedra.allocate(c, c.create(_claim("all", mode="All")), "n1")
    assert len(every["status"]["allocation"]["devices"]["results"]) == 8
    c.delete(RV1B1, "ResourceClaim", "all", "default")
    none = c.create(_claim("big", 1, selectors=['device.attributes["gpu.amd.com"].computePartition == "CPX"']))
    with pytest.raises(ValueError):
        fakedra.allocate(c, none, "n1")
    with pytest.raises(ValueError, match="supported subset"):
        fakedra.cel_match('device.attributes["gpu.amd.com"].productName.startsWith("AMD")', api.DRIVER_NAME, {})
    assert fakedra.quantity("288Gi") == 288 << 30 and fakedra.quantity("1500M") == 1_500_000_000


def test_grpcio_kubelet_calls_the_dra_endpoint(node):
    """The DRA endpoint against grpcio as the kubelet-side client."""
    env, drv, _ = node
    claim = fakedra.allocate(env.client, env.client.create(_claim("g", 1)), "n1")
    i, o, _ = api.DRA_METHODS["NodePrepareResources"]
    ipb, opb = api.protobuf_classes()[0]["NodePrepareResourcesRequest"], \
        api.protobuf_classes()[0]["NodePrepareResourcesResponse"]
    req = ipb()
    req.claims.add(namespace="default", uid=claim["metadata"]["uid"], name="g")
    with grpc.insecure_channel("unix:" + drv.endpoint) as ch:
        call = ch.unary_unary(api.method_path(api.DRA_SERVICE, "NodePrepareResources"),
                              request_serializer=ipb.SerializeToString, response_deserializer=opb.FromString)
        resp = call(req, timeout=5)
        old = ch.unary_unary(api.method_path(api.DRA_SERVICE_V1ALPHA4, "NodePrepareResources"),
                             request_serializer=ipb.SerializeToString, response_deserializer=opb.FromString)
        assert not old(req, timeout=5).claims[claim["metadata"]["uid"]].error  # a 1.31 kubelet's service name
    got = resp.claims[claim["metadata"]["uid"]]  # a real proto3 map on the google.protobuf side
    assert not got.error and got.devices[0].pool_name == "n1" and got.devices[0].cdi_device_ids[0].startswith(
        "gpu.amd.com/claim=")
    assert i and o


def test_codec_matches_google_protobuf_for_dra_messages():
    d_pb, r_pb = api.protobuf_classes()
    ours = api.dra["NodePrepareResourcesResponse"]()
    r = api.dra["NodePrepareResourceResponse"](error="")
    r.devices.add(request_names=["gpus"], pool_name="n1", device_name="gpu-3", cdi_device_ids=["gpu.amd.com/claim=u-gpu-3"])
    ours.claims.add(key="u", value=r)
    theirs = d_pb["NodePrepareResourcesResponse"].FromString(ours.SerializeToString())
    assert theirs.claims["u"].devices[0].device_name == "gpu-3"
    assert api.dra["NodePrepareResourcesResponse"].FromString(theirs.SerializeToString()).claims[0].key == "u"
    info = api.reg["PluginInfo"](type="DRAPlugin", name="gpu.amd.com", endpoint="/x", supported_versions=["v1beta1.DRAPlugin"])
    assert r_pb["PluginInfo"].FromString(info.SerializeToString()).supported_versions == ["v1beta1.DRAPlugin"]


@pytest.mark.parametrize("processes", [False, True], ids=["threads", "processes"])
def test_policy_deploys_the_dra_driver_on_the_simulated_cluster(short_tmp, processes):
    """draDriver.enabled (device plugin off): the operator creates the
    DeviceClass and the driver DaemonSet; the node's ResourceSlice lists its
    GPUs; a claim allocated from it is prepared through the kubelet's DRA
    side into a CDI spec on the node; the policy refuses both advertisers."""
    from amdgpu_operator.api.clusterpolicy import REFERENCE_SET_FLAGS, parse_set_flags, spec_from_values
    from amdgpu_operator.testing.simcluster import NodeSpec, SimCluster

    with pytest.raises(ValueError, match="devicePlugin.enabled=false"):
        spec_from_values(parse_set_flags(REFERENCE_SET_FLAGS + ["draDriver.enabled=true"]))
    flags = REFERENCE_SET_FLAGS + ["draDriver.enabled=true", "devicePlugin.enabled=false"]
    c = SimCluster(str(short_tmp / "c"), [NodeSpec("gpu-1", 4)], fake_gpu=True,
                   process_containers=processes).start()  # processes: the operand images' entry point
    try:
        c.install_operator(parse_set_flags(flags))
        c.wait_ready(60)
        env = c.nodes["gpu-1"].env
        from amdgpu_operator.validator.validate import read_ready

        plug = read_ready(env, "plugin")  # the validator proved the DRA path: a claim for all 4, one pod
        assert plug["pod_mode"] == "dra" and plug["devices_validated"] == 4, plug
        assert not c.client.list(RV1B1, "ResourceClaim")  # its claim is gone again
        from amdgpu_operator.cli.verify import verify

        rep = verify(c.client, c.namespace, expect_gpus_per_node=4)
        assert rep.ok and next(x for x in rep.checks if x.name == "resourceslice[gpu-1]").ok, rep.table()
        import time

        deadline = time.monotonic() + 10  # the kubelet unprepares the claim once the deleted pod has stopped
        while any(f.startswith("gpu.amd.com-claim_") for f in os.listdir(env.cdi_dir)) and time.monotonic() < deadline:
            time.sleep(0.05)
        assert not any(f.startswith("gpu.amd.com-claim_") for f in os.listdir(env.cdi_dir))
        assert not c.nodes["gpu-1"].kubelet.claims  # pod-resources no longer lists the stopped pod's claims
        slices = c.client.list(RV1B1, "ResourceSlice")
        assert len(slices) == 1 and len(slices[0]["spec"]["devices"]) == 4 and slices[0]["spec"]["nodeName"] == "gpu-1"
        assert c.client.get(RV1B1, "DeviceClass", "gpu.amd.com")
        env = c.nodes["gpu-1"].env
        k = fakedra.FakeDraKubelet(os.path.dirname(env.device_plugin_dir.rstrip("/")))
        deadline = time.monotonic() + 10
        while not k.discover() and time.monotonic() < deadline:
            time.sleep(0.05)
        claim = fakedra.allocate(c.client, c.client.create(_claim("train", 4, constraints=[
            {"matchAttribute": "gpu.amd.com/xgmiHive"}])), "gpu-1")
        out = k.prepare(api.DRIVER_NAME, [claim])[claim["metadata"]["uid"]]
        assert not out.error and len(out.devices) == 4
        assert os.path.exists(os.path.join(env.cdi_dir, f"gpu.amd.com-claim_{claim['metadata']['uid']}.json"))
    finally:
        c.stop()


@pytest.mark.gpu
def test_real_mi355x_slice_and_claim(short_tmp):
    """On the MI355X box: the slice built from the real KFD topology, and a
    claim for it prepared into a CDI spec naming the real render node."""
    c = LocalClient(FakeApiServer())
    c.create(R.new("v1", "Node", "box"))
    c.create(device_class())
    env = NodeEnv("box", c, host_root="/", validations_dir=str(short_tmp / "val"), poll_s=0.01,
                  device_plugin_dir=str(short_tmp / "kubelet" / "device-plugins"), cdi_dir=str(short_tmp / "cdi"))
    drv = DraDriver(env)
    drv.serve()
    try:
        s = drv.publish()
        dev = s["spec"]["devices"][0]
        print(json.dumps(s["spec"]))
        assert dev["basic"]["attributes"]["architecture"] == {"string": "gfx950"}
        assert int(dev["basic"]["capacity"]["memory"]["value"][:-2]) > 250_000  # MiB of HBM3E
        k = fakedra.FakeDraKubelet(str(short_tmp / "kubelet"))
        assert k.discover() == {api.DRIVER_NAME: drv.endpoint}
        claim = fakedra.allocate(c, c.create(_claim("one", 1, selectors=[
            'device.attributes["gpu.amd.com"].family == "CDNA4"'])), "box")
        out = k.prepare(api.DRIVER_NAME, [claim])[claim["metadata"]["uid"]]
        assert not out.error
        with open(drv.cdi_path(claim["metadata"]["uid"])) as f:
            spec = json.load(f)
        node = spec["devices"][0]["containerEdits"]["deviceNodes"][0]["path"]
        assert node.startswith("/dev/dri/renderD") and os.path.exists(node)
    finally:
        drv.stop()


@pytest.mark.gpu
def test_real_mi355x_exporter_attributes_the_claim_holder(short_tmp):
    """On the MI355X box: a claim prepared by the DRA driver, reported by the
    kubelet's pod-resources API as the container's dynamic_resources, labels
    the live amd-smi series of exactly that GPU with the pod (the DRA device
    name resolved to the BDF amd-smi reports)."""
    from amdgpu_operator.exporter.metrics import MetricsExporter, PodAttribution, SmiSource, device_id_resolver
    from amdgpu_operator.testing.fakekubelet import FakeKubelet

    c = LocalClient(FakeApiServer())
    c.create(R.new("v1", "Node", "box"))
    c.create(device_class())
    env = NodeEnv("box", c, host_root="/", validations_dir=str(short_tmp / "val"), poll_s=0.01,
                  device_plugin_dir=str(short_tmp / "kubelet" / "device-plugins"), cdi_dir=str(short_tmp / "cdi"))
    drv = DraDriver(env)
    drv.serve()
    sock = str(short_tmp / "podres" / "kubelet.sock")
    kl = FakeKubelet(str(short_tmp / "dp"), sock)
    kl.start()
    src = SmiSource()
    try:
        drv.publish()
        k = fakedra.FakeDraKubelet(str(short_tmp / "kubelet"))
        k.discover()
        claim = fakedra.allocate(c, c.create(_claim("train", 1)), "box")
        out = k.prepare(api.DRIVER_NAME, [claim])[claim["metadata"]["uid"]]
        assert not out.error
        kl.record_claims("ml", "trainer", "main", [{"claim": ("default", "train"), "resources": [
            (api.DRIVER_NAME, d.pool_name, d.device_name, list(d.cdi_device_ids)) for d in out.devices]}])
        held = drv.by_name[out.devices[0].device_name]
        ex = MetricsExporter(src, "box", attribution=PodAttribution(sock, dra_driver=api.DRIVER_NAME,
                                                                     resolve=device_id_resolver("/")))
        ex.collect_once()
        assert ex.errors == 0
        lines = [ln for ln in ex.render().splitlines() if ln.startswith("amd_gpu_power_watts{")]
        print("\n".join(lines))
        mine = [ln for ln in lines if f'bdf="{held.bdf}"' in ln]
        assert mine and all('pod="trainer"' in ln and 'namespace="ml"' in ln for ln in mine), (held.bdf, lines)
        assert not any('pod="trainer"' in ln for ln in lines if ln not in mine)
    finally:
        src.close()
        kl.stop()
        drv.stop()


def test_partition_change_republishes_with_a_new_generation(node):
    env, drv, _ = node
    assert not drv.refresh()
    root = env.sysfs_root()
    import shutil

    shutil.rmtree(os.path.join(root, "sys/class/kfd/kfd/topology/nodes"))
    fakesys.build_node(root, 8, compute_partition="DPX")
    assert drv.refresh()
    s = env.client.get(RV1B1, "ResourceSlice", f"n1-{api.DRIVER_NAME}")
    assert len(s["spec"]["devices"]) == 16 and s["spec"]["pool"]["generation"] == 2
    assert s["spec"]["devices"][1]["basic"]["attributes"]["computePartition"] == {"string": "DPX"}
    # a restarted driver publishing the same devices leaves the slice (and its generation) alone
    rv = s["metadata"]["resourceVersion"]
    again = DraDriver(env).publish()
    assert again["spec"]["pool"]["generation"] == 2 and again["metadata"]["resourceVersion"] == rv


def test_exporter_attributes_dra_claims_via_pod_resources(short_tmp):
    """Pod attribution of GPU metrics with DRA: the kubelet's pod-resources
    List reports a container's prepared claims as dynamic_resources
    (driver/pool/device, kubelet >= 1.31); the exporter maps the DRA device
    names (partitions too) back to the BDF[-pN] IDs its samples carry."""
    from amdgpu_operator.exporter.metrics import PodAttribution, device_id_resolver
    from amdgpu_operator.testing.fakekubelet import FakeKubelet

    root = str(short_tmp / "cpx")
    fakesys.build_node(root, 2, compute_partition="CPX")
    gpus = T.enumerate_gpus(root)
    sock = str(short_tmp / "podres" / "kubelet.sock")
    k = FakeKubelet(str(short_tmp / "dp"), sock)
    k.start()
    try:
        k.assignments[("ml", "legacy", "main")] = ("amd.com/gpu", [gpus[0].device_id_str])
        k.record_claims("ml", "trainer", "main", [{"claim": ("ml", "train-gpus"), "resources": [
            (api.DRIVER_NAME, "n1", "gpu-9", ["gpu.amd.com/claim=u-gpu-9"]),
            (api.DRIVER_NAME, "n1", "gpu-10", ["gpu.amd.com/claim=u-gpu-10"])]}])
        k.record_claims("ml", "other", "main", [{"claim": ("ml", "nic"), "resources": [
            ("rdma.example.com", "n1", "gpu-3", [])]}])  # another driver's device of the same name
        m = PodAttribution(sock, dra_driver=api.DRIVER_NAME, resolve=device_id_resolver(root)).lookup()
        who = {"namespace": "ml", "pod": "trainer", "container": "main"}
        assert m[gpus[9].device_id_str] == who and m[gpus[10].device_id_str] == who
        assert gpus[9].device_id_str.endswith("-p1") and gpus[9].bdf == gpus[10].bdf != gpus[0].bdf
        assert m[gpus[0].device_id_str]["pod"] == "legacy" and gpus[3].device_id_str not in m
        assert not any(v["pod"] == "other" for v in m.values())
        # the plugin's uuid / index deviceIDStrategy IDs resolve to the same BDF[-pN]
        from amdgpu_operator.deviceplugin.server import base_id

        k.assignments[("ml", "by-uuid", "main")] = ("amd.com/gpu", [base_id(gpus[5], "uuid")])
        k.assignments[("ml", "by-index", "main")] = ("amd.com/gpu", [base_id(gpus[12], "index")])
        k.assignments[("ml", "sliced", "main")] = ("amd.com/gpu", [gpus[14].device_id_str + "::3"])
        m = PodAttribution(sock, dra_driver=api.DRIVER_NAME, resolve=device_id_resolver(root)).lookup()
        assert m[gpus[5].device_id_str]["pod"] == "by-uuid" and m[gpus[12].device_id_str]["pod"] == "by-index"
        assert m[gpus[14].device_id_str]["pod"] == "sliced"  # a time-sliced replica counts for its GPU
        for pod in ("by-uuid", "by-index", "sliced"):
            del k.assignments[("ml", pod, "main")]
        # without a DRA driver name only device-plugin allocations count
        assert set(PodAttribution(sock).lookup()) == {gpus[0].device_id_str}
        k.release("ml", "trainer")
        assert gpus[9].device_id_str not in PodAttribution(sock, dra_driver=api.DRIVER_NAME,
                                                            resolve=device_id_resolver(root)).lookup()
    finally:
        k.stop()


def _check_ctr(name, claims, expect):
    return {"name": name, "image": "registry.local/amd-gpu-operator/amd-operator-validator:0.1.0",
            "command": ["amdgpu-gpu-check"], "args": ["--timeout", "30", "--expect-devices", str(expect)],
            "resources": {"claims": [{"name": x} for x in claims]}}


@pytest.mark.parametrize("processes", [False, True], ids=["threads", "processes"])
def test_claims_apply_per_container(short_tmp, processes):
    """A CDI runtime gives a container the devices of the claims its
    ``resources.claims`` names, and composes their specs: one container
    holding two claims sees both GPUs (the specs' edits compose: no
    variable set twice), two containers of one pod holding one claim each
    see one GPU each - different ones - and a container naming no claim
    sees none."""
    from amdgpu_operator.api.clusterpolicy import REFERENCE_SET_FLAGS, parse_set_flags
    from amdgpu_operator.testing.simcluster import NodeSpec, SimCluster

    flags = REFERENCE_SET_FLAGS + ["draDriver.enabled=true", "devicePlugin.enabled=false"]
    c = SimCluster(str(short_tmp / "c"), [NodeSpec("gpu-1", 4)], fake_gpu=True, process_containers=processes).start()
    try:
        c.install_operator(parse_set_flags(flags))
        c.wait_ready(60)
        for n in ("a", "b", "x", "y"):
            c.client.create(_claim(n, 1))

        def pod(name, ctrs, claims):
            return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": "default"},
                    "spec": {"restartPolicy": "Never", "nodeSelector": {"kubernetes.io/hostname": "gpu-1"},
                             "resourceClaims": [{"name": x, "resourceClaimName": x} for x in claims],
                             "containers": ctrs}}

        c.client.create(pod("both", [_check_ctr("check", ["a", "b"], 2)], ["a", "b"]))
        c.client.create(pod("split", [_check_ctr("left", ["x"], 1), _check_ctr("right", ["y"], 1),
                                      _check_ctr("none", [], 0)], ["x", "y"]))
        import time

        def phase(n):
            return (c.client.get("v1", "Pod", n, "default").get("status") or {}).get("phase")

        deadline = time.monotonic() + 30
        while time.monotonic() < deadline and not {phase("both"), phase("split")} <= {"Succeeded", "Failed"}:
            time.sleep(0.05)
        assert phase("both") == "Succeeded", c.client.get("v1", "Pod", "both", "default")["status"]
        assert phase("split") == "Succeeded", c.client.get("v1", "Pod", "split", "default")["status"]
        rep = c.container_reports
        both = rep[("both", "check")]["rocr_visible_devices"].split(",")
        left = rep[("split", "left")]["rocr_visible_devices"].split(",")
        right = rep[("split", "right")]["rocr_visible_devices"].split(",")
        assert len(both) == 2 and len(left) == len(right) == 1 and left != right
        assert rep[("split", "none")]["rocr_visible_devices"] == ""
        alloc = {n: c.client.get(RV1B1, "ResourceClaim", n, "default")["status"]["allocation"]["devices"]["results"][0]
                 ["device"] for n in ("a", "b", "x", "y")}
        assert len(set(alloc.values())) == 4  # four claims, four GPUs
    finally:
        c.stop()


def test_cdi_specs_of_two_claims_compose(node):
    """The driver's per-claim specs, resolved together as a runtime does
    (toolkit/cdi.py, strict): /dev/kfd once, both render nodes, no variable
    set twice.  A spec set that does set one twice fails in strict mode."""
    from amdgpu_operator.toolkit import cdi

    env, drv, kdir = node
    k = fakedra.FakeDraKubelet(kdir)
    k.discover()
    ids = []
    for n in ("p", "q"):
        claim = fakedra.allocate(env.client, env.client.create(_claim(n, 1)), "n1")
        ids += k.prepare(api.DRIVER_NAME, [claim])[claim["metadata"]["uid"]].devices[0].cdi_device_ids
    e = cdi.resolve(env.cdi_dir, ids, strict=True)
    paths = [d["path"] for d in e.device_nodes]
    assert paths.count("/dev/kfd") == 1 and len([p for p in paths if "renderD" in p]) == 2 and not e.conflicts
    with pytest.raises(cdi.CDIError, match="unresolvable"):
        cdi.resolve(env.cdi_dir, ids + ["gpu.amd.com/claim=nope"])
    # the round-4 spec shape (AMD_VISIBLE_DEVICES at spec level) collides when composed
    for i, path in enumerate(sorted(f for f in os.listdir(env.cdi_dir) if f.startswith("gpu.amd.com-claim_"))):
        with open(os.path.join(env.cdi_dir, path)) as f:
            spec = json.load(f)
        spec["containerEdits"]["env"] = [f"AMD_VISIBLE_DEVICES={i}"]
        with open(os.path.join(env.cdi_dir, path), "w") as f:
            json.dump(spec, f)
    assert cdi.resolve(env.cdi_dir, ids).conflicts
    with pytest.raises(cdi.CDIError, match="set a variable twice"):
        cdi.resolve(env.cdi_dir, ids, strict=True)
