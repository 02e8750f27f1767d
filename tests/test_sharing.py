"""Device-plugin config file: GPU time-slicing, device-ID / device-list
strategies, per-node config selection, GFD sharing labels, and the OCI hook's
device-list policy (deviceplugin/config.py, README.md:220 of the reference
points at k8s-device-plugin, whose config shape this follows)."""

import json
import subprocess
import time

import grpc
import pytest

from amdgpu_operator import native
from amdgpu_operator.api.clusterpolicy import REFERENCE_SET_FLAGS, deep_merge, parse_set_flags
from amdgpu_operator.deviceplugin import config as DC
from amdgpu_operator.deviceplugin.server import DevicePluginManager, PluginConfig
from amdgpu_operator.discovery import labels as L
from amdgpu_operator.discovery import topology as T
from amdgpu_operator.testing import fakesys
from amdgpu_operator.testing.fakekubelet import FakeKubelet
from amdgpu_operator.testing.simcluster import NodeSpec, SimCluster

SHARED4 = """
version: v1
sharing:
  timeSlicing:
    resources:
    - name: amd.com/gpu
      replicas: 4
"""


@pytest.fixture
def node(tmp_path):
    root = str(tmp_path / "host")
    fakesys.build_node(root, 8)
    k = FakeKubelet(str(tmp_path / "dp"))
    k.start()
    yield root, str(tmp_path / "dp"), k
    k.stop()


def _start(root, sock_dir, text):
    cfg = PluginConfig(socket_dir=sock_dir, sysfs_root=root, watch_interval_s=0.05, device_config=DC.parse(text))
    m = DevicePluginManager(cfg)
    m.start()
    return m


# ----------------------------------------------------------------- config file
def test_config_defaults_and_validation():
    c = DC.parse("")
    assert c.flags.deviceListStrategy == ["envvar"] and c.sharing_strategy == "none"
    c = DC.parse(SHARED4)
    assert c.shared_for("amd.com/gpu").replicas == 4 and c.sharing_strategy == "time-slicing"
    assert DC.parse("flags: {deviceListStrategy: cdi-cri}").flags.deviceListStrategy == ["cdi-cri"]
    for bad in ("flags: {deviceIDStrategy: serial}", "sharing: {timeSlicing: {resources: [{replicas: 0}]}}",
                "version: v2", "flags: {bogus: 1}", "flags: {deviceListStrategy: []}"):
        with pytest.raises(ValueError):
            DC.parse(bad)


def test_config_selection_by_node_label():
    data = {"default": "", "shared": SHARED4}
    assert DC.select(data, {}, "")[0] == ""
    assert DC.select(data, {}, "default")[0] == "default"
    key, cfg = DC.select(data, {DC.CONFIG_LABEL: "shared"}, "default")
    assert key == "shared" and cfg.shared_for("amd.com/gpu").replicas == 4
    with pytest.raises(KeyError):
        DC.select(data, {DC.CONFIG_LABEL: "missing"}, "default")


# -------------------------------------------------------------- time-slicing
def test_time_slicing_advertises_replicas_and_maps_them_back(node):
    root, sock, k = node
    m = _start(root, sock, SHARED4)
    try:
        assert k.wait_registered("amd.com/gpu", 10, min_devices=32)
        assert k.allocatable("amd.com/gpu") == 32
        ids, resp = k.allocate("amd.com/gpu", 1, pod="a")
        assert "::" in ids[0]
        assert resp.annotations["amd.com/gpu.sharing"] == "time-slicing"
        assert len(resp.envs["AMD_VISIBLE_DEVICES"].split(",")) == 1
        # two replicas of one GPU in one container -> one render node, one index
        srv = m.servers["amd.com/gpu"]
        gpu0 = [i for i in srv._ids_of[m.devices[0].device_id_str]]
        r = srv.container_response(gpu0[:2])
        assert r.envs["AMD_VISIBLE_DEVICES"] == str(m.devices[0].index)
        assert [d.host_path for d in r.devices].count(m.devices[0].render_node) == 1
    finally:
        m.stop()


def test_preferred_allocation_spreads_replicas_least_loaded_first(node):
    root, sock, k = node
    m = _start(root, sock, SHARED4)
    try:
        assert k.wait_registered("amd.com/gpu", 10, min_devices=32)
        srv = m.servers["amd.com/gpu"]
        gpus = []
        for n in range(8):  # eight 1-replica pods land on eight different GPUs
            ids, _ = k.allocate("amd.com/gpu", 1, pod=f"p{n}")
            gpus.append(srv._by_id[ids[0]].device_id_str)
        assert len(set(gpus)) == 8
        ids, _ = k.allocate("amd.com/gpu", 3, pod="multi")  # one container, 3 replicas -> 3 GPUs
        assert len({srv._by_id[i].device_id_str for i in ids}) == 3
    finally:
        m.stop()


def test_fail_requests_greater_than_one_and_rename(node):
    root, sock, k = node
    m = _start(root, sock, """
sharing:
  timeSlicing:
    renameByDefault: true
    failRequestsGreaterThanOne: true
    resources: [{name: amd.com/gpu, replicas: 2}]
""")
    try:
        assert k.wait_registered("amd.com/gpu.shared", 10, min_devices=16)
        assert "amd.com/gpu" not in k.resources
        k.allocate("amd.com/gpu.shared", 1, pod="one")
        with pytest.raises(grpc.RpcError) as e:
            k.allocate("amd.com/gpu.shared", 2, pod="two")
        assert e.value.code() == grpc.StatusCode.INVALID_ARGUMENT
    finally:
        m.stop()


def test_health_flip_marks_every_replica(node):
    root, sock, k = node
    m = _start(root, sock, SHARED4)
    try:
        assert k.wait_registered("amd.com/gpu", 10, min_devices=32)
        before = k.resources["amd.com/gpu"].updates
        m.set_health(m.devices[3].device_id_str, False, "test")
        assert k.wait_update("amd.com/gpu", before, 5)
        assert k.allocatable("amd.com/gpu") == 28
    finally:
        m.stop()


def test_subset_sharing_needs_distinct_names(tmp_path):
    root = str(tmp_path / "h")
    fakesys.build_node(root, 4)
    cfg = PluginConfig(socket_dir=str(tmp_path / "dp"), sysfs_root=root, device_config=DC.parse(
        "sharing: {timeSlicing: {resources: [{name: amd.com/gpu, replicas: 2, devices: [0, 1]}]}}"))
    with pytest.raises(ValueError, match="distinct names"):
        DevicePluginManager(cfg)
    cfg.device_config = DC.parse("sharing: {timeSlicing: {resources: "
                                 "[{name: amd.com/gpu, rename: amd.com/gpu-shared, replicas: 2, devices: [0, 1]}]}}")
    m = DevicePluginManager(cfg)
    assert {r: len(s._by_id) for r, s in m.servers.items()} == {"amd.com/gpu-shared": 4, "amd.com/gpu": 2}


# --------------------------------------------------------- ID / list strategies
@pytest.mark.parametrize("strategy", ["bdf", "uuid", "index"])
def test_device_id_strategies(node, strategy):
    root, sock, k = node
    m = _start(root, sock, f"flags: {{deviceIDStrategy: {strategy}}}")
    try:
        assert k.wait_registered("amd.com/gpu", 10, min_devices=8)
        ids = sorted(k.resources["amd.com/gpu"].devices)
        gpus = T.enumerate_gpus(root)
        want = {"bdf": [g.bdf for g in gpus], "index": [str(g.index) for g in gpus],
                "uuid": [f"GPU-{g.unique_id:016x}" for g in gpus]}[strategy]
        assert ids == sorted(want)
        got, resp = k.allocate("amd.com/gpu", 1, pod="x")
        assert resp.envs["AMD_GPU_DEVICE_IDS"] == got[0]
    finally:
        m.stop()


def test_device_list_strategies_and_no_device_specs(node):
    root, sock, k = node
    m = _start(root, sock, "flags: {deviceListStrategy: [volume-mounts, cdi-annotations, cdi-cri], "
                           "passDeviceSpecs: false}")
    try:
        assert k.wait_registered("amd.com/gpu", 10, min_devices=8)
        _, resp = k.allocate("amd.com/gpu", 2, pod="x")
        assert "AMD_VISIBLE_DEVICES" not in resp.envs and len(resp.devices) == 0
        mounts = sorted(mt.container_path for mt in resp.mounts)
        assert len(mounts) == 2 and all(p.startswith("/var/run/amd-container-devices/") for p in mounts)
        assert all(mt.host_path == "/dev/null" and mt.read_only for mt in resp.mounts)
        ann = resp.annotations["cdi.k8s.io/amd-device-plugin_amd-com-gpu"]
        assert ann.count("amd.com/gpu=") == 2
        assert [c.name for c in resp.cdi_devices] == ann.split(",")
    finally:
        m.stop()


# ------------------------------------------------------------- OCI hook policy
def _bundle(tmp_path, env=None, mounts=None, caps=None):
    b = tmp_path / "bundle"
    b.mkdir(exist_ok=True)
    proc = {"args": ["sh"], "env": env or []}
    if caps is not None:
        proc["capabilities"] = {"bounding": caps}
    spec = {"ociVersion": "1.1.0", "process": proc, "root": {"path": "rootfs"}, "mounts": mounts or [],
            "linux": {"resources": {"devices": []}}}
    (b / "config.json").write_text(json.dumps(spec))
    return str(b)


def _apply(bundle, root, *flags):
    hook = str(native.binary("amdgpu-oci-hook"))
    p = subprocess.run([hook, "apply", "--bundle", bundle, "--root", root, "--dry-run", *flags], capture_output=True,
                       text=True, timeout=30)
    assert p.returncode == 0, p.stderr
    return json.loads(p.stdout)


def test_hook_volume_mount_device_list(tmp_path):
    root = str(tmp_path / "h")
    fakesys.build_node(root, 4)
    mounts = [{"destination": "/var/run/amd-container-devices/2", "source": "/dev/null", "type": "bind"},
              {"destination": "/var/run/amd-container-devices/3", "source": "/dev/null", "type": "bind"}]
    b = _bundle(tmp_path, env=["AMD_VISIBLE_DEVICES=0"], mounts=mounts)
    assert _apply(b, root, "--accept-volume-mounts")["annotations"]["amd.com/gpu.injected"] == "2,3"
    assert _apply(b, root)["annotations"]["amd.com/gpu.injected"] == "0"  # mounts ignored unless accepted


def test_hook_envvar_privileged_only(tmp_path):
    root = str(tmp_path / "h")
    fakesys.build_node(root, 4)
    b = _bundle(tmp_path, env=["AMD_VISIBLE_DEVICES=all"], caps=["CAP_CHOWN"])
    spec = _apply(b, root, "--envvar-privileged-only")
    assert not spec.get("linux", {}).get("devices")  # unprivileged: the env cannot grant GPUs
    b = _bundle(tmp_path, env=["AMD_VISIBLE_DEVICES=all"], caps=["CAP_SYS_ADMIN"])
    assert _apply(b, root, "--envvar-privileged-only")["annotations"]["amd.com/gpu.injected"] == "0,1,2,3"


def test_toolkit_writes_hooks_d_entry_with_policy(tmp_path):
    from amdgpu_operator.toolkit import install as tk

    args = tk.hook_args(accept_volume_mounts=True, envvar_unprivileged=False)
    assert args == ["--accept-volume-mounts", "--envvar-privileged-only"]
    j = json.loads(tk.oci_hook_json("/usr/local/amd/amdgpu-oci-hook", args))
    assert j["hook"]["args"] == ["amdgpu-oci-hook", "precreate", *args] and j["stages"] == ["precreate"]
    drop = tk.dropin_config("amd", "/usr/local/amd/amdgpu-oci-hook", "/var/run/cdi", args)
    assert 'pod_annotations = ["cdi.k8s.io/*"]' in drop and "amd.com/gpu.*" not in drop


# ------------------------------------------------------------ GFD + integration
def test_gfd_sharing_labels():
    base = {"amd.com/gpu.product": "AMD-Instinct-MI355X"}
    out = L.sharing_labels(base, DC.parse(SHARED4))
    assert out["amd.com/gpu.replicas"] == "4" and out["amd.com/gpu.sharing-strategy"] == "time-slicing"
    assert out["amd.com/gpu.product"] == "AMD-Instinct-MI355X-SHARED"
    renamed = DC.parse("sharing: {timeSlicing: {renameByDefault: true, resources: [{replicas: 2}]}}")
    assert L.sharing_labels(base, renamed)["amd.com/gpu.product"] == "AMD-Instinct-MI355X"
    assert L.sharing_labels(base, None)["amd.com/gpu.sharing-strategy"] == "none"


def test_node_label_switches_plugin_config_in_cluster(tmp_path):
    c = SimCluster(str(tmp_path / "c"), [NodeSpec("gpu-1", 2)], fake_gpu=True).start()
    try:
        c.client.create({"apiVersion": "v1", "kind": "ConfigMap",
                         "metadata": {"name": "plugin-config", "namespace": c.namespace},
                         "data": {"default": "version: v1\n", "shared4": SHARED4}})
        values = deep_merge(parse_set_flags(REFERENCE_SET_FLAGS),
                            {"devicePlugin": {"config": {"name": "plugin-config", "default": "default"}},
                             "gfd": {"intervalSeconds": 0.2}})
        c.install_operator(values)
        c.wait_ready(60, {"gpu-1": 2})
        c.client.patch("v1", "Node", "gpu-1", {"metadata": {"labels": {DC.CONFIG_LABEL: "shared4"}}})
        deadline = time.time() + 30
        n = {}
        while time.time() < deadline:
            n = c.client.get("v1", "Node", "gpu-1")
            labels = n["metadata"].get("labels") or {}
            if n["status"]["allocatable"].get("amd.com/gpu") == "8" and labels.get("amd.com/gpu.replicas") == "4":
                break
            time.sleep(0.1)
        assert n["status"]["allocatable"]["amd.com/gpu"] == "8"
        assert n["metadata"]["labels"]["amd.com/gpu.sharing-strategy"] == "time-slicing"
        from amdgpu_operator.cli.verify import verify

        rep = verify(c.client, c.namespace, expect_gpus_per_node=2)  # 2 GPUs x 4 replicas
        assert rep.ok, rep.table()
    finally:
        c.stop()


def test_unknown_config_key_falls_back_to_command_line_flags(tmp_path):
    c = SimCluster(str(tmp_path / "c"), [NodeSpec("gpu-1", 2)], fake_gpu=True).start()
    try:
        c.client.patch("v1", "Node", "gpu-1", {"metadata": {"labels": {DC.CONFIG_LABEL: "no-such-key"}}})
        c.client.create({"apiVersion": "v1", "kind": "ConfigMap",
                         "metadata": {"name": "plugin-config", "namespace": c.namespace}, "data": {"shared4": SHARED4}})
        values = deep_merge(parse_set_flags(REFERENCE_SET_FLAGS),
                            {"devicePlugin": {"config": {"name": "plugin-config"}}})
        c.install_operator(values)
        c.wait_ready(60, {"gpu-1": 2})  # plugin serves unshared GPUs instead of crash-looping
    finally:
        c.stop()


def test_reconfigure_under_concurrent_allocations(node):
    """Config flips (time-slicing on/off) while pods are admitted: no deadlock,
    and the final config is what kubelet sees (SURVEY.md §5.2 race tier)."""
    import threading

    root, sock, k = node
    m = _start(root, sock, "")
    stop = threading.Event()
    done = {"ok": 0, "err": 0}

    def admit():
        n = 0
        while not stop.is_set():
            res = next(iter(k.resources), None)
            try:
                k.allocate(res, 1, pod=f"p{n}")
                k.release("default", f"p{n}")
                done["ok"] += 1
            except Exception:  # noqa: BLE001 - plugin mid-restart / resource renamed: kubelet retries
                done["err"] += 1
            n += 1

    th = threading.Thread(target=admit, daemon=True)
    try:
        assert k.wait_registered("amd.com/gpu", 10, min_devices=8)
        th.start()
        for i in range(6):
            m.reconfigure(DC.parse(SHARED4 if i % 2 == 0 else "flags: {deviceIDStrategy: index}"))
            time.sleep(0.05)
        stop.set()
        th.join(10)
        assert not th.is_alive()
        assert k.wait_registered("amd.com/gpu", 10, min_devices=8)
        deadline = time.time() + 10
        while sorted(k.resources["amd.com/gpu"].devices) != [str(i) for i in range(8)] and time.time() < deadline:
            time.sleep(0.05)
        assert sorted(k.resources["amd.com/gpu"].devices) == [str(i) for i in range(8)]  # last config: index IDs
        assert done["ok"] > 0
        ids, _ = k.allocate("amd.com/gpu", 2, pod="final")
        assert len(ids) == 2
    finally:
        stop.set()
        m.stop()


def test_device_plan_from_kubelet_view():
    from amdgpu_operator.validator.validate import _device_plan

    ids = [f"0000:{i:02x}:00.0" for i in range(4)]
    assert _device_plan({"amd.com/gpu": 4}, {"amd.com/gpu": ids[:3]}) is None
    assert _device_plan({"amd.com/gpu": 4}, {"amd.com/gpu": ids}) == {"amd.com/gpu": 4}
    # time-sliced replicas of 2 GPUs are not 4 GPUs
    reps = [f"{i}::{r}" for i in ids[:2] for r in range(2)]
    assert _device_plan({"amd.com/gpu": 4}, {"amd.com/gpu": reps}) is None
    # renamed by a config file (renameByDefault): one pod per GPU of the renamed resource
    shared = [f"{i}::{r}" for i in ids for r in range(4)]
    assert _device_plan({"amd.com/gpu": 4}, {"amd.com/gpu.shared": shared}) == {"amd.com/gpu.shared": 4}
    assert _device_plan({"amd.com/gpu": 4}, {"amd.com/gpu.shared": shared[:8], "other.io/x": ids}) is None


def test_plugin_validation_with_renamed_shared_resource(tmp_path):
    """A default plugin config that renames the time-sliced resource
    (amd.com/gpu.shared): the validator's --resource flag does not know the
    new name; it reads it from the kubelet and the node still validates."""
    c = SimCluster(str(tmp_path / "c"), [NodeSpec("gpu-1", 2)], fake_gpu=True).start()
    try:
        renamed = "version: v1\nsharing:\n  timeSlicing:\n    renameByDefault: true\n    resources:\n" \
                  "      - name: amd.com/gpu\n        replicas: 4\n"
        c.client.create({"apiVersion": "v1", "kind": "ConfigMap",
                         "metadata": {"name": "plugin-config", "namespace": c.namespace},
                         "data": {"renamed": renamed}})
        values = deep_merge(parse_set_flags(REFERENCE_SET_FLAGS),
                            {"devicePlugin": {"config": {"name": "plugin-config", "default": "renamed"}}})
        c.install_operator(values)
        c.wait_ready(60)
        n = c.client.get("v1", "Node", "gpu-1")
        assert n["status"]["allocatable"].get("amd.com/gpu.shared") == "8"
        from amdgpu_operator.validator.validate import read_ready

        plugin = read_ready(c.nodes["gpu-1"].env, "plugin")
        assert plugin["resources"] == {"amd.com/gpu.shared": 2} and plugin["allocatable_source"] == "kubelet"
    finally:
        c.stop()
