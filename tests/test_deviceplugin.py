"""Device plugin: wire format, gRPC contract against a fake kubelet, allocation
policy, health and kubelet restarts (SURVEY.md §4.2 contract tier)."""

import threading
import time

import pytest

from amdgpu_operator.deviceplugin import api
from amdgpu_operator.deviceplugin.allocator import AllocDevice, TopologyCost, preferred
from amdgpu_operator.deviceplugin.server import DevicePluginManager, PluginConfig
from amdgpu_operator.discovery import topology as T
from amdgpu_operator.testing import fakesys
from amdgpu_operator.testing.fakekubelet import FakeKubelet


def test_wire_format_matches_v1beta1_field_numbers():
    # hand-encoded protobuf for RegisterRequest{version=1, endpoint=2, resource_name=3, options=4{gpaa=2}}
    req = api.pb["RegisterRequest"](version="v1beta1", endpoint="amd.sock", resource_name="amd.com/gpu")
    req.options.get_preferred_allocation_available = True
    assert req.SerializeToString().hex() == "0a07763162657461311208616d642e736f636b1a0b616d642e636f6d2f67707522021001"
    # ContainerAllocateResponse{envs=1 map, devices=3, cdi_devices=5}
    r = api.pb["ContainerAllocateResponse"]()
    r.envs["A"] = "1"
    r.devices.add(container_path="/dev/kfd", host_path="/dev/kfd", permissions="rw")
    r.cdi_devices.add(name="amd.com/gpu=0")
    assert r.SerializeToString().hex() == (
        "0a060a0141120131" "1a180a082f6465762f6b666412082f6465762f6b66641a027277" "2a0f0a0d616d642e636f6d2f6770753d30")
    # Device{ID=1, health=2, topology=3{nodes=1{ID=1}}}
    d = api.pb["Device"](ID="x", health="Healthy")
    d.topology.nodes.add(ID=1)
    assert d.SerializeToString().hex() == "0a0178120748656" + "16c746879" + "1a040a020801"
    pa = api.pb["ContainerPreferredAllocationRequest"](available_deviceIDs=["a"], must_include_deviceIDs=["b"],
                                                      allocation_size=2)
    assert pa.SerializeToString().hex() == "0a016112016218" + "02"


@pytest.fixture
def node(tmp_path):
    root = str(tmp_path / "host")
    fakesys.build_node(root, 8)
    sock_dir = str(tmp_path / "dp")
    k = FakeKubelet(sock_dir, str(tmp_path / "podres" / "kubelet.sock"))
    k.start()
    yield root, sock_dir, k
    k.stop()


def _start(root, sock_dir, **kw):
    cfg = PluginConfig(socket_dir=sock_dir, sysfs_root=root, watch_interval_s=0.05, **kw)
    m = DevicePluginManager(cfg)
    m.start()
    return m


def test_register_and_advertise_all_gpus(node):
    root, sock_dir, k = node
    m = _start(root, sock_dir)
    try:
        assert k.wait_registered("amd.com/gpu", 10, min_devices=8)
        assert k.allocatable("amd.com/gpu") == 8
        numa = k.resources["amd.com/gpu"].numa
        assert all(len(v) == 1 for v in numa.values())
    finally:
        m.stop()


def test_allocate_returns_kfd_and_render_nodes(node):
    root, sock_dir, k = node
    m = _start(root, sock_dir, cdi_enabled=True)
    try:
        assert k.wait_registered("amd.com/gpu", 10, min_devices=8)
        ids, resp = k.allocate("amd.com/gpu", 2, pod="p")
        paths = [d.host_path for d in resp.devices]
        assert paths[0] == "/dev/kfd" and len(paths) == 3
        assert all(p.startswith("/dev/dri/renderD") for p in paths[1:])
        assert resp.envs["AMD_VISIBLE_DEVICES"].count(",") == 1
        assert resp.annotations["amd.com/gpu.memory-bytes"].split(",")[0] == str(fakesys.HBM_BYTES)
        assert [c.name for c in resp.cdi_devices] == [f"amd.com/gpu={i}" for i in resp.envs["AMD_VISIBLE_DEVICES"].split(",")]
        # remaining free devices shrink, double allocation impossible
        assert len(k.free_devices("amd.com/gpu")) == 6
        k.allocate("amd.com/gpu", 6, pod="q")
        with pytest.raises(RuntimeError):
            k.allocate("amd.com/gpu", 1, pod="r")
    finally:
        m.stop()


def test_preferred_allocation_prefers_one_numa_node(node):
    root, sock_dir, k = node
    m = _start(root, sock_dir)
    try:
        assert k.wait_registered("amd.com/gpu", 10, min_devices=8)
        ids, _ = k.allocate("amd.com/gpu", 4, pod="p")
        gpus = {g.device_id_str: g for g in T.enumerate_gpus(root)}
        assert len({gpus[i].numa_node for i in ids}) == 1
    finally:
        m.stop()


def test_health_flip_reaches_kubelet_and_blocks_allocation(node):
    root, sock_dir, k = node
    m = _start(root, sock_dir)
    try:
        assert k.wait_registered("amd.com/gpu", 10, min_devices=8)
        dev = T.enumerate_gpus(root)[3].device_id_str
        before = k.resources["amd.com/gpu"].updates
        m.set_health(dev, False, "ecc_uncorrectable")
        assert k.wait_update("amd.com/gpu", before, 5)
        assert k.allocatable("amd.com/gpu") == 7
        assert dev not in k.free_devices("amd.com/gpu")
        m.set_health(dev, True, "gpu_post_reset")
        assert k.wait_update("amd.com/gpu", before + 1, 5)
        assert k.allocatable("amd.com/gpu") == 8
    finally:
        m.stop()


def test_concurrent_allocate_during_health_flips(node):
    root, sock_dir, k = node
    m = _start(root, sock_dir)
    try:
        assert k.wait_registered("amd.com/gpu", 10, min_devices=8)
        devs = [g.device_id_str for g in T.enumerate_gpus(root)]
        stop = threading.Event()

        def flipper():
            i = 0
            while not stop.is_set():
                m.set_health(devs[7], i % 2 == 1, "flap")
                i += 1
                time.sleep(0.001)

        th = threading.Thread(target=flipper)
        th.start()
        got = []
        for i in range(6):
            ids, _ = k.allocate("amd.com/gpu", 1, pod=f"p{i}")
            got += ids
        stop.set()
        th.join()
        assert len(set(got)) == 6
    finally:
        m.stop()


def test_reregisters_after_kubelet_restart(node):
    root, sock_dir, k = node
    m = _start(root, sock_dir)
    try:
        assert k.wait_registered("amd.com/gpu", 10, min_devices=8)
        k.restart()
        assert k.wait_registered("amd.com/gpu", 10, min_devices=8)
        assert k.register_calls >= 1
        ids, _ = k.allocate("amd.com/gpu", 1)
        assert ids
    finally:
        m.stop()


def test_cpx_mixed_strategy_resources(tmp_path):
    root = str(tmp_path / "host")
    fakesys.build_node(root, 2, "CPX")
    sock_dir = str(tmp_path / "dp")
    k = FakeKubelet(sock_dir)
    k.start()
    m = _start(root, sock_dir, partition_strategy="mixed")
    try:
        assert k.wait_registered("amd.com/gpu-cpx", 10, min_devices=16)
        assert k.allocatable("amd.com/gpu-cpx") == 16
        ids, _ = k.allocate("amd.com/gpu-cpx", 8)
        # 8 CPX partitions fit on one physical GPU: packed, not spread
        assert len({i.rsplit("-p", 1)[0] for i in ids}) == 1
    finally:
        m.stop()
        k.stop()


def test_allocator_cost_model():
    devs = [AllocDevice(f"g{i}", i // 2, 0 if i < 4 else 1) for i in range(8)]
    w = {(f"g{i}", f"g{j}"): 15 for i in range(8) for j in range(8) if i != j}
    # make g0-g1 and g2-g3 "far" (PCIe only)
    for a, b in (("g0", "g2"), ("g0", "g3"), ("g1", "g2"), ("g1", "g3")):
        w[(a, b)] = w[(b, a)] = 60
    cost = TopologyCost(devs, w)
    ids = [d.id for d in devs]
    assert preferred(cost, ids, [], 2) == ["g0", "g1"]  # same physical GPU costs 0
    sel = preferred(cost, ids, ["g4"], 2)
    assert "g4" in sel and sel == ["g4", "g5"]
    assert preferred(cost, ids, [], 0) == []
    assert preferred(cost, ["g0"], [], 3) == ["g0"]
    four = preferred(cost, ids, [], 4)
    assert {devs[int(i[1])].numa for i in four} == {1} or {devs[int(i[1])].numa for i in four} == {0}


def test_allocator_greedy_path_large_pool():
    devs = [AllocDevice(f"d{i:02d}", i // 8, i // 32) for i in range(64)]
    cost = TopologyCost(devs, {})
    sel = preferred(cost, [d.id for d in devs], [], 8)
    assert len({devs[int(i[1:])].physical for i in sel}) == 1


def test_prepared_plugin_does_not_register_before_it_is_told(tmp_path):
    """start(register=False) serves the sockets (the operand's toolkit gate is
    still closed) but must not advertise - not even through the kubelet
    watcher - until register()."""
    import time

    from amdgpu_operator.deviceplugin.server import DevicePluginManager, PluginConfig
    from amdgpu_operator.testing import fakesys
    from amdgpu_operator.testing.fakekubelet import FakeKubelet

    root = str(tmp_path / "h")
    fakesys.build_node(root, 2)
    dp = tmp_path / "dp"
    dp.mkdir()
    k = FakeKubelet(str(dp))
    k.start()
    mgr = DevicePluginManager(PluginConfig(socket_dir=str(dp), sysfs_root=root, watch_interval_s=0.02))
    try:
        mgr.start(register=False)
        time.sleep(0.3)  # several kubelet-watch ticks
        assert k.register_calls == 0
        mgr.register()
        assert k.wait_registered("amd.com/gpu", 5, min_devices=2) and k.register_calls == 1
    finally:
        mgr.stop()
        k.stop()


@pytest.mark.parametrize("strategy,before_toolkit", [("envvar", True), ("cdi-cri", False)])
def test_plugin_advertises_before_the_toolkit_only_when_allocations_need_nothing_from_it(tmp_path, strategy,
                                                                                         before_toolkit):
    """Gated on the toolkit (VALIDATION_GATE=toolkit): with device specs the
    kubelet gives the container /dev/kfd and the render nodes itself, so the
    plugin registers once the driver is up; CDI device names need the
    toolkit's CDI spec, so that plugin waits for toolkit-ready."""
    import threading
    import time

    from amdgpu_operator.cli.operands import run_operand
    from amdgpu_operator.kube.client import LocalClient
    from amdgpu_operator.kube.fakeapi import FakeApiServer
    from amdgpu_operator.nodeenv import NodeEnv
    from amdgpu_operator.testing import fakesys
    from amdgpu_operator.testing.fakekubelet import FakeKubelet
    from amdgpu_operator.validator import validate as V

    root = str(tmp_path / "h")
    fakesys.build_node(root, 2)
    dp = tmp_path / "dp"
    dp.mkdir()
    k = FakeKubelet(str(dp))
    k.start()
    env = NodeEnv("n1", LocalClient(FakeApiServer()), host_root=root, validations_dir=str(tmp_path / "val"),
                  device_plugin_dir=str(dp), poll_s=0.01)
    env.extra["no_health"] = True
    V.write_ready(env, "driver", {"ok": True})
    stop = threading.Event()
    t = threading.Thread(target=run_operand, args=(env, ["device-plugin", "--device-list-strategy", strategy], stop),
                         kwargs={"container_env": {"VALIDATION_GATE": "toolkit"}}, daemon=True)
    t.start()
    try:
        registered = k.wait_registered("amd.com/gpu", 3 if before_toolkit else 0.5, min_devices=2)
        assert registered == before_toolkit
        if not before_toolkit:
            V.write_ready(env, "toolkit", {"ok": True})
            assert k.wait_registered("amd.com/gpu", 5, min_devices=2)
    finally:
        stop.set()
        t.join(10)
        k.stop()
