"""driver.rdma: RDMA NICs beside the GPUs (discovery/rdma.py), the driver's
RDMA-core readiness, the plugin's nearest-NIC report, the GFD labels and the
validator's dma-buf step wiring.  Upstream parity: the NVIDIA GPU Operator's
``driver.rdma.enabled`` / ``useHostMofed`` (off in the reference's install,
/root/reference/README.md:101-110)."""

import os
import sys

import pytest

from amdgpu_operator.api.clusterpolicy import REFERENCE_SET_FLAGS, parse_set_flags, spec_from_values
from amdgpu_operator.controller import manifests as M
from amdgpu_operator.deviceplugin.server import DevicePluginServer, PluginConfig
from amdgpu_operator.discovery import labels as L
from amdgpu_operator.discovery import rdma
from amdgpu_operator.discovery import topology as T
from amdgpu_operator.driver import manager as DM
from amdgpu_operator.kube import resources as R
from amdgpu_operator.kube.client import LocalClient
from amdgpu_operator.kube.fakeapi import FakeApiServer
from amdgpu_operator.nodeenv import NodeEnv, run_local
from amdgpu_operator.testing import fakesys
from amdgpu_operator.validator import validate as V


@pytest.fixture
def node(tmp_path):
    root = str(tmp_path / "host")
    gs = fakesys.build_node(root, 8, pcie_tree=True)
    names = fakesys.add_rdma_nics(root, gs)
    return root, names


def test_each_gpu_finds_the_nic_on_its_own_switch(node):
    root, names = node
    gpus = T.enumerate_gpus(root)
    assert len(gpus) == 8  # the GPUs still enumerate through the PCIe tree's symlinks
    nics = rdma.enumerate_nics(root)
    assert [n.name for n in nics] == names and all(n.active and n.rate_gbps == 400 for n in nics)
    near = rdma.nearest_nics(gpus, nics, root)
    for i, g in enumerate(gpus):
        assert near[g.bdf] == [(names[i], rdma.PIX)]
    assert rdma.allocation_nics(gpus[2:6], nics, root) == names[2:6]


def test_path_classes():
    hb0, hb1 = "pci0000:00", "pci0000:80"
    gpu = (hb0, "0000:00:07.1", "0000:70:00.0", "0000:71:00.0", "0000:72:00.0")
    assert rdma.path_class(gpu, 0, (hb0, "0000:00:07.1", "0000:70:00.0", "0000:71:01.0", "0000:73:00.0"), 0) == rdma.PIX
    # two switches below one root port
    assert rdma.path_class(gpu, 0, (hb0, "0000:00:07.1", "0000:70:00.0", "0000:71:02.0", "0000:74:00.0",
                                    "0000:75:00.0", "0000:76:00.0"), 0) == rdma.PXB
    assert rdma.path_class(gpu, 0, (hb0, "0000:00:05.1", "0000:50:00.0", "0000:51:00.0", "0000:52:00.0"), 0) == rdma.PHB
    assert rdma.path_class(gpu, 0, (hb1, "0000:80:01.1", "0000:81:00.0"), 0) == rdma.NODE
    assert rdma.path_class(gpu, 0, (hb1, "0000:80:01.1", "0000:81:00.0"), 1) == rdma.SYS
    # a flat sysfs copy (no tree): NUMA decides
    assert rdma.path_class(("0000:72:00.0",), 0, ("0000:73:00.0",), 0) == rdma.NODE


def test_nics_on_one_socket_only(tmp_path):
    """Two NICs, both on socket 0: socket-0 GPUs share a host bridge with
    them (PHB), socket-1 GPUs reach them across the sockets (SYS) - and an
    allocation spreads over both NICs instead of piling on one."""
    root = str(tmp_path / "h")
    gs = fakesys.build_node(root, 8, pcie_tree=True)
    fakesys.add_rdma_nics(root, [g for g in gs if g.bdf in ("0000:72:00.0", "0000:0a:00.0")])
    gpus = T.enumerate_gpus(root)
    nics = rdma.enumerate_nics(root)
    near = rdma.nearest_nics(gpus, nics, root)
    by = {g.bdf: g for g in gpus}
    assert near["0000:72:00.0"] == [("ionic_0", rdma.PIX)]
    assert near["0000:5a:00.0"] == [("ionic_0", rdma.PHB), ("ionic_1", rdma.PHB)]
    assert near["0000:f1:00.0"] == [("ionic_0", rdma.SYS), ("ionic_1", rdma.SYS)]
    assert rdma.allocation_nics([by["0000:5a:00.0"], by["0000:23:00.0"]], nics, root) == ["ionic_0", "ionic_1"]
    assert rdma.rdma_labels(gpus, root)["amd.com/gpu.rdma.affinity"] == rdma.SYS


def test_labels_and_readiness(node, tmp_path):
    root, _ = node
    gpus = T.enumerate_gpus(root)
    lab = L.gfd_labels(gpus, root)
    assert lab["amd.com/gpu.rdma.capable"] == "true" and lab["amd.com/gpu.rdma.nics"] == "8"
    assert lab["amd.com/gpu.rdma.link-layer"] == "RoCE" and lab["amd.com/gpu.rdma.rate-gbps"] == "400"
    assert lab["amd.com/gpu.rdma.affinity"] == "PIX" and lab["amd.com/gpu.rdma.dmabuf"] == "true"
    assert rdma.readiness(root)["ok"]
    # no NICs: no RDMA labels at all
    plain = str(tmp_path / "plain")
    fakesys.build_node(plain, 2)
    assert not any(k.startswith("amd.com/gpu.rdma") for k in L.gfd_labels(T.enumerate_gpus(plain), plain))
    # ports down, RDMA core missing, an old kernel
    old = str(tmp_path / "old")
    gs = fakesys.build_node(old, 2, pcie_tree=True, kernel="5.4.0-150-generic")
    fakesys.add_rdma_nics(old, gs, active=False, modules=False)
    st = rdma.readiness(old)
    assert not st["ok"] and not st["dmabuf"]
    assert {"module ib_core not loaded", "module ib_uverbs not loaded", "no RDMA port ACTIVE"} <= set(st["problems"])
    assert L.gfd_labels(T.enumerate_gpus(old), old)["amd.com/gpu.rdma.capable"] == "false"


def _env(tmp_path, kernel="6.8.0-45-generic", modules=True):
    root = str(tmp_path / "drv")
    gs = fakesys.build_node(root, 2, pcie_tree=True, kernel=kernel)
    fakesys.add_rdma_nics(root, gs, modules=modules)
    c = LocalClient(FakeApiServer())
    c.create(R.new("v1", "Node", "n1"))
    env = NodeEnv("n1", c, host_root=root, validations_dir=str(tmp_path / "val"), poll_s=0.01)
    env.extra["kmod"] = fakesys.SimModule(root)
    return env


def test_driver_loads_the_rdma_core_before_it_is_ready(tmp_path):
    env = _env(tmp_path, modules=False)
    out = DM.install(env, timeout=5, cenv={"AMDGPU_RDMA_ENABLED": "true"})
    assert env.extra["kmod"].log == ["load-rdma"] and out["rdma"]["loaded_here"] and out["rdma"]["ok"]
    assert V.read_ready(env, "driver")["rdma"]["nics"] == [f"ionic_{i}" for i in range(2)]
    # without driver.rdma nothing RDMA happens
    env2 = _env(tmp_path / "b", modules=False)
    assert "rdma" not in DM.install(env2, timeout=5, cenv={})
    assert env2.extra["kmod"].log == []


def test_driver_with_host_mofed_waits_for_the_host_stack(tmp_path):
    env = _env(tmp_path, modules=False)
    with pytest.raises(RuntimeError, match="RDMA core not loaded"):
        DM.install(env, timeout=0.3, cenv={"AMDGPU_RDMA_ENABLED": "true", "AMDGPU_RDMA_USE_HOST_MOFED": "true"})
    assert env.extra["kmod"].log == [] and V.read_ready(env, "driver") is None
    fakesys.SimModule(env.sysfs_root()).load_rdma()  # the host's stack comes up
    out = DM.install(env, timeout=5, cenv={"AMDGPU_RDMA_ENABLED": "true", "AMDGPU_RDMA_USE_HOST_MOFED": "true"})
    assert out["rdma"]["ok"] and not out["rdma"]["loaded_here"]


def test_driver_rdma_refuses_a_kernel_without_dmabuf_import(tmp_path):
    env = _env(tmp_path, kernel="5.10.0-28-amd64")
    with pytest.raises(RuntimeError, match="needs >= 5.12"):
        DM.install(env, timeout=5, cenv={"AMDGPU_RDMA_ENABLED": "true"})


def test_plugin_reports_the_nearest_nics_of_an_allocation(node):
    root, names = node
    gpus = T.enumerate_gpus(root)
    for hca_env in (False, True):
        srv = DevicePluginServer(PluginConfig(sysfs_root=root, rdma=True, rdma_hca_env=hca_env), gpus)
        ids = [d.ID for d in srv.device_list()[0].devices]
        r = srv.container_response([ids[1], ids[4]])
        assert r.annotations["amd.com/gpu.rdma-nics"] == f"{names[1]},{names[4]}"
        assert ("NCCL_IB_HCA" in r.envs) == hca_env and (not hca_env or r.envs["NCCL_IB_HCA"] == "ionic_1,ionic_4")
    plain = DevicePluginServer(PluginConfig(sysfs_root=root), gpus)
    assert "amd.com/gpu.rdma-nics" not in plain.container_response([plain.device_list()[0].devices[0].ID]).annotations


def test_policy_switches_rdma_on_in_every_operand():
    spec = spec_from_values(parse_set_flags(REFERENCE_SET_FLAGS + ["driver.rdma.enabled=true",
                                                                   "driver.rdma.hcaEnv=true"]))
    drv = next(d for d in M.state_driver(spec, "ns", []) if d["kind"] == "DaemonSet")
    env = {e["name"]: e.get("value") for c in drv["spec"]["template"]["spec"]["containers"] for e in c["env"]}
    assert env["AMDGPU_RDMA_ENABLED"] == "true" and env["AMDGPU_RDMA_USE_HOST_MOFED"] == "false"
    dp = next(d for d in M.state_device_plugin(spec, "ns", []) if d["kind"] == "DaemonSet")
    args = dp["spec"]["template"]["spec"]["containers"][0]["args"]
    assert "--rdma" in args and "--rdma-hca-env" in args
    val = [d for d in M.state_validator(spec, "ns", []) if d["kind"] == "DaemonSet"][0]["spec"]["template"]["spec"]
    assert any("--dmabuf" in c["args"] for c in val["initContainers"] + val["containers"])
    off = spec_from_values(parse_set_flags(REFERENCE_SET_FLAGS))  # the reference's install: off
    assert not off.driver.rdma.enabled
    val = [d for d in M.state_validator(off, "ns", []) if d["kind"] == "DaemonSet"][0]["spec"]["template"]["spec"]
    assert not any("--dmabuf" in c["args"] for c in val["initContainers"] + val["containers"])


def test_workload_validation_runs_the_dmabuf_step_on_every_device(tmp_path):
    root = str(tmp_path / "h")
    fakesys.build_node(root, 2, compute_partition="DPX")
    env = NodeEnv("n1", None, host_root=root, validations_dir=str(tmp_path / "v"), poll_s=0.01)
    calls = []

    def launcher(argv, e, device, timeout):
        calls.append(argv)
        return run_local([sys.executable, "-m", "amdgpu_operator.testing.fake_validator", *argv[1:]], e, timeout)

    env.launcher = launcher
    out = V.validate_workload(env, ["--peer-timeout", "60", "--dmabuf"])
    assert all("--dmabuf" not in a and "dmabuf" in a[a.index("--steps") + 1].split(",") for a in calls)
    for rank in out["ranks"]:  # each of a GPU's two partitions exported its HBM
        assert sum(1 for s in rank["steps"] if s["name"] == "dmabuf") == 2
    V.validate_workload(env, ["--peer-timeout", "60"])
    assert "dmabuf" not in calls[-1][calls[-1].index("--steps") + 1]


def test_tree_layout_keeps_driver_and_iommu_links(node):
    root, _ = node
    dev = os.path.join(root, "sys/bus/pci/devices/0000:72:00.0")
    assert os.path.islink(dev) and os.path.basename(os.path.realpath(os.path.join(dev, "driver"))) == "amdgpu"
    assert os.path.isdir(os.path.join(dev, "iommu_group"))


def test_rdma_bring_up_on_the_simulated_cluster(tmp_path):
    """driver.rdma end to end: the driver container loads the RDMA core on
    the node, the validator's dmabuf step runs, GFD labels the NICs, the
    config-5 pods' allocations name their nearest NICs, and verify checks it."""
    from amdgpu_operator.cli.verify import verify
    from amdgpu_operator.testing.podworkload import run_pod_workload
    from amdgpu_operator.testing.simcluster import NodeSpec, SimCluster

    c = SimCluster(str(tmp_path / "c"), [NodeSpec("gpu-1", 4, rdma_nics=True)], fake_gpu=True).start()
    try:
        c.install_operator(parse_set_flags(REFERENCE_SET_FLAGS + ["driver.rdma.enabled=true"]))
        c.wait_ready(60, {"gpu-1": 4})
        lab = c.client.get("v1", "Node", "gpu-1")["metadata"]["labels"]
        assert lab["amd.com/gpu.rdma.capable"] == "true" and lab["amd.com/gpu.rdma.affinity"] == "PIX"
        env = c.nodes["gpu-1"].env
        drv = V.read_ready(env, "driver")["rdma"]
        assert drv["ok"] and drv["loaded_here"] and drv["nics"] == [f"ionic_{i}" for i in range(4)]
        wl = V.read_ready(env, "workload")
        assert all(any(s["name"] == "dmabuf" and s["ok"] for s in r["steps"]) for r in wl["ranks"])
        rep = verify(c.client, c.namespace, expect_gpus_per_node=4)
        assert rep.ok and next(x for x in rep.checks if x.name == "rdma[gpu-1]").ok, rep.table()
        out = run_pod_workload(c, "gpu-1", 4, gemm_n=256)
        assert out["all_succeeded"] and out["single_gpu_pods_distinct_devices"]
    finally:
        c.stop()
