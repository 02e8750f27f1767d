"""Synthetic MI355X sysfs / devfs trees for tests and emulated multi-GPU runs.

Modeled on the tree captured from a real MI355X box (tests/fixtures/mi355x:
KFD node 9 = gfx950, 1024 SIMDs, 8 XCCs, 160 KiB LDS, 288 GiB HBM3E
(309,220,868,096 bytes), 7 xGMI io_links of 76,000 MB/s at weight 15, render
minor 184, amdgpu_xcp partition render nodes numbered after the device's own).

``build_node(root, gpus=8, compute_partition="SPX")`` writes:
  sys/module/amdgpu/{initstate,version}, sys/class/kfd/kfd/dev,
  sys/class/kfd/kfd/topology/nodes/<n>/{properties,gpu_id,name,mem_banks,io_links}
  sys/class/drm/renderD<m>/dev, sys/bus/pci/devices/<bdf>/{vendor,device,class,...}
  dev/kfd, dev/dri/renderD<m>   (plain files: tests never open them)
"""

from __future__ import annotations

import os
import shutil
import tarfile
from dataclasses import dataclass

# PCI buses of the 8 OAMs on the captured host, in render-minor order
REAL_BUSES = [0x72, 0x0A, 0x5A, 0x23, 0xF1, 0x8B, 0xD9, 0xA4]
HBM_BYTES = 309220868096
MI355X_DEVICE_ID = 0x75A3
PARTITION_SPLIT = {"SPX": 1, "DPX": 2, "TPX": 3, "QPX": 4, "CPX": 8}
HIVE_ID = 6032565651074706519
IOMMU_GROUP_BASE = 40


def _w(path: str, text: str) -> None:
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as f:
        f.write(text)


def _link(target: str, path: str) -> None:
    os.makedirs(os.path.dirname(path), exist_ok=True)
    if os.path.lexists(path):
        os.unlink(path)
    os.symlink(target, path)


def _props(d: dict) -> str:
    return "".join(f"{k} {v}\n" for k, v in d.items())


@dataclass
class FakeGpu:
    physical: int
    partition: int
    node: int
    bdf: str
    location_id: int
    render_minor: int
    numa: int


def build_node(root: str, gpus: int = 8, compute_partition: str = "SPX", memory_partition: str = "NPS1",
               driver_loaded: bool = True, xgmi: bool = True, sockets: int = 2, hidden_peers: int = 0,
               kernel: str = "6.8.0-45-generic", pcie_tree: bool = False) -> list[FakeGpu]:
    """Write a fake node with ``gpus`` physical MI355X. Returns the GPU nodes.

    ``hidden_peers`` adds that many GPU nodes whose properties are unreadable
    (what a container sees of the other GPUs of the host).  ``pcie_tree``
    places each GPU behind its own PCIe switch (``sys/devices/pci…`` with
    ``sys/bus/pci/devices/<bdf>`` a symlink into it, as on a real host), the
    layout RDMA-NIC affinity reads (:func:`add_rdma_nics`).
    """
    split = PARTITION_SPLIT[compute_partition]
    os.makedirs(root, exist_ok=True)
    _w(f"{root}/proc/sys/kernel/osrelease", kernel + "\n")
    base = os.path.join(root, "sys/class/kfd/kfd/topology/nodes")
    if driver_loaded:
        _w(f"{root}/sys/module/amdgpu/initstate", "live\n")
        _w(f"{root}/sys/module/amdgpu/version", "6.12.12\n")
        _w(f"{root}/sys/class/kfd/kfd/dev", "241:0\n")
        _w(f"{root}/dev/kfd", "")
    _w(f"{root}/sys/class/kfd/kfd/topology/system_properties", "platform_oem 0\nplatform_id 0\nplatform_rev 0\n")

    node = 0
    cpu_nodes = []
    for s in range(sockets):
        _w(f"{base}/{node}/properties", _props({
            "cpu_cores_count": 128, "simd_count": 0, "mem_banks_count": 1, "caches_count": 0, "io_links_count": 0,
            "gfx_target_version": 0, "vendor_id": 0, "device_id": 0, "location_id": 0, "domain": 0,
            "drm_render_minor": 0, "hive_id": 0, "max_engine_clk_ccompute": 5008}))
        _w(f"{base}/{node}/gpu_id", "0\n")
        _w(f"{base}/{node}/name", "\n")
        cpu_nodes.append(node)
        node += 1

    out: list[FakeGpu] = []
    for p in range(gpus):
        bus = REAL_BUSES[p] if p < len(REAL_BUSES) else 0x10 + p
        loc = bus << 8
        bdf = f"0000:{bus:02x}:00.0"
        numa = 0 if bus < 0x80 else min(1, sockets - 1)
        minor0 = 128 + 8 * p
        for k in range(split):
            out.append(FakeGpu(p, k, node, bdf, loc, minor0 + k, numa))
            node += 1
    for g in out:
        nd = f"{base}/{g.node}"
        simd = 1024 // split
        _w(f"{nd}/properties", _props({
            "cpu_cores_count": 0, "simd_count": simd, "mem_banks_count": 1, "caches_count": 0,
            "io_links_count": 0, "p2p_links_count": 0, "cpu_core_id_base": 0, "simd_id_base": 2147487744 + g.node * 16,
            "max_waves_per_simd": 8, "lds_size_in_kb": 160, "gds_size_in_kb": 0, "num_gws": 64, "wave_front_size": 64,
            "array_count": 32 // split, "simd_arrays_per_engine": 1, "cu_per_simd_array": 9, "simd_per_cu": 4,
            "max_slots_scratch_cu": 32, "gfx_target_version": 90500, "vendor_id": 4098, "device_id": MI355X_DEVICE_ID,
            "location_id": g.location_id, "domain": 0, "drm_render_minor": g.render_minor,
            "hive_id": HIVE_ID if xgmi and gpus > 1 else 0, "num_sdma_engines": 2, "num_sdma_xgmi_engines": 14,
            "num_cp_queues": 24, "max_engine_clk_fcompute": 2400, "local_mem_size": 0, "fw_version": 44,
            "unique_id": 0x9048305841F50000 + g.physical * 16 + g.partition, "num_xcc": 8 // split,
            "max_engine_clk_ccompute": 5008}))
        _w(f"{nd}/gpu_id", f"{20000 + g.node * 7}\n")
        _w(f"{nd}/name", "ip discovery\n")
        _w(f"{nd}/mem_banks/0/properties", _props({"heap_type": 1, "size_in_bytes": HBM_BYTES, "flags": 0,
                                                     "width": 8192, "mem_clk_max": 2000}))
        links = [dict(type=2, node_from=g.node, node_to=cpu_nodes[g.numa], weight=20, min_bandwidth=0,
                      max_bandwidth=64000)]
        if xgmi:
            for h in out:
                if h.node == g.node:
                    continue
                same = h.physical == g.physical
                links.append(dict(type=11, node_from=g.node, node_to=h.node, weight=10 if same else 15,
                                  min_bandwidth=76000, max_bandwidth=76000))
        else:
            for h in out:
                if h.node != g.node:
                    links.append(dict(type=2, node_from=g.node, node_to=h.node, weight=40 if h.numa == g.numa else 52,
                                      min_bandwidth=0, max_bandwidth=64000))
        for i, lk in enumerate(links):
            _w(f"{nd}/io_links/{i}/properties", _props({"type": lk["type"], "version_major": 0, "version_minor": 0,
                                                         "node_from": lk["node_from"], "node_to": lk["node_to"],
                                                         "weight": lk["weight"], "min_latency": 0, "max_latency": 0,
                                                         "min_bandwidth": lk["min_bandwidth"],
                                                         "max_bandwidth": lk["max_bandwidth"],
                                                         "recommended_transfer_size": 0, "flags": 1}))
        _w(f"{root}/sys/class/drm/renderD{g.render_minor}/dev", f"226:{g.render_minor}\n")
        _w(f"{root}/dev/dri/renderD{g.render_minor}", "")
        pci = f"{root}/sys/bus/pci/devices/{g.bdf}"
        _w(f"{pci}/vendor", "0x1002\n")
        _w(f"{pci}/device", f"0x{MI355X_DEVICE_ID:04x}\n")
        _w(f"{pci}/class", "0x120000\n")
        _w(f"{pci}/subsystem_vendor", "0x1002\n")
        _w(f"{pci}/subsystem_device", f"0x{MI355X_DEVICE_ID:04x}\n")
        _w(f"{pci}/numa_node", f"{g.numa}\n")
        _w(f"{pci}/current_compute_partition", f"{compute_partition}\n")
        _w(f"{pci}/available_compute_partition", "SPX, DPX, QPX, CPX\n")
        _w(f"{pci}/current_memory_partition", f"{memory_partition}\n")
        _w(f"{pci}/available_memory_partition", "NPS1, NPS2\n")
    for h in range(hidden_peers):
        _w(f"{base}/{node + h}/io_links/0/.hidden", "")
    # PCI driver binding and IOMMU groups (vfio-manager, sandbox workloads):
    # one group per GPU, bound to amdgpu while the module is live
    _w(f"{root}/sys/bus/pci/drivers_probe", "")
    if driver_loaded:
        _w(f"{root}/sys/bus/pci/drivers/amdgpu/unbind", "")
    for n, bdf in enumerate(dict.fromkeys(g.bdf for g in out)):
        group = str(IOMMU_GROUP_BASE + n)
        gdir = f"{root}/sys/kernel/iommu_groups/{group}/devices"
        os.makedirs(gdir, exist_ok=True)
        _link(f"../../../../bus/pci/devices/{bdf}", f"{gdir}/{bdf}")
        _link(f"../../../../kernel/iommu_groups/{group}", f"{root}/sys/bus/pci/devices/{bdf}/iommu_group")
        _w(f"{root}/sys/bus/pci/devices/{bdf}/driver_override", "(null)\n")
        if driver_loaded:
            _link("../../../../bus/pci/drivers/amdgpu", f"{root}/sys/bus/pci/devices/{bdf}/driver")
    # a non-GPU PCI device to make sure discovery filters by vendor/class
    _w(f"{root}/sys/bus/pci/devices/0000:00:01.0/vendor", "0x1022\n")
    _w(f"{root}/sys/bus/pci/devices/0000:00:01.0/class", "0x060000\n")
    _w(f"{root}/sys/bus/pci/devices/0000:00:01.0/device", "0x14a4\n")
    if pcie_tree:
        for bdf, numa in dict.fromkeys((g.bdf, g.numa) for g in out):
            _into_tree(root, bdf, switch_path(bdf, numa) + (bdf,))
    return out


def switch_path(gpu_bdf: str, numa: int) -> tuple[str, ...]:
    """/sys/devices components of the fake PCIe switch above a GPU: host
    bridge (one per socket), root port, switch upstream port, downstream port."""
    bus = int(gpu_bdf.split(":")[1], 16)
    hb = f"{0x00 if numa == 0 else 0x80:02x}"
    return (f"pci0000:{hb}", f"0000:{hb}:{(bus >> 4) & 0x1f:02x}.1", f"0000:{bus - 2:02x}:00.0",
            f"0000:{bus - 1:02x}:00.0")


def _into_tree(root: str, bdf: str, parts: tuple[str, ...]) -> None:
    """Move a flat ``sys/bus/pci/devices/<bdf>`` directory to
    ``sys/devices/<parts>`` and leave the bus entry as a symlink to it; the
    function's own relative symlinks (driver, iommu_group) become absolute so
    they still resolve from the new depth."""
    src = os.path.join(root, "sys/bus/pci/devices", bdf)
    dst = os.path.join(root, "sys/devices", *parts)
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    if os.path.isdir(src) and not os.path.islink(src):
        for name in os.listdir(src):
            p = os.path.join(src, name)
            if os.path.islink(p) and not os.path.isabs(os.readlink(p)):
                target = os.path.normpath(os.path.join(src, os.readlink(p)))
                os.unlink(p)
                os.symlink(target, p)
        shutil.move(src, dst)
    else:
        os.makedirs(dst, exist_ok=True)
    _link(os.path.relpath(dst, os.path.dirname(src)), src)


def add_rdma_nics(root: str, gpus: list[FakeGpu], link_layer: str = "Ethernet", rate_gbps: int = 400,
                  active: bool = True, modules: bool = True, name: str = "ionic_{}") -> list[str]:
    """One RDMA NIC per physical GPU, on the GPU's PCIe switch (build the
    node with ``pcie_tree=True``): ``sys/class/infiniband/<name>`` with one
    port, ``/dev/infiniband/uverbs<n>``, and the RDMA core modules."""
    names = []
    for i, (bdf, numa) in enumerate(dict.fromkeys((g.bdf, g.numa) for g in gpus)):
        bus = int(bdf.split(":")[1], 16)
        nic_bdf = f"0000:{bus + 1:02x}:00.0"
        parts = switch_path(bdf, numa)[:-1] + (f"0000:{bus - 1:02x}:01.0", nic_bdf)
        dev = os.path.join(root, "sys/devices", *parts)
        _w(f"{dev}/vendor", "0x1dd8\n")
        _w(f"{dev}/device", "0x1002\n")
        _w(f"{dev}/class", "0x020000\n")
        _w(f"{dev}/numa_node", f"{numa}\n")
        _link(os.path.relpath(dev, f"{root}/sys/bus/pci/devices"), f"{root}/sys/bus/pci/devices/{nic_bdf}")
        nm = name.format(i)
        ib = f"{root}/sys/class/infiniband/{nm}"
        _link(os.path.relpath(dev, ib), f"{ib}/device")
        _w(f"{ib}/ports/1/state", "4: ACTIVE\n" if active else "1: DOWN\n")
        _w(f"{ib}/ports/1/link_layer", f"{link_layer}\n")
        _w(f"{ib}/ports/1/rate", f"{rate_gbps} Gb/sec (4X NDR)\n")
        _w(f"{root}/dev/infiniband/uverbs{i}", "")
        names.append(nm)
    if modules:
        for m in ("ib_core", "ib_uverbs", "rdma_ucm"):
            _w(f"{root}/sys/module/{m}/initstate", "live\n")
    return names


REAL_FIXTURE = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                            "tests", "fixtures", "mi355x")


def build_from_real_fixture(root: str, driver_loaded: bool = True) -> str:
    """Unpack the sysfs captured on a real MI355X box (1 visible GPU of an
    8-GPU xGMI hive) and add the device nodes / module state the capture could
    not include.  Returns ``root``."""
    os.makedirs(root, exist_ok=True)
    with tarfile.open(os.path.join(REAL_FIXTURE, "sysfs.tar.gz")) as tf:
        tf.extractall(root, filter="data")
    if driver_loaded:
        _w(f"{root}/sys/module/amdgpu/initstate", "live\n")
        _w(f"{root}/sys/class/kfd/kfd/dev", "241:0\n")
        _w(f"{root}/dev/kfd", "")
        _w(f"{root}/dev/dri/renderD128", "")  # the container's re-numbered render node
    return root


class SimModule:
    """Simulated amdgpu kernel module of a fake node (the driver manager's
    module backend in the simulated cluster, ``NodeEnv.extra["kmod"]``).

    ``install`` does what ``deploy/images/amd-driver/install.sh`` does to the
    host: unload a live module, then load the requested version (module
    state, version, ``/dev/kfd``).  ``busy=True`` makes unloading fail, as
    ``modprobe -r`` does while a process holds the device.  ``log`` records
    the operations for tests."""

    def __init__(self, root: str):
        self.root = root
        self.busy = False
        self.log: list[str] = []

    def can_install(self) -> bool:
        return True

    def _live(self) -> bool:
        return os.path.exists(f"{self.root}/sys/module/amdgpu/initstate")

    def unload(self, env=None, timeout: float = 0.0) -> None:
        if self.busy:
            self.log.append("unload-failed")
            raise RuntimeError("modprobe -r amdgpu: Module amdgpu is in use")
        for p in ("sys/module/amdgpu/initstate", "sys/module/amdgpu/version", "dev/kfd"):
            try:
                os.unlink(f"{self.root}/{p}")
            except FileNotFoundError:
                pass
        self.log.append("unload")

    def load_rdma(self, env=None, timeout: float = 0.0) -> None:
        """``modprobe ib_uverbs`` (pulls in ib_core) on the fake node."""
        for m in ("ib_core", "ib_uverbs"):
            _w(f"{self.root}/sys/module/{m}/initstate", "live\n")
        self.log.append("load-rdma")

    def install(self, env, cenv: dict, timeout: float) -> None:
        if self._live():
            self.unload()
        version = cenv.get("AMDGPU_DRIVER_VERSION") or "6.12.12"
        pending = f"{self.root}/.pending-partition"
        if os.path.exists(pending):  # a memory-partition change takes effect at the module load
            import json
            import shutil

            with open(pending) as f:
                p = json.load(f)
            shutil.rmtree(f"{self.root}/sys/class/kfd/kfd/topology/nodes", ignore_errors=True)
            build_node(self.root, p["gpus"], p["compute"], p["memory"])
            os.unlink(pending)
            self.log.append(f"partition {p['compute']}/{p['memory']}")
        _w(f"{self.root}/sys/module/amdgpu/version", f"{version}\n")
        _w(f"{self.root}/sys/module/amdgpu/initstate", "live\n")
        _w(f"{self.root}/dev/kfd", "")
        self.log.append(f"install {version} {cenv.get('AMDGPU_MODULE_PARAMS', '')}".rstrip())


def clear(root: str) -> None:
    shutil.rmtree(root, ignore_errors=True)


class FakePciKernel:
    """The kernel side of PCI driver binding on a fake tree: applies the
    sysfs writes :class:`amdgpu_operator.sandbox.vfio.PciSysfs` makes
    (``driver_override``, ``<driver>/unbind``, ``drivers_probe``) the way
    the PCI core does, and ``modprobe vfio-pci``.  ``busy`` holds fake KFD
    process IDs (GPU users that block an unbind from amdgpu)."""

    def __new__(cls, root: str):
        from ..sandbox.vfio import PciSysfs

        class _Kernel(PciSysfs):
            def write(self, path: str, text: str) -> None:
                super().write(path, text)
                self._apply(os.path.relpath(path, self.path("sys/bus/pci")), text.strip())

            def _dev(self, bdf: str) -> str:
                return self.path("sys/bus/pci/devices", bdf)

            def _apply(self, rel: str, val: str) -> None:
                parts = rel.split(os.sep)
                if rel == "drivers_probe":
                    self._probe(val)
                elif parts[-1] == "unbind":
                    # devices/<bdf>/driver/unbind or drivers/<name>/unbind
                    bdf = parts[1] if parts[0] == "devices" else val
                    link = os.path.join(self._dev(bdf), "driver")
                    if os.path.lexists(link):
                        drv = os.path.basename(os.path.realpath(link))
                        os.unlink(link)
                        if drv == "vfio-pci":
                            grp = self.function(bdf).iommu_group
                            if grp and not any(self.function(b).driver == "vfio-pci" for b in self.group_members(grp)):
                                try:
                                    os.unlink(self.vfio_dev(grp))
                                except OSError:
                                    pass

            def _probe(self, bdf: str) -> None:
                if os.path.lexists(os.path.join(self._dev(bdf), "driver")):
                    return
                try:
                    with open(os.path.join(self._dev(bdf), "driver_override")) as f:
                        override = f.read().strip()
                except OSError:
                    override = ""
                drv = override if override and override != "(null)" else "amdgpu"
                if not self.driver_loaded(drv):
                    return
                _link(f"../../../../bus/pci/drivers/{drv}", os.path.join(self._dev(bdf), "driver"))
                if drv == "vfio-pci":
                    grp = self.function(bdf).iommu_group
                    _w(self.path("dev/vfio/vfio"), "")
                    if grp:
                        _w(self.vfio_dev(grp), "")

            def load_module(self, name: str) -> None:
                self.modprobes.append(name)
                if name in ("vfio-pci", "vfio_pci"):
                    _w(self.path("sys/bus/pci/drivers/vfio-pci/unbind"), "")

            def set_busy(self, pids) -> None:
                procs = self.path("sys/class/kfd/kfd/proc")
                if os.path.isdir(procs):
                    for p in os.listdir(procs):
                        os.rmdir(os.path.join(procs, p))
                for p in pids:
                    os.makedirs(os.path.join(procs, str(p)), exist_ok=True)

        k = _Kernel(root)
        k.modprobes = []
        return k
