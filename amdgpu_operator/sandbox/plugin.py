"""Sandbox device plugin: advertises vfio-bound MI355X GPUs to the kubelet
for VM passthrough.

Counterpart of the NVIDIA operator's sandbox (KubeVirt GPU) device plugin
[EXT]: on a ``vm-passthrough`` node the GPUs are not ``amd.com/gpu`` (no
``/dev/kfd`` for a container) but a per-product resource such as
``amd.com/MI355X`` whose Allocate hands a VM launcher the VFIO group:

* DeviceSpecs ``/dev/vfio/vfio`` (the container) and ``/dev/vfio/<group>``
  for every IOMMU group of the allocated GPUs;
* ``PCI_RESOURCE_AMD_COM_MI355X=<bdf>,<bdf>`` - the env KubeVirt's
  virt-launcher reads to find the host devices of a permitted resource
  (``PCI_RESOURCE_`` + the resource name upper-cased, ``.``/``/`` -> ``_``).

It reuses the kubelet v1beta1 server of :mod:`..deviceplugin.server`
(registration, ListAndWatch, kubelet-restart re-registration, NUMA-aware
preferred allocation); only the device source, health and Allocate differ.
A GPU is healthy while it is bound to vfio-pci and its group's device node
exists (a host-side rebind to amdgpu turns it Unhealthy).
"""

from __future__ import annotations

import os
import threading
from dataclasses import dataclass

from ..deviceplugin import api
from ..deviceplugin.server import DevicePluginServer, PluginConfig
from .vfio import VFIO_DRIVER, PciSysfs

# PCI device ID -> product part of the resource name (labels.PRODUCTS naming)
PRODUCT_NAMES = {0x75A3: "MI355X", 0x75A0: "MI350X", 0x74A1: "MI300X", 0x74A5: "MI325X"}
RESOURCE_PREFIX = "amd.com"


@dataclass
class VfioDevice:
    """A passthrough GPU, shaped like :class:`discovery.topology.GpuDevice`
    where the shared server reads it."""

    index: int
    bdf: str
    device_id: int
    iommu_group: str
    numa_node: int
    unique_id: int = 0
    hive_id: int = 0
    vram_bytes: int = 0
    partition_index: int = 0
    partition_count: int = 1

    @property
    def physical_index(self) -> int:
        return self.index

    @property
    def device_id_str(self) -> str:
        return self.bdf


def resource_name(device_id: int, prefix: str = RESOURCE_PREFIX) -> str:
    return f"{prefix}/{PRODUCT_NAMES.get(device_id, f'AMD_GPU_{device_id:04X}')}"


def kubevirt_env(resource: str) -> str:
    return "PCI_RESOURCE_" + "".join(c if c.isalnum() else "_" for c in resource).upper()


def vfio_devices(pci: PciSysfs) -> list[VfioDevice]:
    """The node's AMD GPUs bound to vfio-pci, in PCI order."""
    out = []
    for f in pci.gpus():
        if f.driver == VFIO_DRIVER and f.iommu_group:
            out.append(VfioDevice(len(out), f.bdf, f.device, f.iommu_group, f.numa_node))
    return out


class VfioPluginServer(DevicePluginServer):
    """One resource (one product) of passthrough GPUs."""

    def __init__(self, cfg: PluginConfig, devices: list[VfioDevice], resource: str):
        super().__init__(cfg, devices, (), resource_name=resource)

    def container_response(self, ids):
        r = api.pb["ContainerAllocateResponse"]()
        devs = list({self._by_id[i].bdf: self._by_id[i] for i in ids}.values())
        r.devices.add(container_path="/dev/vfio/vfio", host_path="/dev/vfio/vfio", permissions="rw")
        for grp in dict.fromkeys(d.iommu_group for d in devs):
            r.devices.add(container_path=f"/dev/vfio/{grp}", host_path=f"/dev/vfio/{grp}", permissions="rw")
        r.envs[kubevirt_env(self.resource_name)] = ",".join(d.bdf for d in devs)
        r.annotations["amd.com/gpu.vfio-groups"] = ",".join(dict.fromkeys(d.iommu_group for d in devs))
        return r


class SandboxPluginManager:
    """Finds the vfio-bound GPUs, serves one resource per product, and keeps
    each device's health in step with its binding."""

    def __init__(self, cfg: PluginConfig, pci: PciSysfs, prefix: str = RESOURCE_PREFIX):
        self.cfg = cfg
        self.pci = pci
        self.devices = vfio_devices(pci)
        by_res: dict[str, list[VfioDevice]] = {}
        for d in self.devices:
            by_res.setdefault(resource_name(d.device_id, prefix), []).append(d)
        self.servers = {}
        for n, (res, devs) in enumerate(sorted(by_res.items())):
            c = PluginConfig(**{**cfg.__dict__, "resource_name": res,
                                "endpoint": f"amd-vfio-{n}.sock" if n else "amd-vfio.sock"})
            self.servers[res] = VfioPluginServer(c, devs, res)
        self._stop = threading.Event()
        self._thread: threading.Thread | None = None

    def check_health(self) -> None:
        for srv in self.servers.values():
            for d in srv.devices:
                f = self.pci.function(d.bdf)
                ok = f.driver == VFIO_DRIVER and os.path.exists(self.pci.vfio_dev(d.iommu_group))
                srv.set_health(d.bdf, ok, "" if ok else f"bound to {f.driver or 'no driver'}")

    def start(self, register: bool = True) -> None:
        for srv in self.servers.values():
            srv.start(register)
        self._thread = threading.Thread(target=self._loop, name="amdgpu-vfio-health", daemon=True)
        self._thread.start()

    def _loop(self) -> None:
        while not self._stop.wait(max(0.05, self.cfg.health_poll_ms / 1000.0)):
            self.check_health()

    def stop(self) -> None:
        self._stop.set()
        for srv in self.servers.values():
            srv.stop()
