"""vfio-manager: hand a node's AMD GPUs to ``vfio-pci`` for VM passthrough,
and back to ``amdgpu``.

The NVIDIA GPU Operator's sandbox mode runs a vfio-manager DaemonSet on nodes
whose ``nvidia.com/gpu.workload.config`` is ``vm-passthrough`` [EXT, SURVEY.md
§0 citation rules: the reference README does not enable it; its
``driver/toolkit/devicePlugin`` flags at /root/reference/README.md:104-106 are
the container half of the same switch].  Here the work is done through the
kernel's PCI sysfs interface, the same on every MI355X host:

* every non-bridge function of a GPU's IOMMU group must be bound to
  ``vfio-pci`` (a VM gets whole groups: ``/dev/vfio/<group>``);
* ``driver_override`` pins the function to ``vfio-pci`` so a later rescan or
  amdgpu reload cannot reclaim it; ``<driver>/unbind`` releases it from
  ``amdgpu``; ``drivers_probe`` binds it to the override;
* a GPU with KFD processes still open (``/sys/class/kfd/kfd/proc/<pid>``) is
  not pulled from under them: the manager waits, bounded, and then fails.

``unbind`` reverses it: override cleared, released from ``vfio-pci``, probed
back to the host driver.  All sysfs writes go through :class:`PciSysfs`; the
simulated kernel (``testing/fakesys.FakePciKernel``) sees the same writes.
"""

from __future__ import annotations

import os
import subprocess
import threading
import time
from dataclasses import dataclass

from ..discovery.labels import AMD_VENDOR, GPU_CLASSES
from ..utils.logs import get_logger

log = get_logger("amdgpu.vfio")

VFIO_DRIVER = "vfio-pci"
HOST_DRIVER = "amdgpu"
BRIDGE_CLASS = "0604"
READY_FILE = "vfio-ready"


class VfioError(RuntimeError):
    pass


@dataclass
class PciFunction:
    bdf: str
    vendor: str       # "1002"
    device: int       # PCI device ID
    cls: str          # 6 hex digits
    driver: str | None
    iommu_group: str | None
    numa_node: int

    @property
    def is_amd_gpu(self) -> bool:
        return self.vendor == AMD_VENDOR and self.cls[:4] in GPU_CLASSES

    @property
    def is_bridge(self) -> bool:
        return self.cls[:4] == BRIDGE_CLASS


def _hex(text: str | None) -> str:
    return (text or "").strip().lower().replace("0x", "")


class PciSysfs:
    """The kernel's PCI driver-binding interface under ``root``."""

    def __init__(self, root: str = "/"):
        self.root = root or "/"

    def path(self, *rel: str) -> str:
        return os.path.join(self.root, *[r.lstrip("/") for r in rel])

    def _read(self, *rel: str) -> str | None:
        try:
            with open(self.path(*rel)) as f:
                return f.read().strip()
        except OSError:
            return None

    def write(self, path: str, text: str) -> None:
        """One sysfs write (the kernel acts on it); errors name the file."""
        try:
            with open(path, "w") as f:
                f.write(text)
        except OSError as e:
            raise VfioError(f"write {text.strip()!r} to {path}: {e.strerror or e}") from e

    # ------------------------------------------------------------ discovery
    def function(self, bdf: str) -> PciFunction:
        d = ("sys/bus/pci/devices", bdf)
        drv = os.path.realpath(self.path(*d, "driver")) if os.path.lexists(self.path(*d, "driver")) else None
        grp = self.path(*d, "iommu_group")
        numa = self._read(*d, "numa_node")
        try:
            dev_id = int(_hex(self._read(*d, "device")) or "0", 16)
        except ValueError:
            dev_id = 0
        return PciFunction(bdf, _hex(self._read(*d, "vendor")), dev_id, _hex(self._read(*d, "class")).zfill(6),
                           os.path.basename(drv) if drv else None,
                           os.path.basename(os.path.realpath(grp)) if os.path.lexists(grp) else None,
                           int(numa) if numa and numa.lstrip("-").isdigit() else -1)

    def functions(self) -> list[PciFunction]:
        try:
            names = sorted(os.listdir(self.path("sys/bus/pci/devices")))
        except OSError:
            return []
        return [self.function(b) for b in names]

    def gpus(self) -> list[PciFunction]:
        return [f for f in self.functions() if f.is_amd_gpu]

    def group_members(self, group: str) -> list[str]:
        try:
            return sorted(os.listdir(self.path("sys/kernel/iommu_groups", group, "devices")))
        except OSError:
            return []

    def driver_loaded(self, name: str) -> bool:
        return os.path.isdir(self.path("sys/bus/pci/drivers", name))

    def vfio_dev(self, group: str) -> str:
        return self.path("dev/vfio", group)

    def kfd_processes(self) -> list[str]:
        try:
            return sorted(p for p in os.listdir(self.path("sys/class/kfd/kfd/proc")) if p.isdigit())
        except OSError:
            return []

    # -------------------------------------------------------------- binding
    def set_override(self, bdf: str, driver: str) -> None:
        self.write(self.path("sys/bus/pci/devices", bdf, "driver_override"), (driver or "") + "\n")

    def unbind(self, bdf: str) -> None:
        if os.path.lexists(self.path("sys/bus/pci/devices", bdf, "driver")):
            self.write(self.path("sys/bus/pci/devices", bdf, "driver", "unbind"), bdf)

    def probe(self, bdf: str) -> None:
        self.write(self.path("sys/bus/pci/drivers_probe"), bdf)

    def load_module(self, name: str) -> None:
        """``modprobe`` into the host kernel: the manager's privileged
        container mounts the host's /lib/modules, like the driver container."""
        r = subprocess.run(["modprobe", name], capture_output=True, text=True, timeout=60)
        if r.returncode != 0:
            raise VfioError(f"modprobe {name}: {r.stderr.strip() or r.returncode}")


@dataclass
class GroupResult:
    group: str
    gpus: list[str]
    functions: list[str]
    driver: str
    changed: bool


def _groups(pci: PciSysfs) -> dict[str, list[PciFunction]]:
    """IOMMU group -> the AMD GPUs in it (a GPU without a group cannot be
    passed through: the IOMMU is off)."""
    out: dict[str, list[PciFunction]] = {}
    for g in pci.gpus():
        if g.iommu_group is None:
            raise VfioError(f"{g.bdf} has no IOMMU group: enable the IOMMU (amd_iommu=on iommu=pt) for passthrough")
        out.setdefault(g.iommu_group, []).append(g)
    return out


def _wait_kfd_idle(pci: PciSysfs, timeout: float, stop: threading.Event | None) -> None:
    deadline = time.monotonic() + timeout
    while True:
        procs = pci.kfd_processes()
        if not procs:
            return
        if time.monotonic() >= deadline or (stop is not None and stop.is_set()):
            raise VfioError(f"GPUs still in use by KFD processes {procs[:8]}: not unbinding them from {HOST_DRIVER}")
        (stop.wait if stop is not None else time.sleep)(0.05)


def bind_all(pci: PciSysfs, timeout: float = 60.0, stop: threading.Event | None = None) -> list[GroupResult]:
    """Bind every AMD GPU (with its IOMMU group) to vfio-pci. Idempotent."""
    groups = _groups(pci)
    if not groups:
        return []
    if not pci.driver_loaded(VFIO_DRIVER):
        pci.load_module("vfio-pci")
        if not pci.driver_loaded(VFIO_DRIVER):
            raise VfioError("vfio-pci driver not available after modprobe")
    todo = {grp: [pci.function(b) for b in pci.group_members(grp) or [g.bdf for g in gpus]]
            for grp, gpus in groups.items()}
    if any(f.driver == HOST_DRIVER for fns in todo.values() for f in fns):
        _wait_kfd_idle(pci, timeout, stop)
    out = []
    for grp, fns in sorted(todo.items(), key=lambda kv: int(kv[0]) if kv[0].isdigit() else kv[0]):
        changed = False
        for f in fns:
            if f.is_bridge or f.driver == VFIO_DRIVER:
                continue
            pci.set_override(f.bdf, VFIO_DRIVER)
            pci.unbind(f.bdf)
            pci.probe(f.bdf)
            now = pci.function(f.bdf).driver
            if now != VFIO_DRIVER:
                raise VfioError(f"{f.bdf}: bound to {now or 'no driver'} after probe, expected {VFIO_DRIVER}")
            changed = True
        gpus = [g.bdf for g in groups[grp]]
        out.append(GroupResult(grp, gpus, [f.bdf for f in fns if not f.is_bridge], VFIO_DRIVER, changed))
        if changed:
            log.info("IOMMU group %s (%s) bound to %s", grp, ",".join(gpus), VFIO_DRIVER)
    return out


def unbind_all(pci: PciSysfs) -> list[GroupResult]:
    """Return every AMD GPU group from vfio-pci to the host driver."""
    out = []
    for grp, gpus in sorted(_groups(pci).items()):
        fns = [pci.function(b) for b in pci.group_members(grp) or [g.bdf for g in gpus]]
        changed = False
        for f in fns:
            if f.is_bridge or f.driver != VFIO_DRIVER:
                continue
            pci.set_override(f.bdf, "")
            pci.unbind(f.bdf)
            pci.probe(f.bdf)
            changed = True
        out.append(GroupResult(grp, [g.bdf for g in gpus], [f.bdf for f in fns if not f.is_bridge],
                               pci.function(gpus[0].bdf).driver or "", changed))
    return out


# <linux/vfio.h>: VFIO_GROUP_GET_STATUS = _IO(';', 100 + 3), struct vfio_group_status {argsz, flags}
VFIO_GROUP_GET_STATUS = (ord(";") << 8) | (100 + 3)
VFIO_GROUP_FLAGS_VIABLE = 1 << 0


def group_viable(dev_path: str) -> bool | None:
    """Ask the kernel whether a VFIO group is viable (every device of the
    group bound to a VFIO driver, so a VM may own it).  None when the path
    is not a VFIO character device (a test tree) or the query is refused."""
    import fcntl
    import stat
    import struct

    try:
        if not stat.S_ISCHR(os.stat(dev_path).st_mode):
            return None
        fd = os.open(dev_path, os.O_RDWR)
    except OSError:
        return None
    try:
        buf = bytearray(struct.pack("II", 8, 0))
        fcntl.ioctl(fd, VFIO_GROUP_GET_STATUS, buf, True)
        return bool(struct.unpack("II", bytes(buf))[1] & VFIO_GROUP_FLAGS_VIABLE)
    except OSError:  # EBUSY: a VM holds the group already; the binding was checked above
        return None
    finally:
        os.close(fd)


def check_bound(pci: PciSysfs) -> tuple[bool, str, list[dict]]:
    """Sandbox validation: every AMD GPU on vfio-pci with its group's device
    node present.  Returns (ok, message, per-GPU detail)."""
    gpus = pci.gpus()
    if not gpus:
        return False, "no AMD GPU on the PCI bus", []
    detail, bad = [], []
    for g in gpus:
        dev = pci.vfio_dev(g.iommu_group) if g.iommu_group else ""
        ok = g.driver == VFIO_DRIVER and bool(dev) and os.path.exists(dev)
        viable = group_viable(dev) if ok else None
        detail.append({"bdf": g.bdf, "driver": g.driver, "iommu_group": g.iommu_group, "vfio_dev": ok,
                       "viable": viable})
        if not ok:
            bad.append(f"{g.bdf} ({g.driver or 'unbound'})")
        elif viable is False:
            bad.append(f"{g.bdf} (IOMMU group {g.iommu_group} not viable: a member is on another driver)")
    if bad:
        return False, f"not ready for passthrough: {', '.join(bad)}", detail
    return True, f"{len(gpus)} GPU(s) bound to {VFIO_DRIVER}", detail
