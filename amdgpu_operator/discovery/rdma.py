"""RDMA NICs next to the GPUs: inventory, PCIe affinity, peer-memory readiness.

Upstream parity: the NVIDIA GPU Operator's ``driver.rdma.enabled`` /
``driver.rdma.useHostMofed`` (GPUDirect RDMA: the driver container loads
``nvidia-peermem`` once the MOFED driver is up, the validator checks it).  The
reference leaves it at its default (off: /root/reference/README.md:101-110
sets neither key); a multi-node MI355X job needs it, because RCCL moves
inter-node traffic NIC <-> HBM directly only when the NIC can address GPU
memory.  On AMD there is no peer-memory module to load: amdgpu exports VRAM
as a dma-buf (``hsa_amd_portable_export_dmabuf``), and the RDMA core imports
it (``ib_umem_dmabuf``, kernel >= 5.12).  Readiness is therefore:

* the RDMA core is up: ``ib_core`` and ``ib_uverbs`` loaded (the host's
  MOFED/inbox stack with ``useHostMofed``, else the driver container loads
  ``ib_uverbs``), and at least one RDMA device with an ACTIVE port;
* the kernel can hand a dma-buf to the NIC (>= 5.12);
* the validator's ``dmabuf`` step exports HBM as a dma-buf and imports it
  back on the device (native/validator/validator_main.cpp step_dmabuf).

Affinity: a GPU should use the NIC nearest to it on the PCIe tree - the same
switch (``PIX``), the same root port hierarchy (``PXB``), the same host
bridge (``PHB``), the same NUMA node (``NODE``), or across sockets (``SYS``),
the path classes RCCL's topology search uses.  The device plugin reports the
nearest NICs of an allocation (annotation, optionally ``NCCL_IB_HCA``).
"""

from __future__ import annotations

import os
import re
from dataclasses import dataclass

# path classes, nearest first
PIX, PXB, PHB, NODE, SYS = "PIX", "PXB", "PHB", "NODE", "SYS"
_RANK = {PIX: 0, PXB: 1, PHB: 2, NODE: 3, SYS: 4}
RDMA_MODULES = ("ib_core", "ib_uverbs")
DMABUF_MIN_KERNEL = (5, 12)


@dataclass(frozen=True)
class RdmaNic:
    name: str  # kernel RDMA device name (mlx5_0, bnxt_re0, ionic_0, ...)
    bdf: str
    numa_node: int
    pci_path: tuple[str, ...]  # /sys/devices components from the host bridge down to the function
    ports: tuple[tuple[int, str, str, float], ...]  # (port, state, link layer, Gb/s)

    @property
    def active(self) -> bool:
        return any(state == "ACTIVE" for _, state, _, _ in self.ports)

    @property
    def link_layer(self) -> str:
        layers = {layer for _, state, layer, _ in self.ports if state == "ACTIVE"}
        return "mixed" if len(layers) > 1 else (layers.pop() if layers else "")

    @property
    def rate_gbps(self) -> float:
        rates = [r for _, state, _, r in self.ports if state == "ACTIVE"]
        return max(rates) if rates else 0.0


def _read(path: str) -> str | None:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def _j(root: str, rel: str) -> str:
    return os.path.join(root or "/", rel.lstrip("/"))


def pci_path(root: str, bdf: str) -> tuple[str, ...]:
    """The PCIe path of a function: the /sys/devices components below
    ``pci<domain>:<bus>`` (host bridge first), from the bus symlink."""
    real = os.path.realpath(_j(root, f"sys/bus/pci/devices/{bdf}"))
    parts = real.split(os.sep)
    for i, p in enumerate(parts):
        if p.startswith("pci") and ":" in p:
            return tuple(parts[i:])
    return (bdf,)  # no tree in this view (a flat sysfs copy): NUMA decides


_RATE_RE = re.compile(r"([\d.]+)\s*Gb/sec")


def enumerate_nics(root: str = "/") -> list[RdmaNic]:
    base = _j(root, "sys/class/infiniband")
    try:
        names = sorted(os.listdir(base))
    except OSError:
        return []
    out = []
    for name in names:
        dev = os.path.join(base, name, "device")
        bdf = os.path.basename(os.path.realpath(dev))
        numa = _read(os.path.join(dev, "numa_node"))
        ports = []
        pdir = os.path.join(base, name, "ports")
        for p in sorted(os.listdir(pdir), key=lambda s: int(s) if s.isdigit() else 0) if os.path.isdir(pdir) else []:
            state = (_read(os.path.join(pdir, p, "state")) or "").split(":")[-1].strip()
            layer = _read(os.path.join(pdir, p, "link_layer")) or ""
            m = _RATE_RE.search(_read(os.path.join(pdir, p, "rate")) or "")
            ports.append((int(p) if p.isdigit() else 0, state, layer, float(m.group(1)) if m else 0.0))
        out.append(RdmaNic(name, bdf, int(numa) if numa and numa.lstrip("-").isdigit() else -1,
                           pci_path(root, bdf), tuple(ports)))
    return out


def path_class(a: tuple[str, ...], a_numa: int, b: tuple[str, ...], b_numa: int) -> str:
    """RCCL-style distance between two PCI functions from their PCIe paths."""
    common = 0
    for x, y in zip(a, b):
        if x != y:
            break
        common += 1
    if common == 0 or len(a) < 2 or len(b) < 2:  # different host bridges (or no tree)
        return NODE if a_numa == b_numa and a_numa >= 0 else SYS
    if common == 1:
        return PHB  # only the host bridge in common
    # below the deepest shared bridge (a switch's upstream port): its
    # downstream port and the function itself on each side = one switch
    return PIX if (len(a) - common) <= 2 and (len(b) - common) <= 2 else PXB


def nearest_nics(gpus, nics: list[RdmaNic], root: str = "/") -> dict[str, list[tuple[str, str]]]:
    """Per GPU (by BDF), the active NICs at the smallest path class:
    ``{bdf: [(nic, class), ...]}``."""
    out = {}
    active = [n for n in nics if n.active] or list(nics)
    for g in gpus:
        gp = pci_path(root, g.bdf)
        ranked = sorted(((path_class(gp, g.numa_node, n.pci_path, n.numa_node), n.name) for n in active),
                        key=lambda t: (_RANK[t[0]], t[1]))
        best = ranked[0][0] if ranked else None
        out[g.bdf] = [(name, cls) for cls, name in ranked if cls == best]
    return out


def allocation_nics(gpus, nics: list[RdmaNic], root: str = "/") -> list[str]:
    """NICs for a set of allocated GPUs: each GPU's nearest NIC, spread so
    GPUs sharing a switch with several NICs take different ones; ordered as
    the GPUs are, deduplicated."""
    near = nearest_nics(gpus, nics, root)
    used: dict[str, int] = {}
    out = []
    for g in gpus:
        cands = [n for n, _ in near.get(g.bdf, [])]
        if not cands:
            continue
        pick = min(cands, key=lambda n: (used.get(n, 0), n))
        used[pick] = used.get(pick, 0) + 1
        if pick not in out:
            out.append(pick)
    return out


def kernel_version(root: str = "/") -> tuple[int, int]:
    rel = _read(_j(root, "proc/sys/kernel/osrelease")) or os.uname().release
    m = re.match(r"(\d+)\.(\d+)", rel)
    return (int(m.group(1)), int(m.group(2))) if m else (0, 0)


def modules_loaded(root: str = "/", names=RDMA_MODULES) -> dict[str, bool]:
    return {m: os.path.isdir(_j(root, f"sys/module/{m}")) for m in names}


def readiness(root: str = "/") -> dict:
    """The node's GPU-RDMA state (what driver.rdma waits for)."""
    nics = enumerate_nics(root)
    mods = modules_loaded(root)
    kv = kernel_version(root)
    problems = [f"module {m} not loaded" for m, ok in mods.items() if not ok]
    if not nics:
        problems.append("no RDMA device (/sys/class/infiniband)")
    elif not any(n.active for n in nics):
        problems.append("no RDMA port ACTIVE")
    if kv < DMABUF_MIN_KERNEL:
        problems.append(f"kernel {kv[0]}.{kv[1]} < 5.12: no dma-buf import in the RDMA core")
    return {"ok": not problems, "problems": problems, "nics": [n.name for n in nics],
            "active": [n.name for n in nics if n.active], "modules": mods, "kernel": f"{kv[0]}.{kv[1]}",
            "dmabuf": kv >= DMABUF_MIN_KERNEL}


def rdma_labels(gpus, root: str = "/", prefix: str = "amd.com") -> dict[str, str]:
    """GFD labels for the node's RDMA side (empty without RDMA devices)."""
    nics = enumerate_nics(root)
    if not nics:
        return {}
    active = [n for n in nics if n.active]
    out = {f"{prefix}/gpu.rdma.capable": "true" if active and all(modules_loaded(root).values()) else "false",
           f"{prefix}/gpu.rdma.nics": str(len(active)),
           f"{prefix}/gpu.rdma.dmabuf": "true" if kernel_version(root) >= DMABUF_MIN_KERNEL else "false"}
    layers = {n.link_layer for n in active}
    if layers:
        out[f"{prefix}/gpu.rdma.link-layer"] = "mixed" if len(layers) > 1 else ("RoCE" if "Ethernet" in layers else
                                                                               layers.pop())
        out[f"{prefix}/gpu.rdma.rate-gbps"] = str(int(min(n.rate_gbps for n in active)))
    if gpus and active:
        near = nearest_nics(gpus, nics, root)
        worst = max((_RANK[c[0][1]] for c in near.values() if c), default=None)
        if worst is not None:
            out[f"{prefix}/gpu.rdma.affinity"] = [k for k, v in _RANK.items() if v == worst][0]
    return out
