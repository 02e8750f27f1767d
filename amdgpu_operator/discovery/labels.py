"""Node feature discovery (C7) and GPU feature discovery (C6) labels.

Reference parity: ``gpu-feature-discovery`` "detects GPUs and labels nodes
that have them" (/root/reference/README.md:108,202,209); GPU nodes are then
selected by label (README.md:119).  Upstream GFD depends on NFD's PCI labels;
here both are implemented natively over the same sysfs view:

* NFD-lite: ``feature.node.kubernetes.io/pci-<class>_<vendor>.present`` (the
  NFD default device label fields) and ``pci-1002.present`` for every AMD
  display / processing-accelerator PCI function, plus
  ``kernel-loadedmodule.amdgpu`` when the module is live.
* GFD: the MI355X capability set - product, CDNA4 family, gfx950 arch, device
  count, HBM per device, CUs/XCCs/LDS, MFMA data types (bf16, fp16, OCP fp8,
  fp6, fp4, f32, f64; no xf32 on gfx950), xGMI hive and link count, compute /
  memory partition mode, driver and ROCm versions; with RDMA NICs on the
  node, their count, link layer, rate and PCIe affinity to the GPUs
  (discovery/rdma.py).
"""

from __future__ import annotations

import os
import re

from .topology import GpuDevice

NFD_PREFIX = "feature.node.kubernetes.io/"
AMD_VENDOR = "1002"
GPU_CLASSES = ("1200", "0380", "0300")  # processing accelerator, display, VGA

PRODUCTS = {
    0x75A3: "AMD-Instinct-MI355X",
    0x75A0: "AMD-Instinct-MI350X",
    0x74A1: "AMD-Instinct-MI300X",
    0x74A5: "AMD-Instinct-MI325X",
}
FAMILIES = {"gfx950": "CDNA4", "gfx942": "CDNA3", "gfx90a": "CDNA2", "gfx908": "CDNA"}
MFMA_TYPES = {
    "CDNA4": {"bf16": True, "fp16": True, "fp8": True, "fp6": True, "fp4": True, "fp32": True, "fp64": True,
              "int8": True, "xf32": False},
    "CDNA3": {"bf16": True, "fp16": True, "fp8": True, "fp6": False, "fp4": False, "fp32": True, "fp64": True,
              "int8": True, "xf32": True},
}
# labels the operator owns (never removed by the GFD sweep)
OPERATOR_OWNED = ("amd.com/gpu.present", "amd.com/gpu.deploy.", "amd.com/gpu.validated", "amd.com/gpu.workload.config",
                  "amd.com/gpu.partition-config", "amd.com/gpu.partition.", "amd.com/gpu.present.source")

_VALUE_RE = re.compile(r"[^A-Za-z0-9_.-]")


def label_value(v) -> str:
    """Kubernetes label value: <= 63 chars of [A-Za-z0-9_.-], alnum at both ends."""
    s = _VALUE_RE.sub("-", str(v))[:63]
    return s.strip("-_.")


def _read(path: str) -> str | None:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def _root_join(root: str, rel: str) -> str:
    return os.path.join(root or "/", rel.lstrip("/"))


def nfd_labels(root: str = "/") -> dict[str, str]:
    labels: dict[str, str] = {}
    pci = _root_join(root, "sys/bus/pci/devices")
    try:
        devs = sorted(os.listdir(pci))
    except OSError:
        devs = []
    for d in devs:
        vendor = (_read(os.path.join(pci, d, "vendor")) or "").lower().replace("0x", "")
        cls = (_read(os.path.join(pci, d, "class")) or "").lower().replace("0x", "")
        if not vendor or not cls:
            continue
        cls4 = cls.zfill(6)[:4]
        labels[f"{NFD_PREFIX}pci-{cls4}_{vendor}.present"] = "true"
        if vendor == AMD_VENDOR and cls4 in GPU_CLASSES:
            labels[f"{NFD_PREFIX}pci-{AMD_VENDOR}.present"] = "true"
    if _read(_root_join(root, "sys/module/amdgpu/initstate")) == "live":
        labels[f"{NFD_PREFIX}kernel-loadedmodule.amdgpu"] = "true"
    # NFD's rdma feature: an RDMA device present / the user-space RDMA modules loaded
    try:
        if os.listdir(_root_join(root, "sys/class/infiniband")):
            labels[f"{NFD_PREFIX}rdma.capable"] = "true"
    except OSError:
        pass
    if all(os.path.isdir(_root_join(root, f"sys/module/{m}")) for m in ("ib_uverbs", "rdma_ucm")):
        labels[f"{NFD_PREFIX}rdma.available"] = "true"
    # a container shares the node's kernel: its own uname is the node's
    ver = _read(_root_join(root, "proc/sys/kernel/osrelease")) or os.uname().release
    if ver:
        labels[f"{NFD_PREFIX}kernel-version.full"] = label_value(ver)
    return labels


def rocm_version(root: str = "/") -> str:
    for p in ("opt/rocm/.info/version", "opt/rocm/.info/version-dev"):
        v = _read(_root_join(root, p))
        if v:
            return v.split("-")[0]
    return os.environ.get("ROCM_VERSION", "")


def _uniform(values, mixed: str = "mixed"):
    """The single value of ``values``, or ``mixed`` when they differ."""
    s = set(values)
    return s.pop() if len(s) == 1 else mixed


def gfd_labels(gpus: list[GpuDevice], root: str = "/", prefix: str = "amd.com") -> dict[str, str]:
    """Node labels from every GPU of the node, not the first one only.

    A property all devices share is labelled with its value; one that
    differs (a node with GPUs in different partition modes, or mixed SKUs)
    reads ``mixed``.  Sizes (memory, CUs, clocks, xGMI links) are the
    minimum over the devices, so a nodeAffinity on them holds for every
    device the scheduler may hand out; an MFMA data type is ``true`` only
    when every device has it.  With mixed partition modes each mode also
    gets ``<prefix>/gpu.<mode>.count`` / ``.memory`` / ``.compute-units`` /
    ``.product`` - the devices the plugin's ``mixed`` strategy advertises as
    ``<prefix>/gpu-<mode>`` (``<prefix>/gpu`` for unpartitioned ones) - and
    mixed SKUs ``<prefix>/gpu.product.<product>.count``."""
    p = f"{prefix}/gpu"
    if not gpus:
        return {}

    def product(g):
        return PRODUCTS.get(g.device_id, f"AMD-GPU-{g.device_id:04x}")

    families = {FAMILIES.get(g.arch, "unknown") for g in gpus}
    physical = len({g.physical_index for g in gpus})
    numa = sorted({g.numa_node for g in gpus if g.numa_node >= 0})
    modes = [g.compute_partition or "SPX" for g in gpus]
    labels = {
        f"{p}.count": str(len(gpus)),
        f"{p}.physical-count": str(physical),
        f"{p}.product": label_value(_uniform(product(g) for g in gpus)),
        f"{p}.device-id": _uniform(f"{g.device_id:04x}" for g in gpus),
        f"{p}.family": _uniform(families),
        f"{p}.arch": label_value(_uniform(g.arch for g in gpus)),
        f"{p}.memory": str(min(g.vram_bytes for g in gpus) // (1024 * 1024)),
        f"{p}.memory-gib": str(round(min(g.vram_bytes for g in gpus) / 2**30)),
        f"{p}.compute-units": str(min(g.cu_count for g in gpus)),
        f"{p}.xcc": str(min(g.num_xcc for g in gpus)),
        f"{p}.lds-kib": str(min(g.lds_size_kib for g in gpus)),
        f"{p}.wavefront-size": "64",
        f"{p}.max-clock-mhz": str(min(g.max_engine_clk_mhz for g in gpus)),
        f"{p}.compute-partition": label_value(_uniform(modes)),
        f"{p}.memory-partition": label_value(_uniform(g.memory_partition or "NPS1" for g in gpus)),
        f"{p}.partition-capable": "true" if families <= {"CDNA4", "CDNA3"} else "false",
        f"{p}.numa-nodes": label_value("-".join(str(n) for n in numa) or "none"),
    }
    for dtype in sorted({d for f in families for d in MFMA_TYPES.get(f, {})}):
        labels[f"{p}.mfma.{dtype}"] = "true" if all(MFMA_TYPES.get(f, {}).get(dtype) for f in families) else "false"
    if len(set(modes)) > 1:
        for mode in sorted(set(modes)):
            group = [g for g, m in zip(gpus, modes) if m == mode]
            m = label_value(mode.lower())
            labels[f"{p}.{m}.count"] = str(len(group))
            labels[f"{p}.{m}.memory"] = str(min(g.vram_bytes for g in group) // (1024 * 1024))
            labels[f"{p}.{m}.compute-units"] = str(min(g.cu_count for g in group))
            labels[f"{p}.{m}.product"] = label_value(_uniform(product(g) for g in group))
    products = [product(g) for g in gpus]
    if len(set(products)) > 1:
        for prod in sorted(set(products)):
            labels[f"{p}.product.{label_value(prod)}.count"] = str(products.count(prod))
    hives = {g.hive_id for g in gpus if g.hive_id}
    labels[f"{p}.xgmi.links"] = str(min(g.xgmi_links for g in gpus))
    labels[f"{p}.xgmi.hive"] = label_value(f"{min(hives):x}") if hives else "none"
    labels[f"{p}.xgmi.hives"] = str(len(hives))
    drv = _read(_root_join(root, "sys/module/amdgpu/version"))
    if drv:
        labels[f"{p}.driver-version"] = label_value(drv)
    rocm = rocm_version(root)
    if rocm:
        labels[f"{p}.rocm-version"] = label_value(rocm)
    from .rdma import rdma_labels  # RDMA NICs beside the GPUs (none: no labels)

    labels.update(rdma_labels(gpus, root, prefix))
    return labels


def sharing_labels(labels: dict[str, str], plugin_config, resource: str = "amd.com/gpu",
                   prefix: str = "amd.com") -> dict[str, str]:
    """GPU-sharing labels from the device-plugin config (deviceplugin/config.py):
    ``gpu.replicas``, ``gpu.sharing-strategy`` and, when the shared GPUs keep
    the plain resource name, ``-SHARED`` on the product label (as upstream GFD
    marks time-sliced GPUs)."""
    p = f"{prefix}/gpu"
    out = dict(labels)
    rule = plugin_config.shared_for(resource) if plugin_config is not None else None
    replicas = rule.replicas if rule is not None else 1
    out[f"{p}.replicas"] = str(replicas)
    out[f"{p}.sharing-strategy"] = "time-slicing" if replicas > 1 else "none"
    if replicas > 1 and plugin_config.shared_name(resource, rule) == resource and f"{p}.product" in out:
        out[f"{p}.product"] = label_value(out[f"{p}.product"] + "-SHARED")
    return out


def sync_node_labels(client, node_name: str, desired: dict[str, str], owned_prefixes: tuple[str, ...],
                     annotations: dict[str, str] | None = None) -> dict:
    """Set ``desired`` and remove stale labels under ``owned_prefixes``
    (operator-owned labels are never removed); ``annotations`` are set in the
    same patch when missing. Returns the applied label patch."""
    node = client.get("v1", "Node", node_name)
    cur_ann = node.get("metadata", {}).get("annotations") or {}
    ann = {k: v for k, v in (annotations or {}).items() if cur_ann.get(k) != v}
    cur = node.get("metadata", {}).get("labels") or {}
    patch: dict = {}
    for k, v in desired.items():
        if cur.get(k) != v:
            patch[k] = v
    for k in cur:
        if k in desired or any(k.startswith(o) for o in OPERATOR_OWNED):
            continue
        if any(k.startswith(pfx) for pfx in owned_prefixes):
            patch[k] = None
    if patch or ann:
        meta: dict = {"labels": patch}
        if ann:
            meta["annotations"] = ann
        client.patch("v1", "Node", node_name, {"metadata": meta})
    return patch
