"""GPU node detection and operand deploy labels.

Reference parity: GPU nodes carry ``nvidia.com/gpu.present=true``
(/root/reference/README.md:119) - set by the operator from NFD's PCI labels.
Here: a node is an AMD GPU node when NFD (ours or upstream) reports PCI vendor
``0x1002`` with a display / processing-accelerator class, or when the node
already advertises ``amd.com/gpu``.  GPU nodes get ``amd.com/gpu.present=true``
and one ``amd.com/gpu.deploy.<operand>`` label per operand; a user-set
``false`` deploy label opts a node out of that operand and is preserved.
"""

from __future__ import annotations

from .. import LABEL_PRESENT, RESOURCE_NAME
from ..api.clusterpolicy import WORKLOAD_OPERANDS, ClusterPolicySpec, operand_enabled
from ..sandbox import WORKLOAD_CONFIG_LABEL, WORKLOADS
from ..utils.logs import get_logger
from .manifests import DEPLOY_LABEL, OPERAND_LABELS

log = get_logger("amdgpu.nodes")
VALIDATED_LABELS = ("amd.com/gpu.validated", "amd.com/gpu.validated.mfma", "amd.com/gpu.validated.mfma-rate")

NFD_PCI_LABELS = (
    "feature.node.kubernetes.io/pci-1002.present",       # vendor only
    "feature.node.kubernetes.io/pci-1200_1002.present",  # processing accelerator (MI series)
    "feature.node.kubernetes.io/pci-0380_1002.present",  # display controller
    "feature.node.kubernetes.io/pci-0300_1002.present",  # VGA
)
# written by our NFD worker (cli/operands.py nfd) with its first label sync: a
# node without it has not been scanned yet, so "no GPU labels" means nothing
from ..wellknown import NFD_SCANNED_ANN  # noqa: E402,F401 - re-exported


def is_gpu_node(node: dict) -> bool:
    labels = node.get("metadata", {}).get("labels") or {}
    if any(labels.get(k) == "true" for k in NFD_PCI_LABELS):
        return True
    cap = (node.get("status") or {}).get("capacity") or {}
    try:
        if int(cap.get(RESOURCE_NAME, "0")) > 0:
            return True
    except ValueError:
        pass
    return labels.get(LABEL_PRESENT) == "true" and labels.get("amd.com/gpu.present.source") == "manual"


def nfd_scanned(node: dict) -> bool:
    """Our NFD worker has run on the node, or another NFD left PCI labels."""
    meta = node.get("metadata") or {}
    if (meta.get("annotations") or {}).get(NFD_SCANNED_ANN):
        return True
    return any(k.startswith("feature.node.kubernetes.io/pci-") for k in meta.get("labels") or {})


def node_workload(node: dict, spec: ClusterPolicySpec) -> str:
    """``container`` or ``vm-passthrough``: the node's
    ``amd.com/gpu.workload.config`` label under ``sandboxWorkloads``, else
    ``sandboxWorkloads.defaultWorkload``; always ``container`` without sandbox mode."""
    if not spec.sandboxWorkloads.enabled:
        return "container"
    val = (node.get("metadata", {}).get("labels") or {}).get(WORKLOAD_CONFIG_LABEL)
    if val in WORKLOADS:
        return val
    if val is not None:
        log.warning("node %s: unknown %s=%r, using %s", node.get("metadata", {}).get("name"), WORKLOAD_CONFIG_LABEL,
                    val, spec.sandboxWorkloads.defaultWorkload)
    return spec.sandboxWorkloads.defaultWorkload


def desired_labels(node: dict, spec: ClusterPolicySpec) -> dict:
    """Label patch (value None = remove) for one node."""
    labels = node.get("metadata", {}).get("labels") or {}
    patch: dict = {}
    gpu = is_gpu_node(node)
    if gpu:
        if labels.get(LABEL_PRESENT) != "true":
            patch[LABEL_PRESENT] = "true"
        mine = WORKLOAD_OPERANDS[node_workload(node, spec)]
        switched = False
        for key, suffix in OPERAND_LABELS.items():
            lbl = DEPLOY_LABEL.format(suffix)
            if not operand_enabled(spec, key) or key not in mine:
                if lbl in labels:
                    patch[lbl] = None
                    switched |= labels[lbl] == "true" and operand_enabled(spec, key)
                continue
            if labels.get(lbl) == "false":
                continue  # user opt-out is sticky
            if (labels.get(lbl) or "").startswith("paused-for-"):
                continue  # paused by a node agent (partition manager) for a change: it restores the label
            if labels.get(lbl) != "true":
                patch[lbl] = "true"
        if switched:
            # the node changed workload (container <-> vm-passthrough): its
            # validation was for the other one
            for lbl in VALIDATED_LABELS:
                if lbl in labels:
                    patch[lbl] = None
    else:
        if LABEL_PRESENT in labels and labels.get("amd.com/gpu.present.source") != "manual":
            patch[LABEL_PRESENT] = None
        for suffix in OPERAND_LABELS.values():
            lbl = DEPLOY_LABEL.format(suffix)
            if lbl in labels:
                patch[lbl] = None
    return patch


def label_nodes(client, spec: ClusterPolicySpec) -> tuple[int, int, int, list[dict]]:
    """Apply GPU/deploy labels to every node. Returns (gpu_nodes, patched,
    nfd_scanned, labels): nfd_scanned counts nodes our NFD worker has
    labelled, labels is each node's label set after this pass."""
    gpu_nodes = patched = scanned = 0
    views = []
    for node in client.list("v1", "Node"):
        if is_gpu_node(node):
            gpu_nodes += 1
        if nfd_scanned(node):
            scanned += 1
        patch = desired_labels(node, spec)
        view = dict(node["metadata"].get("labels") or {})
        if patch:
            client.patch("v1", "Node", node["metadata"]["name"], {"metadata": {"labels": patch}})
            patched += 1
            for k, v in patch.items():
                if v is None:
                    view.pop(k, None)
                else:
                    view[k] = v
        views.append(view)
    return gpu_nodes, patched, scanned, views


def nodes_selected(views: list[dict], selector: dict) -> int:
    return sum(1 for lb in views if all(lb.get(k) == v for k, v in selector.items()))
