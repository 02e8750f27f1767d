"""``amdgpu-operator must-gather``: one archive with what a support case needs.

Reference parity: the reference's troubleshooting is manual - ``kubectl
describe pod`` / ``kubectl logs -c nvidia-driver-ctr`` and "check that the
worker really has a GPU" (/root/reference/README.md:172-187).  This command
collects the same evidence in one go, plus the MI355X node state, into a
``.tar.gz``:

* cluster: ClusterPolicy / AMDGPUDriver objects (spec + status), GPU nodes
  (labels, allocatable, conditions, upgrade state), operand DaemonSets and
  pods (phase, container readiness, restarts), namespace events;
* node (when run on a GPU node, ``--node-root``): KFD topology (GPUs, arch,
  HBM, xGMI links, partitions), the amdgpu module version, the validator's
  ready files (per-step results and durations), live amd-smi metrics;
* ``summary.json``: policy state, GPU nodes not validated, nodes mid driver
  upgrade, operand pods not ready - the first thing to read.
"""

from __future__ import annotations

import io
import json
import os
import tarfile
import time

from ..kube.errors import ApiError


def _list(client, api_version: str, kind: str, namespace: str | None = None) -> list[dict]:
    try:
        return client.list(api_version, kind, namespace)
    except ApiError:
        return []  # kind not served (CRD absent) or not permitted


def _node_view(n: dict) -> dict:
    st = n.get("status") or {}
    return {"name": n["metadata"]["name"], "labels": n["metadata"].get("labels") or {},
            "annotations": {k: v for k, v in (n["metadata"].get("annotations") or {}).items() if k.startswith("amd.com")},
            "unschedulable": bool((n.get("spec") or {}).get("unschedulable")),
            "capacity": st.get("capacity") or {}, "allocatable": st.get("allocatable") or {},
            "conditions": st.get("conditions") or []}


def _pod_view(p: dict) -> dict:
    st = p.get("status") or {}
    return {"name": p["metadata"]["name"], "node": (p.get("spec") or {}).get("nodeName"), "phase": st.get("phase"),
            "reason": st.get("reason"), "message": st.get("message"),
            "containers": [{"name": c.get("name"), "ready": c.get("ready"), "restarts": c.get("restartCount")}
                           for c in st.get("containerStatuses") or []]}


def gather_cluster(client, namespace: str) -> dict:
    from .. import API_GROUP, API_VERSION

    cr_api = f"{API_GROUP}/{API_VERSION}"
    return {
        "clusterpolicies": _list(client, cr_api, "ClusterPolicy"),
        "amdgpudrivers": _list(client, cr_api, "AMDGPUDriver"),
        "nodes": [_node_view(n) for n in _list(client, "v1", "Node")],
        "daemonsets": [{"name": d["metadata"]["name"], "status": d.get("status") or {},
                        "updateStrategy": (d.get("spec") or {}).get("updateStrategy")}
                       for d in _list(client, "apps/v1", "DaemonSet", namespace)],
        "pods": [_pod_view(p) for p in _list(client, "v1", "Pod", namespace)],
        "events": _list(client, "v1", "Event", namespace),
    }


def gather_node(root: str = "/", validations_dir: str | None = None) -> dict:
    from ..discovery import topology as T

    out: dict = {"root": root}
    try:
        out["gpus"] = [g.as_dict() for g in T.enumerate_gpus(root)]
        out["xgmi_links"] = sum(1 for link in T.links(root) if link.is_xgmi)
        out["probe"] = dict(zip(("ok", "message"), T.probe(root)))
    except Exception as e:  # noqa: BLE001 - no KFD on this host
        out["topology_error"] = str(e)
    try:
        with open(os.path.join(root, "sys/module/amdgpu/version")) as f:
            out["amdgpu_version"] = f.read().strip()
    except OSError:
        out["amdgpu_version"] = None
    if validations_dir and os.path.isdir(validations_dir):
        ready = {}
        for fn in sorted(os.listdir(validations_dir)):
            p = os.path.join(validations_dir, fn)
            if os.path.isfile(p):
                try:
                    with open(p) as f:
                        ready[fn] = json.load(f)
                except (OSError, ValueError):
                    ready[fn] = "unreadable"
        out["validations"] = ready
    try:
        with T.Smi() as smi:
            out["metrics"] = [{"index": m.index, "bdf": m.bdf, **m.values} for m in smi.collect()]
    except Exception as e:  # noqa: BLE001 - amd-smi unavailable (CPU host, container without it)
        out["metrics_error"] = str(e)
    return out


def summarize(cluster: dict) -> dict:
    from ..wellknown import DONE, UPGRADE_STATE_LABEL as STATE_LABEL
    from ..validator.validate import VALIDATED_LABEL

    gpu_nodes = [n for n in cluster["nodes"] if n["labels"].get("amd.com/gpu.present") == "true"]
    policies = cluster["clusterpolicies"]
    return {
        "policy_state": [(p["metadata"]["name"], (p.get("status") or {}).get("state")) for p in policies],
        "gpu_nodes": len(gpu_nodes),
        "not_validated": [n["name"] for n in gpu_nodes if n["labels"].get(VALIDATED_LABEL) != "true"],
        "driver_upgrades": {n["name"]: n["labels"][STATE_LABEL] for n in gpu_nodes
                            if n["labels"].get(STATE_LABEL, DONE) != DONE},
        "pods_not_ready": [p["name"] for p in cluster["pods"]
                           if p["phase"] != "Succeeded" and not (p["containers"] and all(c["ready"] for c in p["containers"]))],
        "allocatable": {n["name"]: {k: v for k, v in n["allocatable"].items() if k.startswith("amd.com/gpu")}
                        for n in gpu_nodes},
    }


def must_gather(client, namespace: str, out_path: str, node_root: str | None = None,
                validations_dir: str | None = None) -> dict:
    """Write ``out_path`` (.tar.gz) and return the summary."""
    stamp = time.strftime("%Y%m%dT%H%M%SZ", time.gmtime())
    base = f"amdgpu-must-gather-{stamp}"
    docs: dict[str, object] = {}
    cluster = gather_cluster(client, namespace) if client is not None else None
    if cluster is not None:
        docs.update({f"cluster/{k}.json": v for k, v in cluster.items()})
        summary = summarize(cluster)
    else:
        summary = {}
    if node_root is not None:
        docs["node/node.json"] = gather_node(node_root, validations_dir)
    summary["collected"] = sorted(docs)
    docs["summary.json"] = summary
    os.makedirs(os.path.dirname(os.path.abspath(out_path)) or ".", exist_ok=True)
    with tarfile.open(out_path, "w:gz") as tar:
        for name, obj in docs.items():
            data = json.dumps(obj, indent=1, default=str).encode()
            info = tarfile.TarInfo(f"{base}/{name}")
            info.size = len(data)
            info.mtime = int(time.time())
            tar.addfile(info, io.BytesIO(data))
    return summary
