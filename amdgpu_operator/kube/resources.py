"""Kubernetes resource registry + object helpers (plain dict objects).

Only the small, standard API surface the operator needs (SURVEY.md §7.5 risk 2:
core/v1, apps/v1, rbac, node.k8s.io, apiextensions, batch, and the operator's
own CRD) so the same code talks to the in-memory API server in tests and to a
real apiserver in a cluster.
"""

from __future__ import annotations

import copy
import json
from ..utils.record import record


@record(frozen=True)
class ResourceType:
    group: str
    version: str
    kind: str
    plural: str
    namespaced: bool

    @property
    def api_version(self) -> str:
        return f"{self.group}/{self.version}" if self.group else self.version

    def path(self, namespace: str | None = None, name: str | None = None) -> str:
        base = f"/apis/{self.group}/{self.version}" if self.group else f"/api/{self.version}"
        if self.namespaced and namespace:
            base += f"/namespaces/{namespace}"
        base += f"/{self.plural}"
        if name:
            base += f"/{name}"
        return base


_TYPES = [
    ResourceType("", "v1", "Namespace", "namespaces", False),
    ResourceType("", "v1", "Node", "nodes", False),
    ResourceType("", "v1", "Pod", "pods", True),
    ResourceType("", "v1", "ConfigMap", "configmaps", True),
    ResourceType("", "v1", "Secret", "secrets", True),
    ResourceType("", "v1", "Service", "services", True),
    ResourceType("", "v1", "ServiceAccount", "serviceaccounts", True),
    ResourceType("", "v1", "Event", "events", True),
    ResourceType("apps", "v1", "DaemonSet", "daemonsets", True),
    ResourceType("apps", "v1", "Deployment", "deployments", True),
    ResourceType("batch", "v1", "Job", "jobs", True),
    ResourceType("coordination.k8s.io", "v1", "Lease", "leases", True),
    ResourceType("rbac.authorization.k8s.io", "v1", "ClusterRole", "clusterroles", False),
    ResourceType("rbac.authorization.k8s.io", "v1", "ClusterRoleBinding", "clusterrolebindings", False),
    ResourceType("rbac.authorization.k8s.io", "v1", "Role", "roles", True),
    ResourceType("rbac.authorization.k8s.io", "v1", "RoleBinding", "rolebindings", True),
    ResourceType("node.k8s.io", "v1", "RuntimeClass", "runtimeclasses", False),
    ResourceType("apiextensions.k8s.io", "v1", "CustomResourceDefinition", "customresourcedefinitions", False),
    ResourceType("monitoring.coreos.com", "v1", "ServiceMonitor", "servicemonitors", True),
    ResourceType("amd.com", "v1", "ClusterPolicy", "clusterpolicies", False),
    ResourceType("amd.com", "v1", "AMDGPUDriver", "amdgpudrivers", False),
    # Dynamic Resource Allocation, structured parameters (dra/)
    ResourceType("resource.k8s.io", "v1beta1", "ResourceSlice", "resourceslices", False),
    ResourceType("resource.k8s.io", "v1beta1", "DeviceClass", "deviceclasses", False),
    ResourceType("resource.k8s.io", "v1beta1", "ResourceClaim", "resourceclaims", True),
    ResourceType("resource.k8s.io", "v1beta1", "ResourceClaimTemplate", "resourceclaimtemplates", True),
]

REGISTRY: dict[tuple[str, str], ResourceType] = {(t.api_version, t.kind): t for t in _TYPES}
BY_PLURAL: dict[tuple[str, str, str], ResourceType] = {(t.group, t.version, t.plural): t for t in _TYPES}


def register(t: ResourceType) -> None:
    REGISTRY[(t.api_version, t.kind)] = t
    BY_PLURAL[(t.group, t.version, t.plural)] = t


def rtype(api_version: str, kind: str) -> ResourceType:
    try:
        return REGISTRY[(api_version, kind)]
    except KeyError:
        raise KeyError(f"unknown resource {api_version}/{kind}") from None


def rtype_of(obj: dict) -> ResourceType:
    return rtype(obj["apiVersion"], obj["kind"])


def meta(obj: dict) -> dict:
    return obj.setdefault("metadata", {})


def name_of(obj: dict) -> str:
    return obj.get("metadata", {}).get("name", "")


def ns_of(obj: dict) -> str | None:
    return obj.get("metadata", {}).get("namespace")


def labels_of(obj: dict) -> dict:
    return obj.get("metadata", {}).get("labels") or {}


def key_of(obj: dict) -> tuple:
    t = rtype_of(obj)
    return (t.api_version, t.kind, ns_of(obj) if t.namespaced else None, name_of(obj))


def new(api_version: str, kind: str, name: str, namespace: str | None = None, labels=None, **fields) -> dict:
    o = {"apiVersion": api_version, "kind": kind, "metadata": {"name": name}}
    if namespace:
        o["metadata"]["namespace"] = namespace
    if labels:
        o["metadata"]["labels"] = dict(labels)
    o.update(fields)
    return o


_ATOMS = (str, int, float, bool, type(None))


def deep(obj):
    """Deep copy of a JSON-shaped object (dict / list / scalars): what every
    API object is.  ~6x faster than copy.deepcopy (no memo table), and the
    fake API server copies on every create/get/list/watch event."""
    t = type(obj)
    if t is dict:
        return {k: deep(v) for k, v in obj.items()}
    if t is list:
        return [deep(v) for v in obj]
    if t in _ATOMS:
        return obj
    return copy.deepcopy(obj)  # anything else (tuples, custom objects): the general path


def spec_hash(obj: dict) -> str:
    """Hash of everything but status and server-managed metadata (drift detection)."""
    o = {k: v for k, v in obj.items() if k != "status"}
    m = dict(o.get("metadata", {}))
    for k in ("resourceVersion", "uid", "creationTimestamp", "generation", "managedFields"):
        m.pop(k, None)
    ann = dict(m.get("annotations") or {})
    ann.pop("amd.com/last-applied-hash", None)
    m["annotations"] = ann
    o["metadata"] = m
    import hashlib  # here: an operand's start-up does not need it (~4 ms of import)

    return hashlib.sha256(json.dumps(o, sort_keys=True, default=str).encode()).hexdigest()[:16]


def parse_selector(sel: str | dict | None) -> list[tuple[str, str, object]]:
    """``a=b,c!=d,e,!f,g in (x,y)`` (string) or ``{"a": "b"}`` (matchLabels)."""
    if not sel:
        return []
    if isinstance(sel, dict):
        reqs = [(k, "=", v) for k, v in (sel.get("matchLabels", sel) if "matchLabels" in sel else sel).items()
                if k != "matchExpressions"]
        for e in sel.get("matchExpressions", []) if "matchLabels" in sel or "matchExpressions" in sel else []:
            reqs.append((e["key"], e["operator"].lower(), tuple(e.get("values", []))))
        return reqs
    out = []
    parts, depth, cur = [], 0, ""
    for ch in sel:
        if ch == "(":
            depth += 1
        elif ch == ")":
            depth -= 1
        if ch == "," and depth == 0:
            parts.append(cur)
            cur = ""
        else:
            cur += ch
    parts.append(cur)
    for p in (x.strip() for x in parts):
        if not p:
            continue
        if " notin " in p:
            k, v = p.split(" notin ", 1)
            out.append((k.strip(), "notin", tuple(x.strip() for x in v.strip()[1:-1].split(","))))
        elif " in " in p:
            k, v = p.split(" in ", 1)
            out.append((k.strip(), "in", tuple(x.strip() for x in v.strip()[1:-1].split(","))))
        elif "!=" in p:
            k, v = p.split("!=", 1)
            out.append((k.strip(), "!=", v.strip()))
        elif "==" in p:
            k, v = p.split("==", 1)
            out.append((k.strip(), "=", v.strip()))
        elif "=" in p:
            k, v = p.split("=", 1)
            out.append((k.strip(), "=", v.strip()))
        elif p.startswith("!"):
            out.append((p[1:].strip(), "doesnotexist", None))
        else:
            out.append((p, "exists", None))
    return out


def matches(labels: dict, reqs) -> bool:
    for k, op, v in reqs:
        has = k in labels
        val = labels.get(k)
        if op == "=" and val != v:
            return False
        if op == "!=" and val == v:
            return False
        if op == "exists" and not has:
            return False
        if op == "doesnotexist" and has:
            return False
        if op == "in" and val not in v:
            return False
        if op == "notin" and has and val in v:
            return False
    return True


def merge_patch(target, patch):
    """RFC 7386 JSON merge patch."""
    if not isinstance(patch, dict):
        return deep(patch)
    if not isinstance(target, dict):
        target = {}
    out = dict(target)
    for k, v in patch.items():
        if v is None:
            out.pop(k, None)
        else:
            out[k] = merge_patch(out.get(k), v)
    return out


def node_selector_matches(node: dict, selector: dict | None, affinity: dict | None = None) -> bool:
    labels = labels_of(node)
    if selector and not all(labels.get(k) == v for k, v in selector.items()):
        return False
    terms = (((affinity or {}).get("nodeAffinity") or {}).get("requiredDuringSchedulingIgnoredDuringExecution")
             or {}).get("nodeSelectorTerms")
    if terms:
        ok_any = False
        for t in terms:
            reqs = [(e["key"], e["operator"].lower(), tuple(e.get("values", []))) for e in t.get("matchExpressions", [])]
            if matches(labels, reqs):
                ok_any = True
                break
        if not ok_any:
            return False
    return True


def condition(obj: dict, ctype: str) -> dict | None:
    for c in (obj.get("status") or {}).get("conditions") or []:
        if c.get("type") == ctype:
            return c
    return None


def set_condition(status: dict, ctype: str, value: bool, reason: str = "", message: str = "", now: str = "") -> bool:
    """Set a status condition; returns True when it changed."""
    conds = status.setdefault("conditions", [])
    sval = "True" if value else "False"
    for c in conds:
        if c.get("type") == ctype:
            if c.get("status") == sval and c.get("reason") == reason and c.get("message") == message:
                return False
            if c.get("status") != sval:
                c["lastTransitionTime"] = now
            c.update({"status": sval, "reason": reason, "message": message})
            return True
    conds.append({"type": ctype, "status": sval, "reason": reason, "message": message, "lastTransitionTime": now})
    return True
