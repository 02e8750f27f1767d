"""The cluster side of DRA for tests and the simulated cluster.

* :class:`FakeDraKubelet` - the kubelet's plugin watcher and DRA manager:
  finds registration sockets in ``plugins_registry``, calls ``GetInfo`` and
  ``NotifyRegistrationStatus``, then ``NodePrepareResources`` /
  ``NodeUnprepareResources`` on the endpoint the plugin named.
* :func:`allocate` - the scheduler's structured-parameters allocator for a
  ResourceClaim: requests by DeviceClass with ``ExactCount`` (or ``All``),
  CEL selectors in the subset below, ``matchAttribute`` constraints; writes
  ``status.allocation``.

CEL subset (what the operator's docs and tests use; anything else raises):
``device.driver == "..."``, ``device.attributes["<domain>"].<name> <op>
<literal>`` with ``== != < <= > >=`` on strings, ints and booleans, and
``device.capacity["<domain>"].<name>.compareTo(quantity("<q>")) <op> 0``,
joined with ``&&``.
"""

from __future__ import annotations

import itertools
import os
import re

from ..dra import api
from ..rpc import wire

_Q = {"Ki": 1 << 10, "Mi": 1 << 20, "Gi": 1 << 30, "Ti": 1 << 40, "k": 10**3, "M": 10**6, "G": 10**9, "T": 10**12}


def quantity(q: str) -> int:
    m = re.fullmatch(r"(\d+)([KMGT]i|[kMGT])?", q.strip())
    if not m:
        raise ValueError(f"quantity {q!r}")
    return int(m.group(1)) * _Q.get(m.group(2) or "", 1)


_OPS = {"==": lambda a, b: a == b, "!=": lambda a, b: a != b, "<": lambda a, b: a < b, "<=": lambda a, b: a <= b,
        ">": lambda a, b: a > b, ">=": lambda a, b: a >= b}
_ATTR = re.compile(r'device\.attributes\["([^"]+)"\]\.(\w+)\s*(==|!=|<=|>=|<|>)\s*(.+)')
_CAP = re.compile(r'device\.capacity\["([^"]+)"\]\.(\w+)\.compareTo\(quantity\("([^"]+)"\)\)\s*(==|!=|<=|>=|<|>)\s*0')
_DRV = re.compile(r'device\.driver\s*(==|!=)\s*"([^"]*)"')


def _literal(s: str):
    s = s.strip()
    if s.startswith('"') and s.endswith('"'):
        return s[1:-1]
    if s in ("true", "false"):
        return s == "true"
    return int(s)


def _attr_value(v: dict):
    for k in ("string", "int", "bool", "version"):
        if k in v:
            return v[k]
    return None


def cel_match(expr: str, driver: str, device: dict) -> bool:
    basic = device.get("basic") or {}
    for term in (t.strip() for t in expr.split("&&")):
        if m := _DRV.fullmatch(term):
            ok = (driver == m.group(2)) == (m.group(1) == "==")
        elif m := _ATTR.fullmatch(term):
            dom, name, op, lit = m.groups()
            raw = (basic.get("attributes") or {}).get(name if dom == driver else f"{dom}/{name}")
            val = _attr_value(raw) if raw else None
            ok = val is not None and _OPS[op](val, _literal(lit))
        elif m := _CAP.fullmatch(term):
            dom, name, q, op = m.groups()
            raw = (basic.get("capacity") or {}).get(name if dom == driver else f"{dom}/{name}")
            ok = raw is not None and _OPS[op]((quantity(raw["value"]) > quantity(q)) - (quantity(raw["value"]) < quantity(q)), 0)
        else:
            raise ValueError(f"CEL expression outside the supported subset: {term!r}")
        if not ok:
            return False
    return True


def _candidates(client, node: str | None) -> list[tuple[str, str, dict]]:
    out = []
    for s in client.list("resource.k8s.io/v1beta1", "ResourceSlice"):
        sp = s.get("spec") or {}
        if node and sp.get("nodeName") != node:
            continue
        for d in sp.get("devices") or []:
            out.append((sp["driver"], sp["pool"]["name"], d))
    return out


def allocate(client, claim: dict, node: str | None = None, in_use: set | None = None) -> dict:
    """Allocate ``claim`` from the published slices (``node``: only that
    node's), skipping devices in ``in_use`` (``(driver, pool, device)``) and
    those other allocated claims hold; writes and returns the claim."""
    busy = set(in_use or ())
    for other in client.list("resource.k8s.io/v1beta1", "ResourceClaim"):
        for r in ((((other.get("status") or {}).get("allocation") or {}).get("devices") or {}).get("results") or []):
            busy.add((r["driver"], r["pool"], r["device"]))
    classes = {c["metadata"]["name"]: c for c in client.list("resource.k8s.io/v1beta1", "DeviceClass")}
    devs = [c for c in _candidates(client, node) if (c[0], c[1], c[2]["name"]) not in busy]
    spec = (claim.get("spec") or {}).get("devices") or {}
    results = []
    taken: set = set()
    for req in spec.get("requests") or []:
        cls = classes.get(req.get("deviceClassName", ""))
        if cls is None:
            raise ValueError(f"request {req.get('name')}: no DeviceClass {req.get('deviceClassName')!r}")
        sels = [s["cel"]["expression"] for s in (cls.get("spec") or {}).get("selectors") or []] + \
               [s["cel"]["expression"] for s in req.get("selectors") or []]
        fit = [c for c in devs if (c[0], c[1], c[2]["name"]) not in taken and all(cel_match(e, c[0], c[2]) for e in sels)]
        want = len(fit) if req.get("allocationMode") == "All" else int(req.get("count", 1))
        pick = _constrained(fit, want, spec.get("constraints") or [], req.get("name"))
        if pick is None:
            raise ValueError(f"request {req.get('name')}: {want} device(s) needed, no fitting set among {len(fit)}")
        for drv, pool, d in pick:
            taken.add((drv, pool, d["name"]))
            results.append({"request": req.get("name"), "driver": drv, "pool": pool, "device": d["name"]})
    claim.setdefault("status", {})["allocation"] = {"devices": {"results": results}}
    if node:
        claim["status"]["allocation"]["nodeSelector"] = {"nodeSelectorTerms": [{"matchFields": [
            {"key": "metadata.name", "operator": "In", "values": [node]}]}]}
    return client.update_status(claim)


def _constrained(fit, want: int, constraints: list[dict], request: str | None):
    """The first ``want`` devices (in slice order) satisfying every
    ``matchAttribute`` constraint that names this request (or all)."""
    keys = [c["matchAttribute"] for c in constraints
            if "matchAttribute" in c and (not c.get("requests") or request in c["requests"])]
    if not keys:
        return fit[:want] if len(fit) >= want else None

    def attr(c, key):
        dom, _, name = key.rpartition("/")
        raw = ((c[2].get("basic") or {}).get("attributes") or {}).get(name if dom == c[0] else key)
        return _attr_value(raw) if raw else None

    groups: dict = {}
    for c in fit:
        vals = tuple(attr(c, k) for k in keys)
        if None not in vals:
            groups.setdefault(vals, []).append(c)
    for members in groups.values():
        if len(members) >= want:
            return next(itertools.combinations(members, want))
    return None


class FakeDraKubelet:
    """The kubelet's DRA side on one node (plugin watcher + DRA manager)."""

    def __init__(self, kubelet_dir: str):
        self.registry = os.path.join(kubelet_dir, "plugins_registry")
        self.plugins: dict[str, str] = {}  # driver name -> endpoint

    def discover(self, timeout: float = 5.0) -> dict[str, str]:
        """Register every plugin whose registration socket is present."""
        try:
            socks = [os.path.join(self.registry, n) for n in sorted(os.listdir(self.registry)) if n.endswith(".sock")]
        except FileNotFoundError:
            socks = []
        for s in socks:
            with wire.Channel(s) as ch:
                info = self._call(ch, api.REGISTRATION_SERVICE, api.REGISTRATION_METHODS, "GetInfo",
                                  api.reg["InfoRequest"](), timeout)
                ok = info.type == api.PLUGIN_TYPE and api.DRA_VERSION in info.supported_versions
                err = "" if ok else f"unsupported plugin type {info.type} / versions {list(info.supported_versions)}"
                self._call(ch, api.REGISTRATION_SERVICE, api.REGISTRATION_METHODS, "NotifyRegistrationStatus",
                           api.reg["RegistrationStatus"](plugin_registered=ok, error=err), timeout)
                if ok:
                    self.plugins[info.name] = info.endpoint
        return dict(self.plugins)

    @staticmethod
    def _call(ch, service, methods, name, req, timeout):
        i, o, _ = methods[name]
        return ch.unary_unary(api.method_path(service, name), request_serializer=i.SerializeToString,
                              response_deserializer=o.FromString)(req, timeout=timeout, wait_for_ready=True)

    def prepare(self, driver: str, claims: list[dict], timeout: float = 10.0) -> dict[str, object]:
        """``claims``: ResourceClaim objects; returns uid -> NodePrepareResourceResponse."""
        req = api.dra["NodePrepareResourcesRequest"]()
        for c in claims:
            m = c["metadata"]
            req.claims.add(namespace=m.get("namespace", ""), uid=m["uid"], name=m["name"])
        with wire.Channel(self.plugins[driver]) as ch:
            resp = self._call(ch, api.DRA_SERVICE, api.DRA_METHODS, "NodePrepareResources", req, timeout)
        return {e.key: e.value for e in resp.claims}

    def unprepare(self, driver: str, claims: list[dict], timeout: float = 10.0) -> dict[str, object]:
        req = api.dra["NodeUnprepareResourcesRequest"]()
        for c in claims:
            m = c["metadata"]
            req.claims.add(namespace=m.get("namespace", ""), uid=m["uid"], name=m["name"])
        with wire.Channel(self.plugins[driver]) as ch:
            resp = self._call(ch, api.DRA_SERVICE, api.DRA_METHODS, "NodeUnprepareResources", req, timeout)
        return {e.key: e.value for e in resp.claims}
