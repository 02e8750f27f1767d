"""RBAC authorization for the simulated API server (testing the roles we ship).

The operator's chart grants its ServiceAccount a ClusterRole
(deploy/helm/amd-gpu-operator/templates/rbac.yaml) and the operator grants
each operand's ServiceAccount the rules its manifest names
(controller/manifests.py).  On a real cluster kube-apiserver enforces them;
a missing verb is a ``403 Forbidden`` the simulated cluster would never show.
:class:`Authorizer` evaluates the same objects the way the RBAC authorizer
does [EXT]: the requesting ServiceAccount's RoleBindings (in the request's
namespace) and ClusterRoleBindings, their roles' rules by API group,
resource (``pods``, ``pods/status``, ``*``), verb and ``resourceNames``.
The HTTP front end (kube/httpapi.py) maps bearer tokens to ServiceAccounts
and asks it before every request; ``SimCluster(rbac=True)`` runs the
operator and every operand under their own ServiceAccount.
"""

from __future__ import annotations

SA_PREFIX = "system:serviceaccount:"


def verb_of(method: str, name: str | None, watch: bool) -> str:
    if method == "GET":
        return "watch" if watch else ("get" if name else "list")
    return {"POST": "create", "PUT": "update", "PATCH": "patch", "DELETE": "delete"}[method]


def _rule_allows(rule: dict, verb: str, group: str, resource: str, name: str | None) -> bool:
    groups = rule.get("apiGroups") or []
    resources = rule.get("resources") or []
    verbs = rule.get("verbs") or []
    if "*" not in groups and group not in groups:
        return False
    if "*" not in verbs and verb not in verbs:
        return False
    base = resource.split("/", 1)[0]
    if "*" not in resources and resource not in resources and not (
            "/" in resource and f"{base}/*" in resources):
        return False
    names = rule.get("resourceNames") or []
    return not names or (name is not None and name in names)


class Authorizer:
    def __init__(self, api):
        self.api = api

    def _roles(self, ns: str | None, sa_ns: str, sa: str) -> list[dict]:
        def bound(b):
            return any(s.get("kind") == "ServiceAccount" and s.get("name") == sa
                       and s.get("namespace", "") == sa_ns for s in b.get("subjects") or [])

        out = []
        for b in self.api.list("rbac.authorization.k8s.io/v1", "ClusterRoleBinding"):
            if bound(b):
                out.append(("ClusterRole", b["roleRef"]["name"], None))
        if ns:
            for b in self.api.list("rbac.authorization.k8s.io/v1", "RoleBinding", ns):
                if bound(b):
                    out.append((b["roleRef"]["kind"], b["roleRef"]["name"], ns))
        roles = []
        for kind, name, rns in out:
            try:
                roles.append(self.api.get("rbac.authorization.k8s.io/v1", kind, name, rns if kind == "Role" else None))
            except Exception:  # noqa: BLE001 - a binding to a role that does not exist grants nothing
                continue
        return roles

    def allowed(self, user: str, verb: str, group: str, resource: str, ns: str | None, name: str | None) -> bool:
        if not user.startswith(SA_PREFIX):
            return False
        sa_ns, _, sa = user[len(SA_PREFIX):].partition(":")
        return any(_rule_allows(r, verb, group, resource, name) for role in self._roles(ns, sa_ns, sa)
                   for r in role.get("rules") or [])
