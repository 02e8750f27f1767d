"""Object validation the simulated API server applies like kube-apiserver.

kube-apiserver rejects malformed objects with ``422 Invalid``; the in-memory
API server (kube/fakeapi.py) stored anything, so an object the operator
renders wrongly - a volume mount without its volume, a 16-character port
name, a label value over 63 characters, a DaemonSet whose selector does not
match its template - would pass every simulated bring-up and fail on the
reference's first real command (``helm install --wait``,
/root/reference/README.md:101-111).  This module checks the subset of the
apiserver's validation [EXT: k8s.io/apimachinery validation, pkg/apis/core
validation] that the operator's objects exercise; :func:`install` hooks it
into a FakeApiServer before every create and update.
"""

from __future__ import annotations

import re

_DNS_LABEL = re.compile(r"[a-z0-9]([-a-z0-9]*[a-z0-9])?")
_DNS_SUBDOMAIN = re.compile(r"[a-z0-9]([-a-z0-9]*[a-z0-9])?(\.[a-z0-9]([-a-z0-9]*[a-z0-9])?)*")
_LABEL_NAME = re.compile(r"([A-Za-z0-9][-A-Za-z0-9_.]*)?[A-Za-z0-9]")
_ENV_NAME = re.compile(r"[-._a-zA-Z][-._a-zA-Z0-9]*")
_SVC_NAME = re.compile(r"[a-z0-9]([-a-z0-9]*[a-z0-9])?")
HOSTPATH_TYPES = {"", "DirectoryOrCreate", "Directory", "FileOrCreate", "File", "Socket", "CharDevice", "BlockDevice"}
EFFECTS = {"", "NoSchedule", "PreferNoSchedule", "NoExecute"}
# kinds whose names are DNS-1123 labels rather than subdomains
_LABEL_NAMED = {"Namespace", "Service"}


def _dns_label(s: str) -> bool:
    return isinstance(s, str) and len(s) <= 63 and bool(_DNS_LABEL.fullmatch(s))


def _dns_subdomain(s: str) -> bool:
    return isinstance(s, str) and len(s) <= 253 and bool(_DNS_SUBDOMAIN.fullmatch(s))


def _qualified_name(key: str) -> bool:
    prefix, _, name = key.rpartition("/")
    if prefix and not _dns_subdomain(prefix):
        return False
    return 0 < len(name) <= 63 and bool(_LABEL_NAME.fullmatch(name))


def _label_value(v) -> bool:
    return isinstance(v, str) and len(v) <= 63 and (v == "" or bool(_LABEL_NAME.fullmatch(v)))


def _port_name(s: str) -> bool:
    return (len(s) <= 15 and bool(_SVC_NAME.fullmatch(s)) and "--" not in s and re.search("[a-z]", s) is not None)


def _meta(obj: dict, errs: list[str]) -> None:
    md = obj.get("metadata") or {}
    name = md.get("name", "")
    kind = obj.get("kind", "")
    if not (_dns_label(name) if kind in _LABEL_NAMED else _dns_subdomain(name)):
        errs.append(f"metadata.name {name!r}: not a valid {'DNS-1123 label' if kind in _LABEL_NAMED else 'name'}")
    for k, v in (md.get("labels") or {}).items():
        if not _qualified_name(k):
            errs.append(f"metadata.labels: key {k!r} is not a qualified name")
        if not _label_value(v):
            errs.append(f"metadata.labels[{k}]: value {v!r} is not a valid label value")
    for k in (md.get("annotations") or {}):
        if not _qualified_name(k):
            errs.append(f"metadata.annotations: key {k!r} is not a qualified name")
    size = sum(len(k) + len(str(v)) for k, v in (md.get("annotations") or {}).items())
    if size > 256 * 1024:
        errs.append(f"metadata.annotations: {size} bytes, more than 256 KiB")


def _probe(p: dict | None, path: str, errs: list[str]) -> None:
    if p is None:
        return
    handlers = [h for h in ("exec", "httpGet", "tcpSocket", "grpc") if h in p]
    if len(handlers) != 1:
        errs.append(f"{path}: exactly one handler needed, got {handlers}")


def pod_spec(spec: dict, path: str, errs: list[str], in_template: bool = False, controller: str = "") -> None:
    ctrs = spec.get("containers") or []
    if not ctrs:
        errs.append(f"{path}.containers: at least one container required")
    volumes = {}
    for i, v in enumerate(spec.get("volumes") or []):
        n = v.get("name", "")
        if not _dns_label(n):
            errs.append(f"{path}.volumes[{i}].name {n!r}: not a DNS-1123 label")
        if n in volumes:
            errs.append(f"{path}.volumes[{i}].name {n!r}: duplicate")
        volumes[n] = v
        hp = v.get("hostPath")
        if hp is not None:
            if not str(hp.get("path", "")).startswith("/"):
                errs.append(f"{path}.volumes[{i}].hostPath.path must be absolute")
            if hp.get("type", "") not in HOSTPATH_TYPES:
                errs.append(f"{path}.volumes[{i}].hostPath.type {hp.get('type')!r} not supported")
    claims = set()
    for i, rc in enumerate(spec.get("resourceClaims") or []):
        n = rc.get("name", "")
        if not _dns_label(n):
            errs.append(f"{path}.resourceClaims[{i}].name {n!r}")
        elif n in claims:
            errs.append(f"{path}.resourceClaims[{i}].name {n!r}: duplicate")
        claims.add(n)
        if bool(rc.get("resourceClaimName")) == bool(rc.get("resourceClaimTemplateName")):
            errs.append(f"{path}.resourceClaims[{i}]: exactly one of resourceClaimName, "
                        "resourceClaimTemplateName is required")
    names = set()
    for group in ("initContainers", "containers"):
        for i, c in enumerate(spec.get(group) or []):
            cp = f"{path}.{group}[{i}]"
            n = c.get("name", "")
            if not _dns_label(n):
                errs.append(f"{cp}.name {n!r}: not a DNS-1123 label")
            if n in names:
                errs.append(f"{cp}.name {n!r}: duplicate container name")
            names.add(n)
            if not c.get("image"):
                errs.append(f"{cp}.image: required")
            for j, m in enumerate(c.get("volumeMounts") or []):
                if m.get("name") not in volumes:
                    errs.append(f"{cp}.volumeMounts[{j}].name {m.get('name')!r}: no volume of that name")
                if not str(m.get("mountPath", "")).startswith("/"):
                    errs.append(f"{cp}.volumeMounts[{j}].mountPath must be absolute")
                if m.get("mountPropagation") not in (None, "None", "HostToContainer", "Bidirectional"):
                    errs.append(f"{cp}.volumeMounts[{j}].mountPropagation {m.get('mountPropagation')!r}")
                if m.get("mountPropagation") == "Bidirectional" and not (c.get("securityContext") or {}).get("privileged"):
                    errs.append(f"{cp}.volumeMounts[{j}]: Bidirectional propagation needs a privileged container")
            seen_ports = set()
            for j, p in enumerate(c.get("ports") or []):
                if not 0 < int(p.get("containerPort", 0)) < 65536:
                    errs.append(f"{cp}.ports[{j}].containerPort {p.get('containerPort')!r} out of range")
                pn = p.get("name")
                if pn is not None and not _port_name(pn):
                    errs.append(f"{cp}.ports[{j}].name {pn!r}: not a valid port name (<= 15 chars, IANA_SVC_NAME)")
                if pn is not None and pn in seen_ports:
                    errs.append(f"{cp}.ports[{j}].name {pn!r}: duplicate")
                seen_ports.add(pn)
            for j, e in enumerate(c.get("env") or []):
                en = e.get("name", "")
                if not _ENV_NAME.fullmatch(en):
                    errs.append(f"{cp}.env[{j}].name {en!r}: not a valid environment variable name")
                if "value" in e and "valueFrom" in e:
                    errs.append(f"{cp}.env[{j}]: value and valueFrom are exclusive")
            res = c.get("resources") or {}
            for rname, lim in (res.get("limits") or {}).items():
                if "/" in rname and not rname.startswith(("kubernetes.io/", "requests.")):  # an extended resource
                    req = (res.get("requests") or {}).get(rname, lim)
                    if str(req) != str(lim):
                        errs.append(f"{cp}.resources: extended resource {rname} must request what it limits "
                                    f"({req} != {lim})")
                    if not str(lim).isdigit():
                        errs.append(f"{cp}.resources.limits[{rname}] {lim!r}: must be a whole number")
            for j, rc in enumerate(((c.get("resources") or {}).get("claims")) or []):
                if rc.get("name") not in claims:
                    errs.append(f"{cp}.resources.claims[{j}] {rc.get('name')!r}: not in spec.resourceClaims")
            if group == "containers":
                for pr in ("readinessProbe", "livenessProbe", "startupProbe"):
                    _probe(c.get(pr), f"{cp}.{pr}", errs)
            elif any(c.get(pr) for pr in ("readinessProbe", "livenessProbe")):
                errs.append(f"{cp}: init containers take no readiness/liveness probe")
    for i, t in enumerate(spec.get("tolerations") or []):
        op = t.get("operator", "Equal")
        if op not in ("Exists", "Equal"):
            errs.append(f"{path}.tolerations[{i}].operator {op!r}")
        if op == "Exists" and t.get("value"):
            errs.append(f"{path}.tolerations[{i}]: operator Exists takes no value")
        if t.get("effect", "") not in EFFECTS:
            errs.append(f"{path}.tolerations[{i}].effect {t.get('effect')!r}")
    if controller in ("DaemonSet", "Deployment") and spec.get("restartPolicy", "Always") != "Always":
        errs.append(f"{path}.restartPolicy: {controller} pods must restart Always")
    for k, v in (spec.get("nodeSelector") or {}).items():
        if not _qualified_name(k) or not _label_value(v):
            errs.append(f"{path}.nodeSelector: {k}={v!r} is not a valid label")


def claim_spec(spec: dict, path: str, errs: list[str]) -> None:
    """resource.k8s.io/v1beta1 ResourceClaimSpec: named requests of one
    DeviceClass, ExactCount (count >= 1) or All, CEL selectors, and
    constraints whose matchAttribute is a fully qualified attribute
    (``<domain>/<name>``) over requests that exist."""
    devices = spec.get("devices") or {}
    reqs = devices.get("requests") or []
    names = set()
    for i, r in enumerate(reqs):
        rp = f"{path}.devices.requests[{i}]"
        n = r.get("name", "")
        if not _dns_label(n):
            errs.append(f"{rp}.name {n!r}")
        elif n in names:
            errs.append(f"{rp}.name {n!r}: duplicate")
        names.add(n)
        if not r.get("deviceClassName"):
            errs.append(f"{rp}.deviceClassName: required")
        mode = r.get("allocationMode", "ExactCount")
        if mode not in ("ExactCount", "All"):
            errs.append(f"{rp}.allocationMode {mode!r}: ExactCount or All")
        elif mode == "ExactCount" and int(r.get("count", 1)) < 1:
            errs.append(f"{rp}.count {r.get('count')!r}: must be at least 1")
        elif mode == "All" and "count" in r:
            errs.append(f"{rp}.count: must not be set with allocationMode All")
        for j, sel in enumerate(r.get("selectors") or []):
            if not ((sel.get("cel") or {}).get("expression") or "").strip():
                errs.append(f"{rp}.selectors[{j}].cel.expression: required")
    for i, c in enumerate(devices.get("constraints") or []):
        cp = f"{path}.devices.constraints[{i}]"
        attr = c.get("matchAttribute", "")
        dom, _, nm = str(attr).partition("/")
        if not (dom and nm and _dns_subdomain(dom)):
            errs.append(f"{cp}.matchAttribute {attr!r}: a fully qualified <domain>/<name>")
        for rn in c.get("requests") or []:
            if rn not in names:
                errs.append(f"{cp}.requests: {rn!r} is not a request of this claim")


def validate(obj: dict) -> list[str]:
    """The apiserver's ``Invalid`` causes for ``obj`` (empty: valid)."""
    errs: list[str] = []
    kind = obj.get("kind", "")
    _meta(obj, errs)
    spec = obj.get("spec") or {}
    if kind == "Pod":
        pod_spec(spec, "spec", errs)
    elif kind in ("DaemonSet", "Deployment", "Job"):
        tmpl = spec.get("template") or {}
        pod_spec(tmpl.get("spec") or {}, "spec.template.spec", errs, True, kind)
        tl = (tmpl.get("metadata") or {}).get("labels") or {}
        for k, v in tl.items():
            if not _qualified_name(k) or not _label_value(v):
                errs.append(f"spec.template.metadata.labels: {k}={v!r} is not a valid label")
        if kind != "Job":
            sel = ((spec.get("selector") or {}).get("matchLabels")) or {}
            if not sel:
                errs.append("spec.selector: required")
            elif any(tl.get(k) != v for k, v in sel.items()):
                errs.append(f"spec.template.metadata.labels: do not match spec.selector {sel}")
    elif kind in ("ResourceClaim", "ResourceClaimTemplate"):
        claim_spec(spec.get("spec") or {} if kind == "ResourceClaimTemplate" else spec,
                   "spec.spec" if kind == "ResourceClaimTemplate" else "spec", errs)
    elif kind == "Service":
        ports = spec.get("ports") or []
        pnames = [p.get("name") for p in ports]
        if len(ports) > 1 and (None in pnames or len(set(pnames)) != len(pnames)):
            errs.append("spec.ports: several ports need distinct names")
        for i, p in enumerate(ports):
            if not 0 < int(p.get("port", 0)) < 65536:
                errs.append(f"spec.ports[{i}].port {p.get('port')!r} out of range")
            if p.get("name") and not _port_name(p["name"]) and not _dns_label(p["name"]):
                errs.append(f"spec.ports[{i}].name {p['name']!r}")
    elif kind in ("ClusterRole", "Role"):
        for i, r in enumerate(obj.get("rules") or []):
            if not r.get("verbs"):
                errs.append(f"rules[{i}].verbs: required")
    elif kind in ("ClusterRoleBinding", "RoleBinding"):
        if not (obj.get("roleRef") or {}).get("name"):
            errs.append("roleRef.name: required")
        for i, s in enumerate(obj.get("subjects") or []):
            if s.get("kind") == "ServiceAccount" and not s.get("namespace") and kind == "ClusterRoleBinding":
                errs.append(f"subjects[{i}].namespace: required for a ServiceAccount")
    return errs


def schema_errors(value, schema: dict, path: str = "") -> list[str]:
    """A CR against its CRD's structural openAPIV3Schema, as the apiserver
    checks it: types, enums, required, nested properties and items; fields
    the schema does not know are errors too (the apiserver would prune them
    silently - the operator would never see the value it was given)."""
    errs: list[str] = []
    t = schema.get("type")
    if value is None:
        return [] if schema.get("nullable") else [f"{path or '.'}: null"]
    ok = {"object": isinstance(value, dict), "array": isinstance(value, list), "string": isinstance(value, str),
          "boolean": isinstance(value, bool), "integer": isinstance(value, int) and not isinstance(value, bool),
          "number": isinstance(value, (int, float)) and not isinstance(value, bool)}.get(t, True)
    if schema.get("x-kubernetes-int-or-string"):
        ok = isinstance(value, (int, str)) and not isinstance(value, bool)
    if not ok:
        return [f"{path or '.'}: {type(value).__name__} where the schema has {t}"]
    if "enum" in schema and value not in schema["enum"]:
        errs.append(f"{path}: {value!r} not in {schema['enum']}")
    if isinstance(value, dict) and not schema.get("x-kubernetes-preserve-unknown-fields"):
        props = schema.get("properties")
        addl = schema.get("additionalProperties")
        for k in schema.get("required") or []:
            if k not in value:
                errs.append(f"{path}.{k}: required")
        for k, v in value.items():
            if props is not None and k in props:
                errs += schema_errors(v, props[k], f"{path}.{k}")
            elif isinstance(addl, dict):
                errs += schema_errors(v, addl, f"{path}.{k}")
            elif props is not None or addl is False:
                errs.append(f"{path}.{k}: unknown field")
    if isinstance(value, list) and isinstance(schema.get("items"), dict):
        for i, v in enumerate(value):
            errs += schema_errors(v, schema["items"], f"{path}[{i}]")
    return errs


def install(api) -> None:
    """Validate every create and update of ``api`` (a FakeApiServer)."""
    api.validators.append(validate)
