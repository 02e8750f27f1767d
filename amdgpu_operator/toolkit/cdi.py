"""CDI device resolution, as a container runtime does it.

A runtime with CDI enabled (containerd ``enable_cdi``, CRI-O, the toolkit's
drop-ins: toolkit/install.py) turns each fully-qualified device name a
container is given (``vendor.com/class=name``: the device plugin's CDI
devices, the DRA driver's per-claim devices, dra/driver.py) into edits of
the container's OCI spec.  The rules of the container-device-interface
library (the CDI specification, v0.6):

* every spec file in the spec directories is loaded; a device is found by
  its ``kind`` (``vendor/class``) and ``name``; an unknown name fails the
  container's creation ("unresolvable CDI devices");
* a device's own ``containerEdits`` apply, and its spec's top-level
  ``containerEdits`` apply once for every spec that contributed a device;
* device nodes and mounts are merged by path; environment variables are set
  by name, the later edit replacing the earlier.

The last rule is why two claims of one container must not set the same
variable to different values: the runtime keeps one of them silently.
:func:`resolve` reports such a collision (``conflicts``) and, with
``strict``, fails on it - the simulated kubelet (testing/simcluster.py) runs
strict, so a spec set that would lose a value on a cluster fails its tests.
"""

from __future__ import annotations

import json
import os
from dataclasses import dataclass, field


class CDIError(RuntimeError):
    pass


@dataclass
class Edits:
    device_nodes: list[dict] = field(default_factory=list)
    env: dict[str, str] = field(default_factory=dict)
    mounts: list[dict] = field(default_factory=list)
    hooks: list[dict] = field(default_factory=list)
    conflicts: list[str] = field(default_factory=list)  # "NAME: a -> b" (a later edit replaced a value)
    devices: list[str] = field(default_factory=list)    # the qualified names applied, in order

    def env_list(self) -> list[str]:
        return [f"{k}={v}" for k, v in self.env.items()]


def load_specs(dirs: list[str]) -> dict[str, dict]:
    """kind -> {"spec": top-level edits, "devices": {name: edits}, "path": file}.
    A device name defined by two spec files of one kind is an error, as in
    the CDI registry."""
    out: dict[str, dict] = {}
    for d in dirs:
        try:
            names = sorted(os.listdir(d))
        except OSError:
            continue
        for n in names:
            if not n.endswith((".json", ".yaml", ".yml")) or n.startswith("."):
                continue
            p = os.path.join(d, n)
            try:
                with open(p) as f:
                    if n.endswith(".json"):
                        spec = json.load(f)
                    else:
                        import yaml

                        spec = yaml.safe_load(f)
            except (OSError, ValueError):
                continue
            if not isinstance(spec, dict) or "kind" not in spec:
                continue
            kind = spec["kind"]
            ent = out.setdefault(kind, {"devices": {}, "specs": {}})
            ent["specs"][p] = spec.get("containerEdits") or {}
            for dev in spec.get("devices") or []:
                name = dev.get("name")
                if name in ent["devices"]:
                    raise CDIError(f"CDI device {kind}={name} defined in {ent['devices'][name][0]} and {p}")
                ent["devices"][name] = (p, dev.get("containerEdits") or {})
    return out


def _merge(into: Edits, edits: dict, source: str) -> None:
    for dn in edits.get("deviceNodes") or []:
        if all(x.get("path") != dn.get("path") for x in into.device_nodes):
            into.device_nodes.append(dict(dn))
    for m in edits.get("mounts") or []:
        if all(x.get("containerPath") != m.get("containerPath") for x in into.mounts):
            into.mounts.append(dict(m))
    for h in edits.get("hooks") or []:
        into.hooks.append(dict(h))
    for e in edits.get("env") or []:
        k, _, v = e.partition("=")
        if k in into.env and into.env[k] != v:
            into.conflicts.append(f"{k}: {into.env[k]!r} -> {v!r} ({source})")
        into.env[k] = v


def resolve(dirs: list[str] | str, qualified: list[str], strict: bool = False) -> Edits:
    """The OCI edits for a container given ``qualified`` CDI device names."""
    if isinstance(dirs, str):
        dirs = [dirs]
    specs = load_specs(dirs)
    out = Edits()
    applied_specs: set[str] = set()
    missing = []
    for q in qualified:
        kind, sep, name = q.partition("=")
        if not sep:
            raise CDIError(f"not a qualified CDI device name: {q!r}")
        ent = specs.get(kind)
        if ent is None or name not in ent["devices"]:
            missing.append(q)
            continue
        path, edits = ent["devices"][name]
        if path not in applied_specs:  # the spec's own edits, once per spec that contributes a device
            applied_specs.add(path)
            _merge(out, ent["specs"][path], path)
        _merge(out, edits, f"{q}")
        out.devices.append(q)
    if missing:
        raise CDIError(f"unresolvable CDI devices {', '.join(missing)}")
    if strict and out.conflicts:
        raise CDIError("CDI edits of one container set a variable twice: " + "; ".join(out.conflicts))
    return out
