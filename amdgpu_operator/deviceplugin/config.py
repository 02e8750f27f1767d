"""Device-plugin configuration file: flags + GPU sharing (time-slicing).

Reference parity: the reference points at NVIDIA/k8s-device-plugin
(/root/reference/README.md:220) for the plugin that advertises the GPUs
(README.md:205,211).  That plugin is configured by a versioned config file,
typically delivered as a ConfigMap named in the ClusterPolicy
(``devicePlugin.config.name`` / ``.default``) and selected per node with a node
label; its ``sharing.timeSlicing`` section advertises every GPU N times so N
pods can share it.  Users of the reference moving to MI355X expect the same
knobs, so this module accepts the same shape for ``amd.com/gpu``::

    version: v1
    flags:
      partitionStrategy: single          # single | mixed   (CPX/DPX partitions)
      deviceIDStrategy: bdf              # bdf | uuid | index
      deviceListStrategy: [envvar]       # envvar | volume-mounts | cdi-annotations | cdi-cri
      passDeviceSpecs: true              # /dev/kfd + render nodes as DeviceSpecs
    sharing:
      timeSlicing:
        renameByDefault: false           # true: shared resource is amd.com/gpu.shared
        failRequestsGreaterThanOne: false
        resources:
        - name: amd.com/gpu
          replicas: 4
          devices: all                   # or a list of GPU indices / PCI BDFs

The node label ``amd.com/device-plugin.config=<key>`` picks a key of the
ConfigMap; without it the ClusterPolicy's default key applies, and without
either the built-in defaults (no sharing) do.

MI355X notes: a time-sliced MI355X is shared by whole-GPU context switching;
288 GB of HBM is not partitioned between the replicas (use the partition
manager's DPX/QPX/CPX + NPS modes for hard isolation).  Replicas are spread
over GPUs least-loaded first, so N shared pods land on N different GPUs before
any GPU is doubled up.
"""

from __future__ import annotations

import json
from ..utils.record import asdict, field
from ..utils.record import record as dataclass

from .. import RESOURCE_NAME
from .api import REPLICA_SEP  # noqa: F401 - "<device id>::<replica>"

CONFIG_LABEL = "amd.com/device-plugin.config"
SHARED_SUFFIX = ".shared"

LIST_STRATEGIES = ("envvar", "volume-mounts", "cdi-annotations", "cdi-cri")

# Plain dataclasses with explicit validation: the device plugin imports this
# module at start-up, inside the node's time-to-Ready, and pydantic's import
# alone cost it ~0.1 s (tools/operand_start_probe.py).  Errors are
# ValueError, as pydantic's ValidationError is.


def _check_keys(where: str, data, allowed) -> dict:
    if data is None:
        return {}
    if not isinstance(data, dict):
        raise ValueError(f"{where}: expected a mapping, got {type(data).__name__}")
    extra = set(data) - set(allowed)
    if extra:
        raise ValueError(f"{where}: unknown field(s) {sorted(extra)}")
    return data


def _choice(where: str, v, options):
    if v not in options:
        raise ValueError(f"{where}: {v!r} is not one of {list(options)}")
    return v


def _bool(where: str, v) -> bool:
    if not isinstance(v, bool):
        raise ValueError(f"{where}: expected true/false, got {v!r}")
    return v


@dataclass
class Flags:
    partitionStrategy: str = "single"
    deviceIDStrategy: str = "bdf"
    deviceListStrategy: list = field(default_factory=lambda: ["envvar"])
    passDeviceSpecs: bool = True

    @classmethod
    def from_dict(cls, data) -> "Flags":
        d = _check_keys("flags", data, list(cls.__record_fields__))
        out = cls()
        if "partitionStrategy" in d:
            out.partitionStrategy = _choice("flags.partitionStrategy", d["partitionStrategy"], ("single", "mixed"))
        if "deviceIDStrategy" in d:
            out.deviceIDStrategy = _choice("flags.deviceIDStrategy", d["deviceIDStrategy"], ("bdf", "uuid", "index"))
        if "deviceListStrategy" in d:
            v = d["deviceListStrategy"]
            v = [v] if isinstance(v, str) else v
            if not isinstance(v, list) or not v:
                raise ValueError("deviceListStrategy needs at least one strategy")
            out.deviceListStrategy = list(dict.fromkeys(_choice("flags.deviceListStrategy", x, LIST_STRATEGIES)
                                                        for x in v))
        if "passDeviceSpecs" in d:
            out.passDeviceSpecs = _bool("flags.passDeviceSpecs", d["passDeviceSpecs"])
        return out


@dataclass
class SharedResource:
    replicas: int
    name: str = RESOURCE_NAME
    rename: str = ""
    devices: object = "all"  # "all" or a list of GPU indices / PCI BDFs

    @classmethod
    def from_dict(cls, data) -> "SharedResource":
        d = _check_keys("sharing.timeSlicing.resources[]", data, list(cls.__record_fields__))
        r = d.get("replicas")
        if isinstance(r, bool) or not isinstance(r, int) or not 1 <= r <= 256:
            raise ValueError(f"replicas must be an integer in [1, 256], got {r!r}")
        devices = d.get("devices", "all")
        if devices != "all" and not (isinstance(devices, list) and all(isinstance(x, (int, str)) and not
                                                                         isinstance(x, bool) for x in devices)):
            raise ValueError(f"devices must be 'all' or a list of indices / BDFs, got {devices!r}")
        for k in ("name", "rename"):
            if k in d and not isinstance(d[k], str):
                raise ValueError(f"{k} must be a string")
        return cls(replicas=r, name=d.get("name", RESOURCE_NAME), rename=d.get("rename", ""), devices=devices)

    def selects(self, dev) -> bool:
        if self.devices == "all":
            return True
        return any(sel == dev.index or sel == dev.bdf or sel == str(dev.index) for sel in self.devices)


@dataclass
class TimeSlicing:
    renameByDefault: bool = False
    failRequestsGreaterThanOne: bool = False
    resources: list = field(default_factory=list)

    @classmethod
    def from_dict(cls, data) -> "TimeSlicing":
        d = _check_keys("sharing.timeSlicing", data, list(cls.__record_fields__))
        res = d.get("resources") or []
        if not isinstance(res, list):
            raise ValueError("sharing.timeSlicing.resources must be a list")
        return cls(renameByDefault=_bool("renameByDefault", d.get("renameByDefault", False)),
                   failRequestsGreaterThanOne=_bool("failRequestsGreaterThanOne",
                                                    d.get("failRequestsGreaterThanOne", False)),
                   resources=[SharedResource.from_dict(r) for r in res])


@dataclass
class Sharing:
    timeSlicing: TimeSlicing = field(default_factory=TimeSlicing)

    @classmethod
    def from_dict(cls, data) -> "Sharing":
        d = _check_keys("sharing", data, ["timeSlicing"])
        return cls(timeSlicing=TimeSlicing.from_dict(d.get("timeSlicing")))


@dataclass
class DevicePluginConfig:
    version: str = "v1"
    flags: Flags = field(default_factory=Flags)
    sharing: Sharing = field(default_factory=Sharing)

    @classmethod
    def model_validate(cls, data) -> "DevicePluginConfig":
        d = _check_keys("config", data, ["version", "flags", "sharing"])
        return cls(version=_choice("version", d.get("version", "v1"), ("v1",)), flags=Flags.from_dict(d.get("flags")),
                   sharing=Sharing.from_dict(d.get("sharing")))

    def model_dump(self, mode: str = "json") -> dict:
        return asdict(self)

    def shared_for(self, resource: str) -> SharedResource | None:
        for r in self.sharing.timeSlicing.resources:
            if r.name == resource:
                return r
        return None

    def shared_name(self, resource: str, rule: SharedResource) -> str:
        """Resource name that carries the replicas of ``resource``."""
        if rule.rename:
            return rule.rename
        return resource + SHARED_SUFFIX if self.sharing.timeSlicing.renameByDefault else resource

    def replicas_of(self, resource: str, dev) -> int:
        rule = self.shared_for(resource)
        return rule.replicas if rule is not None and rule.selects(dev) else 1

    @property
    def sharing_strategy(self) -> str:
        return "time-slicing" if any(r.replicas > 1 for r in self.sharing.timeSlicing.resources) else "none"


def parse(text: str) -> DevicePluginConfig:
    """YAML (or JSON) config file -> validated config."""
    import yaml  # only when a config file / ConfigMap key is in use

    data = yaml.safe_load(text) if text.strip() else {}
    return DevicePluginConfig.model_validate(data or {})


def select(data: dict[str, str], node_labels: dict[str, str] | None, default_key: str = "") -> tuple[str, DevicePluginConfig]:
    """Pick the ConfigMap key for this node: its ``amd.com/device-plugin.config``
    label, else ``default_key``, else built-in defaults (key "")."""
    key = (node_labels or {}).get(CONFIG_LABEL) or default_key
    if not key:
        return "", DevicePluginConfig()
    if key not in data:
        raise KeyError(f"device-plugin config {key!r} not in ConfigMap (keys: {sorted(data)})")
    return key, parse(data[key])


def dumps(cfg: DevicePluginConfig) -> str:
    return json.dumps(cfg.model_dump(mode="json"), sort_keys=True)
