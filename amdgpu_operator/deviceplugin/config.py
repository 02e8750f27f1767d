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
from typing import Literal, Union

import yaml
from pydantic import BaseModel, ConfigDict, Field, field_validator

from .. import RESOURCE_NAME
from .api import REPLICA_SEP  # noqa: F401 - "<device id>::<replica>"

CONFIG_LABEL = "amd.com/device-plugin.config"
SHARED_SUFFIX = ".shared"

ListStrategy = Literal["envvar", "volume-mounts", "cdi-annotations", "cdi-cri"]


class _M(BaseModel):
    model_config = ConfigDict(extra="forbid", populate_by_name=True)


class Flags(_M):
    partitionStrategy: Literal["single", "mixed"] = "single"
    deviceIDStrategy: Literal["bdf", "uuid", "index"] = "bdf"
    deviceListStrategy: list[ListStrategy] = Field(default_factory=lambda: ["envvar"])
    passDeviceSpecs: bool = True

    @field_validator("deviceListStrategy", mode="before")
    @classmethod
    def _one_or_many(cls, v):
        return [v] if isinstance(v, str) else v

    @field_validator("deviceListStrategy")
    @classmethod
    def _non_empty(cls, v):
        if not v:
            raise ValueError("deviceListStrategy needs at least one strategy")
        return list(dict.fromkeys(v))


class SharedResource(_M):
    name: str = RESOURCE_NAME
    rename: str = ""
    replicas: int = Field(ge=1, le=256)
    devices: Union[Literal["all"], list[Union[int, str]]] = "all"

    def selects(self, dev) -> bool:
        if self.devices == "all":
            return True
        return any(sel == dev.index or sel == dev.bdf or sel == str(dev.index) for sel in self.devices)


class TimeSlicing(_M):
    renameByDefault: bool = False
    failRequestsGreaterThanOne: bool = False
    resources: list[SharedResource] = Field(default_factory=list)


class Sharing(_M):
    timeSlicing: TimeSlicing = Field(default_factory=TimeSlicing)


class DevicePluginConfig(_M):
    version: Literal["v1"] = "v1"
    flags: Flags = Field(default_factory=Flags)
    sharing: Sharing = Field(default_factory=Sharing)

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
