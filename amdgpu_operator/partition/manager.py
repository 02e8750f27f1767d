"""GPU partition manager (MIG-manager analog, C10) - disabled by default.

Reference parity: ``migManager.enabled=false`` (/root/reference/README.md:109).
Upstream the MIG manager applies a MIG geometry selected by the
``nvidia.com/mig.config`` node label.  On MI355X the equivalent knobs are the
compute partition (SPX / DPX / QPX / CPX: 1 / 2 / 4 / 8 schedulable devices
per GPU, XCDs split between them) and the memory partition (NPS1 / NPS2), set
through ``amdsmi_set_gpu_compute_partition`` / ``amdsmi_set_gpu_memory_partition``
(N3 native binding).  Flow for one node:

1. read ``amd.com/gpu.partition-config=<profile>`` (default profile from the spec);
2. compare with the current mode of every physical GPU (KFD/PCI sysfs);
3. if different: label ``amd.com/gpu.partition.state=pending``, evict pods
   that use ``amd.com/gpu`` on this node, apply memory then compute partition
   on each physical GPU, clear the validation files (the node must revalidate),
   restart the device plugin pod (it re-enumerates the new devices);
4. label ``...partition.state=success|failed`` and ``...partition.applied``.
"""

from __future__ import annotations

import os
from dataclasses import dataclass

from ..nodeenv import NodeEnv
from ..utils.logs import get_logger

log = get_logger("amdgpu.partition")

STATE_LABEL = "amd.com/gpu.partition.state"
APPLIED_LABEL = "amd.com/gpu.partition.applied"
VALID_COMPUTE = ("SPX", "DPX", "TPX", "QPX", "CPX")
VALID_MEMORY = ("NPS1", "NPS2", "NPS4", "NPS8")
# compute modes allowed with each memory mode on MI355X (CPX/QPX need NPS2 for
# per-partition local memory; every mode also works under NPS1)
COMPAT = {"NPS1": set(VALID_COMPUTE), "NPS2": {"DPX", "QPX", "CPX"}, "NPS4": {"QPX", "CPX"}, "NPS8": {"CPX"}}


@dataclass
class Profile:
    compute: str
    memory: str

    def validate(self) -> None:
        if self.compute not in VALID_COMPUTE or self.memory not in VALID_MEMORY:
            raise ValueError(f"bad partition profile {self}")
        if self.compute not in COMPAT[self.memory]:
            raise ValueError(f"compute partition {self.compute} not supported with memory partition {self.memory}")


class SmiBackend:
    """Applies partitions through libamd_smi (root on the node)."""

    def __init__(self):
        from ..discovery.topology import Smi

        self.smi = Smi()

    def current(self, physical_index: int) -> tuple[str, str]:
        return self.smi.partitions(physical_index)

    def apply(self, physical_index: int, profile: Profile) -> None:
        c, m = self.smi.partitions(physical_index)
        if m != profile.memory:
            rc = self.smi.set_memory_partition(physical_index, profile.memory)
            if rc != 0:
                raise RuntimeError(f"set memory partition {profile.memory} on GPU {physical_index}: rc={rc}")
        if c != profile.compute:
            rc = self.smi.set_compute_partition(physical_index, profile.compute)
            if rc != 0:
                raise RuntimeError(f"set compute partition {profile.compute} on GPU {physical_index}: rc={rc}")


class SysfsBackend:
    """Rewrites a (fake) sysfs tree - used by tests and the simulated cluster."""

    def __init__(self, root: str, rebuild):
        self.root = root
        self.rebuild = rebuild  # callable(compute, memory) -> None (re-creates the KFD nodes)

    def current(self, physical_index: int) -> tuple[str, str]:
        from ..discovery import topology

        for g in topology.enumerate_gpus(self.root):
            if g.physical_index == physical_index:
                return g.compute_partition, g.memory_partition
        return "", ""

    def apply(self, physical_index: int, profile: Profile) -> None:
        self.rebuild(profile.compute, profile.memory)


def desired_profile(node: dict, profiles: dict, default: Profile, label: str) -> tuple[str, Profile]:
    name = ((node.get("metadata") or {}).get("labels") or {}).get(label)
    if not name:
        return "default", default
    if name not in profiles:
        raise ValueError(f"unknown partition profile {name!r}")
    p = profiles[name]
    return name, Profile(p.get("compute", default.compute), p.get("memory", default.memory))


def reconcile_node(env: NodeEnv, backend, profiles: dict, default: Profile,
                   label: str = "amd.com/gpu.partition-config", evict: bool = True) -> dict:
    from ..discovery import topology
    from ..validator.validate import clear_ready

    node = env.client.get("v1", "Node", env.node_name)
    name, prof = desired_profile(node, profiles, default, label)
    prof.validate()
    physical = sorted({g.physical_index for g in topology.enumerate_gpus(env.sysfs_root())})
    todo = [p for p in physical if backend.current(p) != (prof.compute, prof.memory)]
    labels = node["metadata"].get("labels") or {}
    if not todo:
        if labels.get(STATE_LABEL) != "success" or labels.get(APPLIED_LABEL) != name:
            env.client.patch("v1", "Node", env.node_name,
                             {"metadata": {"labels": {STATE_LABEL: "success", APPLIED_LABEL: name}}})
        return {"changed": False, "profile": name}
    env.client.patch("v1", "Node", env.node_name, {"metadata": {"labels": {STATE_LABEL: "pending"}}})
    evicted = evict_gpu_pods(env) if evict else []
    try:
        for p in todo:
            backend.apply(p, prof)
    except Exception as e:  # noqa: BLE001
        env.client.patch("v1", "Node", env.node_name, {"metadata": {"labels": {STATE_LABEL: "failed"}}})
        log.error("partition apply failed: %s", e)
        return {"changed": False, "error": str(e), "profile": name}
    clear_ready(env, ("workload", "plugin", "complete"))
    # the plugin re-enumerates the partitions; a fresh validator validates them
    restart_device_plugin(env)
    restart_validator(env)
    env.client.patch("v1", "Node", env.node_name,
                     {"metadata": {"labels": {STATE_LABEL: "success", APPLIED_LABEL: name, "amd.com/gpu.validated": None}}})
    return {"changed": True, "profile": name, "gpus": todo, "evicted": evicted}


def _uses_gpu(pod: dict) -> bool:
    for c in (pod.get("spec") or {}).get("containers", []):
        lim = ((c.get("resources") or {}).get("limits") or {})
        if any(k.startswith("amd.com/gpu") for k in lim):
            return True
    return False


def evict_gpu_pods(env: NodeEnv) -> list[str]:
    out = []
    for pod in env.client.list("v1", "Pod", field_selector=f"spec.nodeName={env.node_name}"):
        if _uses_gpu(pod):
            env.client.delete("v1", "Pod", pod["metadata"]["name"], pod["metadata"].get("namespace"))
            out.append(f"{pod['metadata'].get('namespace')}/{pod['metadata']['name']}")
    return out


def wait_gpu_pods_gone(env: NodeEnv, timeout: float) -> bool:
    """Wait until no GPU pod is left on the node, Terminating ones included
    (they hold ``/dev/kfd`` until their containers exit)."""
    from ..kube.client import wait_for

    _, ok = wait_for(env.client, "v1", "Pod", lambda pods: not any(_uses_gpu(p) for p in pods.values()),
                     field_selector=f"spec.nodeName={env.node_name}", timeout=timeout, poll_s=env.poll_s)
    return ok


def restart_validator(env: NodeEnv) -> None:
    for pod in env.client.list("v1", "Pod", env.namespace, label_selector="app=amd-operator-validator",
                               field_selector=f"spec.nodeName={env.node_name}"):
        env.client.delete("v1", "Pod", pod["metadata"]["name"], env.namespace)


def restart_device_plugin(env: NodeEnv) -> None:
    for pod in env.client.list("v1", "Pod", env.namespace, label_selector="app=amd-device-plugin-daemonset",
                               field_selector=f"spec.nodeName={env.node_name}"):
        env.client.delete("v1", "Pod", pod["metadata"]["name"], env.namespace)


def sysfs_partition_rebuilder(root: str, gpus: int):
    """Rebuilder for :class:`SysfsBackend` on a fakesys tree."""
    from ..testing import fakesys

    def rebuild(compute: str, memory: str) -> None:
        import shutil

        shutil.rmtree(os.path.join(root, "sys/class/kfd/kfd/topology/nodes"), ignore_errors=True)
        fakesys.build_node(root, gpus, compute, memory)

    return rebuild
