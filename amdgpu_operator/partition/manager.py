"""GPU partition manager (MIG-manager analog, C10) - disabled by default.

Reference parity: ``migManager.enabled=false`` (/root/reference/README.md:109).
Upstream the MIG manager applies a MIG geometry selected by the
``nvidia.com/mig.config`` node label.  On MI355X the equivalent knobs are the
compute partition (SPX / DPX / QPX / CPX: 1 / 2 / 4 / 8 schedulable devices
per GPU, the 8 XCDs split between them) and the memory partition (NPS1 /
NPS2), set through ``amdsmi_set_gpu_compute_partition`` /
``amdsmi_set_gpu_memory_partition`` (N3 native binding).  The device must be
idle for either, and a memory-partition change takes effect only after an
amdgpu reload (amdsmi.h: "AMDGPU driver restart is REQUIRED").  Flow for one
node, like the MIG manager's:

1. read ``amd.com/gpu.partition-config=<profile>`` (default profile from the
   spec) and compare with the mode of every physical GPU;
2. label ``amd.com/gpu.partition.state=pending``; evict the pods that use
   ``amd.com/gpu`` on this node and wait until they are gone (Terminating pods
   still hold ``/dev/kfd``);
3. pause the node's own GPU clients - device plugin (amd-smi health watcher),
   metrics exporter (amd-smi), validator - by setting their deploy labels to
   ``paused-for-partition-change`` (their DaemonSets then remove the pods;
   the operator leaves paused labels alone) and wait until those pods are
   gone and ``/sys/class/kfd/kfd/proc`` is empty; hold off the node agents
   that stay (the driver container's amd-smi health poll) through
   ``.smi-hold`` and wait until none is in an amd-smi session
   (utils/smihold.py);
4. apply memory then compute partition on each physical GPU; on a memory
   change ask the node's driver container to reload amdgpu
   (``.driver-reload-request``, driver/manager.py) and wait for the fresh
   ``driver-ready``; verify every GPU reports the profile;
5. clear the validations, restore the paused deploy labels (a fresh device
   plugin enumerates the new devices, a fresh validator validates them) and
   label ``...partition.state=success|failed`` and ``...partition.applied``.
   The paused labels are restored on failure too.
"""

from __future__ import annotations

import json
import os
import time
from dataclasses import dataclass

from ..nodeenv import NodeEnv
from ..utils.logs import get_logger

log = get_logger("amdgpu.partition")

STATE_LABEL = "amd.com/gpu.partition.state"
APPLIED_LABEL = "amd.com/gpu.partition.applied"
# what MI355X offers: compute SPX/DPX/QPX/CPX, memory NPS1/NPS2 (TPX and
# NPS4/NPS8 are MI300X modes, refused here)
VALID_COMPUTE = ("SPX", "DPX", "QPX", "CPX")
VALID_MEMORY = ("NPS1", "NPS2")
# compute modes allowed with each memory mode (NPS2 splits the HBM in two:
# at least one compute partition per memory partition)
COMPAT = {"NPS1": set(VALID_COMPUTE), "NPS2": {"DPX", "QPX", "CPX"}}
PAUSED = "paused-for-partition-change"
# operands holding amd-smi / KFD handles on the node during a change
PAUSE_OPERANDS = ("devicePlugin", "dcgmExporter", "validator")
RELOAD_REQUEST = ".driver-reload-request"


class PartitionBusy(RuntimeError):
    """The device is in use (amd-smi AMDSMI_STATUS_BUSY / KFD users)."""


@dataclass
class Profile:
    compute: str
    memory: str

    def validate(self) -> None:
        if self.compute not in VALID_COMPUTE or self.memory not in VALID_MEMORY:
            raise ValueError(f"bad partition profile {self}: MI355X offers compute {VALID_COMPUTE}, "
                             f"memory {VALID_MEMORY}")
        if self.compute not in COMPAT[self.memory]:
            raise ValueError(f"compute partition {self.compute} not supported with memory partition {self.memory}")


AMDSMI_STATUS_BUSY = 30


class SmiBackend:
    """Applies partitions through libamd_smi (root on the node).  The session
    is opened on use and closed around a driver reload (:meth:`close`): an
    amd-smi session keeps the GPUs' DRM nodes open, which would keep amdgpu
    in use and fail every unload a memory-partition change needs."""

    def __init__(self):
        self._smi = None

    @property
    def smi(self):
        if self._smi is None:
            from ..discovery.topology import Smi

            self._smi = Smi()
        return self._smi

    def close(self) -> None:
        if self._smi is not None:
            self._smi.close()
            self._smi = None

    def current(self, physical_index: int) -> tuple[str, str]:
        return self.smi.partitions(physical_index)

    def apply(self, physical_index: int, profile: Profile) -> None:
        c, m = self.smi.partitions(physical_index)
        if m != profile.memory:
            rc = self.smi.set_memory_partition(physical_index, profile.memory)
            if rc == AMDSMI_STATUS_BUSY:
                raise PartitionBusy(f"GPU {physical_index} busy: memory partition {profile.memory} not set")
            if rc != 0:
                raise RuntimeError(f"set memory partition {profile.memory} on GPU {physical_index}: rc={rc}")
        if c != profile.compute:
            rc = self.smi.set_compute_partition(physical_index, profile.compute)
            if rc == AMDSMI_STATUS_BUSY:
                raise PartitionBusy(f"GPU {physical_index} busy: compute partition {profile.compute} not set")
            if rc != 0:
                raise RuntimeError(f"set compute partition {profile.compute} on GPU {physical_index}: rc={rc}")


class SysfsBackend:
    """A fake node's partitions (tests, the simulated cluster), with the
    hardware's rules: a change is refused while KFD users exist (the fake
    tree's ``sys/class/kfd/kfd/proc``) or an amd-smi client of the node is
    in a session (its lease in ``validations_dir``, utils/smihold.py), a
    compute change takes effect at once, a memory change only at the next
    amdgpu load (the fake module, fakesys.SimModule, applies
    ``.pending-partition``)."""

    def __init__(self, root: str, rebuild, validations_dir: str | None = None):
        self.root = root
        self.rebuild = rebuild  # callable(compute, memory) -> None (re-creates the KFD nodes)
        self.validations_dir = validations_dir

    def current(self, physical_index: int) -> tuple[str, str]:
        from ..discovery import topology

        for g in topology.enumerate_gpus(self.root):
            if g.physical_index == physical_index:
                return g.compute_partition, g.memory_partition
        return "", ""

    def apply(self, physical_index: int, profile: Profile) -> None:
        procs = os.path.join(self.root, "sys/class/kfd/kfd/proc")
        users = [p for p in (os.listdir(procs) if os.path.isdir(procs) else []) if p.isdigit()]
        if users:
            raise PartitionBusy(f"GPU {physical_index} busy: KFD users {users[:8]}")
        if self.validations_dir:
            from ..utils import smihold

            clients = smihold.live_clients(self.validations_dir)
            if clients:
                raise PartitionBusy(f"GPU {physical_index} busy: amd-smi clients {clients[:8]}")
        c, m = self.current(physical_index)
        if m != profile.memory:
            from ..discovery import topology

            gpus = len({g.physical_index for g in topology.enumerate_gpus(self.root)})
            with open(os.path.join(self.root, ".pending-partition"), "w") as f:
                json.dump({"compute": profile.compute, "memory": profile.memory, "gpus": gpus}, f)
        elif c != profile.compute:
            self.rebuild(profile.compute, profile.memory)


def desired_profile(node: dict, profiles: dict, default: Profile, label: str) -> tuple[str, Profile]:
    name = ((node.get("metadata") or {}).get("labels") or {}).get(label)
    if not name:
        return "default", default
    if name not in profiles:
        raise ValueError(f"unknown partition profile {name!r}")
    p = profiles[name]
    return name, Profile(p.get("compute", default.compute), p.get("memory", default.memory))


def _deploy_label(operand: str) -> str:
    from ..wellknown import DEPLOY_LABEL, OPERAND_LABELS

    return DEPLOY_LABEL.format(OPERAND_LABELS[operand])


def _app(operand: str) -> str:
    return {"devicePlugin": "amd-device-plugin-daemonset", "dcgmExporter": "amd-metrics-exporter",
            "validator": "amd-operator-validator"}[operand]


def pause_operands(env: NodeEnv, operands=PAUSE_OPERANDS) -> list[str]:
    """Deploy labels of ``operands`` that are on (``true``) set to
    ``paused-for-partition-change``; returns the operands paused."""
    labels = (env.client.get("v1", "Node", env.node_name)["metadata"].get("labels") or {})
    paused = [o for o in operands if labels.get(_deploy_label(o)) in ("true", PAUSED)]
    if paused:
        env.client.patch("v1", "Node", env.node_name,
                         {"metadata": {"labels": {_deploy_label(o): PAUSED for o in paused}}})
    return paused


def resume_operands(env: NodeEnv, paused: list[str]) -> None:
    if paused:
        env.client.patch("v1", "Node", env.node_name,
                         {"metadata": {"labels": {_deploy_label(o): "true" for o in paused}}})


def wait_operands_gone(env: NodeEnv, operands: list[str], timeout: float) -> bool:
    """The paused operands' pods have left this node."""
    from ..kube.client import wait_for

    apps = {_app(o) for o in operands}
    if not apps:
        return True
    _, ok = wait_for(env.client, "v1", "Pod",
                     lambda pods: not any(((p["metadata"].get("labels") or {}).get("app") in apps) for p in pods.values()),
                     namespace=env.namespace, field_selector=f"spec.nodeName={env.node_name}", timeout=timeout,
                     poll_s=env.poll_s)
    return ok


def kfd_idle(env: NodeEnv, timeout: float) -> list[str]:
    """Wait until no process has the GPU open; returns the PIDs left."""
    from ..driver.manager import kfd_users

    deadline = time.monotonic() + timeout
    for delay in env.waits(cap_s=0.05):
        users = kfd_users(env)
        if not users or time.monotonic() >= deadline:
            return users
        time.sleep(delay)
    return []


def request_driver_reload(env: NodeEnv, reason: str, timeout: float) -> bool:
    """Ask the node's driver container to reload amdgpu and wait for the
    driver-ready it writes afterwards."""
    from ..validator.validate import read_ready

    os.makedirs(env.validations_dir, exist_ok=True)
    req = env.validation_file(RELOAD_REQUEST)
    t0 = time.time()
    with open(req + ".tmp", "w") as f:
        json.dump({"reason": reason, "time": t0}, f)
    os.replace(req + ".tmp", req)
    deadline = time.monotonic() + timeout
    for delay in env.waits(cap_s=0.05):
        if not os.path.exists(req) and (read_ready(env, "driver") or {}).get("time", 0) >= t0:
            return True
        if time.monotonic() >= deadline:
            return False
        time.sleep(delay)
    return False


def reconcile_node(env: NodeEnv, backend, profiles: dict, default: Profile,
                   label: str = "amd.com/gpu.partition-config", evict: bool = True, timeout: float = 300.0) -> dict:
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

    def fail(why: str) -> dict:
        env.client.patch("v1", "Node", env.node_name, {"metadata": {"labels": {STATE_LABEL: "failed"}}})
        log.error("partition %s not applied: %s", name, why)
        return {"changed": False, "error": why, "profile": name}

    from ..utils import smihold

    env.client.patch("v1", "Node", env.node_name, {"metadata": {"labels": {STATE_LABEL: "pending"}}})
    evicted = evict_gpu_pods(env) if evict else []
    if evict and not wait_gpu_pods_gone(env, timeout):
        return fail("GPU pods still on the node")
    memory_change = any(backend.current(p)[1] != prof.memory for p in todo)
    paused = pause_operands(env)
    # the node agents that stay (amd-driver-health's amd-smi poll) are held off
    # the devices for the change (utils/smihold.py)
    smihold.hold(env.validations_dir, f"partition {name}")
    try:
        if not wait_operands_gone(env, paused, timeout):
            return fail(f"paused operands {paused} still running on the node")
        users = kfd_idle(env, timeout)
        if users:
            return fail(f"GPU still open by process(es) {users[:8]}")
        clients = smihold.wait_clients_gone(env.validations_dir, timeout)
        if clients:
            return fail(f"amd-smi clients {clients[:8]} still in a session")
        try:
            for p in todo:
                backend.apply(p, prof)
        except Exception as e:  # noqa: BLE001 - PartitionBusy or an amd-smi error: nothing more is changed
            return fail(str(e))
        if memory_change:
            clear_ready(env, ("workload", "plugin", "complete"))
            if hasattr(backend, "close"):
                backend.close()  # our own amd-smi session would keep amdgpu from unloading
            if not request_driver_reload(env, f"memory partition {prof.memory}", timeout):
                return fail("the driver container did not reload amdgpu for the memory partition change")
        left = [p for p in todo if backend.current(p) != (prof.compute, prof.memory)]
        if left:
            return fail(f"GPUs {left} do not report {prof.compute}/{prof.memory} after the change")
        clear_ready(env, ("workload", "plugin", "complete"))
        env.client.patch("v1", "Node", env.node_name,
                         {"metadata": {"labels": {STATE_LABEL: "success", APPLIED_LABEL: name,
                                                  "amd.com/gpu.validated": None}}})
        return {"changed": True, "profile": name, "gpus": todo, "evicted": evicted, "paused": paused,
                "driver_reloaded": memory_change}
    finally:
        smihold.release(env.validations_dir)
        # the device plugin comes back on the new devices, a fresh validator validates them
        resume_operands(env, paused)


def _uses_gpu(pod: dict, client=None) -> bool:
    """A pod holding the node's GPUs: amd.com/gpu, or a gpu.amd.com DRA claim
    (wellknown.uses_gpu) - a partition switch re-creates the devices both hold."""
    from ..wellknown import uses_gpu

    get = (lambda ns, n: client.get("resource.k8s.io/v1beta1", "ResourceClaim", n, ns)) if client is not None else None
    return uses_gpu(pod, get)


def evict_gpu_pods(env: NodeEnv) -> list[str]:
    out = []
    for pod in env.client.list("v1", "Pod", field_selector=f"spec.nodeName={env.node_name}"):
        if _uses_gpu(pod, env.client):
            env.client.delete("v1", "Pod", pod["metadata"]["name"], pod["metadata"].get("namespace"))
            out.append(f"{pod['metadata'].get('namespace')}/{pod['metadata']['name']}")
    return out


def wait_gpu_pods_gone(env: NodeEnv, timeout: float) -> bool:
    """Wait until no GPU pod is left on the node, Terminating ones included
    (they hold ``/dev/kfd`` until their containers exit)."""
    from ..kube.client import wait_for

    _, ok = wait_for(env.client, "v1", "Pod", lambda pods: not any(_uses_gpu(p, env.client) for p in pods.values()),
                     field_selector=f"spec.nodeName={env.node_name}", timeout=timeout, poll_s=env.poll_s)
    return ok


def sysfs_partition_rebuilder(root: str, gpus: int):
    """Rebuilder for :class:`SysfsBackend` on a fakesys tree."""
    from ..testing import fakesys

    def rebuild(compute: str, memory: str) -> None:
        import shutil

        shutil.rmtree(os.path.join(root, "sys/class/kfd/kfd/topology/nodes"), ignore_errors=True)
        fakesys.build_node(root, gpus, compute, memory)

    return rebuild
