"""The MI355X DRA driver (``gpu.amd.com``): structured parameters for GPUs.

What it does on a node, the kubelet-plugin half of Dynamic Resource
Allocation (dra/api.py has the wire API):

1. **Publish** one ``ResourceSlice`` with every schedulable device - a whole
   MI355X in SPX, each compute partition otherwise - and the attributes a
   claim's CEL selectors and ``matchAttribute`` constraints use: product,
   architecture, family, partition modes, physical GPU index, PCI address,
   NUMA node, xGMI hive, driver version, plus ``memory`` and
   ``computeUnits`` capacity.  The scheduler allocates claims from these; the
   kubelet never sees a device count.
2. **Register** with the kubelet's plugin watcher (``GetInfo`` names the DRA
   endpoint and ``v1beta1.DRAPlugin``).
3. **Prepare** a claim the scheduler allocated on this node: read it from the
   API server (uid checked), take the results for this driver and pool, and
   write a CDI spec for the claim (``gpu.amd.com/claim=<uid>-<device>``: the
   device's render node, ``/dev/kfd``), returned as the claim's CDI device
   ids - the container runtime injects them.  The spec sets no environment
   variable: a container holding two claims gets both specs' edits, and two
   values of one variable would leave it one of them (toolkit/cdi.py); the
   device nodes compose, and ROCm finds the GPUs by them.  Prepared
   claims are checkpointed, so a repeated call (kubelet restart) answers the
   same and a driver restart keeps them; **unprepare** removes the spec.

The device plugin (deviceplugin/) advertises the same GPUs as
``amd.com/gpu``; a GPU must be handed out by one of the two, so the policy
enables one per cluster (api/clusterpolicy.py).
"""

from __future__ import annotations

import json
import os
import threading
import time

from ..rpc import wire
from ..utils.logs import get_logger
from . import api

log = get_logger("amdgpu.dra")
CDI_KIND = f"{api.DRIVER_NAME}/claim"


def device_name(g) -> str:
    return f"gpu-{g.index}"


def _semver(v: str) -> str | None:
    parts = (v or "").split(".")
    return v if len(parts) == 3 and all(p.isdigit() for p in parts) else None


def device_entry(g, driver_version: str = "") -> dict:
    from ..discovery.labels import FAMILIES, PRODUCTS

    attrs = {
        "productName": {"string": PRODUCTS.get(g.device_id, f"AMD-GPU-{g.device_id:04x}")},
        "architecture": {"string": g.arch},
        "family": {"string": FAMILIES.get(g.arch, "unknown")},
        "computePartition": {"string": g.compute_partition or "SPX"},
        "memoryPartition": {"string": g.memory_partition or "NPS1"},
        "physicalIndex": {"int": g.physical_index},
        "partitionIndex": {"int": g.partition_index},
        "index": {"int": g.index},
        "pciBusID": {"string": g.bdf},
        "numaNode": {"int": g.numa_node},
        "xgmiHive": {"string": f"{g.hive_id:x}" if g.hive_id else "none"},
        "uuid": {"string": f"GPU-{g.unique_id:016x}"},
    }
    if _semver(driver_version):
        attrs["driverVersion"] = {"version": driver_version}
    return {"name": device_name(g), "basic": {
        "attributes": attrs,
        "capacity": {"memory": {"value": f"{g.vram_bytes // (1 << 20)}Mi"},
                     "computeUnits": {"value": str(g.cu_count)}}}}


def resource_slice(node_name: str, gpus, node_uid: str = "", driver_version: str = "", generation: int = 1) -> dict:
    meta = {"name": f"{node_name}-{api.DRIVER_NAME}", "labels": {"app.kubernetes.io/managed-by": "amd-gpu-operator"}}
    if node_uid:  # removed with the node
        meta["ownerReferences"] = [{"apiVersion": "v1", "kind": "Node", "name": node_name, "uid": node_uid,
                                    "controller": True}]
    return {"apiVersion": "resource.k8s.io/v1beta1", "kind": "ResourceSlice", "metadata": meta,
            "spec": {"driver": api.DRIVER_NAME, "nodeName": node_name,
                     "pool": {"name": node_name, "generation": generation, "resourceSliceCount": 1},
                     "devices": [device_entry(g, driver_version) for g in gpus]}}


def device_class(name: str = api.DRIVER_NAME) -> dict:
    return {"apiVersion": "resource.k8s.io/v1beta1", "kind": "DeviceClass", "metadata": {"name": name},
            "spec": {"selectors": [{"cel": {"expression": f'device.driver == "{api.DRIVER_NAME}"'}}]}}


class DraDriver:
    """One node's DRA driver: slices, kubelet registration, prepare/unprepare."""

    def __init__(self, env, gpus=None, kubelet_dir: str | None = None):
        from ..discovery import topology

        self.env = env
        self.gpus = list(gpus) if gpus is not None else topology.enumerate_gpus(env.sysfs_root())
        self.by_name = {device_name(g): g for g in self.gpus}
        kdir = kubelet_dir or os.path.dirname(env.device_plugin_dir.rstrip("/"))
        self.registry_socket = os.path.join(kdir, "plugins_registry", f"{api.DRIVER_NAME}-reg.sock")
        self.plugin_dir = os.path.join(kdir, "plugins", api.DRIVER_NAME)
        self.endpoint = os.path.join(self.plugin_dir, "dra.sock")
        self.checkpoint_path = os.path.join(self.plugin_dir, "checkpoint.json")
        self._lock = threading.Lock()
        self.prepared: dict[str, dict] = self._load_checkpoint()
        self.registered = threading.Event()
        self.registration_error = ""
        self._servers: list[wire.Server] = []

    # ------------------------------------------------------------- slices
    def publish(self) -> dict:
        """Create or update this node's ResourceSlice (one pool, one slice)."""
        from ..driver.manager import loaded_version
        from ..kube.errors import NotFound

        c = self.env.client
        node = c.get("v1", "Node", self.env.node_name)
        want = resource_slice(self.env.node_name, self.gpus, node["metadata"].get("uid", ""), loaded_version(self.env))
        name = want["metadata"]["name"]
        try:
            cur = c.get("resource.k8s.io/v1beta1", "ResourceSlice", name)
        except NotFound:
            return c.create(want)
        gen = int(((cur.get("spec") or {}).get("pool") or {}).get("generation", 1))

        def content(spec):  # what is published, apart from the pool's generation counter
            return {**spec, "pool": {k: v for k, v in (spec.get("pool") or {}).items() if k != "generation"}}

        if content(cur.get("spec") or {}) == content(want["spec"]):
            return cur  # unchanged (a driver restart): the generation stays
        # new devices (a partition change): a new pool generation
        want["spec"]["pool"]["generation"] = gen + 1
        want["metadata"]["resourceVersion"] = cur["metadata"].get("resourceVersion")
        return c.update(want)

    def refresh(self) -> bool:
        """Re-read the node's devices (a partition change re-creates them) and
        republish when the set changed; True when it did."""
        from ..discovery import topology

        gpus = topology.enumerate_gpus(self.env.sysfs_root())
        if [(device_name(g), g.bdf, g.compute_partition) for g in gpus] == \
                [(device_name(g), g.bdf, g.compute_partition) for g in self.gpus]:
            return False
        self.gpus = gpus
        self.by_name = {device_name(g): g for g in gpus}
        self.publish()
        log.info("devices changed: %d now published", len(gpus))
        return True

    def withdraw(self) -> None:
        from ..kube.errors import NotFound

        try:
            self.env.client.delete("resource.k8s.io/v1beta1", "ResourceSlice", f"{self.env.node_name}-{api.DRIVER_NAME}")
        except NotFound:
            pass

    # --------------------------------------------------------- checkpoint
    def _load_checkpoint(self) -> dict:
        try:
            with open(self.checkpoint_path) as f:
                return json.load(f).get("claims", {})
        except (OSError, ValueError):
            return {}

    def _save_checkpoint(self) -> None:
        os.makedirs(self.plugin_dir, exist_ok=True)
        tmp = self.checkpoint_path + ".tmp"
        with open(tmp, "w") as f:
            json.dump({"claims": self.prepared}, f)
        os.replace(tmp, self.checkpoint_path)

    def cdi_path(self, uid: str) -> str:
        return os.path.join(self.env.cdi_dir, f"{api.DRIVER_NAME}-claim_{uid}.json")

    def _write_cdi(self, uid: str, devices: list[str]) -> list[str]:
        spec = {"cdiVersion": "0.6.0", "kind": CDI_KIND,
                "containerEdits": {"deviceNodes": [{"path": "/dev/kfd", "type": "c", "permissions": "rw"}]},
                "devices": [{"name": f"{uid}-{d}", "containerEdits": {"deviceNodes": [
                    {"path": self.by_name[d].render_node, "type": "c", "permissions": "rw"}]}} for d in devices]}
        os.makedirs(self.env.cdi_dir, exist_ok=True)
        path = self.cdi_path(uid)
        with open(path + ".tmp", "w") as f:
            json.dump(spec, f, indent=1)
        os.replace(path + ".tmp", path)
        return [f"{CDI_KIND}={uid}-{d}" for d in devices]

    # ------------------------------------------------------ prepare paths
    def prepare(self, namespace: str, name: str, uid: str) -> tuple[list[dict], str]:
        """(devices, error) of one claim; idempotent."""
        with self._lock:
            if uid in self.prepared:
                return self.prepared[uid]["devices"], ""
        from ..kube.errors import NotFound

        try:
            claim = self.env.client.get("resource.k8s.io/v1beta1", "ResourceClaim", name, namespace)
        except NotFound:
            return [], f"claim {namespace}/{name} not found"
        if claim["metadata"].get("uid") != uid:
            return [], f"claim {namespace}/{name} has uid {claim['metadata'].get('uid')}, kubelet asked for {uid}"
        results = [r for r in ((((claim.get("status") or {}).get("allocation") or {}).get("devices") or {})
                               .get("results") or []) if r.get("driver") == api.DRIVER_NAME]
        mine = [r for r in results if r.get("pool") == self.env.node_name]
        if not mine:
            return [], f"claim {namespace}/{name} has no {api.DRIVER_NAME} device allocated on {self.env.node_name}"
        unknown = [r["device"] for r in mine if r.get("device") not in self.by_name]
        if unknown:
            return [], f"claim {namespace}/{name}: unknown devices {unknown} (slice out of date?)"
        devs = list(dict.fromkeys(r["device"] for r in mine))
        ids = dict(zip(devs, self._write_cdi(uid, devs)))
        out = [{"request_names": [r.get("request", "")], "pool_name": self.env.node_name, "device_name": r["device"],
                "cdi_device_ids": [ids[r["device"]]]} for r in mine]
        with self._lock:
            self.prepared[uid] = {"namespace": namespace, "name": name, "devices": out, "time": time.time()}
            self._save_checkpoint()
        log.info("prepared claim %s/%s: %s", namespace, name, devs)
        return out, ""

    def unprepare(self, uid: str) -> str:
        with self._lock:
            self.prepared.pop(uid, None)
            self._save_checkpoint()
        try:
            os.unlink(self.cdi_path(uid))
        except FileNotFoundError:
            pass
        return ""

    # ------------------------------------------------------------- gRPC
    def NodePrepareResources(self, request, context):
        out = api.dra["NodePrepareResourcesResponse"]()
        for c in request.claims:
            devs, err = self.prepare(c.namespace, c.name, c.uid)
            r = api.dra["NodePrepareResourceResponse"](error=err)
            for d in devs:
                r.devices.add(**d)
            out.claims.add(key=c.uid, value=r)
        return out

    def NodeUnprepareResources(self, request, context):
        out = api.dra["NodeUnprepareResourcesResponse"]()
        for c in request.claims:
            out.claims.add(key=c.uid, value=api.dra["NodeUnprepareResourceResponse"](error=self.unprepare(c.uid)))
        return out

    def GetInfo(self, request, context):
        return api.reg["PluginInfo"](type=api.PLUGIN_TYPE, name=api.DRIVER_NAME, endpoint=self.endpoint,
                                     supported_versions=list(api.DRA_VERSIONS))

    def NotifyRegistrationStatus(self, request, context):
        self.registration_error = request.error
        if request.plugin_registered:
            self.registered.set()
            log.info("registered with the kubelet as %s", api.DRIVER_NAME)
        else:
            log.error("kubelet refused the registration: %s", request.error)
        return api.reg["RegistrationStatusResponse"]()

    def serve(self) -> None:
        """DRA endpoint first, then the registration socket the kubelet's
        plugin watcher picks up (it dials the endpoint right after GetInfo)."""
        for path, services, methods in ((self.endpoint, (api.DRA_SERVICE, api.DRA_SERVICE_V1ALPHA4), api.DRA_METHODS),
                                        (self.registry_socket, (api.REGISTRATION_SERVICE,), api.REGISTRATION_METHODS)):
            os.makedirs(os.path.dirname(path), exist_ok=True)
            wire.remove_socket(path)
            srv = wire.Server({api.method_path(svc, n): wire.MethodHandler(getattr(self, n), i.FromString,
                                                                           o.SerializeToString, s)
                               for svc in services for n, (i, o, s) in methods.items()}, name="amdgpu-dra")
            srv.add_unix(path)
            srv.start()
            self._servers.append(srv)

    def stop(self, withdraw: bool = False) -> None:
        for srv in self._servers:
            srv.stop(grace=0.5).wait()
        self._servers = []
        for path in (self.registry_socket, self.endpoint):
            wire.remove_socket(path)
        if withdraw:
            self.withdraw()
