"""AMD GPU device plugin: advertises ``amd.com/gpu`` to kubelet.

Reference parity: ``nvidia-device-plugin-daemonset`` "advertises the number of
available GPUs on the node to Kubernetes" (/root/reference/README.md:205,211),
which surfaces as Allocatable ``nvidia.com/gpu`` (README.md:122).  This server
implements the kubelet ``v1beta1`` DevicePlugin service over a unix socket:

* ``Register`` with kubelet (``kubelet.sock``) and re-register whenever the
  kubelet socket is re-created (kubelet restart);
* ``ListAndWatch`` streams the device list and every health change
  (N6 health watcher: amd-smi events, ECC / xGMI deltas; or an injected source);
* ``GetPreferredAllocation`` uses the xGMI/NUMA/partition cost model
  (:mod:`.allocator`);
* ``Allocate`` returns ``/dev/kfd`` + the render nodes as DeviceSpecs, the
  ``AMD_VISIBLE_DEVICES`` env consumed by the OCI hook, annotations (HBM size,
  xGMI hive) and, when enabled, CDI device names for containerd;
* ``PreStartContainer`` is a no-op (not required).

GPU sharing, device-ID and device-list strategies come from the plugin config
file (:mod:`.config`, the k8s-device-plugin config shape): a time-sliced GPU is
advertised as ``<id>::<k>`` replicas, Allocate maps replicas back to the
physical GPU, and preferred allocation spreads replicas least-loaded first.

The plugin is stateless: kubelet checkpoints assignments.
gRPC runs on the operator's own HTTP/2 transport (:mod:`..rpc.wire`): grpcio's
import was ~0.1 s of the plugin's start-up, before its kubelet registration.
"""

from __future__ import annotations

import os
import threading
import time
from ..utils.record import field
from ..utils.record import record as dataclass
from typing import Callable

from .. import RESOURCE_NAME
from . import api
from .allocator import from_topology, preferred
from .config import REPLICA_SEP, DevicePluginConfig
from ..rpc import wire
from ..utils.logs import get_logger

log = get_logger("amdgpu.deviceplugin")


@dataclass
class PluginConfig:
    resource_name: str = RESOURCE_NAME
    socket_dir: str = api.DEVICE_PLUGIN_PATH
    kubelet_socket: str | None = None
    endpoint: str = "amd-gpu.sock"
    sysfs_root: str = "/"
    cdi_enabled: bool = False
    cdi_kind: str = "amd.com/gpu"
    partition_strategy: str = "single"  # single | mixed
    health_poll_ms: int = 1000
    watch_interval_s: float = 0.5
    rocm_mount: str | None = None
    extra_env: dict = field(default_factory=dict)
    device_config: DevicePluginConfig | None = None  # config file: flags + sharing
    rdma: bool = False  # driver.rdma: annotate allocations with their nearest RDMA NICs
    rdma_hca_env: bool = False  # ... and set NCCL_IB_HCA to them

    @property
    def config(self) -> DevicePluginConfig:
        return self.device_config or DevicePluginConfig()

    @property
    def id_strategy(self) -> str:
        return self.config.flags.deviceIDStrategy

    @property
    def list_strategies(self) -> list[str]:
        out = list(self.config.flags.deviceListStrategy)
        if self.cdi_enabled and "cdi-cri" not in out:  # legacy --cdi flag
            out.append("cdi-cri")
        return out

    @property
    def pass_device_specs(self) -> bool:
        return self.config.flags.passDeviceSpecs

    @property
    def kubelet_path(self) -> str:
        return self.kubelet_socket or os.path.join(self.socket_dir, "kubelet.sock")

    @property
    def endpoint_path(self) -> str:
        return os.path.join(self.socket_dir, self.endpoint)


CONTAINER_DEVICES_DIR = "/var/run/amd-container-devices"  # volume-mounts list strategy (read by the OCI hook)


def base_id(dev, strategy: str) -> str:
    """kubelet device ID of a GPU (or partition) under ``deviceIDStrategy``."""
    if strategy == "index":
        return str(dev.index)
    if strategy == "uuid" and dev.unique_id:
        u = f"GPU-{dev.unique_id:016x}"
        return u if dev.partition_count <= 1 else f"{u}-p{dev.partition_index}"
    return dev.device_id_str


def resource_for(dev, cfg: PluginConfig) -> str:
    """Resource name of a device under the partition strategy.

    ``single``: every device (whole GPU or partition) is ``amd.com/gpu``.
    ``mixed``: partitioned devices are ``amd.com/gpu-<mode>`` (e.g. ``-cpx``)."""
    from ..discovery import topology

    return topology.partition_resource(dev, cfg.resource_name, cfg.partition_strategy)


class DevicePluginServer:
    """One kubelet device-plugin endpoint serving one resource name."""

    def __init__(self, cfg: PluginConfig, devices, links=(), resource_name: str | None = None, replicas: int = 1,
                 fail_requests_gt_one: bool = False):
        self.cfg = cfg
        self.resource_name = resource_name or cfg.resource_name
        self.devices = list(devices)
        self.replicas = max(1, int(replicas))
        self.fail_requests_gt_one = fail_requests_gt_one and self.replicas > 1
        self._ids_of: dict[str, list[str]] = {}  # physical key (device_id_str) -> advertised ids
        self._by_id = {}
        for d in self.devices:
            b = base_id(d, cfg.id_strategy)
            ids = [b] if self.replicas == 1 else [f"{b}{REPLICA_SEP}{k}" for k in range(self.replicas)]
            self._ids_of[d.device_id_str] = ids
            for i in ids:
                self._by_id[i] = d
        self._order = {d.device_id_str: n for n, d in enumerate(self.devices)}
        self._health = {i: api.HEALTHY for i in self._by_id}
        self._cost = from_topology(self.devices, links, lambda g: self._ids_of[g.device_id_str][0])
        self._cv = threading.Condition()
        self._version = 0
        self._stop = threading.Event()
        self._server: wire.Server | None = None
        self._watch_thread: threading.Thread | None = None
        self._nics = None  # RDMA NICs (cfg.rdma), enumerated at the first allocation
        self._kubelet_ino = None
        self.registrations = 0
        self.allocations = 0
        self.events: list[dict] = []

    # ------------------------------------------------------------------ health
    def set_health(self, device_id: str, healthy: bool, reason: str = "") -> None:
        """``device_id``: a physical GPU (every replica of it) or one advertised ID."""
        state = api.HEALTHY if healthy else api.UNHEALTHY
        ids = self._ids_of.get(device_id) or ([device_id] if device_id in self._health else [])
        with self._cv:
            ids = [i for i in ids if self._health[i] != state]
            if not ids:
                return
            for i in ids:
                self._health[i] = state
            self._version += 1
            self.events.append({"t": time.time(), "device": device_id, "health": state, "reason": reason,
                                "ids": len(ids)})
            self._cv.notify_all()
        log.warning("device %s -> %s %s", device_id, state, reason)

    def healthy_count(self) -> int:
        with self._cv:
            return sum(1 for h in self._health.values() if h == api.HEALTHY)

    def device_list(self):
        with self._cv:
            resp = api.pb["ListAndWatchResponse"]()
            for d in self.devices:
                for i in self._ids_of[d.device_id_str]:
                    dev = resp.devices.add(ID=i, health=self._health[i])
                    if d.numa_node >= 0:
                        dev.topology.nodes.add(ID=d.numa_node)
            return resp, self._version

    # ------------------------------------------------------------ gRPC methods
    def GetDevicePluginOptions(self, request, context):
        return api.pb["DevicePluginOptions"](pre_start_required=False, get_preferred_allocation_available=True)

    def ListAndWatch(self, request, context):
        done = threading.Event()
        context.add_callback(done.set)
        resp, ver = self.device_list()
        yield resp
        while not self._stop.is_set() and not done.is_set():
            with self._cv:
                if self._version == ver:
                    self._cv.wait(timeout=0.5)
                changed = self._version != ver
            if changed:
                resp, ver = self.device_list()
                yield resp

    def GetPreferredAllocation(self, request, context):
        out = api.pb["PreferredAllocationResponse"]()
        for creq in request.container_requests:
            with self._cv:
                avail = [i for i in creq.available_deviceIDs if self._health.get(i) == api.HEALTHY]
            must = list(creq.must_include_deviceIDs)
            if self.replicas > 1:
                ids = self._preferred_replicas(avail, must, creq.allocation_size)
            else:
                ids = preferred(self._cost, avail, must, creq.allocation_size)
            out.container_responses.add(deviceIDs=ids)
        return out

    def _preferred_replicas(self, avail: list[str], must: list[str], size: int) -> list[str]:
        """Time-sliced GPUs: take replicas from GPUs not yet in this request,
        then from the GPU with the most free replicas (least loaded), then in
        device order - N shared pods land on N different GPUs first."""
        chosen = [i for i in must if i in self._by_id]
        free: dict[str, list[str]] = {}
        for i in avail:
            if i in self._by_id and i not in chosen:
                free.setdefault(self._by_id[i].device_id_str, []).append(i)
        in_request: dict[str, int] = {}
        for i in chosen:
            k = self._by_id[i].device_id_str
            in_request[k] = in_request.get(k, 0) + 1
        while len(chosen) < size and free:
            k = min(free, key=lambda g: (in_request.get(g, 0), -len(free[g]), self._order[g]))
            chosen.append(free[k].pop(0))
            in_request[k] = in_request.get(k, 0) + 1
            if not free[k]:
                del free[k]
        return chosen

    def container_response(self, ids):
        r = api.pb["ContainerAllocateResponse"]()
        devs = list({self._by_id[i].device_id_str: self._by_id[i] for i in ids}.values())  # replicas -> GPU
        if self.cfg.pass_device_specs:
            r.devices.add(container_path="/dev/kfd", host_path="/dev/kfd", permissions="rw")
            for d in devs:
                r.devices.add(container_path=d.render_node, host_path=d.render_node, permissions="rw")
        indices = ",".join(str(d.index) for d in devs)
        strategies = self.cfg.list_strategies
        if "envvar" in strategies:
            r.envs["AMD_VISIBLE_DEVICES"] = indices
            r.envs["AMD_GPU_DEVICE_IDS"] = ",".join(ids)
        if "volume-mounts" in strategies:  # unprivileged pods cannot forge a mount list (OCI hook reads it)
            for d in devs:
                r.mounts.add(container_path=f"{CONTAINER_DEVICES_DIR}/{d.index}", host_path="/dev/null",
                             read_only=True)
        if "cdi-annotations" in strategies:
            key = "cdi.k8s.io/amd-device-plugin_" + "".join(c if c.isalnum() else "-" for c in self.resource_name)
            r.annotations[key] = ",".join(f"{self.cfg.cdi_kind}={d.index}" for d in devs)
        if self.replicas > 1:
            r.annotations["amd.com/gpu.sharing"] = "time-slicing"
            r.annotations["amd.com/gpu.replicas"] = ",".join(ids)
        for k, v in self.cfg.extra_env.items():
            r.envs[k] = v
        r.annotations["amd.com/gpu.devices"] = indices
        r.annotations["amd.com/gpu.memory-bytes"] = ",".join(str(d.vram_bytes) for d in devs)
        hives = sorted({str(d.hive_id) for d in devs if d.hive_id})
        if hives:
            r.annotations["amd.com/gpu.xgmi-hive"] = ",".join(hives)
        if self.cfg.rdma:
            nics = self._rdma_nics(devs)
            if nics:
                r.annotations["amd.com/gpu.rdma-nics"] = ",".join(nics)
                if self.cfg.rdma_hca_env:
                    r.envs["NCCL_IB_HCA"] = ",".join(nics)
        if self.cfg.rocm_mount:
            r.mounts.add(container_path=self.cfg.rocm_mount, host_path=self.cfg.rocm_mount, read_only=True)
        if "cdi-cri" in strategies:
            for d in devs:
                r.cdi_devices.add(name=f"{self.cfg.cdi_kind}={d.index}")
        return r

    def _rdma_nics(self, devs) -> list[str]:
        """The allocation's nearest RDMA NICs (PCIe switch first), read once:
        NICs do not come and go under a running plugin."""
        if self._nics is None:
            from ..discovery import rdma

            try:
                self._nics = rdma.enumerate_nics(self.cfg.sysfs_root)
            except OSError as e:
                log.warning("RDMA NICs not readable: %s", e)
                self._nics = []
        if not self._nics:
            return []
        from ..discovery import rdma

        return rdma.allocation_nics(devs, self._nics, self.cfg.sysfs_root)

    def Allocate(self, request, context):
        out = api.pb["AllocateResponse"]()
        for creq in request.container_requests:
            ids = list(creq.devices_ids)
            unknown = [i for i in ids if i not in self._by_id]
            if unknown:
                context.abort(wire.StatusCode.INVALID_ARGUMENT, f"unknown device ids {unknown}")
            if self.fail_requests_gt_one and len(ids) > 1:
                context.abort(wire.StatusCode.INVALID_ARGUMENT,
                              f"time-sliced {self.resource_name}: request for {len(ids)} replicas, at most 1 allowed "
                              "(failRequestsGreaterThanOne)")
            with self._cv:
                bad = [i for i in ids if self._health[i] != api.HEALTHY]
            if bad:
                context.abort(wire.StatusCode.FAILED_PRECONDITION, f"unhealthy devices {bad}")
            out.container_responses.append(self.container_response(ids))
        self.allocations += 1
        return out

    def PreStartContainer(self, request, context):
        return api.pb["PreStartContainerResponse"]()

    # --------------------------------------------------------------- lifecycle
    def _handlers(self) -> dict[str, wire.MethodHandler]:
        return {api.method_path(api.DEVICE_PLUGIN_SERVICE, name):
                wire.MethodHandler(getattr(self, name), req.FromString, resp.SerializeToString, stream)
                for name, (req, resp, stream) in api.DEVICE_PLUGIN_METHODS.items()}

    def serve(self) -> None:
        os.makedirs(self.cfg.socket_dir, exist_ok=True)
        path = os.path.join(self.cfg.socket_dir, self._endpoint())
        if os.path.exists(path):
            os.unlink(path)
        self._server = wire.Server(self._handlers(), name="amdgpu-dp")
        self._server.add_unix(path)
        self._server.start()

    def _endpoint(self) -> str:
        if self.resource_name == self.cfg.resource_name:
            return self.cfg.endpoint
        tail = self.resource_name[len(self.cfg.resource_name):] if self.resource_name.startswith(
            self.cfg.resource_name) else self.resource_name
        tail = "".join(c if c.isalnum() else "-" for c in tail).strip("-")
        return self.cfg.endpoint.replace(".sock", "-" + tail + ".sock")

    def register(self, timeout: float = 5.0) -> None:
        t0 = time.perf_counter()
        with wire.Channel(self.cfg.kubelet_path) as ch:
            req_cls, resp_cls, _ = api.REGISTRATION_METHODS["Register"]
            call = ch.unary_unary(api.method_path(api.REGISTRATION_SERVICE, "Register"),
                                  request_serializer=req_cls.SerializeToString, response_deserializer=resp_cls.FromString)
            req = req_cls(version=api.VERSION, endpoint=self._endpoint(), resource_name=self.resource_name)
            req.options.get_preferred_allocation_available = True
            call(req, timeout=timeout, wait_for_ready=True)
        self.registrations += 1
        self._kubelet_ino = self._kubelet_identity()
        log.info("registered %s with kubelet (%d devices) in %.3f s", self.resource_name, len(self.devices),
                 time.perf_counter() - t0)

    def _kubelet_identity(self):
        """(inode, ctime) of kubelet.sock: a re-created socket may reuse the
        inode number, but not the change time."""
        try:
            st = os.stat(self.cfg.kubelet_path)
        except OSError:
            return None
        return (st.st_ino, st.st_ctime_ns)

    def _watch_kubelet(self) -> None:
        """Re-register when kubelet.sock is re-created (kubelet restart)."""
        while not self._stop.wait(self.cfg.watch_interval_s):
            if not self.registrations:
                continue  # prepared but not yet advertised (DevicePluginManager.register)
            ident = self._kubelet_identity()
            if ident is None:
                self._kubelet_ino = None  # socket gone: re-register when it returns
                continue
            if ident != self._kubelet_ino and not self._stop.is_set():
                try:
                    self.register()
                except wire.RpcError as e:  # kubelet not ready yet: retry next tick
                    log.warning("re-register failed: %s", e)

    def start(self, register: bool = True) -> None:
        self.serve()
        if register:
            self.register()
        self._watch_thread = threading.Thread(target=self._watch_kubelet, name="amdgpu-dp-watch", daemon=True)
        self._watch_thread.start()

    def stop(self) -> None:
        self._stop.set()
        with self._cv:
            self._cv.notify_all()
        th = self._watch_thread
        if th is not None and th is not threading.current_thread():
            th.join(timeout=6.0)  # a re-registration in flight ends within its 5 s deadline
        if self._server is not None:
            self._server.stop(grace=0.5).wait()
            self._server = None
        path = os.path.join(self.cfg.socket_dir, self._endpoint())
        if os.path.exists(path):
            os.unlink(path)


class DevicePluginManager:
    """Enumerates the node's GPUs (N3) and runs one server per resource name;
    routes N6 health events to the owning server."""

    def __init__(self, cfg: PluginConfig, devices=None, links=None,
                 health_poll: Callable[[int], list] | None = None,
                 health_factory: Callable[[], Callable[[int], list]] | None = None):
        """``health_poll`` polls N6 health events; ``health_factory`` makes
        that poll function on the health thread instead (amd-smi start-up
        then overlaps registration instead of delaying it)."""
        from ..discovery import topology

        self.cfg = cfg
        if cfg.device_config is not None:  # the config file's flags win over the command line
            cfg.partition_strategy = cfg.device_config.flags.partitionStrategy
        self.devices = devices if devices is not None else topology.enumerate_gpus(cfg.sysfs_root)
        self.links = links if links is not None else topology.links(cfg.sysfs_root)
        self.servers = self._build_servers()
        self._health_poll = health_poll
        self._health_factory = health_factory
        self._stop = threading.Event()
        self._thread: threading.Thread | None = None
        self._registered = True
        self._lock = threading.Lock()

    def _build_servers(self) -> dict[str, DevicePluginServer]:
        """One server per resource name: partition strategy first, then the
        time-slicing rule of that resource (replicas, optional rename)."""
        dc = self.cfg.config
        ts = dc.sharing.timeSlicing
        groups: dict[str, tuple[list, int]] = {}
        for d in self.devices:
            res = resource_for(d, self.cfg)
            rule = dc.shared_for(res)
            reps = 1
            if rule is not None and rule.selects(d):
                res, reps = dc.shared_name(res, rule), rule.replicas
            devs, r0 = groups.setdefault(res, ([], reps))
            if r0 != reps:
                raise ValueError(f"{res}: GPUs with different replica counts ({r0}, {reps}) need distinct names "
                                 "(set rename or renameByDefault)")
            devs.append(d)
        return {r: DevicePluginServer(self.cfg, devs, self.links, r, replicas=reps,
                                      fail_requests_gt_one=ts.failRequestsGreaterThanOne)
                for r, (devs, reps) in groups.items()}

    def reconfigure(self, device_config: DevicePluginConfig | None) -> bool:
        """Apply a new config file (node label or ConfigMap changed): stop the
        servers, rebuild them for the new resource layout, register again.
        Returns False when the config is unchanged."""
        from .config import dumps

        if dumps(device_config or DevicePluginConfig()) == dumps(self.cfg.config):
            return False
        with self._lock:
            old = self.servers
            self.cfg.device_config = device_config
            if device_config is not None:
                self.cfg.partition_strategy = device_config.flags.partitionStrategy
            self.servers = self._build_servers()
            for s in old.values():
                s.stop()
            for s in self.servers.values():
                s.start(register=self._registered)
        log.info("device-plugin config applied: %s", sorted(self.servers))
        return True

    def start(self, register: bool = True) -> None:
        self._registered = register
        for s in self.servers.values():
            s.start(register=register)
        if self._health_poll is not None or self._health_factory is not None:
            self._thread = threading.Thread(target=self._health_loop, name="amdgpu-dp-health", daemon=True)
            self._thread.start()

    def register(self) -> None:
        """Advertise: register every server with the kubelet (after a
        ``start(register=False)`` that prepared them)."""
        with self._lock:
            self._registered = True
            for s in self.servers.values():
                if not s.registrations:
                    s.register()

    def _health_loop(self) -> None:
        if self._health_poll is None:
            try:
                self._health_poll = self._health_factory()
            except Exception as e:  # noqa: BLE001 - no amd-smi (CPU box): serve without health events
                log.info("health watcher unavailable: %s", e)
                return
            log.info("health watcher live")
        by_index = {d.index: d for d in self.devices}
        while not self._stop.is_set():
            try:
                events = self._health_poll(self.cfg.health_poll_ms)
            except Exception as e:  # noqa: BLE001 - keep serving on a watcher error
                log.error("health poll failed: %s", e)
                self._stop.wait(1.0)
                continue
            for ev in events:
                d = by_index.get(ev.index)
                if d is None:
                    continue
                healthy = not ev.critical if ev.kind != "gpu_post_reset" else True
                if ev.critical or ev.kind == "gpu_post_reset":
                    for s in list(self.servers.values()):
                        s.set_health(d.device_id_str, healthy, f"{ev.kind}: {ev.message}")

    def set_health(self, device_id: str, healthy: bool, reason: str = "") -> None:
        for s in list(self.servers.values()):
            s.set_health(device_id, healthy, reason)

    def stop(self) -> None:
        self._stop.set()
        for s in self.servers.values():
            s.stop()
