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

The plugin is stateless: kubelet checkpoints assignments.
"""

from __future__ import annotations

import logging
import os
import threading
import time
from concurrent import futures
from dataclasses import dataclass, field
from typing import Callable

import grpc

from .. import RESOURCE_NAME
from . import api
from .allocator import from_topology, preferred

log = logging.getLogger("amdgpu.deviceplugin")


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

    @property
    def kubelet_path(self) -> str:
        return self.kubelet_socket or os.path.join(self.socket_dir, "kubelet.sock")

    @property
    def endpoint_path(self) -> str:
        return os.path.join(self.socket_dir, self.endpoint)


def resource_for(dev, cfg: PluginConfig) -> str:
    """Resource name of a device under the partition strategy.

    ``single``: every device (whole GPU or partition) is ``amd.com/gpu``.
    ``mixed``: partitioned devices are ``amd.com/gpu-<mode>`` (e.g. ``-cpx``)."""
    if cfg.partition_strategy == "mixed" and dev.partition_count > 1 and dev.compute_partition:
        return f"{cfg.resource_name}-{dev.compute_partition.lower()}"
    return cfg.resource_name


class DevicePluginServer:
    """One kubelet device-plugin endpoint serving one resource name."""

    def __init__(self, cfg: PluginConfig, devices, links=(), resource_name: str | None = None):
        self.cfg = cfg
        self.resource_name = resource_name or cfg.resource_name
        self.devices = list(devices)
        self._by_id = {d.device_id_str: d for d in self.devices}
        self._health = {d.device_id_str: api.HEALTHY for d in self.devices}
        self._cost = from_topology(self.devices, links, lambda g: g.device_id_str)
        self._cv = threading.Condition()
        self._version = 0
        self._stop = threading.Event()
        self._server: grpc.Server | None = None
        self._watch_thread: threading.Thread | None = None
        self._kubelet_ino = None
        self.registrations = 0
        self.allocations = 0
        self.events: list[dict] = []

    # ------------------------------------------------------------------ health
    def set_health(self, device_id: str, healthy: bool, reason: str = "") -> None:
        state = api.HEALTHY if healthy else api.UNHEALTHY
        with self._cv:
            if device_id not in self._health or self._health[device_id] == state:
                return
            self._health[device_id] = state
            self._version += 1
            self.events.append({"t": time.time(), "device": device_id, "health": state, "reason": reason})
            self._cv.notify_all()
        log.warning("device %s -> %s %s", device_id, state, reason)

    def healthy_count(self) -> int:
        with self._cv:
            return sum(1 for h in self._health.values() if h == api.HEALTHY)

    def device_list(self):
        with self._cv:
            resp = api.pb["ListAndWatchResponse"]()
            for d in self.devices:
                dev = resp.devices.add(ID=d.device_id_str, health=self._health[d.device_id_str])
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
            ids = preferred(self._cost, avail, list(creq.must_include_deviceIDs), creq.allocation_size)
            out.container_responses.add(deviceIDs=ids)
        return out

    def container_response(self, ids):
        r = api.pb["ContainerAllocateResponse"]()
        devs = [self._by_id[i] for i in ids]
        r.devices.add(container_path="/dev/kfd", host_path="/dev/kfd", permissions="rw")
        for d in devs:
            r.devices.add(container_path=d.render_node, host_path=d.render_node, permissions="rw")
        indices = ",".join(str(d.index) for d in devs)
        r.envs["AMD_VISIBLE_DEVICES"] = indices
        r.envs["AMD_GPU_DEVICE_IDS"] = ",".join(ids)
        for k, v in self.cfg.extra_env.items():
            r.envs[k] = v
        r.annotations["amd.com/gpu.devices"] = indices
        r.annotations["amd.com/gpu.memory-bytes"] = ",".join(str(d.vram_bytes) for d in devs)
        hives = sorted({str(d.hive_id) for d in devs if d.hive_id})
        if hives:
            r.annotations["amd.com/gpu.xgmi-hive"] = ",".join(hives)
        if self.cfg.rocm_mount:
            r.mounts.add(container_path=self.cfg.rocm_mount, host_path=self.cfg.rocm_mount, read_only=True)
        if self.cfg.cdi_enabled:
            for d in devs:
                r.cdi_devices.add(name=f"{self.cfg.cdi_kind}={d.index}")
        return r

    def Allocate(self, request, context):
        out = api.pb["AllocateResponse"]()
        for creq in request.container_requests:
            ids = list(creq.devices_ids)
            unknown = [i for i in ids if i not in self._by_id]
            if unknown:
                context.abort(grpc.StatusCode.INVALID_ARGUMENT, f"unknown device ids {unknown}")
            with self._cv:
                bad = [i for i in ids if self._health[i] != api.HEALTHY]
            if bad:
                context.abort(grpc.StatusCode.FAILED_PRECONDITION, f"unhealthy devices {bad}")
            out.container_responses.append(self.container_response(ids))
        self.allocations += 1
        return out

    def PreStartContainer(self, request, context):
        return api.pb["PreStartContainerResponse"]()

    # --------------------------------------------------------------- lifecycle
    def _handlers(self):
        handlers = {}
        for name, (req, resp, stream) in api.DEVICE_PLUGIN_METHODS.items():
            fn = getattr(self, name)
            mk = grpc.unary_stream_rpc_method_handler if stream else grpc.unary_unary_rpc_method_handler
            handlers[name] = mk(fn, request_deserializer=req.FromString, response_serializer=resp.SerializeToString)
        return grpc.method_handlers_generic_handler(api.DEVICE_PLUGIN_SERVICE, handlers)

    def serve(self) -> None:
        os.makedirs(self.cfg.socket_dir, exist_ok=True)
        path = os.path.join(self.cfg.socket_dir, self._endpoint())
        if os.path.exists(path):
            os.unlink(path)
        self._server = grpc.server(futures.ThreadPoolExecutor(max_workers=8, thread_name_prefix="amdgpu-dp"))
        self._server.add_generic_rpc_handlers((self._handlers(),))
        self._server.add_insecure_port("unix:" + path)
        self._server.start()

    def _endpoint(self) -> str:
        if self.resource_name == self.cfg.resource_name:
            return self.cfg.endpoint
        return self.cfg.endpoint.replace(".sock", "-" + self.resource_name.rsplit("-", 1)[-1] + ".sock")

    def register(self, timeout: float = 5.0) -> None:
        with grpc.insecure_channel("unix:" + self.cfg.kubelet_path) as ch:
            req_cls, resp_cls, _ = api.REGISTRATION_METHODS["Register"]
            call = ch.unary_unary(api.method_path(api.REGISTRATION_SERVICE, "Register"),
                                  request_serializer=req_cls.SerializeToString, response_deserializer=resp_cls.FromString)
            req = req_cls(version=api.VERSION, endpoint=self._endpoint(), resource_name=self.resource_name)
            req.options.get_preferred_allocation_available = True
            call(req, timeout=timeout, wait_for_ready=True)
        self.registrations += 1
        self._kubelet_ino = self._kubelet_identity()
        log.info("registered %s with kubelet (%d devices)", self.resource_name, len(self.devices))

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
            ident = self._kubelet_identity()
            if ident is None:
                self._kubelet_ino = None  # socket gone: re-register when it returns
                continue
            if ident != self._kubelet_ino:
                try:
                    self.register()
                except grpc.RpcError as e:  # kubelet not ready yet: retry next tick
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
                 health_poll: Callable[[int], list] | None = None):
        from ..discovery import topology

        self.cfg = cfg
        self.devices = devices if devices is not None else topology.enumerate_gpus(cfg.sysfs_root)
        self.links = links if links is not None else topology.links(cfg.sysfs_root)
        groups: dict[str, list] = {}
        for d in self.devices:
            groups.setdefault(resource_for(d, cfg), []).append(d)
        self.servers = {r: DevicePluginServer(cfg, devs, self.links, r) for r, devs in groups.items()}
        self._health_poll = health_poll
        self._stop = threading.Event()
        self._thread: threading.Thread | None = None

    def start(self, register: bool = True) -> None:
        for s in self.servers.values():
            s.start(register=register)
        if self._health_poll is not None:
            self._thread = threading.Thread(target=self._health_loop, name="amdgpu-dp-health", daemon=True)
            self._thread.start()

    def _health_loop(self) -> None:
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
                    for s in self.servers.values():
                        s.set_health(d.device_id_str, healthy, f"{ev.kind}: {ev.message}")

    def set_health(self, device_id: str, healthy: bool, reason: str = "") -> None:
        for s in self.servers.values():
            s.set_health(device_id, healthy, reason)

    def stop(self) -> None:
        self._stop.set()
        for s in self.servers.values():
            s.stop()
