"""In-process fake kubelet: device-plugin Registration server + device manager
+ pod-resources server, over real gRPC on unix sockets.

Used by the contract tests, the fake-cluster integration and the bench
(neither kind nor kubectl exists in the build environment).
It behaves like kubelet's device manager where the plugin can observe it:

* serves ``v1beta1.Registration/Register`` on ``<dir>/kubelet.sock``;
* on registration dials ``<dir>/<endpoint>``, calls GetDevicePluginOptions and
  keeps a ``ListAndWatch`` stream open, updating the resource's device health;
* ``allocatable(resource)`` = healthy devices (what lands in node
  ``status.allocatable``, /root/reference/README.md:122);
* ``allocate(resource, n, pod)`` = GetPreferredAllocation (if offered) over the
  free healthy devices, then Allocate; assignments are remembered (the
  checkpoint) and exposed through ``v1.PodResourcesLister/List``;
* ``restart()`` re-creates ``kubelet.sock`` (new inode) and forgets
  registrations, like a kubelet restart.
"""

from __future__ import annotations

import json
import os
import threading
import time
from concurrent import futures
from dataclasses import dataclass, field

import grpc

from ..deviceplugin import api


@dataclass
class _Resource:
    name: str
    endpoint: str
    channel: grpc.Channel
    options: object
    devices: dict = field(default_factory=dict)  # id -> health
    numa: dict = field(default_factory=dict)
    updates: int = 0
    stream_thread: threading.Thread | None = None
    cv: threading.Condition = field(default_factory=threading.Condition)


class FakeKubelet:
    def __init__(self, socket_dir: str, pod_resources_socket: str | None = None):
        self.dir = socket_dir
        self.sock = os.path.join(socket_dir, "kubelet.sock")
        self.podres_sock = pod_resources_socket
        self.resources: dict[str, _Resource] = {}
        self.assignments: dict[tuple[str, str, str], tuple[str, list[str]]] = {}  # (ns,pod,ctr) -> (res, ids)
        # (ns,pod,ctr) -> DRA claims the DRA manager prepared for it:
        # [{"claim": (ns, name), "resources": [(driver, pool, device, [cdi ids])]}]
        self.claims: dict[tuple[str, str, str], list[dict]] = {}
        self.register_calls = 0
        self.register_seconds: list[float] = []  # handler time per Register call
        self.register_walls: list[float] = []  # wall time each Register call arrived
        self.first_list_walls: dict[str, float] = {}  # resource -> wall time of its first ListAndWatch answer
        self._lock = threading.Lock()
        self._alloc_lock = threading.Lock()
        self._server: grpc.Server | None = None
        self._podres_server: grpc.Server | None = None
        self._registered = threading.Condition()

    # ----------------------------------------------------------- Registration
    def _register(self, request, context):
        t0 = time.perf_counter()
        self.register_walls.append(time.time())
        if request.version != api.VERSION:
            context.abort(grpc.StatusCode.INVALID_ARGUMENT, f"unsupported version {request.version}")
        ep = os.path.join(self.dir, request.endpoint)
        ch = grpc.insecure_channel("unix:" + ep)
        opt_req, opt_resp, _ = api.DEVICE_PLUGIN_METHODS["GetDevicePluginOptions"]
        opts = ch.unary_unary(api.method_path(api.DEVICE_PLUGIN_SERVICE, "GetDevicePluginOptions"),
                              request_serializer=opt_req.SerializeToString,
                              response_deserializer=opt_resp.FromString)(opt_req(), timeout=5, wait_for_ready=True)
        res = _Resource(request.resource_name, request.endpoint, ch, opts)
        with self._lock:
            old = self.resources.get(request.resource_name)
            self.resources[request.resource_name] = res
            self.register_calls += 1
        if old is not None:
            old.channel.close()
        res.stream_thread = threading.Thread(target=self._watch, args=(res,), daemon=True,
                                             name=f"fake-kubelet-law-{request.resource_name}")
        res.stream_thread.start()
        with self._registered:
            self._registered.notify_all()
        self.register_seconds.append(time.perf_counter() - t0)
        return api.pb["Empty"]()

    def _watch(self, res: _Resource) -> None:
        req, resp, _ = api.DEVICE_PLUGIN_METHODS["ListAndWatch"]
        stream = res.channel.unary_stream(api.method_path(api.DEVICE_PLUGIN_SERVICE, "ListAndWatch"),
                                          request_serializer=req.SerializeToString, response_deserializer=resp.FromString)
        try:
            for msg in stream(req(), wait_for_ready=True):
                self.first_list_walls.setdefault(res.name, time.time())
                with res.cv:
                    res.devices = {d.ID: d.health for d in msg.devices}
                    res.numa = {d.ID: [n.ID for n in d.topology.nodes] for d in msg.devices}
                    res.updates += 1
                    res.cv.notify_all()
                self._write_checkpoint()
        except grpc.RpcError:
            pass  # plugin went away or channel closed
        with self._lock:
            current = self.resources.get(res.name) is res
        if current:  # endpoint gone without a new registration: kubelet marks its devices unhealthy
            with res.cv:
                res.devices = {i: api.UNHEALTHY for i in res.devices}
                res.updates += 1
                res.cv.notify_all()

    CHECKPOINT = "kubelet_internal_checkpoint"

    def _write_checkpoint(self) -> None:
        """Like the kubelet's device manager: every device-list update and
        allocation is checkpointed in the device-plugins directory (temp file
        + rename), which is what a watcher of that directory sees."""
        with self._lock:
            data = {"RegisteredDevices": {r: list(res.devices) for r, res in self.resources.items()},
                    "PodDeviceEntries": [{"PodUID": f"{k[0]}/{k[1]}", "ContainerName": k[2], "ResourceName": v[0],
                                          "DeviceIDs": list(v[1])} for k, v in self.assignments.items()]}
        path = os.path.join(self.dir, self.CHECKPOINT)
        tmp = f"{path}.tmp.{threading.get_ident()}"
        try:
            with open(tmp, "w") as f:
                json.dump({"Data": data}, f)
            os.replace(tmp, path)
        except OSError:
            pass

    # -------------------------------------------------------------- lifecycle
    def start(self) -> None:
        os.makedirs(self.dir, exist_ok=True)
        if os.path.exists(self.sock):
            os.unlink(self.sock)
        req, resp, _ = api.REGISTRATION_METHODS["Register"]
        handler = grpc.method_handlers_generic_handler(api.REGISTRATION_SERVICE, {
            "Register": grpc.unary_unary_rpc_method_handler(self._register, request_deserializer=req.FromString,
                                                            response_serializer=resp.SerializeToString)})
        self._server = grpc.server(futures.ThreadPoolExecutor(max_workers=4, thread_name_prefix="fake-kubelet"))
        self._server.add_generic_rpc_handlers((handler,))
        self._server.add_insecure_port("unix:" + self.sock)
        self._server.start()
        if self.podres_sock:
            self._start_podres()

    def _start_podres(self) -> None:
        os.makedirs(os.path.dirname(self.podres_sock), exist_ok=True)
        if os.path.exists(self.podres_sock):
            os.unlink(self.podres_sock)
        handlers = {}
        for name, (req, resp, _) in api.POD_RESOURCES_METHODS.items():
            fn = self._podres_list if name == "List" else self._podres_allocatable
            handlers[name] = grpc.unary_unary_rpc_method_handler(fn, request_deserializer=req.FromString,
                                                                 response_serializer=resp.SerializeToString)
        self._podres_server = grpc.server(futures.ThreadPoolExecutor(max_workers=2))
        self._podres_server.add_generic_rpc_handlers(
            (grpc.method_handlers_generic_handler(api.POD_RESOURCES_SERVICE, handlers),))
        self._podres_server.add_insecure_port("unix:" + self.podres_sock)
        self._podres_server.start()

    def _podres_list(self, request, context):
        out = api.podres["ListPodResourcesResponse"]()
        pods: dict[tuple[str, str], object] = {}
        with self._lock:
            items = list(self.assignments.items())
            claims = dict(self.claims)
        ctrs: dict[tuple[str, str, str], object] = {}

        def container(ns, pod, ctr):
            if (ns, pod, ctr) not in ctrs:
                pr = pods.get((ns, pod))
                if pr is None:
                    pr = pods[(ns, pod)] = out.pod_resources.add(name=pod, namespace=ns)
                ctrs[(ns, pod, ctr)] = pr.containers.add(name=ctr)
            return ctrs[(ns, pod, ctr)]

        for (ns, pod, ctr), (res, ids) in items:
            container(ns, pod, ctr).devices.add(resource_name=res, device_ids=ids)
        for (ns, pod, ctr), held in claims.items():
            c = container(ns, pod, ctr)
            for h in held:
                dr = c.dynamic_resources.add(claim_namespace=h["claim"][0], claim_name=h["claim"][1])
                for drv, pool, dev, cdi in h["resources"]:
                    cr = dr.claim_resources.add(driver_name=drv, pool_name=pool, device_name=dev)
                    for n in cdi:
                        cr.cdi_devices.add(name=n)
        return out

    def _podres_allocatable(self, request, context):
        out = api.podres["AllocatableResourcesResponse"]()
        for name, res in list(self.resources.items()):
            with res.cv:  # like the kubelet's device manager: every reported device, healthy or not
                ids = list(res.devices)
            out.devices.add(resource_name=name, device_ids=ids)
        return out

    def stop(self) -> None:
        for srv in (self._server, self._podres_server):
            if srv is not None:
                srv.stop(grace=0.2).wait()
        self._server = self._podres_server = None
        with self._lock:
            for r in self.resources.values():
                r.channel.close()

    def restart(self) -> None:
        """kubelet restart: registrations are lost; kubelet.sock gets a new inode."""
        self.stop()
        with self._lock:
            self.resources.clear()
        self.start()

    # ------------------------------------------------------------------ views
    def wait_registered(self, resource: str, timeout: float = 10.0, min_devices: int = 0) -> bool:
        import time

        deadline = time.monotonic() + timeout
        with self._registered:
            while resource not in self.resources:
                left = deadline - time.monotonic()
                if left <= 0:
                    return False
                self._registered.wait(left)
        res = self.resources[resource]
        with res.cv:
            while res.updates == 0 or len(res.devices) < min_devices:
                left = deadline - time.monotonic()
                if left <= 0:
                    return False
                res.cv.wait(left)
        return True

    def wait_update(self, resource: str, after: int, timeout: float = 10.0) -> bool:
        import time

        res = self.resources[resource]
        deadline = time.monotonic() + timeout
        with res.cv:
            while res.updates <= after:
                left = deadline - time.monotonic()
                if left <= 0:
                    return False
                res.cv.wait(left)
        return True

    def capacity(self, resource: str) -> int:
        res = self.resources.get(resource)
        return 0 if res is None else len(res.devices)

    def allocatable(self, resource: str) -> int:
        res = self.resources.get(resource)
        if res is None:
            return 0
        with res.cv:
            return sum(1 for h in res.devices.values() if h == api.HEALTHY)

    def free_devices(self, resource: str) -> list[str]:
        res = self.resources[resource]
        with self._lock:
            used = {i for (r, ids) in self.assignments.values() if r == resource for i in ids}
        with res.cv:
            return [i for i, h in res.devices.items() if h == api.HEALTHY and i not in used]

    # ------------------------------------------------------------- allocation
    def allocate(self, resource: str, count: int, namespace: str = "default", pod: str = "pod",
                 container: str = "main", must_include: list[str] | None = None):
        # kubelet's device manager admits one pod at a time (devicemanager mutex)
        with self._alloc_lock:
            return self._allocate(resource, count, namespace, pod, container, must_include)

    def _allocate(self, resource, count, namespace, pod, container, must_include):
        res = self.resources[resource]
        free = self.free_devices(resource)
        if count > len(free):
            with self._lock:
                holders = sorted({k[1] for k, (r, _) in self.assignments.items() if r == resource})
            raise RuntimeError(f"insufficient {resource}: want {count}, free {len(free)} "
                               f"(devices {len(res.devices)}, healthy {self.allocatable(resource)}, held by {holders})")
        ids = free[:count]
        if res.options.get_preferred_allocation_available:
            req, resp, _ = api.DEVICE_PLUGIN_METHODS["GetPreferredAllocation"]
            call = res.channel.unary_unary(api.method_path(api.DEVICE_PLUGIN_SERVICE, "GetPreferredAllocation"),
                                           request_serializer=req.SerializeToString, response_deserializer=resp.FromString)
            r = req()
            r.container_requests.add(available_deviceIDs=free, must_include_deviceIDs=must_include or [],
                                     allocation_size=count)
            pref = list(call(r, timeout=5).container_responses[0].deviceIDs)
            if len(pref) == count and set(pref) <= set(free):
                ids = pref
        req, resp, _ = api.DEVICE_PLUGIN_METHODS["Allocate"]
        call = res.channel.unary_unary(api.method_path(api.DEVICE_PLUGIN_SERVICE, "Allocate"),
                                       request_serializer=req.SerializeToString, response_deserializer=resp.FromString)
        r = req()
        r.container_requests.add(devices_ids=ids)
        out = call(r, timeout=5)
        with self._lock:
            self.assignments[(namespace, pod, container)] = (resource, ids)
        self._write_checkpoint()
        return ids, out.container_responses[0]

    def release(self, namespace: str, pod: str) -> None:
        with self._lock:
            for k in [k for k in self.assignments if k[0] == namespace and k[1] == pod]:
                del self.assignments[k]
            for k in [k for k in self.claims if k[0] == namespace and k[1] == pod]:
                del self.claims[k]

    def record_claims(self, namespace: str, pod: str, container: str, held: list[dict]) -> None:
        """The DRA manager prepared ``held`` for this container (what
        pod-resources List reports as its dynamic_resources)."""
        with self._lock:
            self.claims[(namespace, pod, container)] = held
