"""Python view of the native device/topology library (N3/N4/N6).

``libamdgpu_topo.so`` (``native/topology``) enumerates MI355X GPUs from KFD /
PCI / DRM sysfs, collects amd-smi metrics and watches health events.  This
module turns its C structs into dataclasses for the control plane.  Every
function takes ``root`` so it runs unchanged against captured or synthetic
sysfs trees (``tests/fakesys.py``) - the MI355X counterpart of the NVML
queries behind ``nvidia-smi`` (/root/reference/README.md:152,158-167).
"""

from __future__ import annotations

import ctypes
import threading
from ..utils.record import asdict, field, record

from .. import native

LIB = "libamdgpu_topo.so"
LINK_PCIE = 2
LINK_XGMI = 11


class _Gpu(ctypes.Structure):
    _fields_ = [
        ("kfd_node", ctypes.c_int32),
        ("gpu_id", ctypes.c_uint32),
        ("gfx_target_version", ctypes.c_uint32),
        ("arch", ctypes.c_char * 16),
        ("simd_count", ctypes.c_uint32),
        ("simd_per_cu", ctypes.c_uint32),
        ("cu_count", ctypes.c_uint32),
        ("num_xcc", ctypes.c_uint32),
        ("max_waves_per_simd", ctypes.c_uint32),
        ("wave_front_size", ctypes.c_uint32),
        ("lds_size_kib", ctypes.c_uint32),
        ("max_engine_clk_mhz", ctypes.c_uint32),
        ("vram_bytes", ctypes.c_uint64),
        ("drm_render_minor", ctypes.c_uint32),
        ("domain", ctypes.c_uint32),
        ("location_id", ctypes.c_uint32),
        ("bdf", ctypes.c_char * 16),
        ("vendor_id", ctypes.c_uint32),
        ("device_id", ctypes.c_uint32),
        ("unique_id", ctypes.c_uint64),
        ("hive_id", ctypes.c_uint64),
        ("num_xgmi_links", ctypes.c_uint32),
        ("numa_node", ctypes.c_int32),
        ("physical_index", ctypes.c_int32),
        ("partition_index", ctypes.c_int32),
        ("partition_count", ctypes.c_int32),
        ("compute_partition", ctypes.c_char * 8),
        ("memory_partition", ctypes.c_char * 8),
    ]


class _Link(ctypes.Structure):
    _fields_ = [
        ("from_gpu", ctypes.c_int32),
        ("to_gpu", ctypes.c_int32),
        ("type", ctypes.c_uint32),
        ("weight", ctypes.c_uint32),
        ("min_bandwidth_mbps", ctypes.c_uint32),
        ("max_bandwidth_mbps", ctypes.c_uint32),
    ]


class _Metrics(ctypes.Structure):
    _fields_ = [
        ("index", ctypes.c_int32),
        ("bdf", ctypes.c_char * 16),
        ("uuid", ctypes.c_char * 64),
        ("market_name", ctypes.c_char * 64),
        ("vram_total_bytes", ctypes.c_uint64),
        ("vram_used_bytes", ctypes.c_uint64),
        ("gfx_activity_pct", ctypes.c_uint32),
        ("umc_activity_pct", ctypes.c_uint32),
        ("mm_activity_pct", ctypes.c_uint32),
        ("socket_power_w", ctypes.c_double),
        ("power_limit_w", ctypes.c_double),
        ("temp_hotspot_c", ctypes.c_double),
        ("temp_mem_c", ctypes.c_double),
        ("temp_edge_c", ctypes.c_double),
        ("gfx_clk_mhz", ctypes.c_uint32),
        ("mem_clk_mhz", ctypes.c_uint32),
        ("energy_j", ctypes.c_double),
        ("ecc_correctable", ctypes.c_uint64),
        ("ecc_uncorrectable", ctypes.c_uint64),
        ("ecc_deferred", ctypes.c_uint64),
        ("xgmi_links_total", ctypes.c_uint32),
        ("xgmi_links_up", ctypes.c_uint32),
        ("xgmi_links_error", ctypes.c_uint32),
        ("bad_pages", ctypes.c_uint32),
        ("num_processes", ctypes.c_uint32),
        ("xgmi_read_bytes", ctypes.c_uint64),
        ("xgmi_write_bytes", ctypes.c_uint64),
        ("pcie_bandwidth_gbps", ctypes.c_uint64),
        ("pcie_replay_count", ctypes.c_uint64),
        ("pcie_nak_sent", ctypes.c_uint64),
        ("pcie_nak_rcvd", ctypes.c_uint64),
        ("prochot_residency", ctypes.c_uint64),
        ("ppt_residency", ctypes.c_uint64),
        ("socket_thermal_residency", ctypes.c_uint64),
        ("hbm_thermal_residency", ctypes.c_uint64),
        ("vram_max_bandwidth_gbps", ctypes.c_uint64),
        ("xgmi_link_speed_gbps", ctypes.c_uint32),
        ("xgmi_link_width", ctypes.c_uint32),
        ("pcie_link_width", ctypes.c_uint32),
        ("pcie_link_speed_mts", ctypes.c_uint32),
        ("throttle_status", ctypes.c_uint32),
        ("valid_mask", ctypes.c_uint32),
    ]


class _Event(ctypes.Structure):
    _fields_ = [
        ("index", ctypes.c_int32),
        ("kind", ctypes.c_int32),
        ("critical", ctypes.c_int32),
        ("message", ctypes.c_char * 128),
    ]


M_VRAM, M_ACTIVITY, M_POWER, M_TEMP, M_CLOCK, M_ENERGY, M_ECC, M_XGMI, M_BADPAGES, M_PROCS, M_GPU_METRICS = (
    1 << i for i in range(11))

EVENT_NAMES = {
    1: "vm_fault",
    2: "thermal_throttle",
    3: "gpu_pre_reset",
    4: "gpu_post_reset",
    100: "ecc_uncorrectable",
    101: "xgmi_link_error",
    102: "device_lost",
    103: "bad_pages",
}


def _lib() -> ctypes.CDLL:
    lib = native.load(LIB)
    if getattr(lib, "_at_typed", False):
        return lib
    c = ctypes
    lib.at_abi_version.restype = c.c_int
    lib.at_enumerate.argtypes = [c.c_char_p, c.POINTER(_Gpu), c.c_int, c.POINTER(c.c_int)]
    lib.at_links.argtypes = [c.c_char_p, c.POINTER(_Link), c.c_int, c.POINTER(c.c_int)]
    lib.at_probe.argtypes = [c.c_char_p, c.c_int, c.c_char_p, c.c_int]
    lib.at_smi_open.restype = c.c_int
    lib.at_smi_count.restype = c.c_int
    lib.at_smi_collect.argtypes = [c.POINTER(_Metrics), c.c_int, c.POINTER(c.c_int)]
    lib.at_smi_driver_version.argtypes = [c.c_char_p, c.c_int]
    lib.at_smi_set_compute_partition.argtypes = [c.c_int, c.c_char_p]
    lib.at_smi_set_memory_partition.argtypes = [c.c_int, c.c_char_p]
    lib.at_smi_get_partitions.argtypes = [c.c_int, c.c_char_p, c.c_int, c.c_char_p, c.c_int]
    lib.at_health_poll.argtypes = [c.c_int, c.POINTER(_Event), c.c_int, c.POINTER(c.c_int)]
    lib._at_typed = True
    return lib


def _s(b: bytes) -> str:
    return b.decode("utf-8", "replace")


@record(frozen=True)
class GpuDevice:
    """One schedulable GPU (a whole MI355X in SPX, one partition in DPX/QPX/CPX)."""

    index: int
    kfd_node: int
    gpu_id: int
    arch: str
    gfx_target_version: int
    cu_count: int
    simd_count: int
    num_xcc: int
    lds_size_kib: int
    max_engine_clk_mhz: int
    vram_bytes: int
    render_minor: int
    bdf: str
    vendor_id: int
    device_id: int
    unique_id: int
    hive_id: int
    xgmi_links: int
    numa_node: int
    physical_index: int
    partition_index: int
    partition_count: int
    compute_partition: str
    memory_partition: str

    @property
    def render_node(self) -> str:
        return f"/dev/dri/renderD{self.render_minor}"

    @property
    def device_id_str(self) -> str:
        """Stable kubelet device ID: PCI BDF (+ partition suffix when partitioned)."""
        return self.bdf if self.partition_count <= 1 else f"{self.bdf}-p{self.partition_index}"

    def as_dict(self) -> dict:
        return asdict(self)


@record(frozen=True)
class GpuLink:
    src: int
    dst: int
    type: int
    weight: int
    min_bandwidth_mbps: int
    max_bandwidth_mbps: int

    @property
    def is_xgmi(self) -> bool:
        return self.type == LINK_XGMI


def _root(root: str | None) -> bytes:
    return (root or "/").encode()


def partition_resource(dev: GpuDevice, resource_name: str, strategy: str = "single") -> str:
    """Extended-resource name a device is advertised under: ``resource_name``,
    or ``<resource_name>-<mode>`` for a partitioned GPU under the ``mixed``
    strategy (the device plugin's and the validator's shared rule)."""
    if strategy == "mixed" and dev.partition_count > 1 and dev.compute_partition:
        return f"{resource_name}-{dev.compute_partition.lower()}"
    return resource_name


def enumerate_gpus(root: str | None = None) -> list[GpuDevice]:
    lib = _lib()
    n = ctypes.c_int(0)
    lib.at_enumerate(_root(root), None, 0, ctypes.byref(n))
    if n.value == 0:
        return []
    arr = (_Gpu * n.value)()
    cnt = ctypes.c_int(0)
    rc = lib.at_enumerate(_root(root), arr, n.value, ctypes.byref(cnt))
    if rc != 0:
        raise RuntimeError(f"at_enumerate failed rc={rc}")
    out = []
    for i in range(cnt.value):
        g = arr[i]
        out.append(GpuDevice(
            index=i, kfd_node=g.kfd_node, gpu_id=g.gpu_id, arch=_s(g.arch), gfx_target_version=g.gfx_target_version,
            cu_count=g.cu_count, simd_count=g.simd_count, num_xcc=g.num_xcc, lds_size_kib=g.lds_size_kib,
            max_engine_clk_mhz=g.max_engine_clk_mhz, vram_bytes=g.vram_bytes, render_minor=g.drm_render_minor,
            bdf=_s(g.bdf), vendor_id=g.vendor_id, device_id=g.device_id, unique_id=g.unique_id, hive_id=g.hive_id,
            xgmi_links=g.num_xgmi_links, numa_node=g.numa_node, physical_index=g.physical_index,
            partition_index=g.partition_index, partition_count=g.partition_count,
            compute_partition=_s(g.compute_partition), memory_partition=_s(g.memory_partition)))
    return out


def links(root: str | None = None) -> list[GpuLink]:
    lib = _lib()
    n = ctypes.c_int(0)
    lib.at_links(_root(root), None, 0, ctypes.byref(n))
    if n.value == 0:
        return []
    arr = (_Link * n.value)()
    cnt = ctypes.c_int(0)
    lib.at_links(_root(root), arr, n.value, ctypes.byref(cnt))
    return [GpuLink(l.from_gpu, l.to_gpu, l.type, l.weight, l.min_bandwidth_mbps, l.max_bandwidth_mbps)
            for l in arr[: cnt.value]]


def visible_devices_env(devices: list["GpuDevice"], all_devices: list["GpuDevice"] | None = None) -> dict:
    """Environment that limits a process's ROCm runtime to ``devices``.

    ``ROCR_VISIBLE_DEVICES`` with the GPUs' KFD unique ids (ROCr's
    "GPU-<id>" UUIDs) keeps the HSA runtime from initialising every other GPU
    of the node - at N = 8 a validator process otherwise sets up all eight
    agents, and 3N such processes start together (tools/storm_probe.py).
    Inside, the first listed device is HIP device 0.  Devices without a
    unique id, or ids shared by several devices (partitions of one GPU),
    fall back to HIP-level ordinals (``HIP_VISIBLE_DEVICES``: same device
    numbering inside, no runtime saving)."""
    ids = [d.unique_id for d in devices]
    seen = [d.unique_id for d in (all_devices or devices)]
    if all(ids) and all(seen.count(i) == 1 for i in ids):
        return {"ROCR_VISIBLE_DEVICES": ",".join(f"GPU-{i:016x}" for i in ids)}
    return {"HIP_VISIBLE_DEVICES": ",".join(str(d.index) for d in devices)}


def probe(root: str | None = None, expect_gpus: int = 0) -> tuple[bool, str]:
    """N1 driver readiness (amdgpu live, /dev/kfd, KFD GPU nodes, render nodes)."""
    buf = ctypes.create_string_buffer(256)
    rc = _lib().at_probe(_root(root), expect_gpus, buf, len(buf))
    return rc == 0, _s(buf.value)


@record
class GpuMetrics:
    index: int
    bdf: str
    uuid: str
    market_name: str
    values: dict = field(default_factory=dict)


_METRIC_FIELDS = {
    M_VRAM: ("vram_total_bytes", "vram_used_bytes"),
    M_ACTIVITY: ("gfx_activity_pct", "umc_activity_pct", "mm_activity_pct"),
    M_POWER: ("socket_power_w", "power_limit_w"),
    M_TEMP: ("temp_hotspot_c", "temp_mem_c", "temp_edge_c"),
    M_CLOCK: ("gfx_clk_mhz", "mem_clk_mhz"),
    M_ENERGY: ("energy_j",),
    M_ECC: ("ecc_correctable", "ecc_uncorrectable", "ecc_deferred"),
    M_XGMI: ("xgmi_links_total", "xgmi_links_up", "xgmi_links_error"),
    M_BADPAGES: ("bad_pages",),
    M_PROCS: ("num_processes",),
    M_GPU_METRICS: ("xgmi_read_bytes", "xgmi_write_bytes", "pcie_bandwidth_gbps", "pcie_replay_count", "pcie_nak_sent",
                    "pcie_nak_rcvd", "prochot_residency", "ppt_residency", "socket_thermal_residency",
                    "hbm_thermal_residency", "vram_max_bandwidth_gbps", "xgmi_link_speed_gbps", "xgmi_link_width",
                    "pcie_link_width", "pcie_link_speed_mts", "throttle_status"),
}


class Smi:
    """N4 collector handle (libamd_smi via the native library)."""

    def __init__(self):
        self._lib = _lib()
        rc = self._lib.at_smi_open()
        if rc != 0:
            raise native.NativeUnavailable(f"amd-smi unavailable (rc={rc})")
        self._open = True

    def close(self) -> None:
        if self._open:
            self._lib.at_smi_close()
            self._open = False

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def count(self) -> int:
        return max(0, self._lib.at_smi_count())

    def collect(self) -> list[GpuMetrics]:
        n = self.count()
        if n == 0:
            return []
        arr = (_Metrics * n)()
        cnt = ctypes.c_int(0)
        rc = self._lib.at_smi_collect(arr, n, ctypes.byref(cnt))
        if rc != 0:
            raise RuntimeError(f"at_smi_collect rc={rc}")
        out = []
        for m in arr[: cnt.value]:
            vals = {}
            for bit, names in _METRIC_FIELDS.items():
                if m.valid_mask & bit:
                    for nm in names:
                        vals[nm] = getattr(m, nm)
            out.append(GpuMetrics(m.index, _s(m.bdf), _s(m.uuid), _s(m.market_name), vals))
        return out

    def driver_version(self) -> str:
        buf = ctypes.create_string_buffer(256)
        return _s(buf.value) if self._lib.at_smi_driver_version(buf, len(buf)) == 0 else ""

    def partitions(self, index: int) -> tuple[str, str]:
        c = ctypes.create_string_buffer(32)
        m = ctypes.create_string_buffer(32)
        self._lib.at_smi_get_partitions(index, c, 32, m, 32)
        return _s(c.value), _s(m.value)

    def set_compute_partition(self, index: int, mode: str) -> int:
        return self._lib.at_smi_set_compute_partition(index, mode.encode())

    def set_memory_partition(self, index: int, mode: str) -> int:
        return self._lib.at_smi_set_memory_partition(index, mode.encode())


@record(frozen=True)
class HealthEvent:
    index: int
    kind: str
    critical: bool
    message: str


class HealthWatcher:
    """N6: amd-smi event notifications + ECC/xGMI/bad-page deltas."""

    def __init__(self):
        self._lib = _lib()
        rc = self._lib.at_health_start()
        if rc != 0:
            raise native.NativeUnavailable(f"health watcher unavailable (rc={rc})")

    def poll(self, timeout_ms: int = 1000) -> list[HealthEvent]:
        arr = (_Event * 64)()
        cnt = ctypes.c_int(0)
        self._lib.at_health_poll(timeout_ms, arr, 64, ctypes.byref(cnt))
        return [HealthEvent(e.index, EVENT_NAMES.get(e.kind, str(e.kind)), bool(e.critical), _s(e.message))
                for e in arr[: min(cnt.value, 64)]]

    def close(self) -> None:
        self._lib.at_health_stop()


class HealthHub:
    """One N6 event client per process, fanned out to every subscriber.

    amd-smi delivers each event notification to one reader, and N6's counter
    deltas are computed against one baseline, so two watchers in a process
    (the device plugin's health loop and the exporter's XID-equivalent
    series, both threads of one process in the simulated cluster's thread
    mode) would split the stream between them.  The hub owns the only
    :class:`HealthWatcher`, polls it on one thread, and queues every event
    for each :class:`HealthSubscription`; the watcher closes when the last
    subscription does.  ``factory`` builds the watcher (tests pass a fake)."""

    _lock = threading.Lock()
    _inst: "HealthHub | None" = None

    def __init__(self, factory):
        self._watcher = factory()
        self._subs: list[HealthSubscription] = []
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._run, name="amdgpu-health-hub", daemon=True)
        self._thread.start()

    @classmethod
    def subscribe(cls, factory=None) -> "HealthSubscription":
        """A new subscription on the process's hub (started on first use;
        raises what the watcher raises when amd-smi is unavailable)."""
        with cls._lock:
            if cls._inst is None:
                cls._inst = HealthHub(factory or HealthWatcher)
            sub = HealthSubscription(cls._inst)
            cls._inst._subs.append(sub)
            return sub

    def _release(self, sub: "HealthSubscription") -> None:
        with HealthHub._lock:
            if sub in self._subs:
                self._subs.remove(sub)
            if self._subs or HealthHub._inst is not self:
                return
            HealthHub._inst = None
        self._stop.set()
        self._thread.join(timeout=5.0)
        try:
            self._watcher.close()
        except Exception:  # noqa: BLE001 - closing a watcher of a vanished device
            pass

    def _run(self) -> None:
        while not self._stop.is_set():
            try:
                events = self._watcher.poll(200)
            except Exception as e:  # noqa: BLE001 - handed to every subscriber's poll
                events = e
            with HealthHub._lock:
                subs = list(self._subs)
            if isinstance(events, Exception):
                for s in subs:
                    s._q.put(events)
                self._stop.wait(1.0)
                continue
            if events:
                for s in subs:
                    s._q.put(list(events))


class HealthSubscription:
    """A subscriber's view of the process's :class:`HealthHub`: ``poll``
    has :meth:`HealthWatcher.poll`'s signature and returns every event since
    the previous call (waiting up to ``timeout_ms`` for the first)."""

    def __init__(self, hub: HealthHub):
        import queue

        self._hub = hub
        self._q: "queue.Queue[list[HealthEvent] | Exception]" = queue.Queue()
        self._closed = False

    def poll(self, timeout_ms: int = 1000) -> list[HealthEvent]:
        import queue

        out: list[HealthEvent] = []
        try:
            item = self._q.get(timeout=max(0.0, timeout_ms / 1000.0))
        except queue.Empty:
            return out
        while True:
            if isinstance(item, Exception):
                if out:
                    return out
                raise item
            out.extend(item)
            try:
                item = self._q.get_nowait()
            except queue.Empty:
                return out

    def close(self) -> None:
        if not self._closed:
            self._closed = True
            self._hub._release(self)
