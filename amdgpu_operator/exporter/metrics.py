"""GPU metrics exporter (DCGM-exporter equivalent, C9) and node-status
exporter (C8), both serving Prometheus text format on ``/metrics``.

Reference parity: ``nvidia-dcgm-exporter`` "collects GPU metrics for
monitoring" (/root/reference/README.md:204,213) and ``nodeStatusExporter`` is
enabled (README.md:107).  The MI355X exporter reads every GPU through the N4
native collector (libamd_smi, one native call per interval for all GPUs and
fields), attributes GPUs to pods through the kubelet pod-resources API, and
caches the snapshot so a scrape never touches the hardware.

Metric names (``amd_gpu_*``) and their DCGM counterparts
(``--dcgm-names`` additionally emits the DCGM_FI_DEV_* aliases):

====================================  ==================================
amd_gpu_gfx_activity_percent          DCGM_FI_DEV_GPU_UTIL
amd_gpu_umc_activity_percent          DCGM_FI_DEV_MEM_COPY_UTIL
amd_gpu_vram_used_bytes / _free       DCGM_FI_DEV_FB_USED / _FREE (MiB)
amd_gpu_power_watts                   DCGM_FI_DEV_POWER_USAGE
amd_gpu_energy_joules_total           DCGM_FI_DEV_TOTAL_ENERGY_CONSUMPTION (mJ)
amd_gpu_temperature_hotspot_celsius   DCGM_FI_DEV_GPU_TEMP
amd_gpu_temperature_memory_celsius    DCGM_FI_DEV_MEMORY_TEMP
amd_gpu_gfx_clock_mhz / mem_clock     DCGM_FI_DEV_SM_CLOCK / _MEM_CLOCK
amd_gpu_ecc_uncorrectable_total       DCGM_FI_DEV_ECC_DBE_VOL_TOTAL
amd_gpu_ecc_correctable_total         DCGM_FI_DEV_ECC_SBE_VOL_TOTAL
amd_gpu_retired_pages                 DCGM_FI_DEV_RETIRED_DBE
amd_gpu_xgmi_links_up / _link_errors  DCGM_FI_DEV_NVLINK_* (link health)
amd_gpu_xgmi_{read,write}_bytes_total (NVLink traffic: per-GPU xGMI bytes)
amd_gpu_pcie_replay_total             DCGM_FI_DEV_PCIE_REPLAY_COUNTER
amd_gpu_pcie_link_width               DCGM_FI_DEV_PCIE_LINK_WIDTH
amd_gpu_throttle_*_residency_total    (DCGM_FI_DEV_*_VIOLATION analogs)
amd_gpu_last_critical_event_code      DCGM_FI_DEV_XID_ERRORS (last critical
                                      N6 event; :class:`HealthCounters`)
amd_gpu_reset_total, _vm_fault_total, (XID-class events, per GPU)
_*_events_total, _health_critical
====================================  ==================================

Metric selection (``--metrics-config`` / ``dcgmExporter.config``): the
dcgm-exporter counters CSV format, one ``NAME, type, help`` line per series.
NAME is an ``amd_gpu_*`` metric or the DCGM field it stands for, so an existing
dcgm-exporter CSV keeps producing the series its dashboards query; DCGM fields
with no MI355X source (e.g. ENC/DEC utilisation) are reported and skipped.
"""

from __future__ import annotations

import json
import os
import threading
import time
from dataclasses import dataclass
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

from ..utils.logs import get_logger

log = get_logger("amdgpu.exporter")

# (metric, field, type, help, dcgm alias, dcgm scale)
FIELDS = [
    ("amd_gpu_gfx_activity_percent", "gfx_activity_pct", "gauge", "Graphics/compute engine activity (%)",
     "DCGM_FI_DEV_GPU_UTIL", 1.0),
    ("amd_gpu_umc_activity_percent", "umc_activity_pct", "gauge", "Memory controller activity (%)",
     "DCGM_FI_DEV_MEM_COPY_UTIL", 1.0),
    ("amd_gpu_mm_activity_percent", "mm_activity_pct", "gauge", "Multimedia engine activity (%)", None, 1.0),
    ("amd_gpu_vram_total_bytes", "vram_total_bytes", "gauge", "HBM capacity (bytes)", None, 1.0),
    ("amd_gpu_vram_used_bytes", "vram_used_bytes", "gauge", "HBM in use (bytes)", "DCGM_FI_DEV_FB_USED", 1 / 2**20),
    ("amd_gpu_vram_free_bytes", "vram_free_bytes", "gauge", "HBM free (bytes)", "DCGM_FI_DEV_FB_FREE", 1 / 2**20),
    ("amd_gpu_power_watts", "socket_power_w", "gauge", "Socket power (W)", "DCGM_FI_DEV_POWER_USAGE", 1.0),
    ("amd_gpu_power_limit_watts", "power_limit_w", "gauge", "Socket power limit (W)", None, 1.0),
    ("amd_gpu_temperature_hotspot_celsius", "temp_hotspot_c", "gauge", "Hotspot temperature (C)",
     "DCGM_FI_DEV_GPU_TEMP", 1.0),
    ("amd_gpu_temperature_memory_celsius", "temp_mem_c", "gauge", "HBM temperature (C)", "DCGM_FI_DEV_MEMORY_TEMP", 1.0),
    ("amd_gpu_temperature_edge_celsius", "temp_edge_c", "gauge", "Edge temperature (C)", None, 1.0),
    ("amd_gpu_gfx_clock_mhz", "gfx_clk_mhz", "gauge", "Graphics clock (MHz)", "DCGM_FI_DEV_SM_CLOCK", 1.0),
    ("amd_gpu_mem_clock_mhz", "mem_clk_mhz", "gauge", "Memory clock (MHz)", "DCGM_FI_DEV_MEM_CLOCK", 1.0),
    ("amd_gpu_energy_joules_total", "energy_j", "counter", "Energy consumed (J)",
     "DCGM_FI_DEV_TOTAL_ENERGY_CONSUMPTION", 1000.0),
    ("amd_gpu_ecc_correctable_total", "ecc_correctable", "counter", "Correctable ECC errors",
     "DCGM_FI_DEV_ECC_SBE_VOL_TOTAL", 1.0),
    ("amd_gpu_ecc_uncorrectable_total", "ecc_uncorrectable", "counter", "Uncorrectable ECC errors",
     "DCGM_FI_DEV_ECC_DBE_VOL_TOTAL", 1.0),
    ("amd_gpu_ecc_deferred_total", "ecc_deferred", "counter", "Deferred ECC errors", None, 1.0),
    ("amd_gpu_xgmi_links_total", "xgmi_links_total", "gauge", "xGMI links", None, 1.0),
    ("amd_gpu_xgmi_links_up", "xgmi_links_up", "gauge", "xGMI links up", None, 1.0),
    ("amd_gpu_xgmi_link_errors", "xgmi_links_error", "gauge", "xGMI links in error", None, 1.0),
    ("amd_gpu_retired_pages", "bad_pages", "gauge", "Retired (bad) HBM pages", "DCGM_FI_DEV_RETIRED_DBE", 1.0),
    ("amd_gpu_processes", "num_processes", "gauge", "Processes using the GPU", None, 1.0),
    # PMFW metrics table (amdsmi_get_gpu_metrics_info)
    ("amd_gpu_xgmi_read_bytes_total", "xgmi_read_bytes", "counter", "Bytes read over xGMI, all links", None, 1.0),
    ("amd_gpu_xgmi_write_bytes_total", "xgmi_write_bytes", "counter", "Bytes written over xGMI, all links", None, 1.0),
    ("amd_gpu_xgmi_link_speed_gbps", "xgmi_link_speed_gbps", "gauge", "xGMI link bit rate (Gb/s)", None, 1.0),
    ("amd_gpu_pcie_bandwidth_gbps", "pcie_bandwidth_gbps", "gauge", "PCIe bandwidth, instantaneous (GB/s)", None, 1.0),
    ("amd_gpu_pcie_replay_total", "pcie_replay_count", "counter", "PCIe replays",
     "DCGM_FI_DEV_PCIE_REPLAY_COUNTER", 1.0),
    ("amd_gpu_pcie_nak_sent_total", "pcie_nak_sent", "counter", "PCIe NAKs sent", None, 1.0),
    ("amd_gpu_pcie_nak_received_total", "pcie_nak_rcvd", "counter", "PCIe NAKs received", None, 1.0),
    ("amd_gpu_pcie_link_width", "pcie_link_width", "gauge", "PCIe link width (lanes)", "DCGM_FI_DEV_PCIE_LINK_WIDTH",
     1.0),
    ("amd_gpu_pcie_link_speed_mts", "pcie_link_speed_mts", "gauge", "PCIe link speed (MT/s)", None, 1.0),
    ("amd_gpu_throttle_prochot_residency_total", "prochot_residency", "counter", "PROCHOT throttle residency",
     None, 1.0),
    ("amd_gpu_throttle_ppt_residency_total", "ppt_residency", "counter", "Package power throttle residency", None,
     1.0),
    ("amd_gpu_throttle_socket_thermal_residency_total", "socket_thermal_residency", "counter",
     "Socket thermal throttle residency", None, 1.0),
    ("amd_gpu_throttle_hbm_thermal_residency_total", "hbm_thermal_residency", "counter",
     "HBM thermal throttle residency", None, 1.0),
    ("amd_gpu_throttle_status", "throttle_status", "gauge", "Throttle status bitmask", None, 1.0),
    ("amd_gpu_vram_max_bandwidth_gbps", "vram_max_bandwidth_gbps", "gauge", "HBM bandwidth at max memory clock (GB/s)",
     None, 1.0),
    # the XID equivalent (:class:`HealthCounters`): N6 health events per GPU
    ("amd_gpu_reset_total", "health_gpu_pre_reset", "counter", "GPU resets (amd-smi GPU pre-reset events)", None, 1.0),
    ("amd_gpu_reset_recovered_total", "health_gpu_post_reset", "counter",
     "GPU reset recoveries (amd-smi GPU post-reset events)", None, 1.0),
    ("amd_gpu_vm_fault_total", "health_vm_fault", "counter", "GPU VM (page) faults (amd-smi events)", None, 1.0),
    ("amd_gpu_thermal_throttle_events_total", "health_thermal_throttle", "counter",
     "Thermal throttle events (amd-smi events)", None, 1.0),
    ("amd_gpu_ecc_uncorrectable_events_total", "health_ecc_uncorrectable", "counter",
     "Polls that found new uncorrectable ECC errors", None, 1.0),
    ("amd_gpu_xgmi_link_error_events_total", "health_xgmi_link_error", "counter",
     "Polls that found more xGMI links in error", None, 1.0),
    ("amd_gpu_device_lost_events_total", "health_device_lost", "counter", "The GPU stopped answering amd-smi",
     None, 1.0),
    ("amd_gpu_bad_page_events_total", "health_bad_pages", "counter", "Polls that found newly retired HBM pages",
     None, 1.0),
    ("amd_gpu_health_critical", "health_critical", "gauge",
     "A critical health event (reset, uncorrectable ECC, xGMI link error, device lost) and no recovery since",
     None, 1.0),
    ("amd_gpu_last_critical_event_code", "health_last_critical_code", "gauge",
     "Code of the last critical health event (3 GPU reset, 100 uncorrectable ECC, 101 xGMI link error, "
     "102 device lost; 0 none)", "DCGM_FI_DEV_XID_ERRORS", 1.0),
]
# DCGM fields with no MI355X source: accepted in a metrics CSV, reported as unsupported
DCGM_UNSUPPORTED = {"DCGM_FI_DEV_ENC_UTIL", "DCGM_FI_DEV_DEC_UTIL",
                    "DCGM_FI_DEV_VGPU_LICENSE_STATUS", "DCGM_FI_DEV_NVLINK_BANDWIDTH_TOTAL"}
HEALTH_KINDS = ("gpu_pre_reset", "gpu_post_reset", "vm_fault", "thermal_throttle", "ecc_uncorrectable",
                "xgmi_link_error", "device_lost", "bad_pages")
# N6 event kinds (native/include/amdgpu_topo.h AT_EV_*), the code the XID alias carries
HEALTH_CODES = {"vm_fault": 1, "thermal_throttle": 2, "gpu_pre_reset": 3, "gpu_post_reset": 4,
                "ecc_uncorrectable": 100, "xgmi_link_error": 101, "device_lost": 102, "bad_pages": 103}


class HealthCounters:
    """The exporter's XID-equivalent series: N6's health events
    (native/topology/health.cpp - amd-smi GPU reset, VM-fault and thermal
    notifications, and the ECC / xGMI / bad-page / device-lost deltas of its
    polls) counted per GPU, a ``health_critical`` gauge that a critical event
    raises and a reset recovery (post-reset) clears, and the last critical
    event's code, which the ``DCGM_FI_DEV_XID_ERRORS`` alias carries as the
    dcgm-exporter's XID gauge carries the last XID.  The reference's exporter
    "collects GPU metrics for monitoring" (/root/reference/README.md:204,213);
    GPU alerting keys on the XID series.

    ``poll`` is a :class:`~amdgpu_operator.discovery.topology.HealthSubscription`
    poll (the process's one amd-smi event client, shared with the device
    plugin's health loop when both run in one process)."""

    def __init__(self):
        self._lock = threading.Lock()
        self._by_gpu: dict[int, dict] = {}
        self.unattributed = 0
        self.live = False
        self.events = 0

    def ingest(self, events) -> None:
        with self._lock:
            for ev in events:
                self.events += 1
                if ev.index is None or ev.index < 0:
                    self.unattributed += 1
                    continue
                g = self._by_gpu.setdefault(ev.index, {})
                if ev.kind in HEALTH_KINDS:
                    g[f"health_{ev.kind}"] = g.get(f"health_{ev.kind}", 0) + 1
                if ev.critical:
                    g["health_critical"] = 1
                    g["health_last_critical_code"] = HEALTH_CODES.get(ev.kind, 0)
                    g["health_last_message"] = str(ev.message)[:200]
                elif ev.kind == "gpu_post_reset":
                    g["health_critical"] = 0

    def values(self, index: int) -> dict:
        """Every health field of one GPU (0 where nothing happened)."""
        with self._lock:
            g = dict(self._by_gpu.get(index, {}))
        out = {f"health_{k}": float(g.get(f"health_{k}", 0)) for k in HEALTH_KINDS}
        out["health_critical"] = float(g.get("health_critical", 0))
        out["health_last_critical_code"] = float(g.get("health_last_critical_code", 0))
        return out

    def run(self, poll, stop: threading.Event, timeout_ms: int = 500) -> None:
        """Feed from ``poll`` until ``stop``."""
        self.live = True
        try:
            while not stop.is_set():
                try:
                    evs = poll(timeout_ms)
                except Exception as e:  # noqa: BLE001 - keep serving the counts so far
                    log.warning("health events: %s", e)
                    stop.wait(1.0)
                    continue
                if evs:
                    self.ingest(evs)
        finally:
            self.live = False


@dataclass(frozen=True)
class Series:
    name: str
    field: str
    type: str
    help: str
    scale: float


def parse_metrics_csv(text: str) -> tuple[list[Series], list[str]]:
    """dcgm-exporter counters CSV (``NAME, type, help``; ``#`` comments) ->
    (series to export, names with no MI355X source)."""
    by_name = {}
    for metric, fld, mtype, help_, alias, scale in FIELDS:
        by_name[metric] = Series(metric, fld, mtype, help_, 1.0)
        if alias:
            by_name[alias] = Series(alias, fld, mtype, help_, scale)
    out, missing = [], []
    for raw in text.splitlines():
        line = raw.strip()
        if not line or line.startswith("#"):
            continue
        parts = [p.strip() for p in line.split(",", 2)]
        name = parts[0]
        base = by_name.get(name)
        if base is None:
            missing.append(name)
            continue
        mtype = parts[1] if len(parts) > 1 and parts[1] in ("gauge", "counter") else base.type
        help_ = parts[2] if len(parts) > 2 and parts[2] else base.help
        out.append(Series(name, base.field, mtype, help_, base.scale))
    return out, missing


def _esc(v: str) -> str:
    return str(v).replace("\\", "\\\\").replace("\n", "\\n").replace('"', '\\"')


def _labels(d: dict) -> str:
    return "{" + ",".join(f'{k}="{_esc(v)}"' for k, v in d.items()) + "}" if d else ""


@dataclass
class Sample:
    index: int
    bdf: str
    uuid: str
    product: str
    values: dict


class FixtureSource:
    """Metrics from an ``amd-smi metric --json`` capture (tests / demos)."""

    def __init__(self, path: str, gpus: int | None = None):
        with open(path) as f:
            self.doc = json.load(f)
        self.gpus = gpus

    @staticmethod
    def _v(x):
        if isinstance(x, dict):
            x = x.get("value")
        try:
            return float(x)
        except (TypeError, ValueError):
            return None

    def collect(self) -> list[Sample]:
        out = []
        entries = self.doc if isinstance(self.doc, list) else self.doc.get("gpu_data", [self.doc])
        n = self.gpus or len(entries)
        for i in range(n):
            e = entries[i % len(entries)]
            usage = e.get("usage") or {}
            power = e.get("power") or {}
            temp = e.get("temperature") or {}
            clock = e.get("clock") or {}
            mem = e.get("mem_usage") or {}
            ecc = e.get("ecc") or {}
            pcie = e.get("pcie") or {}
            throttle = e.get("throttle") or {}
            vals = {
                "gfx_activity_pct": self._v(usage.get("gfx_activity")),
                "umc_activity_pct": self._v(usage.get("umc_activity")),
                "mm_activity_pct": self._v(usage.get("mm_activity")),
                "socket_power_w": self._v(power.get("socket_power")),
                "temp_hotspot_c": self._v(temp.get("hotspot")),
                "temp_mem_c": self._v(temp.get("mem")),
                "temp_edge_c": self._v(temp.get("edge")),
                "gfx_clk_mhz": self._v(((clock.get("gfx_0") or {}).get("clk"))),
                "mem_clk_mhz": self._v(((clock.get("mem_0") or {}).get("clk"))),
                "vram_total_bytes": (self._v(mem.get("total_vram")) or 0) * 2**20 or None,
                "vram_used_bytes": (self._v(mem.get("used_vram")) or 0) * 2**20,
                "ecc_correctable": self._v(ecc.get("total_correctable_count")) or 0.0,
                "ecc_uncorrectable": self._v(ecc.get("total_uncorrectable_count")) or 0.0,
                "ecc_deferred": self._v(ecc.get("total_deferred_count")) or 0.0,
                "pcie_link_width": self._v(pcie.get("width")),
                "pcie_link_speed_mts": (self._v(pcie.get("speed")) or 0) * 1000 or None,
                "pcie_replay_count": self._v(pcie.get("replay_count")),
                "pcie_nak_sent": self._v(pcie.get("nak_sent_count")),
                "pcie_nak_rcvd": self._v(pcie.get("nak_received_count")),
                "prochot_residency": self._v(throttle.get("prochot_accumulated")),
                "ppt_residency": self._v(throttle.get("ppt_accumulated")),
                "socket_thermal_residency": self._v(throttle.get("socket_thermal_accumulated")),
                "hbm_thermal_residency": self._v(throttle.get("hbm_thermal_accumulated")),
            }
            out.append(Sample(i, f"0000:{0x72 + i:02x}:00.0", f"fixture-{i}", "AMD-Instinct-MI355X",
                              {k: v for k, v in vals.items() if v is not None}))
        return out


class SmiSource:
    """Live metrics via the N4 native collector (libamd_smi)."""

    def __init__(self):
        from ..discovery.topology import Smi

        self.smi = Smi()

    def collect(self) -> list[Sample]:
        return [Sample(m.index, m.bdf, m.uuid, self._product(m.bdf, m.market_name), m.values)
                for m in self.smi.collect()]

    _names: dict = {}

    @classmethod
    def _product(cls, bdf: str, market_name: str) -> str:
        """amd-smi's market name comes from libdrm's amdgpu.ids; where that
        table is missing or does not know the part it says "AMD Radeon
        Graphics" (seen on MI355X hosts).  The PCI device ID names it then,
        as the node labels do (discovery/labels.py PRODUCTS)."""
        if market_name and market_name != "AMD Radeon Graphics":
            return market_name
        if bdf not in cls._names:
            from ..discovery.labels import PRODUCTS

            try:
                with open(f"/sys/bus/pci/devices/{bdf}/device") as f:
                    cls._names[bdf] = PRODUCTS.get(int(f.read().strip(), 16), market_name)
            except (OSError, ValueError):
                cls._names[bdf] = market_name
        return cls._names[bdf]

    def close(self):
        self.smi.close()


class PodAttribution:
    """Maps device IDs (PCI BDF[-pN]) to pods via the kubelet pod-resources API.

    Device-plugin allocations arrive as ``devices`` (the plugin's IDs);
    DRA allocations as ``dynamic_resources`` (claim -> driver/pool/device,
    kubelet >= 1.31).  ``resolve`` turns DRA device names (``gpu-<index>``,
    dra/driver.py) and the plugin's uuid/index IDs into the BDF[-pN] IDs the
    samples carry (:func:`device_id_resolver`)."""

    def __init__(self, socket_path: str, resource_prefix: str = "amd.com/gpu", dra_driver: str = "",
                 resolve=None):
        self.socket_path = socket_path
        self.prefix = resource_prefix
        self.dra_driver = dra_driver
        self.resolve = resolve  # allocation name -> BDF[-pN] (None: the name itself)

    def lookup(self) -> dict[str, dict]:
        from ..deviceplugin import api
        from ..rpc import wire

        if not os.path.exists(self.socket_path):
            return {}
        req, resp, _ = api.POD_RESOURCES_METHODS["List"]
        with wire.Channel(self.socket_path) as ch:
            call = ch.unary_unary(api.method_path(api.POD_RESOURCES_SERVICE, "List"),
                                  request_serializer=req.SerializeToString, response_deserializer=resp.FromString)
            out = call(req(), timeout=2)
        m: dict[str, dict] = {}
        for pr in out.pod_resources:
            for c in pr.containers:
                who = {"namespace": pr.namespace, "pod": pr.name, "container": c.name}
                for d in c.devices:
                    if not d.resource_name.startswith(self.prefix):
                        continue
                    for dev in d.device_ids:
                        base = dev.split(api.REPLICA_SEP, 1)[0]  # a time-sliced replica: its GPU
                        m[(self.resolve(base) if self.resolve else None) or base] = who
                if not self.dra_driver:
                    continue
                for dr in c.dynamic_resources:
                    for cr in dr.claim_resources:
                        if cr.driver_name == self.dra_driver and cr.device_name:
                            key = self.resolve(cr.device_name) if self.resolve else cr.device_name
                            if key:
                                m[key] = who
        return m


def device_id_resolver(sysfs_root: str):
    """``resolve`` for :class:`PodAttribution`: any name the node's GPUs go
    by in an allocation -> their BDF[-pN] ID.  DRA device names
    (``gpu-<index>``) and the device plugin's ``uuid`` and ``index``
    deviceIDStrategy IDs (deviceplugin/server.py base_id) all map to it; the
    table is re-read from the KFD topology when a name is unknown
    (partitions change the device set)."""
    from ..deviceplugin.server import base_id
    from ..discovery import topology
    from ..dra.driver import device_name

    cache: dict[str, str] = {}

    def resolve(name: str) -> str | None:
        if name not in cache:
            cache.clear()
            for g in topology.enumerate_gpus(sysfs_root):
                for alias in (device_name(g), base_id(g, "uuid"), base_id(g, "index"), g.device_id_str):
                    cache[alias] = g.device_id_str
        return cache.get(name)

    return resolve


class MetricsExporter:
    def __init__(self, source, node_name: str = "", interval_s: float = 1.0, attribution: PodAttribution | None = None,
                 dcgm_names: bool = False, selection: list[Series] | None = None,
                 health: HealthCounters | None = None):
        self.source = source
        self.health = health  # the XID-equivalent series (None: not exported)
        self.selection = selection  # None = every field (plus DCGM aliases with dcgm_names)
        self.node = node_name
        self.interval = interval_s
        self.attribution = attribution
        self.dcgm_names = dcgm_names
        self._snapshot: list[Sample] = []
        self._pods: dict[str, dict] = {}
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self.collections = 0
        self.last_collect_s = 0.0
        self.errors = 0

    def collect_once(self) -> None:
        t0 = time.perf_counter()
        try:
            snap = self.source.collect()
            for smp in snap:
                v = smp.values
                if "vram_total_bytes" in v and "vram_used_bytes" in v and "vram_free_bytes" not in v:
                    smp.values = dict(v, vram_free_bytes=max(0.0, float(v["vram_total_bytes"]) - v["vram_used_bytes"]))
            pods = self.attribution.lookup() if self.attribution else {}
        except Exception as e:  # noqa: BLE001 - keep serving the last snapshot
            self.errors += 1
            log.warning("collect failed: %s", e)
            return
        with self._lock:
            self._snapshot, self._pods = snap, pods
            self.collections += 1
            self.last_collect_s = time.perf_counter() - t0

    def run(self) -> None:
        while not self._stop.is_set():
            self.collect_once()
            self._stop.wait(self.interval)

    def stop(self) -> None:
        self._stop.set()

    def _series(self) -> list[Series]:
        if self.selection is not None:
            return self.selection
        out = []
        for metric, fld, mtype, help_, alias, scale in FIELDS:
            out.append(Series(metric, fld, mtype, help_, 1.0))
            if self.dcgm_names and alias:
                out.append(Series(alias, fld, mtype, help_, scale))
        return out

    def render(self) -> str:
        with self._lock:
            snap, pods = list(self._snapshot), dict(self._pods)
        if self.health is not None:
            snap = [Sample(s.index, s.bdf, s.uuid, s.product, {**s.values, **self.health.values(s.index)})
                    for s in snap]
        lines = []
        for ser in self._series():
            rows = [s for s in snap if ser.field in s.values]
            if not rows:
                continue
            lines.append(f"# HELP {ser.name} {ser.help}")
            lines.append(f"# TYPE {ser.name} {ser.type}")
            for s in rows:
                lab = {"gpu": str(s.index), "bdf": s.bdf, "uuid": s.uuid, "product": s.product}
                if self.node:
                    lab["node"] = self.node
                pod = pods.get(s.bdf) or next((v for k, v in pods.items() if k.startswith(s.bdf + "-p")), None)
                if pod:
                    lab.update(pod)
                lines.append(f"{ser.name}{_labels(lab)} {s.values[ser.field] * ser.scale:.6g}")
        lines += [
            "# HELP amd_gpu_exporter_collections_total Completed collection passes",
            "# TYPE amd_gpu_exporter_collections_total counter",
            f"amd_gpu_exporter_collections_total {self.collections}",
            "# HELP amd_gpu_exporter_collect_seconds Duration of the last collection pass",
            "# TYPE amd_gpu_exporter_collect_seconds gauge",
            f"amd_gpu_exporter_collect_seconds {self.last_collect_s:.6g}",
            "# HELP amd_gpu_exporter_errors_total Failed collection passes",
            "# TYPE amd_gpu_exporter_errors_total counter",
            f"amd_gpu_exporter_errors_total {self.errors}",
        ]
        if self.health is not None:
            lines += [
                "# HELP amd_gpu_exporter_health_events_live The amd-smi health event stream is being read",
                "# TYPE amd_gpu_exporter_health_events_live gauge",
                f"amd_gpu_exporter_health_events_live {int(self.health.live)}",
                "# HELP amd_gpu_health_unattributed_events_total Health events naming no known GPU",
                "# TYPE amd_gpu_health_unattributed_events_total counter",
                f"amd_gpu_health_unattributed_events_total {self.health.unattributed}",
            ]
        return "\n".join(lines) + "\n"


class NodeStatusExporter:
    """Operand readiness / validation metrics from the validations directory."""

    STEPS = ("driver", "toolkit", "workload", "plugin", "complete")

    def __init__(self, validations_dir: str, node_name: str = ""):
        self.dir = validations_dir
        self.node = node_name
        self.scrapes = 0

    def render(self) -> str:
        from ..driver.manager import LOST_MARKER
        from ..validator.validate import READY_FILES

        self.scrapes += 1
        lab_node = {"node": self.node} if self.node else {}
        lines = ["# HELP amd_gpu_operator_node_validation_ready Validation step completed (1) or not (0)",
                 "# TYPE amd_gpu_operator_node_validation_ready gauge"]
        secs = []
        for s in self.STEPS:
            p = os.path.join(self.dir, READY_FILES[s])
            ok = os.path.exists(p)
            lines.append(f"amd_gpu_operator_node_validation_ready{_labels({**lab_node, 'step': s})} {int(ok)}")
            if ok:
                try:
                    with open(p) as f:
                        d = json.load(f)
                    if isinstance(d.get("seconds"), (int, float)):
                        secs.append((s, d["seconds"]))
                except (OSError, ValueError):
                    pass
        lines += ["# HELP amd_gpu_operator_node_validation_seconds Duration of each validation step",
                  "# TYPE amd_gpu_operator_node_validation_seconds gauge"]
        for s, v in secs:
            lines.append(f"amd_gpu_operator_node_validation_seconds{_labels({**lab_node, 'step': s})} {v:.6g}")
        validated = os.path.exists(os.path.join(self.dir, READY_FILES["complete"]))
        lines += ["# HELP amd_gpu_operator_node_validated Node passed every validation step",
                  "# TYPE amd_gpu_operator_node_validated gauge",
                  f"amd_gpu_operator_node_validated{_labels(lab_node)} {int(validated)}",
                  "# HELP amd_gpu_operator_node_driver_lost The amdgpu driver went away and is not back yet",
                  "# TYPE amd_gpu_operator_node_driver_lost gauge",
                  f"amd_gpu_operator_node_driver_lost{_labels(lab_node)} "
                  f"{int(os.path.exists(os.path.join(self.dir, LOST_MARKER)))}",
                  "# HELP amd_gpu_operator_node_status_scrapes_total Scrapes served",
                  "# TYPE amd_gpu_operator_node_status_scrapes_total counter",
                  f"amd_gpu_operator_node_status_scrapes_total{_labels(lab_node)} {self.scrapes}"]
        return "\n".join(lines) + "\n"


class MetricsHttpServer:
    """``/metrics`` + ``/healthz`` for any object with ``render() -> str``."""

    def __init__(self, renderer, host: str = "0.0.0.0", port: int = 9400):
        r = renderer

        class H(BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def do_GET(self):
                if self.path.startswith("/metrics"):
                    body = r.render().encode()
                    ctype = "text/plain; version=0.0.4; charset=utf-8"
                elif self.path.startswith("/healthz"):
                    body, ctype = b"ok\n", "text/plain"
                else:
                    self.send_response(404)
                    self.end_headers()
                    return
                self.send_response(200)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

        self.httpd = ThreadingHTTPServer((host, port), H)
        self.httpd.daemon_threads = True
        self.thread = threading.Thread(target=self.httpd.serve_forever, daemon=True, name="metrics-http")

    @property
    def port(self) -> int:
        return self.httpd.server_address[1]

    def start(self) -> "MetricsHttpServer":
        self.thread.start()
        return self

    def stop(self) -> None:
        self.httpd.shutdown()
        self.httpd.server_close()
