"""Control-plane latencies of the operator's node agents.

The reference only observes its operands after the fact (pod AGE, README.md:
138-139, 202-206); these are the per-request costs behind time-to-Ready and
behind a pod getting its GPU:

* device plugin (C5), over real gRPC on unix sockets against the fake
  kubelet: registration -> ``amd.com/gpu: N`` advertised; one pod admission
  (GetPreferredAllocation + Allocate) for 1/2/4/8 GPUs on an 8-GPU xGMI node
  and on a CPX node (64 partitions); health flip -> kubelet update;
* metrics exporter (C9): one collect+render cycle and one HTTP scrape, from the
  captured MI355X amd-smi fixture (CPU) or live libamd_smi (``--live``, GPU box).

Prints one JSON document.  ``python tools/plane_bench.py [--live] [--reps N]``
"""

from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import tempfile
import time
import urllib.request

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from amdgpu_operator.deviceplugin.server import DevicePluginManager, PluginConfig  # noqa: E402
from amdgpu_operator.discovery import topology as T  # noqa: E402
from amdgpu_operator.exporter.metrics import FixtureSource, MetricsExporter, MetricsHttpServer  # noqa: E402
from amdgpu_operator.testing import fakesys  # noqa: E402
from amdgpu_operator.testing.fakekubelet import FakeKubelet  # noqa: E402


def stats_ms(xs: list[float]) -> dict:
    xs = sorted(xs)
    return {"n": len(xs), "p50_ms": round(1e3 * statistics.median(xs), 3),
            "p99_ms": round(1e3 * xs[min(len(xs) - 1, int(0.99 * len(xs)))], 3),
            "max_ms": round(1e3 * xs[-1], 3)}


def plugin_bench(gpus: int, partition: str, resource: str, sizes, reps: int) -> dict:
    work = tempfile.mkdtemp(prefix="pb-")
    root = os.path.join(work, "host")
    fakesys.build_node(root, gpus, partition)
    k = FakeKubelet(os.path.join(work, "dp"))
    k.start()
    strategy = "single" if partition == "SPX" else "mixed"
    n_dev = len(T.enumerate_gpus(root))
    t0 = time.perf_counter()
    m = DevicePluginManager(PluginConfig(socket_dir=os.path.join(work, "dp"), sysfs_root=root,
                                         watch_interval_s=0.05, partition_strategy=strategy))
    m.start()
    out: dict = {"node": f"{gpus}x MI355X {partition}", "resource": resource, "devices": n_dev}
    try:
        assert k.wait_registered(resource, 30, min_devices=n_dev), "plugin did not register"
        out["register_to_advertised_ms"] = round(1e3 * (time.perf_counter() - t0), 2)
        out["allocatable"] = k.allocatable(resource)
        for size in sizes:
            if size > n_dev:
                continue
            lat = []
            for i in range(reps):
                t = time.perf_counter()
                ids, _ = k.allocate(resource, size, pod=f"p{i}")
                lat.append(time.perf_counter() - t)
                assert len(ids) == size
                k.release("default", f"p{i}")
            out[f"admit_{size}"] = stats_ms(lat)
        dev = sorted(k.resources[resource].devices)[0]
        lat = []
        for i in range(20):
            before = k.resources[resource].updates
            t = time.perf_counter()
            m.set_health(dev, i % 2 == 1, "bench")
            assert k.wait_update(resource, before, 5)
            lat.append(time.perf_counter() - t)
        out["health_flip_to_kubelet"] = stats_ms(lat)
    finally:
        m.stop()
        k.stop()
    return out


def exporter_bench(live: bool, reps: int) -> dict:
    if live:
        from amdgpu_operator.exporter.metrics import SmiSource

        src = SmiSource()
        label = "live libamd_smi"
    else:
        src = FixtureSource(os.path.join(fakesys.REAL_FIXTURE, "amd-smi-metric.json"), gpus=8)
        label = "amd-smi fixture, 8 GPUs"
    ex = MetricsExporter(src, "bench-node", dcgm_names=True)
    out: dict = {"source": label}
    try:
        coll, rend = [], []
        for _ in range(reps):
            t = time.perf_counter()
            ex.collect_once()
            coll.append(time.perf_counter() - t)
            t = time.perf_counter()
            text = ex.render()
            rend.append(time.perf_counter() - t)
        out["collect"] = stats_ms(coll)
        out["render"] = stats_ms(rend)
        out["series"] = sum(1 for ln in text.splitlines() if ln and not ln.startswith("#"))
        srv = MetricsHttpServer(ex, "127.0.0.1", 0).start()
        try:
            lat = []
            for _ in range(reps):
                t = time.perf_counter()
                body = urllib.request.urlopen(f"http://127.0.0.1:{srv.port}/metrics", timeout=5).read()
                lat.append(time.perf_counter() - t)
            out["http_scrape"] = stats_ms(lat)
            out["scrape_bytes"] = len(body)
        finally:
            srv.stop()
    finally:
        if hasattr(src, "close"):
            src.close()
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--live", action="store_true", help="exporter on the real GPUs (libamd_smi)")
    ap.add_argument("--reps", type=int, default=100)
    a = ap.parse_args()
    t0 = time.time()
    res = {
        "device_plugin": [
            plugin_bench(8, "SPX", "amd.com/gpu", (1, 2, 4, 8), a.reps),
            plugin_bench(8, "CPX", "amd.com/gpu-cpx", (1, 8, 16), max(10, a.reps // 4)),
        ],
        "metrics_exporter": exporter_bench(a.live, a.reps),
    }
    res["wall_s"] = round(time.time() - t0, 2)
    print(json.dumps(res, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
