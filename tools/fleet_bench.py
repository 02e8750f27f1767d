"""Fleet bring-up: time-to-Ready and API load as the node count grows.

bench.py measures one node with real MI355X GPUs.  This measures the part
that grows with the cluster: the operator's reconcile passes and the API
requests every component makes while N GPU nodes (8 synthetic MI355X each,
CPU-only stand-in validators) go from ``helm install`` to validated, with the
reference's ``--set`` flags (/root/reference/README.md:101-110).

Prints one JSON document: per N, time-to-Ready of the whole fleet, reconcile
passes, and API requests by verb and by component thread.

``python tools/fleet_bench.py [--nodes 1,8,32] [--timeout 300]``
"""

from __future__ import annotations

import argparse
import collections
import json
import os
import shutil
import sys
import tempfile
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from amdgpu_operator.api.clusterpolicy import REFERENCE_SET_FLAGS, parse_set_flags  # noqa: E402
from amdgpu_operator.kube.client import LocalClient  # noqa: E402
from amdgpu_operator.testing.simcluster import NodeSpec, SimCluster  # noqa: E402

VERBS = ("create", "get", "list", "update", "update_status", "patch", "delete", "watch")


class CountingClient(LocalClient):
    """LocalClient that counts requests per (verb, kind) and per calling thread."""

    def __init__(self, server):
        super().__init__(server)
        self.by_verb: collections.Counter = collections.Counter()
        self.by_thread: collections.Counter = collections.Counter()
        self._lock = threading.Lock()
        for verb in VERBS:
            setattr(self, verb, self._counted(verb, getattr(LocalClient, verb)))

    def _counted(self, verb, fn):
        def call(*a, **kw):
            kind = a[0].get("kind") if a and isinstance(a[0], dict) else (a[1] if len(a) > 1 else "?")
            role = threading.current_thread().name
            role = role.split("-")[0] + "-" + role.split("-")[1] if "-" in role else role
            with self._lock:
                self.by_verb[f"{verb} {kind}"] += 1
                self.by_thread[role] += 1
            return fn(self, *a, **kw)
        return call

    def reset(self):
        with self._lock:
            self.by_verb.clear()
            self.by_thread.clear()


def bring_up(n_nodes: int, timeout: float) -> dict:
    work = tempfile.mkdtemp(prefix="fleet-")
    nodes = [NodeSpec(f"n{i:03d}", gpus=8) for i in range(n_nodes)]
    cluster = SimCluster(work, nodes, fake_gpu=True, poll_s=0.01)
    cluster.client = cluster.agent_client = CountingClient(cluster.api)
    cluster.start()
    try:
        cluster.client.reset()
        passes = []
        t0 = time.perf_counter()
        cluster.install_operator(parse_set_flags(REFERENCE_SET_FLAGS))
        orig = cluster.reconciler.reconcile

        def counted():
            passes.append(time.perf_counter())
            return orig()

        cluster.reconciler.reconcile = counted
        ttr = cluster.wait_ready(timeout, {n.name: 8 for n in nodes})
        total = sum(cluster.client.by_verb.values())
        return {"nodes": n_nodes, "gpus": 8 * n_nodes, "time_to_ready_s": round(ttr, 3),
                "wall_s": round(time.perf_counter() - t0, 3), "reconcile_passes": len(passes),
                "api_requests": total, "api_requests_per_node": round(total / n_nodes, 1),
                "top_requests": dict(cluster.client.by_verb.most_common(12)),
                "by_component": dict(cluster.client.by_thread.most_common(12))}
    finally:
        cluster.stop()
        shutil.rmtree(work, ignore_errors=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", default="1,8,32")
    ap.add_argument("--timeout", type=float, default=300.0)
    args = ap.parse_args()
    out = [bring_up(int(n), args.timeout) for n in args.nodes.split(",")]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
