"""The synthetic pod-scheduling workload of BASELINE.json config 5.

"8 x MI355X: 8 pods @1 GPU each, topology-aware alloc" - what the node is for
once the operator reports it Ready (the reference's post-install check is that
the node advertises schedulable GPUs, /root/reference/README.md:122,211).
After a bring-up, user-shaped pods are created on the node:

* N pods x 1 GPU, all at once (each must land on its own GPU), then
* one pod x N GPUs (the whole node: xGMI-consistent by construction), and
* on nodes of 8 GPUs, two pods x 4 GPUs at once (GetPreferredAllocation must
  give each a NUMA-local, xGMI-linked half).

Every pod goes the production way: kubelet admission -> the device plugin's
GetPreferredAllocation -> Allocate -> the OCI hook edits the container spec ->
the container runs ``amdgpu-validator --all-devices`` with ``hip,gemm``: a
random-init bf16 GEMM (4096^3 by default) on the hand-written MFMA kernel of
every GPU it was given, Freivalds-checked, and ``--expect-devices`` so a GPU
the runtime left out fails the pod.  The per-pod times come from the
simulated kubelet's trace (pod created -> devices allocated -> spec hooked ->
report out = kernel done).
"""

from __future__ import annotations

import json
import os
import time

from .. import RESOURCE_NAME

POD_LABEL = "amd.com/pod-workload"


def _pct(xs: list[float], q: float) -> float | None:
    if not xs:
        return None
    s = sorted(xs)
    return round(s[min(len(s) - 1, max(0, int(round(q * (len(s) - 1)))))], 4)


def _pod(name: str, node: str, namespace: str, run_id: str, count: int, gemm_n: int,
         resource: str = RESOURCE_NAME) -> dict:
    return {
        "apiVersion": "v1", "kind": "Pod",
        "metadata": {"name": name, "namespace": namespace, "labels": {"app": "gpu-job", POD_LABEL: run_id}},
        "spec": {
            "nodeName": node, "restartPolicy": "Never",
            "tolerations": [{"key": resource, "operator": "Exists", "effect": "NoSchedule"}],
            "containers": [{"name": "gemm", "image": "amd-operator-validator",
                            "command": ["amdgpu-validator"],
                            "args": ["--all-devices", "--expect-devices", str(count), "--steps", "hip,gemm",
                                     "--gemm", str(gemm_n), "--gemm-iters", "1"],
                            "resources": {"limits": {resource: str(count)}, "requests": {resource: str(count)}}}],
        },
    }


def _run_batch(cluster, node: str, namespace: str, shapes: list[int], gemm_n: int, timeout: float) -> list[dict]:
    """Create one pod per entry of ``shapes`` (its GPU count) at once, wait for
    all, collect their record, delete them."""
    from ..kube.client import wait_for

    run_id = os.urandom(3).hex()
    names = [f"gpu-job-{run_id}-{i}x{k}" for i, k in enumerate(shapes)]
    created = {}
    for name, k in zip(names, shapes):
        created[name] = time.perf_counter()
        cluster.client.create(_pod(name, node, namespace, run_id, k, gemm_n))
    objs, ok = wait_for(cluster.client, "v1", "Pod", lambda o: all(
        n in o and ((o[n].get("status") or {}).get("phase") in ("Succeeded", "Failed")) for n in names),
        namespace=namespace, label_selector=f"{POD_LABEL}={run_id}", timeout=timeout, poll_s=0.01)
    events = {}
    for t, what, detail in list(cluster.events):
        if detail in created and what in ("gpu-pod-allocated", "gpu-pod-hooked", "gpu-pod-reported"):
            events.setdefault(detail, {}).setdefault(what, t)
    topo = {}
    try:
        from ..discovery import topology

        root = cluster.nodes[node].env.sysfs_root()
        topo = {g.device_id_str: g for g in topology.enumerate_gpus(root)}
    except Exception:  # noqa: BLE001 - record the device ids only
        pass
    out = []
    for name, k in zip(names, shapes):
        o = objs.get(name) or {}
        ev = events.get(name, {})
        rec = {"pod": name, "gpus": k, "phase": (o.get("status") or {}).get("phase", "Missing")}
        alloc = ((o.get("metadata") or {}).get("annotations") or {}).get("amd.com/gpu.allocated", "")
        rec["devices"] = [d for d in alloc.split(",") if d]
        gs = [topo[d] for d in rec["devices"] if d in topo]
        if gs:
            rec["numa_nodes"] = sorted({g.numa_node for g in gs})
            rec["physical_gpus"] = sorted({g.physical_index for g in gs})
        t0 = created[name]
        if "gpu-pod-allocated" in ev:
            rec["admitted_allocated_s"] = round(ev["gpu-pod-allocated"] - t0, 4)
        if "gpu-pod-hooked" in ev:
            rec["hooked_s"] = round(ev["gpu-pod-hooked"] - t0, 4)
        if "gpu-pod-reported" in ev:
            rec["kernel_done_s"] = round(ev["gpu-pod-reported"] - t0, 4)
        rep = (getattr(cluster, "pod_reports", {}) or {}).get(name) or {}
        gemms = [s for s in rep.get("steps", []) if s.get("name") == "gemm"]
        if gemms:
            rec["gemm_ok"] = all(s.get("ok") for s in gemms) and rep.get("ok") is True
            rec["gemm_tflops"] = [s.get("tflops") for s in gemms]
            rec["freivalds_rel_err"] = max((s.get("freivalds_rel_err") or 0.0) for s in gemms)
            rec["simulated"] = bool(rep.get("simulated"))
        elif rep:
            rec["gemm_ok"] = rep.get("ok") is True
            rec["simulated"] = bool(rep.get("simulated"))
        out.append(rec)
    for name in names:
        try:
            cluster.client.delete("v1", "Pod", name, namespace)
        except Exception:  # noqa: BLE001
            pass
    if not ok:
        raise TimeoutError(f"pod workload did not finish in {timeout} s: {[r['phase'] for r in out]}")
    # the next batch starts once the kubelet released these pods' devices
    kubelet = cluster.nodes[node].kubelet
    deadline = time.monotonic() + timeout
    while time.monotonic() < deadline and any(k[1] in names for k in list(kubelet.assignments)):
        time.sleep(0.01)
    return out


def run_pod_workload(cluster, node: str, n_gpus: int, gemm_n: int = 4096, timeout: float = 120.0,
                     namespace: str = "default") -> dict:
    """Config 5 on a validated node; returns the ``pod_workload`` block."""
    t0 = time.perf_counter()
    batches = {"single": _run_batch(cluster, node, namespace, [1] * n_gpus, gemm_n, timeout),
               "whole_node": _run_batch(cluster, node, namespace, [n_gpus], gemm_n, timeout)}
    if n_gpus == 8:
        batches["two_halves"] = _run_batch(cluster, node, namespace, [4, 4], gemm_n, timeout)
    pods = [p for b in batches.values() for p in b]
    single = batches["single"]
    done = [p["kernel_done_s"] for p in single if "kernel_done_s" in p]
    out = {
        "pods": len(pods),
        "all_succeeded": all(p["phase"] == "Succeeded" for p in pods),
        "gemm_correct": all(p.get("gemm_ok") for p in pods),
        "gemm_n": gemm_n,
        "single_gpu_pods_distinct_devices": len({d for p in single for d in p["devices"]}) == n_gpus,
        "admission_to_kernel_done_p50_s": _pct(done, 0.5),
        "admission_to_kernel_done_p99_s": _pct(done, 0.99),
        "admission_to_allocated_p50_s": _pct([p["admitted_allocated_s"] for p in single
                                              if "admitted_allocated_s" in p], 0.5),
        "whole_node_kernel_done_s": batches["whole_node"][0].get("kernel_done_s"),
        "seconds": round(time.perf_counter() - t0, 3),
        "batches": batches,
    }
    if "two_halves" in batches:
        halves = batches["two_halves"]
        out["two_halves_numa_local"] = all(len(p.get("numa_nodes", [])) == 1 for p in halves)
        out["two_halves_disjoint"] = not (set(halves[0]["devices"]) & set(halves[1]["devices"]))
    return out


def summary_line(block: dict) -> str:
    """One line for logs."""
    keep = {k: v for k, v in block.items() if k != "batches"}
    return json.dumps(keep)
