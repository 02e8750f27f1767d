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

With the DRA driver instead of the device plugin (``dra=True``) the same
batches are ResourceClaims: one claim per pod (``count: k``; the whole node
as ``allocationMode: All``; the two halves with a ``matchAttribute`` on
``gpu.amd.com/numaNode`` so each half is NUMA-local), allocated by the
scheduler from the node's ResourceSlice, prepared by the node's DRA driver
through the kubelet's DRA manager, and injected from the claim's CDI spec.
"""

from __future__ import annotations

import json
import os
import time

from .. import RESOURCE_NAME
from ..api.clusterpolicy import DEFAULT_REPOSITORY, DEFAULT_VERSION, validator_pod_image

POD_LABEL = "amd.com/pod-workload"


DEFAULT_IMAGE = f"{DEFAULT_REPOSITORY}/amd-operator-validator:{DEFAULT_VERSION}"

def _pct(xs: list[float], q: float) -> float | None:
    if not xs:
        return None
    s = sorted(xs)
    return round(s[min(len(s) - 1, max(0, int(round(q * (len(s) - 1)))))], 4)


def _pod(name: str, node: str, namespace: str, run_id: str, count: int, gemm_n: int,
         resource: str = RESOURCE_NAME, image: str = DEFAULT_IMAGE) -> dict:
    return {
        "apiVersion": "v1", "kind": "Pod",
        "metadata": {"name": name, "namespace": namespace, "labels": {"app": "gpu-job", POD_LABEL: run_id}},
        "spec": {
            # through the scheduler, as a user's pod goes: it counts the GPUs of
            # pods still terminating on the node (the plugin-validation pod the
            # validator deleted once it had its result) and binds once they are
            # free, where a pod bound by nodeName would fail kubelet admission
            "nodeSelector": {"kubernetes.io/hostname": node}, "restartPolicy": "Never",
            "tolerations": [{"key": resource, "operator": "Exists", "effect": "NoSchedule"}],
            "containers": [{"name": "gemm", "image": image,
                            "command": ["amdgpu-validator"],
                            "args": ["--all-devices", "--expect-devices", str(count), "--steps", "hip,gemm",
                                     "--gemm", str(gemm_n), "--gemm-iters", "1"],
                            "resources": {"limits": {resource: str(count)}, "requests": {resource: str(count)}}}],
        },
    }


def _dra_pod(name: str, node: str, namespace: str, run_id: str, count: int, gemm_n: int, n_gpus: int,
             image: str = DEFAULT_IMAGE) -> list[dict]:
    """A ResourceClaim for ``count`` devices and the pod using it (scheduled
    by the scheduler, which allocates the claim on ``node``)."""
    from ..dra.api import DRIVER_NAME

    req = {"name": "gpus", "deviceClassName": DRIVER_NAME}
    if count == n_gpus:
        req["allocationMode"] = "All"
    else:
        req["count"] = count
    constraints = [{"requests": ["gpus"], "matchAttribute": f"{DRIVER_NAME}/numaNode"}] if 1 < count < n_gpus else []
    claim = {"apiVersion": "resource.k8s.io/v1beta1", "kind": "ResourceClaim",
             "metadata": {"name": name, "namespace": namespace, "labels": {POD_LABEL: run_id}},
             "spec": {"devices": {"requests": [req], "constraints": constraints}}}
    pod = _pod(name, node, namespace, run_id, count, gemm_n, image=image)
    spec = pod["spec"]
    del spec["tolerations"]
    spec["resourceClaims"] = [{"name": "gpus", "resourceClaimName": name}]
    spec["containers"][0]["resources"] = {"claims": [{"name": "gpus"}]}
    return [claim, pod]


def _run_batch(cluster, node: str, namespace: str, shapes: list[int], gemm_n: int, timeout: float,
               dra: bool = False, n_gpus: int = 0, image: str = DEFAULT_IMAGE) -> list[dict]:
    """Create one pod per entry of ``shapes`` (its GPU count) at once, wait for
    all, collect their record, delete them."""
    from ..kube.client import wait_for

    run_id = os.urandom(3).hex()
    names = [f"gpu-job-{run_id}-{i}x{k}" for i, k in enumerate(shapes)]
    created = {}
    for name, k in zip(names, shapes):
        created[name] = time.perf_counter()
        for obj in (_dra_pod(name, node, namespace, run_id, k, gemm_n, n_gpus, image=image) if dra
                    else [_pod(name, node, namespace, run_id, k, gemm_n, image=image)]):
            cluster.client.create(obj)
    objs, ok = wait_for(cluster.client, "v1", "Pod", lambda o: all(
        n in o and ((o[n].get("status") or {}).get("phase") in ("Succeeded", "Failed")) for n in names),
        namespace=namespace, label_selector=f"{POD_LABEL}={run_id}", timeout=timeout, poll_s=0.01)
    events = {}
    for t, what, detail in list(cluster.events):
        if detail in created and what in ("gpu-pod-allocated", "gpu-pod-hooked", "gpu-pod-reported"):
            events.setdefault(detail, {}).setdefault(what, t)
    topo, by_dra_name = {}, {}
    try:
        from ..discovery import topology
        from ..dra.driver import device_name

        root = cluster.nodes[node].env.sysfs_root()
        gpus = topology.enumerate_gpus(root)
        topo = {g.device_id_str: g for g in gpus}
        by_dra_name = {device_name(g): g.device_id_str for g in gpus}
    except Exception:  # noqa: BLE001 - record the device ids only
        pass
    claims = {}
    if dra:
        claims = {c["metadata"]["name"]: c for c in cluster.client.list(
            "resource.k8s.io/v1beta1", "ResourceClaim", namespace, label_selector=f"{POD_LABEL}={run_id}")}
    out = []
    for name, k in zip(names, shapes):
        o = objs.get(name) or {}
        ev = events.get(name, {})
        rec = {"pod": name, "gpus": k, "phase": (o.get("status") or {}).get("phase", "Missing")}
        if dra:
            res = ((((claims.get(name) or {}).get("status") or {}).get("allocation") or {}).get("devices")
                   or {}).get("results") or []
            rec["devices"] = [by_dra_name.get(r["device"], r["device"]) for r in res]
        else:
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
        for kind in (("v1", "Pod"),) + ((("resource.k8s.io/v1beta1", "ResourceClaim"),) if dra else ()):
            try:
                cluster.client.delete(*kind, name, namespace)
            except Exception:  # noqa: BLE001
                pass
    if not ok:
        raise TimeoutError(f"pod workload did not finish in {timeout} s: {[r['phase'] for r in out]}")
    # the next batch starts once the kubelet released these pods' devices
    # (DRA: and the driver unprepared their claims, removing the CDI specs)
    kubelet = cluster.nodes[node].kubelet
    cdi_dir = cluster.nodes[node].env.cdi_dir
    uids = {c["metadata"].get("uid") for c in claims.values()}

    def held():
        if any(k[1] in names for k in list(kubelet.assignments) + list(kubelet.claims)):
            return True
        try:
            return dra and any(f.split("claim_", 1)[-1][:-5] in uids for f in os.listdir(cdi_dir))
        except OSError:
            return False

    deadline = time.monotonic() + timeout
    while time.monotonic() < deadline and held():
        time.sleep(0.01)
    return out


def run_pod_workload(cluster, node: str, n_gpus: int, gemm_n: int = 4096, timeout: float = 120.0,
                     namespace: str = "default", dra: bool = False) -> dict:
    """Config 5 on a validated node; returns the ``pod_workload`` block."""
    t0 = time.perf_counter()
    # the user's GEMM image: the validator image of the installed policy (a bare
    # name would not be in the registry, SimCluster.known_images)
    image = validator_pod_image(((cluster.policy() or {}).get("spec")) or {})["image"]

    def batch(shapes):
        return _run_batch(cluster, node, namespace, shapes, gemm_n, timeout, dra=dra, n_gpus=n_gpus, image=image)

    batches = {"single": batch([1] * n_gpus), "whole_node": batch([n_gpus])}
    if n_gpus == 8:
        batches["two_halves"] = batch([4, 4])
    pods = [p for b in batches.values() for p in b]
    single = batches["single"]
    done = [p["kernel_done_s"] for p in single if "kernel_done_s" in p]
    out = {
        "allocation": "dra" if dra else "device-plugin",
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
