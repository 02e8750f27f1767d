"""Randomized fault injection on the simulated cluster (CPU, fake GPUs).

Two 2-GPU nodes and a CPU node under one ClusterPolicy with sandbox mode on.
Each step injects one fault, lets it land, then requires the cluster to be
Ready again with the allocatable each node's workload implies:

  delpod      delete a random operand pod on a GPU node (the DaemonSet replaces it)
  driverloss  the amdgpu module vanishes and comes back (driver monitor pass)
  kubelet     the node's kubelet restarts (device plugins re-register)
  switch      flip a node between container and vm-passthrough
  spec        toggle gfd / the metrics exporter in the ClusterPolicy
  upgrade     change driver.driverVersion (node-by-node driver upgrade)
  partition   flip a container node between SPX and CPX (partition manager: 2 or 16 devices)
  partbusy    the same while a process holds the GPU (a KFD user the node's
              agents do not own): the change must wait until it is gone
  noop        (--inject-noop only) claims to revalidate but does nothing: the
              harness must catch it

With ``--dra`` the GPUs are advertised by the DRA driver instead of the
device plugin (draDriver.enabled, devicePlugin.enabled=false): Ready means
the node's ResourceSlice lists every device (2 or 16 per node), a kubelet
restart makes the plugin watcher register the driver again, there is no
vm-passthrough switch, and one more fault runs a user's workload:

  claimpod    a ResourceClaim for one device and a pod using it (amdgpu-gpu-check
              --expect-devices 1) must Succeed; both are deleted again

Ready again is not enough to pass a step: a fault that must revalidate the
node (validator pod deleted, driver loss, partition change, driver upgrade,
workload switch) must leave a strictly newer validation record on it - the
``workload-ready`` / ``sandbox-validated`` time - and on ``--real-gpu`` that
record's GEMM step must carry ``counter_gate: pass``.  A kubelet restart must
show the device plugin registered again.  Each step prints the revalidation
delay (new record minus fault time).

    python tools/chaos_sim.py --seeds 1-5 --steps 10

Prints one line per step and, on a step that never converges, the cluster
diagnostics; exits 1 if any seed failed.
"""

from __future__ import annotations

import argparse
import os
import random
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from amdgpu_operator.api.clusterpolicy import (REFERENCE_SET_FLAGS, deep_merge, parse_set_flags,  # noqa: E402
                                              validator_pod_image)
from amdgpu_operator.driver.manager import monitor_once  # noqa: E402
from amdgpu_operator.sandbox import WORKLOAD_CONFIG_LABEL  # noqa: E402
from amdgpu_operator.testing.simcluster import NodeSpec, SimCluster  # noqa: E402
from amdgpu_operator.utils import record  # noqa: E402

FAULTS = ("delpod", "delpod", "driverloss", "kubelet", "switch", "switch", "spec", "upgrade", "partition", "partbusy")
REVALIDATE = ("driverloss", "partition", "partbusy", "upgrade", "switch", "noop")


REAL_GPU_FAULTS = ("delpod", "delpod", "kubelet", "spec")  # no root on a GPU box: no module, PCI or partition changes
DRA_FAULTS = ("delpod", "delpod", "driverloss", "kubelet", "spec", "upgrade", "partition", "partbusy", "claimpod",
              "claimpod")
REAL_GPU_DRA_FAULTS = ("delpod", "delpod", "kubelet", "spec", "claimpod")
RV1B1 = "resource.k8s.io/v1beta1"


def slice_devices(c, node: str) -> int:
    try:
        return len((c.client.get(RV1B1, "ResourceSlice", f"{node}-gpu.amd.com").get("spec") or {}).get("devices") or [])
    except Exception:  # noqa: BLE001 - not published (yet)
        return 0


def claim_pod(c, node: str, timeout: float) -> tuple[bool, str]:
    """A user's one-GPU DRA workload on ``node``: claim + pod, Succeeded?"""
    name = f"chaos-{os.urandom(3).hex()}"
    c.client.create({"apiVersion": RV1B1, "kind": "ResourceClaim", "metadata": {"name": name, "namespace": "default"},
                     "spec": {"devices": {"requests": [{"name": "gpu", "deviceClassName": "gpu.amd.com"}]}}})
    c.client.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": "default"},
                     "spec": {"restartPolicy": "Never", "nodeSelector": {"kubernetes.io/hostname": node},
                              "resourceClaims": [{"name": "gpu", "resourceClaimName": name}],
                              "containers": [{"name": "check", "image": validator_pod_image(
                                  (c.policy() or {}).get("spec") or {})["image"],
                                              "command": ["amdgpu-gpu-check"],
                                              "args": ["--timeout", "30", "--expect-devices", "1"],
                                              "resources": {"claims": [{"name": "gpu"}]}}]}})
    deadline = time.time() + timeout
    st = {}
    while time.time() < deadline:
        st = c.client.get("v1", "Pod", name, "default").get("status") or {}
        if st.get("phase") in ("Succeeded", "Failed"):
            break
        time.sleep(0.05)
    for kind in (("v1", "Pod"), (RV1B1, "ResourceClaim")):
        try:
            c.client.delete(*kind, name, "default")
        except Exception:  # noqa: BLE001
            pass
    return st.get("phase") == "Succeeded", f"{name} {st.get('phase')} {st.get('message', '')[:200]}"


def validation_record(c, node: str) -> dict:
    """The node's latest validation: workload (container) or sandbox time."""
    from amdgpu_operator.validator.validate import read_ready

    env = c.nodes[node].env
    wl = read_ready(env, "workload") or {}
    sb = read_ready(env, "sandbox") or {}
    return {"time": max(wl.get("time", 0.0), sb.get("time", 0.0)), "workload": wl}


def gemm_gate_passed(record: dict) -> bool:
    ranks = (record.get("workload") or {}).get("ranks") or []
    gemms = [s for r in ranks for s in r.get("steps", []) if s.get("name") == "gemm"]
    return bool(gemms) and all(s.get("counter_gate") == "pass" for s in gemms)


def run_seed(seed: int, steps: int, settle_s: float, timeout: float, http_api: bool = False,
             real_gpu: bool = False, inject_noop: int = -1, processes: bool = False, rbac: bool = False,
             dra: bool = False) -> bool:
    rnd = random.Random(seed)
    d = tempfile.mkdtemp(prefix="chaos-")
    if real_gpu:  # one node, this machine's GPU(s): every validation runs on the real device
        from amdgpu_operator.discovery import topology

        n_gpus = len(topology.enumerate_gpus("/"))
        nodes, gpu_nodes = [NodeSpec("g0", n_gpus, sysfs_root="/")], ["g0"]
    else:
        n_gpus = 2
        nodes, gpu_nodes = [NodeSpec("g0", 2), NodeSpec("g1", 2), NodeSpec("cpu", 0)], ["g0", "g1"]
    c = SimCluster(os.path.join(d, "c"), nodes, fake_gpu=not real_gpu,
                   poll_s=0.005, agent_poll_s=0.05, termination_s=0.0,  # kubelet-confirmed pod deletes
                   http_api=http_api, process_containers=processes, rbac=rbac).start()
    mode = {n: "container" for n in gpu_nodes}
    cpx = {n: False for n in gpu_nodes}
    from amdgpu_operator.partition import manager as PM

    if not real_gpu:
        for n in mode:  # partition changes act on the fake sysfs tree
            env = c.nodes[n].env
            env.extra["partition_backend"] = PM.SysfsBackend(env.host_root,
                                                             PM.sysfs_partition_rebuilder(env.host_root, 2),
                                                             validations_dir=env.validations_dir)

    def devices(n):
        return 8 * n_gpus if cpx[n] else n_gpus

    def expect():
        if dra:  # no amd.com/gpu: the slice is checked instead (wait_ready below)
            return {}
        return {n: (devices(n) if m == "container" else {"amd.com/MI355X": n_gpus}) for n, m in mode.items()}

    def wait_ready():
        c.wait_ready(timeout, expect())
        deadline = time.time() + timeout
        while dra and any(slice_devices(c, n) != devices(n) for n in gpu_nodes):
            if time.time() > deadline:
                raise TimeoutError(f"ResourceSlices {[(n, slice_devices(c, n), devices(n)) for n in gpu_nodes]}")
            time.sleep(0.05)

    try:
        extra = [] if real_gpu else ["migManager.enabled=true"]
        extra += ["draDriver.enabled=true", "devicePlugin.enabled=false"] if dra else []
        c.install_operator(deep_merge(parse_set_flags(REFERENCE_SET_FLAGS + extra),
                                      {} if real_gpu or dra else {"sandboxWorkloads": {"enabled": True}}))
        wait_ready()
        faults = (REAL_GPU_DRA_FAULTS if dra else REAL_GPU_FAULTS) if real_gpu else (DRA_FAULTS if dra else FAULTS)
        for i in range(steps):
            fault, node = rnd.choice(faults), rnd.choice(gpu_nodes)
            if i == inject_noop:
                fault = "noop"
            info = ""
            before = {n: validation_record(c, n)["time"] for n in gpu_nodes}
            regs_before = c.nodes[node].kubelet.register_calls
            t_fault = time.time()
            must = {node} if fault in REVALIDATE else set()
            if fault == "delpod":
                pods = [p for p in c.pods() if p["spec"].get("nodeName") == node]
                p = rnd.choice(pods)
                info = p["metadata"]["name"]
                if info.startswith("amd-operator-validator"):
                    must = {node}  # its replacement validates the node again
                c.client.delete("v1", "Pod", info, c.namespace)
            elif fault == "driverloss" and mode[node] == "container":
                env = c.nodes[node].env
                f = os.path.join(env.host_root, "sys/module/amdgpu/initstate")
                os.rename(f, f + ".gone")
                # the driver container's health monitor notices (run here with the harness's own
                # client: under --rbac the node env's HTTP client carries no ServiceAccount token)
                monitor_once(record.replace(env, client=c.client))
                os.rename(f + ".gone", f)
            elif fault == "kubelet":
                c.nodes[node].kubelet.restart()
                c.nodes[node].dra = None  # the plugin watcher starts over and registers the DRA driver again
            elif fault == "claimpod":
                ok, info = claim_pod(c, node, timeout)
                if not ok:
                    print(f"seed {seed} step {i} claimpod {node}: the workload did not succeed: {info}", flush=True)
                    return False
            elif fault == "switch":
                mode[node] = "vm-passthrough" if mode[node] == "container" else "container"
                c.client.patch("v1", "Node", node, {"metadata": {"labels": {WORKLOAD_CONFIG_LABEL: mode[node]}}})
                info = mode[node]
            elif fault == "spec":
                cp = c.policy()
                key = rnd.choice(["gfd", "dcgmExporter"])
                cp["spec"][key]["enabled"] = not cp["spec"][key]["enabled"]
                c.client.update(cp)
                info = f"{key}={cp['spec'][key]['enabled']}"
            elif fault in ("partition", "partbusy") and mode[node] == "container":
                env = c.nodes[node].env
                holder = os.path.join(env.host_root, "sys/class/kfd/kfd/proc/4242")
                if fault == "partbusy":  # a process outside the operator's reach holds the GPU
                    os.makedirs(holder, exist_ok=True)
                applied_before = (c.client.get("v1", "Node", node)["metadata"].get("labels") or {}).get(PM.APPLIED_LABEL)
                cpx[node] = not cpx[node]
                c.client.patch("v1", "Node", node, {"metadata": {"labels": {
                    "amd.com/gpu.partition-config": "all-cpx" if cpx[node] else "all-spx"}}})
                info = "CPX" if cpx[node] else "SPX"
                if fault == "partbusy":
                    time.sleep(1.0)
                    applied = (c.client.get("v1", "Node", node)["metadata"].get("labels") or {}).get(PM.APPLIED_LABEL)
                    if applied != applied_before:
                        print(f"seed {seed} step {i} partbusy {node}: partition applied while the GPU was held",
                              flush=True)
                        return False
                    os.rmdir(holder)  # the holder exits: the change may go ahead
                    info += " (held 1 s)"
            elif fault in ("partition", "partbusy"):
                must = set()  # vm-passthrough node: nothing to partition
            elif fault == "noop":
                info = "claims a revalidation, does nothing"
            elif fault == "upgrade":
                cp = c.policy()
                cp["spec"]["driver"]["driverVersion"] = "6.14.0" if cp["spec"]["driver"]["driverVersion"] != "6.14.0" \
                    else "6.12.12"
                c.client.update(cp)
                info = cp["spec"]["driver"]["driverVersion"]
                must = {n for n, m in mode.items() if m == "container"}
            elif fault == "driverloss":
                must = set()  # a vm-passthrough node has no driver to lose
            time.sleep(settle_s)
            t0 = time.time()
            try:
                if fault == "upgrade":  # ready is not enough: every container node runs the new driver
                    want = info
                    deadline = time.time() + timeout
                    while time.time() < deadline and not all(
                            (c.client.get("v1", "Node", n)["metadata"].get("annotations") or {}).get(
                                "amd.com/gpu-driver.version") == want for n, m in mode.items() if m == "container"):
                        time.sleep(0.05)
                wait_ready()
                # the fault must have landed: a fresh validation of every node it concerns
                deadline = time.time() + timeout
                while time.time() < deadline and any(validation_record(c, n)["time"] <= before[n] for n in must):
                    time.sleep(0.05)
                    wait_ready()
                while fault == "kubelet" and not dra and time.time() < deadline \
                        and c.nodes[node].kubelet.register_calls <= regs_before:
                    time.sleep(0.05)  # the plugin sees the new kubelet.sock within its watch interval
            except TimeoutError as e:
                print(f"seed {seed} step {i} {fault} {node} {info}: NOT READY after {timeout:.0f} s\n{e}", flush=True)
                for t, what, detail in c.trace_since(0)[-120:]:
                    print(f"  trace {t:9.3f} {what} {detail}")
                return False
            stale = [n for n in must if validation_record(c, n)["time"] <= before[n]]
            if stale:
                print(f"seed {seed} step {i} {fault} {node} {info}: Ready, but no fresh validation on {stale}: "
                      "the fault did not land", flush=True)
                return False
            if real_gpu and must and not all(gemm_gate_passed(validation_record(c, n)) for n in must):
                print(f"seed {seed} step {i} {fault} {node}: revalidated without a passing GEMM counter gate", flush=True)
                return False
            if fault == "kubelet" and dra and claim_pod(c, node, timeout)[0] is False:
                print(f"seed {seed} step {i} kubelet {node}: no DRA workload after the restart", flush=True)
                return False
            if fault == "kubelet" and not dra and c.nodes[node].kubelet.register_calls <= regs_before:
                print(f"seed {seed} step {i} kubelet {node}: the device plugin did not register again", flush=True)
                return False
            reval = " ".join(f"{n} revalidated +{validation_record(c, n)['time'] - t_fault:.2f} s" for n in sorted(must))
            print(f"seed {seed} step {i} {fault} {node} {info}: ready {time.time() - t0:.2f} s after settling"
                  + (f"; {reval}" if reval else ""), flush=True)
        if rbac and c._http.denied:  # a request the shipped roles do not grant (kube/rbac.py)
            for d in sorted(set(c._http.denied)):
                print(f"seed {seed}: RBAC denied {d}", flush=True)
            return False
        return True
    finally:
        c.stop()


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", default="1-3", help="N or A-B")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--settle-s", type=float, default=0.5, help="let the fault land before checking readiness")
    ap.add_argument("--timeout", type=float, default=60.0)
    ap.add_argument("--http-api", action="store_true", help="operator and operands over HTTP (RestClient, informers)")
    ap.add_argument("--real-gpu", action="store_true", help="one node on this machine's GPUs (pod/kubelet/spec faults)")
    ap.add_argument("--processes", action="store_true",
                    help="the operator and every operand container as its own process (bench.py's headline mode)")
    ap.add_argument("--rbac", action="store_true",
                    help="with --processes: every request authorized against the shipped roles (kube/rbac.py)")
    ap.add_argument("--dra", action="store_true",
                    help="the DRA driver advertises the GPUs (device plugin off); adds the claimpod fault")
    ap.add_argument("--inject-noop", type=int, default=-1, metavar="STEP",
                    help="make step STEP a no-op fault that claims a revalidation (the harness must fail)")
    a = ap.parse_args()
    if a.rbac and not a.processes:
        ap.error("--rbac needs --processes (a ServiceAccount per operand process)")
    lo, _, hi = a.seeds.partition("-")
    ok = all([run_seed(s, a.steps, a.settle_s, a.timeout, a.http_api, a.real_gpu, a.inject_noop, a.processes, a.rbac,
                        a.dra)
              for s in range(int(lo), int(hi or lo) + 1)])
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
