"""``amdgpu-operator verify``: the reference's manual checks, machine-asserted (C13).

The reference verifies the install by hand (/root/reference/README.md):

=====================================================  =====================================
reference command                                      assertion here
=====================================================  =====================================
kubectl get nodes -o wide (README.md:80)               every node Ready
kubectl get pods -n gpu-operator-resources (:116,195)   every operand pod Running / Completed
kubectl get nodes -l nvidia.com/gpu.present=true (:119)  >= 1 node labelled amd.com/gpu.present
describe nodes | grep Allocatable nvidia.com/gpu (:122)  Allocatable amd.com/gpu > 0 per GPU node
get pods -A | grep nvidia-driver-daemonset (:132)       driver pods 2/2 Running, 0 restarts
exec ... -c nvidia-driver-ctr -- nvidia-smi (:152)      amd-driver-ctr present, and the driver
                                                        image's amd-smi reports live power and
                                                        temperature for every GPU (the health
                                                        container's amd.com/gpu.driver-smi)
(validator "Completed", :199)                           node labelled amd.com/gpu.validated
(``--run-pod``: a user's first GPU pod)                 per GPU node, one pod asking for one GPU
                                                        (amd.com/gpu, or a ResourceClaim with the
                                                        DRA driver) runs a kernel on exactly the
                                                        GPU it was given and Succeeds
=====================================================  =====================================

Output: one JSON document (``--json``) or a table; exit 0 only if all pass.
"""

from __future__ import annotations

import json
import os
import time
from dataclasses import asdict, dataclass, field

from .. import LABEL_PRESENT, RESOURCE_NAME
from ..kube import resources as R
from ..wellknown import DRIVER_SMI_ANN

EXPECTED_OPERANDS = {
    "amd-driver-daemonset": "driver",
    "amd-container-toolkit-daemonset": "toolkit",
    "amd-device-plugin-daemonset": "devicePlugin",
    "amd-dra-driver": "draDriver",
    "amd-operator-validator": "validator",
    "gpu-feature-discovery": "gfd",
    "amd-metrics-exporter": "dcgmExporter",
    "amd-node-status-exporter": "nodeStatusExporter",
    "node-feature-discovery-worker": "nfd",
}
OFF_BY_DEFAULT = {"draDriver"}  # operands a policy without the key does not run
# vm-passthrough nodes (sandboxWorkloads) run these instead of the container operands
EXPECTED_SANDBOX_OPERANDS = {
    "amd-vfio-manager": "vfioManager",
    "amd-sandbox-validator": "validator",
    "amd-sandbox-device-plugin-daemonset": "sandboxDevicePlugin",
}
PASSTHROUGH_LABEL = "amd.com/gpu.deploy.vfio-manager"


def _passthrough(node: dict) -> bool:
    return (node["metadata"].get("labels") or {}).get(PASSTHROUGH_LABEL) == "true"


def _count(allocs: dict, match) -> int:
    n = 0
    for k, v in allocs.items():
        if match(k):
            try:
                n += int(v)
            except ValueError:
                pass
    return n


@dataclass
class Check:
    name: str
    ok: bool
    detail: str = ""
    reference: str = ""


@dataclass
class Report:
    checks: list[Check] = field(default_factory=list)

    @property
    def ok(self) -> bool:
        return all(c.ok for c in self.checks)

    def add(self, name: str, ok: bool, detail: str = "", reference: str = "") -> None:
        self.checks.append(Check(name, bool(ok), detail, reference))

    def as_dict(self) -> dict:
        return {"ok": self.ok, "checks": [asdict(c) for c in self.checks]}

    def table(self) -> str:
        w = max(len(c.name) for c in self.checks) if self.checks else 10
        lines = [f"{'CHECK'.ljust(w)}  RESULT  DETAIL"]
        for c in self.checks:
            lines.append(f"{c.name.ljust(w)}  {'PASS' if c.ok else 'FAIL':6s}  {c.detail}")
        lines.append(f"overall: {'PASS' if self.ok else 'FAIL'}")
        return "\n".join(lines)


def _pod_ok(p: dict) -> tuple[bool, str]:
    st = p.get("status") or {}
    phase = st.get("phase", "Pending")
    cs = st.get("containerStatuses") or []
    ready = sum(1 for c in cs if c.get("ready"))
    restarts = sum(int(c.get("restartCount", 0)) for c in cs)
    ok = phase == "Succeeded" or (phase == "Running" and ready == len(cs) and len(cs) > 0)
    return ok, f"{phase} {ready}/{len(cs)} restarts={restarts}"


def _allocatable_check(rep: "Report", name: str, labels: dict, allocs: dict, expect_gpus_per_node: int | None) -> None:
    # amd.com/gpu, partition (-cpx ...) and time-sliced (.shared / renamed) resources all count;
    # time-slicing multiplies the advertised devices by the replicas GFD publishes
    count = _count(allocs, lambda k: k == RESOURCE_NAME or k.startswith((RESOURCE_NAME + "-", RESOURCE_NAME + ".")))
    try:
        replicas = max(1, int(labels.get("amd.com/gpu.replicas", "1")))
    except ValueError:
        replicas = 1
    want = expect_gpus_per_node * replicas if expect_gpus_per_node else None
    ok = count > 0 and (want is None or count == want)
    rep.add(f"allocatable[{name}]", ok, f"{RESOURCE_NAME}*={count}" + (f" (expected {want})" if want else ""),
            "README.md:122")


def pod_image_of(spec: dict, override: str | None = None) -> dict:
    """The image a verification pod runs: the live ClusterPolicy's validator
    image (``{repository}/{image}:{version}``, its pull policy and pull
    secrets: api/clusterpolicy.py validator_pod_image, as the validator's own
    plugin pods), or ``override`` (``--pod-image``) with the policy's pull
    settings.  A bare name would be pulled from Docker Hub on a cluster."""
    from ..api.clusterpolicy import ClusterPolicySpec, validator_pod_image

    try:
        img = validator_pod_image(ClusterPolicySpec.model_validate(spec or {}))
    except Exception:  # noqa: BLE001 - a policy this version cannot parse: its validator block only
        v = (spec or {}).get("validator") or {}
        from ..api.clusterpolicy import DEFAULT_REPOSITORY, DEFAULT_VERSION

        img = {"image": f"{v.get('repository', DEFAULT_REPOSITORY)}/{v.get('image') or 'amd-operator-validator'}:"
                        f"{v.get('version', DEFAULT_VERSION)}",
               "pull_policy": v.get("imagePullPolicy", "IfNotPresent"), "pull_secrets": v.get("imagePullSecrets") or []}
    if override:
        img["image"] = override
    return img


def run_gpu_pod(client, node: str, namespace: str, dra: bool, image: str | dict,
                timeout: float = 120.0, device_class: str | None = None) -> tuple[bool, str]:
    """One pod on ``node`` asking for one GPU - through the device plugin
    (``amd.com/gpu: 1``) or, with the DRA driver, a ResourceClaim for one
    device of the policy's DeviceClass - running ``amdgpu-gpu-check
    --expect-devices 1`` from the validator image (:func:`pod_image_of`);
    (passed, detail).  Pod and claim are deleted afterwards."""
    from ..dra.api import DRIVER_NAME

    img = image if isinstance(image, dict) else {"image": image}
    name = f"amd-gpu-verify-{os.urandom(3).hex()}"
    ctr = {"name": "check", "image": img["image"], "imagePullPolicy": img.get("pull_policy") or "IfNotPresent",
           "command": ["amdgpu-gpu-check"], "args": ["--timeout", "30", "--expect-devices", "1"]}
    spec = {"restartPolicy": "Never", "containers": [ctr]}
    if img.get("pull_secrets"):
        spec["imagePullSecrets"] = [{"name": x} for x in img["pull_secrets"]]
    objs = []
    if dra:
        objs.append({"apiVersion": "resource.k8s.io/v1beta1", "kind": "ResourceClaim",
                     "metadata": {"name": name, "namespace": namespace},
                     "spec": {"devices": {"requests": [{"name": "gpu",
                                                        "deviceClassName": device_class or DRIVER_NAME}]}}})
        spec["nodeSelector"] = {"kubernetes.io/hostname": node}
        spec["resourceClaims"] = [{"name": "gpu", "resourceClaimName": name}]
        ctr["resources"] = {"claims": [{"name": "gpu"}]}
    else:
        spec["nodeSelector"] = {"kubernetes.io/hostname": node}
        spec["tolerations"] = [{"key": RESOURCE_NAME, "operator": "Exists", "effect": "NoSchedule"}]
        ctr["resources"] = {"limits": {RESOURCE_NAME: "1"}}
    objs.append({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": namespace,
                                                                  "labels": {"app": "amd-gpu-verify"}}, "spec": spec})
    t0 = time.monotonic()
    try:
        for o in objs:
            client.create(o)
        phase, st = "Pending", {}
        while time.monotonic() - t0 < timeout:
            st = client.get("v1", "Pod", name, namespace).get("status") or {}
            phase = st.get("phase", "Pending")
            if phase in ("Succeeded", "Failed"):
                break
            time.sleep(0.05)
        detail = f"{'dra claim' if dra else RESOURCE_NAME + '=1'}: {phase} in {time.monotonic() - t0:.2f} s"
        if phase != "Succeeded" and st.get("message"):
            detail += f" ({st['message'][:300]})"
        waiting = [((c.get("state") or {}).get("waiting") or {}) for c in st.get("containerStatuses") or []]
        if phase != "Succeeded" and any(w.get("reason") for w in waiting):  # ErrImagePull, ImagePullBackOff, ...
            w = next(w for w in waiting if w.get("reason"))
            detail += f" ({w['reason']}: {str(w.get('message', ''))[:300]}; image {img['image']})"
        return phase == "Succeeded", detail
    finally:
        for o in reversed(objs):
            try:
                client.delete(o["apiVersion"], o["kind"], name, namespace)
            except Exception:  # noqa: BLE001 - already gone
                pass


def verify(client, namespace: str, expect_gpus_per_node: int | None = None, run_pods: bool = False,
           pod_image: str | None = None, pod_timeout: float = 120.0) -> Report:
    rep = Report()
    nodes = client.list("v1", "Node")
    not_ready = [n["metadata"]["name"] for n in nodes
                 if (R.condition(n, "Ready") or {}).get("status") not in ("True", None)]
    rep.add("nodes-ready", not not_ready, f"{len(nodes)} node(s), not ready: {not_ready or 'none'}", "README.md:80")

    try:
        cp = client.list("amd.com/v1", "ClusterPolicy")
    except Exception:  # noqa: BLE001 - CRD missing
        cp = []
    spec = (cp[0].get("spec") if cp else {}) or {}
    gpu_nodes = [n for n in nodes if (n["metadata"].get("labels") or {}).get(LABEL_PRESENT) == "true"]
    rep.add("gpu-nodes-labelled", bool(gpu_nodes), f"{len(gpu_nodes)} node(s) with {LABEL_PRESENT}=true", "README.md:119")

    for n in gpu_nodes:
        name = n["metadata"]["name"]
        labels = n["metadata"].get("labels") or {}
        allocs = (n.get("status") or {}).get("allocatable") or {}
        if _passthrough(n):
            # VM passthrough: the GPUs are amd.com/<product> (vfio-pci), not amd.com/gpu
            from ..sandbox.plugin import PRODUCT_NAMES

            names = {f"amd.com/{p}" for p in PRODUCT_NAMES.values()}
            count = _count(allocs, lambda k: k in names or k.startswith("amd.com/AMD_GPU_"))
            want = expect_gpus_per_node
            rep.add(f"allocatable[{name}]", count > 0 and (want is None or count == want),
                    f"vm-passthrough amd.com/<product>={count}" + (f" (expected {want})" if want else ""),
                    "README.md:122")
            validated = labels.get("amd.com/gpu.validated") == "true"
            rep.add(f"validated[{name}]", validated, "GPUs on vfio-pci" if validated else "not validated",
                    "README.md:199")
            continue
        if (spec.get("draDriver") or {}).get("enabled"):
            # DRA: the node's GPUs are devices of its ResourceSlice, not amd.com/gpu
            try:
                sl = client.get("resource.k8s.io/v1beta1", "ResourceSlice", f"{name}-gpu.amd.com")
                count = len((sl.get("spec") or {}).get("devices") or [])
            except Exception:  # noqa: BLE001 - no slice
                count = 0
            want = expect_gpus_per_node
            rep.add(f"resourceslice[{name}]", count > 0 and (want is None or count == want),
                    f"gpu.amd.com devices={count}" + (f" (expected {want})" if want else ""), "README.md:122 (DRA)")
        else:
            _allocatable_check(rep, name, labels, allocs, expect_gpus_per_node)
        # what the reference reads off `nvidia-smi` in the driver container
        # (README.md:152-166: product, memory, GPU count) comes from GFD labels
        prod, mem, arch = (labels.get("amd.com/gpu.product"), labels.get("amd.com/gpu.memory"),
                           labels.get("amd.com/gpu.arch"))
        cnt = labels.get("amd.com/gpu.count")
        inv_ok = bool(prod and mem and arch) and (cnt is None or int(cnt) > 0)
        rep.add(f"gpu-inventory[{name}]", inv_ok,
                f"product={prod} arch={arch} memory={mem}MiB count={cnt}", "README.md:152-166")
        validated = labels.get("amd.com/gpu.validated") == "true"
        rep.add(f"validated[{name}]", validated, "amd.com/gpu.validated=true" if validated else "not validated",
                "README.md:199")
        if ((spec.get("driver") or {}).get("rdma") or {}).get("enabled"):
            # driver.rdma: NICs that can reach GPU memory (discovery/rdma.py labels)
            cap, nics, aff = (labels.get("amd.com/gpu.rdma.capable"), labels.get("amd.com/gpu.rdma.nics"),
                              labels.get("amd.com/gpu.rdma.affinity"))
            rep.add(f"rdma[{name}]", cap == "true", f"capable={cap} nics={nics} affinity={aff}",
                    "driver.rdma (upstream GPUDirect RDMA; not set in README.md:101-110)")
        if (spec.get("driver") or {}).get("enabled", True):
            smi = (n["metadata"].get("annotations") or {}).get(DRIVER_SMI_ANN, "")
            rep.add(f"driver-smi[{name}]", smi.startswith("ok"), smi or "not reported by amd-driver-health",
                    "README.md:152-167")
        if run_pods:
            dra = (spec.get("draDriver") or {})
            ok, detail = run_gpu_pod(client, name, namespace, bool(dra.get("enabled")), pod_image_of(spec, pod_image),
                                     pod_timeout, dra.get("deviceClass"))
            rep.add(f"gpu-pod[{name}]", ok, detail, "README.md:147-152 (a GPU workload runs)")

    pods = client.list("v1", "Pod", namespace)
    bad = []
    for p in pods:
        ok, d = _pod_ok(p)
        if not ok:
            bad.append(f"{p['metadata']['name']}: {d}")
    rep.add("operand-pods-running", bool(pods) and not bad,
            f"{len(pods)} pod(s) in {namespace}; failing: {bad or 'none'}", "README.md:116,195-207")

    container_nodes = [n for n in gpu_nodes if not _passthrough(n)]
    vm_nodes = [n for n in gpu_nodes if _passthrough(n)]
    drv = [p for p in pods if p["metadata"]["name"].startswith("amd-driver-daemonset")]
    drv_ok = bool(drv) or not container_nodes
    details = []
    for p in drv:
        ok, d = _pod_ok(p)
        names = [c["name"] for c in p["spec"].get("containers", [])]
        drv_ok &= ok and len(names) == 2 and "amd-driver-ctr" in names
        details.append(f"{p['metadata']['name']} {d} containers={names}")
    rep.add("driver-daemonset", drv_ok, "; ".join(details) or "no driver pods", "README.md:132-143,152")

    present = {p["metadata"].get("labels", {}).get("app") for p in pods}
    if drv:  # per-kernel (usePrecompiled) and per-pool (AMDGPUDriver) driver DaemonSets count as the driver
        present.add("amd-driver-daemonset")
    missing = [ds for ds, key in EXPECTED_OPERANDS.items()
               if (spec.get(key) or {}).get("enabled", key not in OFF_BY_DEFAULT) and ds not in present
               and (container_nodes if key != "nfd" else gpu_nodes)]
    missing += [ds for ds, key in EXPECTED_SANDBOX_OPERANDS.items()
                if vm_nodes and (spec.get(key) or {}).get("enabled", True) and ds not in present]
    rep.add("operands-deployed", not missing, f"missing: {missing or 'none'}", "README.md:201-207")
    state = ((cp[0].get("status") or {}).get("state") if cp else "absent")
    rep.add("cluster-policy-ready", state == "ready", f"ClusterPolicy state={state}", "README.md:101 (--wait)")
    return rep


def main_verify(client, namespace: str, as_json: bool, expect: int | None, run_pods: bool = False,
                pod_image: str | None = None, pod_timeout: float = 120.0) -> int:
    rep = verify(client, namespace, expect, run_pods, pod_image, pod_timeout)
    print(json.dumps(rep.as_dict(), indent=1) if as_json else rep.table())
    return 0 if rep.ok else 1
