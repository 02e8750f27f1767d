"""Names shared by the operator (controller/) and the node operands.

Labels, annotations and state values both sides read or write live here, in
a module with no imports: operand processes import it at start-up, inside
the node's time-to-Ready, and the controller modules that define the
operator's behaviour pull in the ClusterPolicy model (pydantic, ~0.2 s of
imports no operand needs).  controller/ re-exports these names.
"""

# per-node operand selection: amd.com/gpu.deploy.<operand>=true
DEPLOY_LABEL = "amd.com/gpu.deploy.{}"
# ClusterPolicy operand key -> deploy-label suffix
OPERAND_LABELS = {
    "driver": "driver",
    "toolkit": "container-toolkit",
    "validator": "operator-validator",
    "devicePlugin": "device-plugin",
    "draDriver": "dra-driver",
    "dcgmExporter": "metrics-exporter",
    "gfd": "gpu-feature-discovery",
    "migManager": "partition-manager",
    "nodeStatusExporter": "node-status-exporter",
    "vfioManager": "vfio-manager",
    "sandboxValidator": "sandbox-validator",
    "sandboxDevicePlugin": "sandbox-device-plugin",
}

# written by the NFD worker on each node it scanned
NFD_SCANNED_ANN = "nfd.amd.com/scanned"

# driver upgrade (controller/upgrade.py): the node's state label and values
UPGRADE_STATE_LABEL = "amd.com/gpu-driver-upgrade-state"
REQUIRED, CORDON, POD_DELETION, POD_RESTART = ("upgrade-required", "cordon-required", "pod-deletion-required",
                                               "pod-restart-required")
VALIDATION, UNCORDON, DONE, FAILED = "validation-required", "uncordon-required", "upgrade-done", "upgrade-failed"
ACTIVE = (CORDON, POD_DELETION, POD_RESTART, VALIDATION, UNCORDON)
# written by the driver container once the module it installed is live
LOADED_HASH_ANN = "amd.com/gpu-driver.spec-hash"
LOADED_VERSION_ANN = "amd.com/gpu-driver.version"

# the driver health container's amd-smi status line (driver/manager.py publish_smi,
# checked by `amdgpu-operator verify`)
DRIVER_SMI_ANN = "amd.com/gpu.driver-smi"

# the DRA driver's name (dra/api.py DRIVER_NAME): ResourceClaim results it allocated
DRA_DRIVER = "gpu.amd.com"


def uses_gpu(pod: dict, get_claim=None) -> bool:
    """Does this pod hold GPUs of the node - through the device plugin
    (``amd.com/gpu*`` limits or requests of any container) or through the DRA
    driver (a ResourceClaim that one of its containers names)?  A partition
    change, a driver upgrade and a drain must take both kinds off the node.
    ``get_claim(namespace, name)``: the claim, to skip claims another DRA
    driver (a NIC's) allocated; without it, or when a claim cannot be read or
    is not allocated yet, any claim counts (the safe side: evict)."""
    spec = pod.get("spec") or {}
    ctrs = list(spec.get("containers") or []) + list(spec.get("initContainers") or [])
    for c in ctrs:
        res = c.get("resources") or {}
        if any(k.startswith("amd.com/gpu") for part in ("limits", "requests") for k in (res.get(part) or {})):
            return True
    entries = spec.get("resourceClaims") or []
    if not entries or not any((c.get("resources") or {}).get("claims") for c in ctrs):
        return False
    if get_claim is None:
        return True
    ns = (pod.get("metadata") or {}).get("namespace", "default")
    generated = {s.get("name"): s.get("resourceClaimName")
                 for s in (pod.get("status") or {}).get("resourceClaimStatuses") or []}
    for e in entries:
        name = e.get("resourceClaimName") or generated.get(e.get("name"))
        if not name:
            return True  # a template's claim not created yet
        try:
            claim = get_claim(ns, name)
        except Exception:  # noqa: BLE001 - unreadable: count it
            return True
        results = ((((claim or {}).get("status") or {}).get("allocation") or {}).get("devices") or {}).get("results")
        if not results or any(r.get("driver") == DRA_DRIVER for r in results):
            return True
    return False
