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
