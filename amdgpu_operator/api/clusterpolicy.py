"""ClusterPolicy (``amd.com/v1``) spec and the Helm values that produce it.

Reference parity: the reference installs the operator with seven value
overrides (/root/reference/README.md:104-110)::

    driver.enabled=true  toolkit.enabled=true  devicePlugin.enabled=true
    nodeStatusExporter.enabled=true  gfd.enabled=true  migManager.enabled=false
    operator.cleanupCRD=true

The same keys are accepted here with the same meaning (``migManager`` is the
MI355X partition manager; ``partitionManager`` is accepted as an alias, as is
``metricsExporter`` for ``dcgmExporter``), plus AMD-specific keys.  Values map
1:1 onto the ClusterPolicy spec and are validated with
pydantic; unknown keys are rejected so typos fail the install instead of being
silently ignored.
"""

from __future__ import annotations

from typing import Literal

from pydantic import BaseModel, ConfigDict, Field, model_validator

from .. import API_GROUP, API_VERSION, DEFAULT_NAMESPACE, RESOURCE_NAME

DEFAULT_REPOSITORY = "registry.local/amd-gpu-operator"
DEFAULT_VERSION = "0.1.0"
ROCM_VERSION = "7.2.0"


class _M(BaseModel):
    model_config = ConfigDict(extra="forbid", populate_by_name=True)


class Image(_M):
    repository: str = DEFAULT_REPOSITORY
    image: str = ""
    version: str = DEFAULT_VERSION
    imagePullPolicy: Literal["Always", "IfNotPresent", "Never"] = "IfNotPresent"
    imagePullSecrets: list[str] = Field(default_factory=list)

    def ref(self, default_image: str) -> str:
        return f"{self.repository}/{self.image or default_image}:{self.version}"


class Resources(_M):
    requests: dict[str, str] = Field(default_factory=dict)
    limits: dict[str, str] = Field(default_factory=dict)


class Operand(Image):
    enabled: bool = True
    env: list[dict] = Field(default_factory=list)
    args: list[str] = Field(default_factory=list)
    resources: Resources = Field(default_factory=Resources)


class UpgradePolicy(_M):
    autoUpgrade: bool = True
    maxParallelUpgrades: int = 1
    drainEnabled: bool = True
    drainTimeoutSeconds: int = 300
    podDeletionForce: bool = False


class RdmaSpec(_M):
    """GPU memory for RDMA NICs (upstream ``driver.rdma``; off, as the
    reference leaves it: README.md:101-110).  On MI355X: amdgpu's dma-buf
    export imported by the RDMA core - no peer-memory module (discovery/rdma.py)."""

    enabled: bool = False
    # the host's MOFED / inbox RDMA stack loads the RDMA core; the driver
    # container waits for it instead of loading ib_uverbs itself
    useHostMofed: bool = False
    # the device plugin also sets NCCL_IB_HCA to the allocation's nearest NICs
    # (always: the amd.com/gpu.rdma-nics annotation)
    hcaEnv: bool = False


class DriverSpec(Operand):
    """amdgpu DKMS + ROCm userspace for gfx950 (README.md:104,212)."""

    image: str = "amd-driver"
    rocmVersion: str = ROCM_VERSION
    driverVersion: str = "6.12.12"
    usePrecompiled: bool = False
    blacklistAmdgpuInbox: bool = True
    kernelModuleParams: dict[str, str] = Field(default_factory=dict)
    packageRepository: str = ""  # package mirror for air-gapped clusters (default repo.radeon.com)
    startupProbeTimeoutSeconds: int = 600
    # unload the module this driver container installed when the container
    # stops (not while GPU processes hold it; never a host-managed module)
    unloadOnExit: bool = True
    upgradePolicy: UpgradePolicy = Field(default_factory=UpgradePolicy)
    # per-node-pool drivers: one driver DaemonSet per AMDGPUDriver object
    # (api/driver_cr.py) instead of the single ClusterPolicy-wide one
    useDriverCRD: bool = False
    rdma: RdmaSpec = Field(default_factory=RdmaSpec)


class CDISpec(_M):
    enabled: bool = True
    default: bool = False
    specDir: str = "/var/run/cdi"


class ToolkitSpec(Operand):
    """OCI hook + CDI spec + containerd patch (README.md:105,210)."""

    image: str = "amd-container-toolkit"
    installDir: str = "/usr/local/amd"
    runtime: Literal["containerd", "docker", "crio"] = "containerd"
    containerdConfig: str = "/etc/containerd/config.toml"
    containerdSocket: str = "/run/containerd/containerd.sock"
    crioConfigDir: str = "/etc/crio/crio.conf.d"  # runtime: crio
    dockerConfig: str = "/etc/docker/daemon.json"  # runtime: docker
    runtimeClass: str = "amd"
    cdi: CDISpec = Field(default_factory=CDISpec)
    mountRocm: bool = False
    # OCI-hook device-list policy (the NVIDIA toolkit's
    # accept-nvidia-visible-devices-as-volume-mounts / -envvar-when-unprivileged)
    acceptDeviceListAsVolumeMounts: bool = False
    acceptEnvvarUnprivileged: bool = True
    setAsDefault: bool = False  # make the amd runtime containerd's default_runtime_name
    cleanupOnExit: bool = True  # restore the runtime config when the toolkit pod goes (helm uninstall)


class DevicePluginConfigRef(_M):
    """ConfigMap of device-plugin config files (deviceplugin/config.py): ``name``
    in the operator namespace, ``default`` key for nodes without the
    ``amd.com/device-plugin.config`` label.  Same shape as the NVIDIA
    operator's ``devicePlugin.config`` (time-slicing lives there)."""

    name: str = ""
    default: str = ""


class DraDriverSpec(Operand):
    """DRA driver ``gpu.amd.com`` (dra/): GPUs as ResourceSlice devices for
    ResourceClaims (Kubernetes >= 1.32, resource.k8s.io/v1beta1) instead of
    the amd.com/gpu extended resource.  Off by default - the reference's
    cluster is v1.28 (README.md:45-46) and advertises through the device
    plugin (README.md:106,211); a GPU is handed out by one of the two."""

    enabled: bool = False
    image: str = "amd-device-plugin"  # the operand image that carries the device plugin
    deviceClass: str = "gpu.amd.com"  # the DeviceClass the operator creates


class DevicePluginSpec(Operand):
    """kubelet device plugin for amd.com/gpu (README.md:106,211)."""

    image: str = "amd-device-plugin"
    resourceName: str = RESOURCE_NAME
    partitionStrategy: Literal["single", "mixed"] = "single"
    deviceIDStrategy: Literal["bdf", "uuid", "index"] = "bdf"
    deviceListStrategy: list[Literal["envvar", "volume-mounts", "cdi-annotations", "cdi-cri"]] = Field(
        default_factory=lambda: ["envvar"])
    passDeviceSpecs: bool = True
    cdiAnnotations: bool = False
    healthPollMs: int = 1000
    # open the amd-smi health event client once the node is validated (not beside the validator)
    healthStart: Literal["afterValidation", "immediate"] = "afterValidation"
    config: DevicePluginConfigRef = Field(default_factory=DevicePluginConfigRef)


class ServiceMonitor(_M):
    enabled: bool = False
    interval: str = "15s"
    additionalLabels: dict[str, str] = Field(default_factory=dict)


class MetricsConfigRef(_M):
    """ConfigMap holding a dcgm-exporter style counters CSV (``key``) that
    selects the exported series; empty ``name`` = every series."""

    name: str = ""
    key: str = "metrics.csv"


class MetricsExporterSpec(Operand):
    """amd-smi based DCGM-exporter equivalent (README.md:204,213)."""

    image: str = "amd-metrics-exporter"
    port: int = 9400
    intervalSeconds: float = 1.0
    podAttribution: bool = True
    dcgmNames: bool = False  # also emit DCGM_FI_DEV_* series for existing dashboards
    # the XID-equivalent series (amd-smi reset / VM-fault / thermal events, ECC / xGMI deltas)
    healthEvents: bool = True
    serviceMonitor: ServiceMonitor = Field(default_factory=ServiceMonitor)
    config: MetricsConfigRef = Field(default_factory=lambda: MetricsConfigRef())


class NodeStatusExporterSpec(Operand):
    """Operand / validation readiness metrics (README.md:107)."""

    image: str = "amd-node-status-exporter"
    port: int = 8000


class GFDSpec(Operand):
    """GPU feature discovery labels (README.md:108,202,209)."""

    image: str = "gpu-feature-discovery"
    intervalSeconds: float = 60.0
    labelPrefix: str = "amd.com"


class NFDSpec(Operand):
    """Node feature discovery (PCI vendor 0x1002 scan)."""

    image: str = "node-feature-discovery"
    intervalSeconds: float = 60.0


class PartitionManagerSpec(Operand):
    """MIG-manager analog: compute (SPX/DPX/QPX/CPX) + memory (NPS1/NPS2) partitions.
    Disabled by default, as in the reference (README.md:109)."""

    enabled: bool = False
    image: str = "amd-partition-manager"
    defaultComputePartition: Literal["SPX", "DPX", "TPX", "QPX", "CPX"] = "SPX"
    defaultMemoryPartition: Literal["NPS1", "NPS2", "NPS4", "NPS8"] = "NPS1"
    configLabel: str = "amd.com/gpu.partition-config"
    profiles: dict[str, dict[str, str]] = Field(default_factory=lambda: {
        "all-spx": {"compute": "SPX", "memory": "NPS1"},
        "all-dpx": {"compute": "DPX", "memory": "NPS2"},
        "all-qpx": {"compute": "QPX", "memory": "NPS1"},
        "all-cpx": {"compute": "CPX", "memory": "NPS2"},
    })


class SandboxWorkloadsSpec(_M):
    """VM passthrough next to containers (the NVIDIA operator's
    ``sandboxWorkloads``): a GPU node's ``amd.com/gpu.workload.config`` label
    (``container`` | ``vm-passthrough``, default ``defaultWorkload``) picks
    which operands it runs.  Off by default: every GPU node is a container node."""

    enabled: bool = False
    defaultWorkload: Literal["container", "vm-passthrough"] = "container"


class VFIOManagerSpec(Operand):
    """Binds a passthrough node's GPUs (whole IOMMU groups) to vfio-pci."""

    image: str = "amd-vfio-manager"
    kfdIdleTimeoutSeconds: int = 300  # wait this long for GPU users before unbinding from amdgpu


class SandboxDevicePluginSpec(Operand):
    """Advertises vfio-bound GPUs per product (``amd.com/MI355X``) for VMs."""

    image: str = "amd-sandbox-device-plugin"
    resourcePrefix: str = "amd.com"


class WorkloadSpec(_M):
    gemmN: int = 4096
    gemmIters: int = 3
    hbmBytes: int = 1 << 30
    rcclElems: int = 1 << 24
    xgmiElems: int = 1 << 22
    # Ready-gate floors, for a whole MI355X (256 CUs; a compute partition is
    # held to its share of the CUs).  Derived (tools/floor_calibration.py,
    # profiles/r6_floors, table in BASELINE.md) from 60 validator runs on an
    # MI355X at the shipped kernels and sizes: floor = min(0.72 x median,
    # 0.90 x the slowest healthy run), i.e. ~72 % of the typical rate with a
    # 10 % margin under the slowest run for clocks and temperature.  A GPU
    # held at low clocks or a capped power limit, a slow HBM stack or fenced-off
    # CUs fails the node.  The floors apply at gemmN >= 4096 / hbmBytes >=
    # 1 GiB (smaller runs are launch-bound and report their rate only); 0 =
    # report only.
    minGemmTflops: float = 1080.0   # bf16: median 1,505.5 TF/s
    minHbmGbps: float = 4270.0      # 1 GiB copy: median 5,944 GB/s
    # the mfma-rate check (validator steps gemm_fp8, gemm_fp4, gemm_fp6 and
    # gemm_mxfp4, label amd.com/gpu.validated.mfma-rate): OCP e4m3, FP4 (e2m1),
    # FP6 (e2m3) and block-scaled MXFP4 GEMMs on the gfx950 f8f6f4 MFMA at
    # mfmaRateGemmN^3, held to these floors and counted by the gate
    # (SQ_INSTS_VALU_MFMA_MOPS_F8 / _F6F4)
    mfmaRateCheck: bool = True
    # the validator takes multiples of 256 (its 256 x 256 tiles), and >= 512 for fp4
    mfmaRateGemmN: int = Field(default=4096, ge=512, multiple_of=256)
    minFp8Tflops: float = 1940.0    # median 2,706 TF/s
    minFp4Tflops: float = 3100.0    # median 4,313 TF/s
    minFp6Tflops: float = 2540.0    # median 3,534 TF/s
    minMxfp4Tflops: float = 2830.0  # median 3,939 TF/s
    # counter-gate floor on MFMA busy cycles per SIMD-cycle of the counted
    # bf16 GEMM (native/include/gate_policy.h): median 0.62 at 4096^3
    minMfmaUtil: float = 0.44
    # the same per low-precision data type (their 4096^3 GEMMs keep the MFMA
    # pipes busy a smaller share of the time: medians 0.46 / 0.30 / 0.29 / 0.29)
    # N7 gate lock (native/include/gate_lock.h): the counted dispatch holds a
    # per-GPU lock that the plugin pod's check and the RCCL processes share
    gateLock: bool = True
    # count the GEMMs after the kernel steps (validator_main.cpp PendingGate)
    # instead of inside each step: the first counted window rarely waits for
    # the plugin pod's hold on the gate lock (-2.5 ms median time-to-Ready),
    # but back-to-back GEMM trials read fp6 / MXFP4 3-9 % lower
    # (profiles/r6_defer), so off by default
    deferGates: bool = False
    minMfmaUtilByDtype: dict[str, float] = Field(
        default_factory=lambda: {"fp8": 0.33, "fp4": 0.21, "fp6": 0.20, "mxfp4": 0.20})
    # N >= 2 throughput floors from the xGMI link model (validator/validate.py
    # fabric_floors): a rank's links to its N-1 peers carry 76 GB/s each per
    # direction on MI355X (KFD io_links), 532 GB/s at N = 8.  RCCL fp32
    # all-reduce busBW >= this fraction of that sum x B/(B + 16 MiB) at the
    # validated size B (64 MiB: 0.8) - 85 GB/s at N = 8, 12 GB/s at N = 2; a
    # PCIe-routed node (no xGMI) gets ~20-60 GB/s in total and fails
    rcclBusbwLinkFraction: float = 0.2
    # K4 one-shot all-reduce: the peer reads (N-1 buffers at once, one per
    # link) >= this fraction of the same sum - 133 GB/s at N = 8
    xgmiReadLinkFraction: float = 0.25
    # multi-GPU nodes: every pair of GPUs joined by an xGMI link in the KFD
    # topology and amd-smi reporting the links up, none in error, each trained
    # to >= minXgmiLinkFraction of the KFD nominal rate (rate x width: a link
    # that came back at half its rate or width is "up" and fails here)
    requireXgmiLinks: bool = True
    minXgmiLinkFraction: float = 0.9
    # N >= 2: a rank not alive within this long is missing (also bounds the
    # RCCL communicator set-up); a collective not done within
    # collectiveTimeoutSeconds aborts the communicator
    peerTimeoutSeconds: float = 30.0
    collectiveTimeoutSeconds: float = 30.0
    counterGate: bool = True
    # how the gate reads the counters: "aql" - AQL profiling packets around one
    # more dispatch of the GEMM on the validator's own HSA queue (no profiler
    # runtime in the process); "sdk" - the rocprofiler-sdk tool library
    counterGateMode: Literal["aql", "sdk"] = "aql"
    # run the RCCL check (own process, world 1) on a single-GPU node too: the
    # multi-GPU critical path, rehearsed where there is no xGMI peer
    rcclSingleGpu: bool = False
    # one validator process per physical GPU runs the kernel checks of every
    # device of the GPU (its partitions, concurrently), the xGMI one-shot and
    # RCCL ("shared", default); "separate" puts xGMI + RCCL in a second process
    # per GPU when that stays within maxGpuProcesses (the storm probe measured
    # one process per GPU faster at N = 5: profiles/r3_storm)
    rcclProcess: Literal["separate", "shared"] = "shared"
    # concurrent GPU processes one node's validation may start (workload
    # processes + plugin-validation pods): a GPU box admits few processes per
    # user on its devices (16 measured), and each one's HIP start-up stretches
    # the others'
    maxGpuProcesses: int = Field(default=16, ge=2)
    # start the validator processes while the driver is still being validated:
    # they load their libraries and wait behind a start gate, so process start
    # is off the time-to-Ready critical path (no GPU call before the gate opens)
    prespawn: bool = True


class ValidatorSpec(Operand):
    """Operator validator: driver, toolkit, workload (HIP + MFMA + RCCL), plugin."""

    image: str = "amd-operator-validator"
    workload: WorkloadSpec = Field(default_factory=WorkloadSpec)
    pluginValidation: bool = True
    # what a plugin-validation pod runs on the GPUs it was allocated: "hsa" -
    # amdgpu-gpu-check, a kernel per GPU on the HSA runtime alone (~0.08 s to
    # its report on MI355X); "hip" - amdgpu-validator hip,vecadd (HIP runtime
    # and context, ~0.1-0.2 s; profiles/r3_pod_check)
    pluginPodCheck: Literal["hsa", "hip"] = "hsa"
    # plugin-validation pods: one per resource holding all of its devices
    # ("perResource", default: fewest processes in the start-up storm), or one
    # 1-device pod per device ("perDevice": N pods x 1 GPU, each its own
    # GetPreferredAllocation/Allocate/hook, started at most workload.
    # maxGpuProcesses - workload processes at a time)
    pluginPods: Literal["perResource", "perDevice"] = "perResource"
    validationsDir: str = "/run/amd/validations"


class OperatorSpec(_M):
    defaultRuntime: Literal["containerd", "docker", "crio"] = "containerd"
    runtimeClass: str = "amd"
    cleanupCRD: bool = False  # README.md:110 sets it true
    upgradeCRD: bool = True
    logLevel: Literal["debug", "info", "warning", "error"] = "info"
    reconcileIntervalSeconds: float = 30.0


class DaemonsetsSpec(_M):
    priorityClassName: str = "system-node-critical"
    tolerations: list[dict] = Field(default_factory=lambda: [
        {"key": "amd.com/gpu", "operator": "Exists", "effect": "NoSchedule"}])
    labels: dict[str, str] = Field(default_factory=dict)
    annotations: dict[str, str] = Field(default_factory=dict)
    updateStrategy: Literal["RollingUpdate", "OnDelete"] = "RollingUpdate"
    maxUnavailable: str = "1"
    # Operands wait for their prerequisite validation (driver-ready,
    # toolkit-ready) inside their own container instead of behind an init
    # container, the driver container runs the upgrade check itself, and the
    # validator validates in its main container: every operand process starts
    # with the pod and is imported and waiting when its gate opens.  Each init
    # container is one more container start on the time-to-Ready critical
    # path (~0.35 s of interpreter + imports per operand process on the
    # MI355X box, profiles/r3_ttr); false = the init-container layout.
    inContainerGates: bool = True


class PSASpec(_M):
    """Pod Security Admission: label the operand namespace ``privileged`` (the
    driver, toolkit and plugin pods need host access)."""

    enabled: bool = False


class ClusterPolicySpec(_M):
    operator: OperatorSpec = Field(default_factory=OperatorSpec)
    psa: PSASpec = Field(default_factory=PSASpec)
    daemonsets: DaemonsetsSpec = Field(default_factory=DaemonsetsSpec)
    driver: DriverSpec = Field(default_factory=DriverSpec)
    toolkit: ToolkitSpec = Field(default_factory=ToolkitSpec)
    devicePlugin: DevicePluginSpec = Field(default_factory=DevicePluginSpec)
    draDriver: DraDriverSpec = Field(default_factory=DraDriverSpec)
    dcgmExporter: MetricsExporterSpec = Field(default_factory=MetricsExporterSpec, alias="metricsExporter")
    nodeStatusExporter: NodeStatusExporterSpec = Field(default_factory=NodeStatusExporterSpec)
    gfd: GFDSpec = Field(default_factory=GFDSpec)
    nfd: NFDSpec = Field(default_factory=NFDSpec)
    migManager: PartitionManagerSpec = Field(default_factory=PartitionManagerSpec, alias="partitionManager")
    validator: ValidatorSpec = Field(default_factory=ValidatorSpec)
    sandboxWorkloads: SandboxWorkloadsSpec = Field(default_factory=SandboxWorkloadsSpec)
    vfioManager: VFIOManagerSpec = Field(default_factory=VFIOManagerSpec)
    sandboxDevicePlugin: SandboxDevicePluginSpec = Field(default_factory=SandboxDevicePluginSpec)

    @model_validator(mode="before")
    @classmethod
    def _aliases(cls, data):
        if isinstance(data, dict):
            data = dict(data)
            for alias, key in (("metricsExporter", "dcgmExporter"), ("partitionManager", "migManager")):
                if alias in data and key in data:
                    raise ValueError(f"set either {alias} or {key}, not both")
                if alias in data:
                    data[key] = data.pop(alias)
        return data

    @model_validator(mode="after")
    def _consistency(self):
        if self.draDriver.enabled and self.devicePlugin.enabled:
            raise ValueError("draDriver.enabled needs devicePlugin.enabled=false: both would hand out the same GPUs "
                             "(ResourceClaims and amd.com/gpu)")
        if self.devicePlugin.enabled and not self.driver.enabled and not self.toolkit.enabled:
            pass  # host-installed driver/toolkit is a supported setup
        if self.migManager.enabled and self.devicePlugin.partitionStrategy == "single":
            pass  # partitions are advertised as amd.com/gpu
        return self


# operand state order, also the order a reconcile pass
# applies them in: node feature discovery first - its labels are what makes
# a node a GPU node, so every other operand of a bring-up waits for it
STATES = [
    ("pre-requisites", None),
    ("state-node-feature-discovery", "nfd"),
    ("state-driver", "driver"),
    ("state-container-toolkit", "toolkit"),
    ("state-operator-validation", "validator"),
    ("state-device-plugin", "devicePlugin"),
    ("state-dra-driver", "draDriver"),
    ("state-metrics-exporter", "dcgmExporter"),
    ("state-gpu-feature-discovery", "gfd"),
    ("state-partition-manager", "migManager"),
    ("state-node-status-exporter", "nodeStatusExporter"),
    # sandboxWorkloads (vm-passthrough nodes)
    ("state-vfio-manager", "vfioManager"),
    ("state-sandbox-validation", "sandboxValidator"),
    ("state-sandbox-device-plugin", "sandboxDevicePlugin"),
]

SANDBOX_OPERANDS = ("vfioManager", "sandboxValidator", "sandboxDevicePlugin")
# which operands a GPU node runs for its amd.com/gpu.workload.config
WORKLOAD_OPERANDS = {
    "container": ("driver", "toolkit", "validator", "devicePlugin", "draDriver", "dcgmExporter", "gfd", "migManager",
                  "nodeStatusExporter"),
    "vm-passthrough": SANDBOX_OPERANDS,
}


def operand_enabled(spec: ClusterPolicySpec, key: str | None) -> bool:
    """Is the operand of a state (``STATES`` key) switched on by the spec?
    Sandbox operands need ``sandboxWorkloads.enabled``; the sandbox validator
    follows ``validator.enabled``."""
    if key is None:
        return True
    if key in SANDBOX_OPERANDS:
        own = spec.validator.enabled if key == "sandboxValidator" else getattr(spec, key).enabled
        return spec.sandboxWorkloads.enabled and own
    return getattr(spec, key).enabled


class HelmValues(_M):
    """Top-level chart values (``deploy/helm/amd-gpu-operator/values.yaml``)."""

    model_config = ConfigDict(extra="allow", populate_by_name=True)
    namespace: str = DEFAULT_NAMESPACE
    operator: dict = Field(default_factory=dict)


def spec_from_values(values: dict) -> ClusterPolicySpec:
    """Helm values -> ClusterPolicy spec (chart-only keys are dropped)."""
    v = dict(values or {})
    for chart_only in ("namespace", "nameOverride", "fullnameOverride", "crds", "rbac", "serviceAccount",
                       "operatorImage", "nodeSelector", "podSecurityContext"):
        v.pop(chart_only, None)
    op = dict(v.get("operator") or {})
    for chart_only in ("image", "repository", "version", "imagePullPolicy", "resources", "replicas", "leaderElection"):
        op.pop(chart_only, None)
    if op or "operator" in v:
        v["operator"] = op
    return ClusterPolicySpec.model_validate(v)


def parse_set_flags(flags: list[str]) -> dict:
    """``--set a.b=c`` strings -> nested values dict (bools/ints parsed like Helm)."""
    out: dict = {}
    for f in flags:
        key, _, raw = f.partition("=")
        val: object = raw
        if raw in ("true", "false"):
            val = raw == "true"
        else:
            try:
                val = int(raw)
            except ValueError:
                try:
                    val = float(raw)
                except ValueError:
                    val = raw
        cur = out
        parts = key.split(".")
        for p in parts[:-1]:
            cur = cur.setdefault(p, {})
        cur[parts[-1]] = val
    return out


def deep_merge(base: dict, over: dict) -> dict:
    out = dict(base)
    for k, v in over.items():
        if isinstance(v, dict) and isinstance(out.get(k), dict):
            out[k] = deep_merge(out[k], v)
        else:
            out[k] = v
    return out


def cluster_policy(name: str = "cluster-policy", spec: ClusterPolicySpec | dict | None = None) -> dict:
    if isinstance(spec, dict) or spec is None:
        spec = ClusterPolicySpec.model_validate(spec or {})
    return {
        "apiVersion": f"{API_GROUP}/{API_VERSION}",
        "kind": "ClusterPolicy",
        "metadata": {"name": name},
        "spec": spec.model_dump(mode="json", by_alias=False),
    }


# the exact install command of the reference, as values (README.md:101-110)
REFERENCE_SET_FLAGS = [
    "driver.enabled=true",
    "toolkit.enabled=true",
    "devicePlugin.enabled=true",
    "nodeStatusExporter.enabled=true",
    "gfd.enabled=true",
    "migManager.enabled=false",
    "operator.cleanupCRD=true",
]


def policy_images(spec: ClusterPolicySpec | dict) -> dict[str, str]:
    """Every image the policy can run, by spec path (``driver``,
    ``validator``, ...): what a node pulls, what an air-gapped registry must
    mirror, and what the simulated kubelet can pull (testing/simcluster.py)."""
    if isinstance(spec, dict):
        spec = ClusterPolicySpec.model_validate(spec)
    out = {}
    for name in type(spec).model_fields:
        v = getattr(spec, name)
        if isinstance(v, Image):
            out[name] = v.ref(v.image)
    return out


def validator_pod_image(spec: ClusterPolicySpec | dict) -> dict:
    """The image a GPU check pod runs (plugin validation, ``verify --run-pod``,
    the example workloads): the validator's, with its pull policy and pull
    secrets - the same resolution the operand DaemonSets use."""
    if isinstance(spec, dict):
        spec = ClusterPolicySpec.model_validate(spec)
    v = spec.validator
    return {"image": v.ref(v.image), "pull_policy": v.imagePullPolicy, "pull_secrets": list(v.imagePullSecrets)}
