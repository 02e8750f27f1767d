"""Operand manifests rendered from the ClusterPolicy spec, one bundle per state.

Names follow the reference's operand pods (/root/reference/README.md:132,152,
184,201-207) with the AMD prefix:

  nvidia-driver-daemonset / nvidia-driver-ctr   -> amd-driver-daemonset / amd-driver-ctr (2/2 containers)
  nvidia-container-toolkit-daemonset            -> amd-container-toolkit-daemonset
  nvidia-device-plugin-daemonset                -> amd-device-plugin-daemonset
  nvidia-dcgm-exporter                          -> amd-metrics-exporter
  gpu-feature-discovery                         -> gpu-feature-discovery
  (node status exporter, validator, NFD, MIG mgr)-> amd-node-status-exporter, amd-operator-validator,
                                                    node-feature-discovery-worker, amd-partition-manager

Every operand container runs the same ``amdgpu-operator`` entry point with a
sub-command (``amdgpu_operator/cli/main.py``).  GPU operands are scheduled by
the per-node ``amd.com/gpu.deploy.<operand>=true`` labels the operator sets.
Ordering between operands is enforced on the node by init containers that
wait for validation files in the host's ``/run/amd/validations`` directory
(driver-ready -> toolkit-ready -> workload-ready -> plugin-ready).
"""

from __future__ import annotations

import os

from ..api.clusterpolicy import ClusterPolicySpec
from ..wellknown import DEPLOY_LABEL, OPERAND_LABELS  # noqa: F401 - re-exported

APP_LABEL = "app"
VALIDATIONS_HOST_DIR = "/run/amd/validations"


def owner_ref(cp: dict) -> list[dict]:
    md = cp["metadata"]
    return [{"apiVersion": cp["apiVersion"], "kind": cp["kind"], "name": md["name"], "uid": md.get("uid", ""),
             "controller": True, "blockOwnerDeletion": True}]


def _meta(name: str, ns: str | None, labels: dict, owner: list[dict] | None, extra_labels=None, annotations=None):
    m = {"name": name, "labels": {**labels, **(extra_labels or {})}}
    if ns:
        m["namespace"] = ns
    if owner:
        m["ownerReferences"] = owner
    if annotations:
        m["annotations"] = dict(annotations)
    return m


def _hostpath(name: str, path: str, type_: str = "DirectoryOrCreate") -> dict:
    return {"name": name, "hostPath": {"path": path, "type": type_}}


def _mount(name: str, path: str, ro: bool = False, propagation: str | None = None) -> dict:
    m = {"name": name, "mountPath": path}
    if ro:
        m["readOnly"] = True
    if propagation:
        m["mountPropagation"] = propagation
    return m


def _container(name: str, image: str, pull: str, args: list[str], mounts=None, env=None, privileged=False,
               resources=None, readiness=None, ports=None, command: str = "amdgpu-operator") -> dict:
    c = {"name": name, "image": image, "imagePullPolicy": pull, "command": [command], "args": list(args),
         "env": [{"name": "NODE_NAME", "valueFrom": {"fieldRef": {"fieldPath": "spec.nodeName"}}},
                 {"name": "OPERATOR_NAMESPACE", "valueFrom": {"fieldRef": {"fieldPath": "metadata.namespace"}}},
                 # which pod instance an operand is (the driver container's module ownership)
                 {"name": "POD_NAME", "valueFrom": {"fieldRef": {"fieldPath": "metadata.name"}}},
                 {"name": "POD_UID", "valueFrom": {"fieldRef": {"fieldPath": "metadata.uid"}}}]
         + list(env or []),
         "volumeMounts": list(mounts or [])}
    if privileged:
        c["securityContext"] = {"privileged": True}
    if resources and (resources.get("requests") or resources.get("limits")):
        c["resources"] = {k: v for k, v in resources.items() if v}
    if readiness:
        c["readinessProbe"] = readiness
    if ports:
        c["ports"] = ports
    return c


def _wait_init(name: str, image: str, pull: str, what: str, extra_args=(), env=None, mounts=()) -> dict:
    """Init container that blocks until a validation file exists on the host."""
    return _container(name, image, pull, ["validate", what, *extra_args],
                      mounts=[_mount("run-amd-validations", VALIDATIONS_HOST_DIR, propagation="HostToContainer"),
                              *_host_view(), *mounts],
                      env=env, privileged=True)


def _gate(spec: ClusterPolicySpec, ctr: dict, init: dict, step: str) -> list[dict]:
    """The prerequisite of an operand container: an init container (``init``)
    or, with ``daemonsets.inContainerGates``, the same wait inside ``ctr``
    (cli/operands.py VALIDATION_GATE) with the mounts the wait needs.
    Returns the init containers to use."""
    if not spec.daemonsets.inContainerGates:
        return [init]
    ctr["env"].append({"name": "VALIDATION_GATE", "value": step})
    have = {m["name"] for m in ctr["volumeMounts"]}
    ctr["volumeMounts"] += [m for m in init["volumeMounts"] if m["name"] not in have]
    return []


# the kubelet's pod-resources socket: the validator reads the device
# manager's allocatable devices there (deviceplugin/podresources.py)
POD_RESOURCES_MOUNT = {"name": "pod-resources", "mountPath": "/var/lib/kubelet/pod-resources", "readOnly": True}
# ...and watches the device-plugins directory, where the kubelet checkpoints
# each device-list update (validate.py _wait_kubelet_devices)
DEVICE_PLUGINS_MOUNT = {"name": "device-plugin", "mountPath": "/var/lib/kubelet/device-plugins", "readOnly": True}


def _workload_pod_env(v, image: str) -> list[dict]:
    """What the plugin-validation pods the validator creates run: its own image."""
    return [{"name": "VALIDATOR_IMAGE", "value": image}, {"name": "VALIDATOR_IMAGE_PULL_POLICY", "value": v.imagePullPolicy},
            {"name": "VALIDATOR_IMAGE_PULL_SECRETS", "value": ",".join(v.imagePullSecrets)}]


def _host_view() -> list[dict]:
    """/host/sys + /host/dev: what the N1 probe and the topology reader need
    (NodeEnv.host_root = /host inside operand containers)."""
    return [_mount("host-sys", "/host/sys", ro=True), _mount("host-dev", "/host/dev", ro=True)]


def _daemonset(spec: ClusterPolicySpec, ns: str, owner, name: str, operand_key: str | None, sa: str,
               containers: list, init_containers: list = (), volumes: list = (), host_pid: bool = False,
               host_network: bool = False, node_selector: dict | None = None, extra_labels=None,
               operand=None) -> dict:
    ds = spec.daemonsets
    operand = operand if operand is not None else (getattr(spec, operand_key) if operand_key else None)
    labels = {APP_LABEL: name, "app.kubernetes.io/part-of": "amd-gpu-operator",
              "app.kubernetes.io/managed-by": "amd-gpu-operator"}
    if node_selector is None:
        node_selector = {DEPLOY_LABEL.format(OPERAND_LABELS[operand_key]): "true"} if operand_key else {}
    volumes = list(volumes)
    # the host's /sys and /dev as the N1 probe reads them (NodeEnv host_root
    # "/host"): any container mounting them gets the volume without each
    # state builder repeating it
    have = {v["name"] for v in volumes}
    mounted = {m["name"] for c in [*containers, *init_containers] for m in c.get("volumeMounts", [])}
    for vol_name, host_path in (("host-sys", "/sys"), ("host-dev", "/dev")):
        if vol_name in mounted and vol_name not in have:
            volumes.append(_hostpath(vol_name, host_path, "Directory"))
    tmpl_spec = {
        "serviceAccountName": sa,
        "priorityClassName": ds.priorityClassName,
        "tolerations": [dict(t) for t in ds.tolerations],
        "nodeSelector": node_selector,
        "hostPID": host_pid,
        "hostNetwork": host_network,
        "initContainers": list(init_containers),
        "containers": list(containers),
        "volumes": volumes,
    }
    if operand is not None and operand.imagePullSecrets:  # private registries (<operand>.imagePullSecrets)
        tmpl_spec["imagePullSecrets"] = [{"name": n} for n in operand.imagePullSecrets]
    strategy = {"type": ds.updateStrategy}
    if ds.updateStrategy == "RollingUpdate":
        strategy["rollingUpdate"] = {"maxUnavailable": ds.maxUnavailable}
    return {
        "apiVersion": "apps/v1",
        "kind": "DaemonSet",
        "metadata": _meta(name, ns, labels, owner, {**ds.labels, **(extra_labels or {})}, ds.annotations),
        "spec": {
            "selector": {"matchLabels": {APP_LABEL: name}},
            "updateStrategy": strategy,
            "template": {"metadata": {"labels": {**labels, **ds.labels}, "annotations": dict(ds.annotations)},
                         "spec": tmpl_spec},
        },
    }


def _sa(name: str, ns: str, owner) -> dict:
    return {"apiVersion": "v1", "kind": "ServiceAccount", "metadata": _meta(name, ns, {APP_LABEL: name}, owner)}


def _cluster_role(name: str, rules: list[dict], owner) -> dict:
    return {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRole",
            "metadata": _meta(name, None, {APP_LABEL: name}, owner), "rules": rules}


def _cluster_binding(name: str, sa: str, ns: str, owner) -> dict:
    return {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRoleBinding",
            "metadata": _meta(name, None, {APP_LABEL: name}, owner),
            "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "ClusterRole", "name": name},
            "subjects": [{"kind": "ServiceAccount", "name": sa, "namespace": ns}]}


def _service(name: str, ns: str, owner, port: int, port_name: str = "metrics") -> dict:
    return {"apiVersion": "v1", "kind": "Service",
            "metadata": _meta(name, ns, {APP_LABEL: name}, owner),
            "spec": {"selector": {APP_LABEL: name}, "ports": [{"name": port_name, "port": port, "targetPort": port,
                                                                "protocol": "TCP"}],
                     "type": "ClusterIP"}}


NODE_RW_RULES = [
    {"apiGroups": [""], "resources": ["nodes"], "verbs": ["get", "list", "watch", "patch", "update"]},
    {"apiGroups": [""], "resources": ["pods"], "verbs": ["get", "list", "watch", "create", "delete"]},
    {"apiGroups": [""], "resources": ["events"], "verbs": ["create", "patch"]},
]
PLUGIN_CONFIG_RULES = [
    {"apiGroups": [""], "resources": ["nodes"], "verbs": ["get", "list", "watch"]},
    {"apiGroups": [""], "resources": ["configmaps"], "verbs": ["get", "list", "watch"]},
]


# ------------------------------------------------------------------ states ----

def state_prerequisites(spec: ClusterPolicySpec, ns: str, owner) -> list[dict]:
    objs = []
    rc = spec.operator.runtimeClass
    if spec.toolkit.enabled and rc:
        objs.append({"apiVersion": "node.k8s.io/v1", "kind": "RuntimeClass",
                     "metadata": _meta(rc, None, {APP_LABEL: "amd-gpu-operator"}, owner), "handler": rc})
    return objs


def state_driver(spec: ClusterPolicySpec, ns: str, owner, name: str = "amd-driver-daemonset",
                 node_selector: dict | None = None, kernel: str | None = None) -> list[dict]:
    """The driver DaemonSet: policy-wide, per AMDGPUDriver pool
    (``node_selector``), or per node kernel (``kernel``, usePrecompiled: the
    image tagged ``<driverVersion>-<kernel>`` holds modules built for it)."""
    from .upgrade import HASH_LABEL, driver_spec_hash

    d = spec.driver
    sa = "amd-driver"
    image = d.ref("amd-driver")
    if kernel is not None:
        image = f"{d.repository}/{d.image or 'amd-driver'}:{d.driverVersion}-{kernel}"
    spec_hash = driver_spec_hash(spec)
    env = [{"name": "ROCM_VERSION", "value": d.rocmVersion}, {"name": "AMDGPU_DRIVER_VERSION", "value": d.driverVersion},
           {"name": "AMDGPU_DRIVER_SPEC_HASH", "value": spec_hash},
           {"name": "AMDGPU_USE_PRECOMPILED", "value": str(d.usePrecompiled).lower()},
           {"name": "AMDGPU_BLACKLIST_INBOX", "value": str(d.blacklistAmdgpuInbox).lower()},
           {"name": "AMDGPU_MODULE_PARAMS", "value": " ".join(f"{k}={v}" for k, v in sorted(d.kernelModuleParams.items()))},
           {"name": "AMDGPU_WAIT_SECONDS", "value": str(d.startupProbeTimeoutSeconds)},
           {"name": "AMDGPU_UNLOAD_ON_EXIT", "value": str(d.unloadOnExit).lower()},
           {"name": "AMDGPU_RDMA_ENABLED", "value": str(d.rdma.enabled).lower()},
           {"name": "AMDGPU_RDMA_USE_HOST_MOFED", "value": str(d.rdma.useHostMofed).lower()}
           ] + ([{"name": "AMDGPU_REPO_BASE", "value": d.packageRepository}] if d.packageRepository else []) + list(d.env)
    mounts = [_mount("run-amd", "/run/amd", propagation="Bidirectional"), _mount("host-root", "/host", ro=True,
                                                                                 propagation="HostToContainer"),
              _mount("lib-modules", "/lib/modules"), _mount("dev", "/dev"), _mount("host-sys", "/host/sys", ro=True),
              _mount("run-amd-validations", VALIDATIONS_HOST_DIR)]
    if not d.usePrecompiled:  # DKMS builds against the node's kernel headers (install.sh ensure_headers)
        mounts.append(_mount("host-usr-src", "/host/usr/src", ro=True))
    readiness = {"exec": {"command": ["amdgpu-probe", "--root", "/host", "--ready-file",
                                      f"{VALIDATIONS_HOST_DIR}/driver-ready"]},
                 "initialDelaySeconds": 5, "periodSeconds": 10, "failureThreshold": 60}
    drain_env = [{"name": "DRAIN_ENABLED", "value": str(d.upgradePolicy.drainEnabled).lower()},
                 {"name": "DRAIN_TIMEOUT_SECONDS", "value": str(d.upgradePolicy.drainTimeoutSeconds)}]
    gated = spec.daemonsets.inContainerGates  # the upgrade check runs in amd-driver-ctr itself
    ctr = _container("amd-driver-ctr", image, d.imagePullPolicy,
                     ["driver", "install", *(["--prepare-upgrade"] if gated else []), *d.args], mounts,
                     env + (drain_env if gated else []), True, d.resources.model_dump(), readiness)
    health = _container("amd-driver-health", image, d.imagePullPolicy, ["driver", "monitor"],
                        [*_host_view(), _mount("run-amd-validations", VALIDATIONS_HOST_DIR)], privileged=True)
    # the init container compares the live module with this spec and unloads it
    # on a mismatch, so it gets the same driver env as amd-driver-ctr
    init = _container("amd-driver-manager", image, d.imagePullPolicy, ["driver", "prepare-upgrade"],
                      [_mount("run-amd", "/run/amd"), _mount("lib-modules", "/lib/modules"), *_host_view()],
                      env + drain_env, True)
    vols = [_hostpath("run-amd", "/run/amd"), _hostpath("host-root", "/", "Directory"),
            _hostpath("lib-modules", "/lib/modules"), _hostpath("dev", "/dev", "Directory"),
            _hostpath("host-sys", "/sys", "Directory"), _hostpath("run-amd-validations", VALIDATIONS_HOST_DIR)]
    if not d.usePrecompiled:
        vols.append(_hostpath("host-usr-src", "/usr/src", "DirectoryOrCreate"))
    sel = None
    if kernel is not None:  # one DaemonSet per kernel: the image was built for it
        sel = {DEPLOY_LABEL.format(OPERAND_LABELS["driver"]): "true", KERNEL_LABEL: kernel}
    elif node_selector is not None:  # AMDGPUDriver pool: the driver deploy label plus the pool's selector
        sel = {DEPLOY_LABEL.format(OPERAND_LABELS["driver"]): "true", **node_selector}
    ds = _daemonset(spec, ns, owner, name, "driver", sa, [ctr, health], [] if gated else [init], vols, host_pid=True,
                    node_selector=sel)
    # what the pods install, for the upgrade controller (controller/upgrade.py)
    ds["spec"]["template"]["metadata"]["labels"][HASH_LABEL] = spec_hash
    if kernel is not None:
        ds["metadata"]["labels"][KERNEL_DS_LABEL] = ds["spec"]["template"]["metadata"]["labels"][KERNEL_DS_LABEL] = \
            kernel_suffix(kernel)
    if d.upgradePolicy.autoUpgrade and node_selector is None:  # node-by-node rollout (controller/upgrade.py)
        ds["spec"]["updateStrategy"] = {"type": "OnDelete"}
    return [_sa(sa, ns, owner), _cluster_role(sa, NODE_RW_RULES, owner), _cluster_binding(sa, sa, ns, owner), ds]


def state_toolkit(spec: ClusterPolicySpec, ns: str, owner) -> list[dict]:
    t = spec.toolkit
    name, sa = "amd-container-toolkit-daemonset", "amd-container-toolkit"
    image = t.ref("amd-container-toolkit")
    env = [{"name": "RUNTIME", "value": t.runtime}, {"name": "CONTAINERD_CONFIG", "value": t.containerdConfig},
           {"name": "CONTAINERD_SOCKET", "value": t.containerdSocket}, {"name": "RUNTIME_CLASS", "value": t.runtimeClass},
           {"name": "INSTALL_DIR", "value": t.installDir}, {"name": "CDI_ENABLED", "value": str(t.cdi.enabled).lower()},
           {"name": "CDI_SPEC_DIR", "value": t.cdi.specDir}, {"name": "MOUNT_ROCM", "value": str(t.mountRocm).lower()},
           {"name": "ACCEPT_DEVICE_LIST_AS_VOLUME_MOUNTS", "value": str(t.acceptDeviceListAsVolumeMounts).lower()},
           {"name": "ACCEPT_ENVVAR_UNPRIVILEGED", "value": str(t.acceptEnvvarUnprivileged).lower()},
           {"name": "CONTAINERD_SET_AS_DEFAULT", "value": str(t.setAsDefault).lower()},
           {"name": "CLEANUP_ON_EXIT", "value": str(t.cleanupOnExit).lower()},
           ] + list(t.env)
    # the runtime's host directories are mounted at their host paths, so the
    # paths the installer writes into the runtime's configuration (imports,
    # hooks dirs, CDI dirs) are the paths the runtime itself reads
    if t.runtime == "containerd":
        runtime_dirs = [os.path.dirname(t.containerdConfig), os.path.dirname(t.containerdSocket)]
        env.append({"name": "RUNTIME_PID_FILE", "value": os.path.join(os.path.dirname(t.containerdSocket),
                                                                        "containerd.pid")})
    elif t.runtime == "crio":
        runtime_dirs = [t.crioConfigDir]
    else:
        runtime_dirs = [os.path.dirname(t.dockerConfig)]
    env += [{"name": "CRIO_CONFIG_DIR", "value": t.crioConfigDir}, {"name": "DOCKER_CONFIG", "value": t.dockerConfig}]
    runtime_mounts = [(f"runtime-dir-{i}", d) for i, d in enumerate(dict.fromkeys(runtime_dirs))]
    mounts = [_mount(n, d) for n, d in runtime_mounts] + [
        _mount("install-dir", t.installDir), _mount("cdi-dir", t.cdi.specDir),
        *_host_view(), _mount("run-amd-validations", VALIDATIONS_HOST_DIR)]
    ctr = _container("amd-container-toolkit-ctr", image, t.imagePullPolicy, ["toolkit", "install", *t.args], mounts, env,
                     True, t.resources.model_dump())
    inits = _gate(spec, ctr, _wait_init("driver-validation", image, t.imagePullPolicy, "driver"), "driver")
    vols = [_hostpath(n, d, "DirectoryOrCreate") for n, d in runtime_mounts] + [
        _hostpath("install-dir", t.installDir), _hostpath("cdi-dir", t.cdi.specDir),
        _hostpath("host-sys", "/sys", "Directory"), _hostpath("run-amd-validations", VALIDATIONS_HOST_DIR)]
    return [_sa(sa, ns, owner), _daemonset(spec, ns, owner, name, "toolkit", sa, [ctr], inits, vols, host_pid=True)]


def state_validator(spec: ClusterPolicySpec, ns: str, owner) -> list[dict]:
    v = spec.validator
    name, sa = "amd-operator-validator", "amd-operator-validator"
    image = v.ref("amd-operator-validator")
    w = v.workload
    wl_args = ["--gemm", str(w.gemmN), "--gemm-iters", str(w.gemmIters), "--hbm-bytes", str(w.hbmBytes),
               "--rccl-elems", str(w.rcclElems), "--xgmi-elems", str(w.xgmiElems)]
    if w.mfmaRateCheck:
        wl_args += ["--fp8-gemm", str(w.mfmaRateGemmN), "--fp4-gemm", str(w.mfmaRateGemmN)]
    else:
        wl_args += ["--no-mfma-rate"]
    for flag, val in (("--min-gemm-tflops", w.minGemmTflops), ("--min-hbm-gbps", w.minHbmGbps),
                      ("--min-fp8-tflops", w.minFp8Tflops if w.mfmaRateCheck else 0),
                      ("--min-fp4-tflops", w.minFp4Tflops if w.mfmaRateCheck else 0),
                      ("--min-fp6-tflops", w.minFp6Tflops if w.mfmaRateCheck else 0),
                      ("--min-mxfp4-tflops", w.minMxfp4Tflops if w.mfmaRateCheck else 0),
                      ("--min-mfma-util", w.minMfmaUtil), ("--rccl-busbw-link-fraction", w.rcclBusbwLinkFraction),
                      ("--xgmi-read-link-fraction", w.xgmiReadLinkFraction)):
        if val:
            wl_args += [flag, f"{val:g}"]
    if not w.gateLock:
        wl_args.append("--no-gate-lock")
    if w.deferGates:
        wl_args.append("--defer-gates")
    util = {k: v for k, v in w.minMfmaUtilByDtype.items() if w.mfmaRateCheck or k == "bf16"}
    if util:
        wl_args += ["--min-mfma-util-by-dtype", ",".join(f"{k}={v:g}" for k, v in sorted(util.items()))]
    wl_args += ["--peer-timeout", f"{w.peerTimeoutSeconds:g}", "--collective-timeout", f"{w.collectiveTimeoutSeconds:g}",
                "--max-gpu-processes", str(w.maxGpuProcesses)]
    if w.requireXgmiLinks:
        wl_args += ["--require-xgmi-links", "--min-xgmi-link-fraction", f"{w.minXgmiLinkFraction:g}"]
    if w.counterGate:
        wl_args += ["--counter-gate"] + (["--gate-mode", "sdk"] if w.counterGateMode == "sdk" else [])
    if w.rcclSingleGpu:
        wl_args += ["--rccl-single-gpu"]
    if w.rcclProcess == "separate":
        wl_args += ["--rccl-separate-process"]
    if spec.driver.rdma.enabled:  # HBM exported as a dma-buf, what the RDMA NICs import
        wl_args += ["--dmabuf"]
    inits = [_wait_init("driver-validation", image, v.imagePullPolicy, "driver")]
    # the plugin pods request what the device plugin advertises (its resource
    # name, and amd.com/gpu-<mode> for partitioned GPUs under "mixed")
    plugin_res = ["--resource", spec.devicePlugin.resourceName,
                  "--partition-strategy", spec.devicePlugin.partitionStrategy, "--pod-check", v.pluginPodCheck,
                  "--plugin-pods", v.pluginPods]
    # the GPUs' advertiser: the device plugin, or the DRA driver (a claim and a pod through the scheduler)
    advertiser = spec.devicePlugin.enabled or spec.draDriver.enabled
    if spec.draDriver.enabled:
        plugin_res += ["--dra", "--dra-device-class", spec.draDriver.deviceClass]
    if v.pluginValidation and advertiser and w.prespawn:
        # one init container validates the driver and, meanwhile, starts the
        # workload processes behind their start gate (validate.py validate_gpu)
        extra = [*plugin_res, "--with-driver"] + (["--wait-toolkit"] if spec.toolkit.enabled else [])
        inits = [_wait_init("gpu-validation", image, v.imagePullPolicy, "gpu", [*extra, *wl_args],
                            env=_workload_pod_env(v, image), mounts=[POD_RESOURCES_MOUNT, DEVICE_PLUGINS_MOUNT])]
    elif v.pluginValidation and advertiser:  # (validation pods: _workload_pod_env)
        # workload (all GPUs, RCCL over xGMI) and plugin (1-GPU pods through the
        # device plugin + OCI hook) validation run concurrently.  The workload
        # needs only the driver (its processes run in this pod, not through the
        # runtime hook), so it overlaps the toolkit install; the plugin pods
        # wait for the toolkit inside the step.
        extra = plugin_res + (["--wait-toolkit"] if spec.toolkit.enabled else [])
        inits.append(_wait_init("gpu-validation", image, v.imagePullPolicy, "gpu", [*extra, *wl_args],
                                env=_workload_pod_env(v, image), mounts=[POD_RESOURCES_MOUNT, DEVICE_PLUGINS_MOUNT]))
    else:
        if spec.toolkit.enabled:
            inits.append(_wait_init("toolkit-validation", image, v.imagePullPolicy, "toolkit"))
        inits.append(_wait_init("workload-validation", image, v.imagePullPolicy, "workload", wl_args))
    ctr = _container("amd-operator-validator", image, v.imagePullPolicy, ["validate", "complete"],
                     [_mount("run-amd-validations", VALIDATIONS_HOST_DIR)], list(v.env), True,
                     v.resources.model_dump())
    if spec.daemonsets.inContainerGates and len(inits) == 1 and inits[0]["name"] == "gpu-validation":
        # the main container validates (driver, workload, plugin) and then
        # completes: one container start instead of two
        gi = inits.pop()
        ctr["args"] = [*gi["args"], "--complete"]
        ctr["env"] = gi["env"] + list(v.env)
        ctr["volumeMounts"] = gi["volumeMounts"]
    vols = [_hostpath("run-amd-validations", VALIDATIONS_HOST_DIR), _hostpath("host-sys", "/sys", "Directory")]
    if any(m["name"] == "pod-resources" for c in [*inits, ctr] for m in c["volumeMounts"]):
        vols += [_hostpath("pod-resources", "/var/lib/kubelet/pod-resources"),
                 _hostpath("device-plugin", "/var/lib/kubelet/device-plugins")]
    rules = NODE_RW_RULES + (VALIDATOR_DRA_RULES if spec.draDriver.enabled else [])
    return [_sa(sa, ns, owner), _cluster_role(sa, rules, owner), _cluster_binding(sa, sa, ns, owner),
            _daemonset(spec, ns, owner, name, "validator", sa, [ctr], inits, vols)]


# validate.py validate_dra: the node's slice, and a claim it creates and deletes
VALIDATOR_DRA_RULES = [
    {"apiGroups": ["resource.k8s.io"], "resources": ["resourceslices"], "verbs": ["get", "list", "watch"]},
    {"apiGroups": ["resource.k8s.io"], "resources": ["resourceclaims"],
     "verbs": ["get", "list", "watch", "create", "delete"]},
]


def state_device_plugin(spec: ClusterPolicySpec, ns: str, owner) -> list[dict]:
    p = spec.devicePlugin
    name, sa = "amd-device-plugin-daemonset", "amd-device-plugin"
    image = p.ref("amd-device-plugin")
    args = ["device-plugin", "--resource-name", p.resourceName, "--partition-strategy", p.partitionStrategy,
            "--health-poll-ms", str(p.healthPollMs), "--device-id-strategy", p.deviceIDStrategy,
            "--device-list-strategy", ",".join(p.deviceListStrategy),
            "--health-start", "after-validation" if p.healthStart == "afterValidation" else "immediate"]
    if spec.toolkit.enabled and spec.toolkit.cdi.enabled and p.cdiAnnotations:
        args.append("--cdi")
    if not p.passDeviceSpecs:
        args.append("--no-device-specs")
    if spec.driver.rdma.enabled:  # nearest RDMA NICs of each allocation (discovery/rdma.py)
        args += ["--rdma"] + (["--rdma-hca-env"] if spec.driver.rdma.hcaEnv else [])
    rbac = []
    if p.config.name:  # config-manager loop: reads the ConfigMap and this node's config label
        args += ["--config-map", f"{ns}/{p.config.name}", "--config-default", p.config.default]
        rbac = [_cluster_role(sa, PLUGIN_CONFIG_RULES, owner), _cluster_binding(sa, sa, ns, owner)]
    ctr = _container("amd-device-plugin", image, p.imagePullPolicy, args + list(p.args),
                     [_mount("device-plugin", "/var/lib/kubelet/device-plugins"), *_host_view()],
                     list(p.env), True, p.resources.model_dump())
    gate = "toolkit" if spec.toolkit.enabled else "driver"
    inits = _gate(spec, ctr, _wait_init("toolkit-validation", image, p.imagePullPolicy, gate), gate)
    vols = [_hostpath("device-plugin", "/var/lib/kubelet/device-plugins"), _hostpath("host-sys", "/sys", "Directory"),
            _hostpath("run-amd-validations", VALIDATIONS_HOST_DIR)]
    return [_sa(sa, ns, owner), *rbac, _daemonset(spec, ns, owner, name, "devicePlugin", sa, [ctr], inits, vols)]


DRA_RULES = [
    {"apiGroups": [""], "resources": ["nodes"], "verbs": ["get"]},
    {"apiGroups": ["resource.k8s.io"], "resources": ["resourceslices"],
     "verbs": ["get", "list", "watch", "create", "update", "delete"]},
    {"apiGroups": ["resource.k8s.io"], "resources": ["resourceclaims"], "verbs": ["get"]},
]


def state_dra_driver(spec: ClusterPolicySpec, ns: str, owner) -> list[dict]:
    """DRA driver gpu.amd.com (dra/driver.py): publishes the node's
    ResourceSlice, registers with the kubelet's plugin watcher and prepares
    claims as CDI specs; plus the DeviceClass claims name."""
    from ..dra.driver import device_class

    d = spec.draDriver
    name, sa = "amd-dra-driver", "amd-dra-driver"
    image = d.ref("amd-device-plugin")
    ctr = _container("amd-dra-driver", image, d.imagePullPolicy, ["dra-driver", *d.args],
                     [_mount("kubelet-plugins", "/var/lib/kubelet/plugins"),
                      _mount("kubelet-registry", "/var/lib/kubelet/plugins_registry"),
                      _mount("cdi-dir", spec.toolkit.cdi.specDir), *_host_view()],
                     [{"name": "CDI_SPEC_DIR", "value": spec.toolkit.cdi.specDir}, *d.env], True,
                     d.resources.model_dump())
    # claims are injected as CDI devices: the runtime must have CDI on (the toolkit) before devices are published
    gate = "toolkit" if spec.toolkit.enabled else "driver"
    inits = _gate(spec, ctr, _wait_init("toolkit-validation", image, d.imagePullPolicy, gate), gate)
    vols = [_hostpath("kubelet-plugins", "/var/lib/kubelet/plugins"),
            _hostpath("kubelet-registry", "/var/lib/kubelet/plugins_registry"),
            _hostpath("cdi-dir", spec.toolkit.cdi.specDir), _hostpath("host-sys", "/sys", "Directory"),
            _hostpath("run-amd-validations", VALIDATIONS_HOST_DIR)]
    dc = device_class(d.deviceClass)
    dc["metadata"]["ownerReferences"] = owner
    return [_sa(sa, ns, owner), _cluster_role(sa, DRA_RULES, owner), _cluster_binding(sa, sa, ns, owner), dc,
            _daemonset(spec, ns, owner, name, "draDriver", sa, [ctr], inits, vols)]


def state_metrics_exporter(spec: ClusterPolicySpec, ns: str, owner) -> list[dict]:
    m = spec.dcgmExporter
    name, sa = "amd-metrics-exporter", "amd-metrics-exporter"
    image = m.ref("amd-metrics-exporter")
    args = ["metrics-exporter", "--port", str(m.port), "--interval", str(m.intervalSeconds)]
    if m.podAttribution:
        args.append("--pod-attribution")
    if m.dcgmNames:
        args.append("--dcgm-names")
    if not m.healthEvents:
        args.append("--no-health-events")
    rbac = []
    if m.config.name:
        args += ["--metrics-config-map", f"{ns}/{m.config.name}/{m.config.key}"]
        rbac = [_cluster_role(sa, PLUGIN_CONFIG_RULES[1:], owner), _cluster_binding(sa, sa, ns, owner)]
    ctr = _container("amd-metrics-exporter", image, m.imagePullPolicy, args + list(m.args),
                     [_mount("pod-resources", "/var/lib/kubelet/pod-resources", ro=True),
                      *_host_view()], list(m.env), True, m.resources.model_dump(),
                     ports=[{"name": "metrics", "containerPort": m.port}])
    inits = _gate(spec, ctr, _wait_init("driver-validation", image, m.imagePullPolicy, "driver"), "driver")
    vols = [_hostpath("pod-resources", "/var/lib/kubelet/pod-resources"), _hostpath("host-sys", "/sys", "Directory"),
            _hostpath("run-amd-validations", VALIDATIONS_HOST_DIR)]
    objs = [_sa(sa, ns, owner), *rbac, _daemonset(spec, ns, owner, name, "dcgmExporter", sa, [ctr], inits, vols),
            _service(name, ns, owner, m.port)]
    if m.serviceMonitor.enabled:
        objs.append({"apiVersion": "monitoring.coreos.com/v1", "kind": "ServiceMonitor",
                     "metadata": _meta(name, ns, {APP_LABEL: name}, owner, m.serviceMonitor.additionalLabels),
                     "spec": {"selector": {"matchLabels": {APP_LABEL: name}},
                              "endpoints": [{"port": "metrics", "interval": m.serviceMonitor.interval}]}})
    return objs


def state_nfd(spec: ClusterPolicySpec, ns: str, owner) -> list[dict]:
    n = spec.nfd
    name, sa = "node-feature-discovery-worker", "node-feature-discovery"
    image = n.ref("node-feature-discovery")
    # the native worker (native/nfd/nfd_worker.cpp): the first operand of every
    # bring-up, so no interpreter start on the critical path
    ctr = _container("nfd-worker", image, n.imagePullPolicy, ["--interval", str(n.intervalSeconds)],
                     [_mount("host-sys", "/host/sys", ro=True)], list(n.env), False, n.resources.model_dump(),
                     command="amdgpu-nfd")
    vols = [_hostpath("host-sys", "/sys", "Directory")]
    # runs on every node: it is what identifies the GPU nodes in the first place
    ds = _daemonset(spec, ns, owner, name, None, sa, [ctr], [], vols, node_selector={}, operand=n)
    ds["spec"]["template"]["spec"]["tolerations"].append({"operator": "Exists"})
    return [_sa(sa, ns, owner), _cluster_role(sa, NODE_RW_RULES, owner), _cluster_binding(sa, sa, ns, owner), ds]


def state_gfd(spec: ClusterPolicySpec, ns: str, owner) -> list[dict]:
    g = spec.gfd
    name, sa = "gpu-feature-discovery", "gpu-feature-discovery"
    image = g.ref("gpu-feature-discovery")
    args = ["gfd", "--interval", str(g.intervalSeconds), "--label-prefix", g.labelPrefix]
    if spec.devicePlugin.config.name:  # sharing labels follow the device-plugin config
        args += ["--device-plugin-config-map", f"{ns}/{spec.devicePlugin.config.name}",
                 "--device-plugin-config-default", spec.devicePlugin.config.default]
    ctr = _container("gpu-feature-discovery", image, g.imagePullPolicy, args + list(g.args),
                     [_mount("host-sys", "/host/sys", ro=True)], list(g.env), False, g.resources.model_dump())
    inits = _gate(spec, ctr, _wait_init("driver-validation", image, g.imagePullPolicy, "driver"), "driver")
    vols = [_hostpath("host-sys", "/sys", "Directory"), _hostpath("run-amd-validations", VALIDATIONS_HOST_DIR)]
    return [_sa(sa, ns, owner), _cluster_role(sa, NODE_RW_RULES + PLUGIN_CONFIG_RULES[1:], owner),
            _cluster_binding(sa, sa, ns, owner), _daemonset(spec, ns, owner, name, "gfd", sa, [ctr], inits, vols)]


def state_partition_manager(spec: ClusterPolicySpec, ns: str, owner) -> list[dict]:
    p = spec.migManager
    name, sa = "amd-partition-manager", "amd-partition-manager"
    image = p.ref("amd-partition-manager")
    ctr = _container("amd-partition-manager", image, p.imagePullPolicy,
                     ["partition-manager", "--config-label", p.configLabel, "--default-compute",
                      p.defaultComputePartition, "--default-memory", p.defaultMemoryPartition] + list(p.args),
                     [_mount("host-sys", "/host/sys"), _mount("run-amd-validations", VALIDATIONS_HOST_DIR)],
                     list(p.env), True, p.resources.model_dump())
    inits = _gate(spec, ctr, _wait_init("driver-validation", image, p.imagePullPolicy, "driver"), "driver")
    vols = [_hostpath("host-sys", "/sys", "Directory"), _hostpath("run-amd-validations", VALIDATIONS_HOST_DIR)]
    return [_sa(sa, ns, owner), _cluster_role(sa, NODE_RW_RULES, owner), _cluster_binding(sa, sa, ns, owner),
            _daemonset(spec, ns, owner, name, "migManager", sa, [ctr], inits, vols, host_pid=True)]


def state_node_status_exporter(spec: ClusterPolicySpec, ns: str, owner) -> list[dict]:
    n = spec.nodeStatusExporter
    name, sa = "amd-node-status-exporter", "amd-node-status-exporter"
    image = n.ref("amd-node-status-exporter")
    ctr = _container("amd-node-status-exporter", image, n.imagePullPolicy,
                     ["node-status-exporter", "--port", str(n.port)] + list(n.args),
                     [_mount("run-amd-validations", VALIDATIONS_HOST_DIR, ro=True)], list(n.env), False,
                     n.resources.model_dump(), ports=[{"name": "metrics", "containerPort": n.port}])
    vols = [_hostpath("run-amd-validations", VALIDATIONS_HOST_DIR)]
    return [_sa(sa, ns, owner), _daemonset(spec, ns, owner, name, "nodeStatusExporter", sa, [ctr], [], vols),
            _service(name, ns, owner, n.port)]


def state_vfio_manager(spec: ClusterPolicySpec, ns: str, owner) -> list[dict]:
    """vm-passthrough nodes: GPUs (whole IOMMU groups) to vfio-pci (sandbox/vfio.py)."""
    m = spec.vfioManager
    name, sa = "amd-vfio-manager", "amd-vfio-manager"
    image = m.ref("amd-vfio-manager")
    ctr = _container("amd-vfio-manager", image, m.imagePullPolicy,
                     ["vfio-manager", "bind", "--kfd-idle-timeout", str(m.kfdIdleTimeoutSeconds)] + list(m.args),
                     [_mount("host-sys", "/host/sys"), _mount("host-dev", "/host/dev", ro=True),
                      _mount("lib-modules", "/lib/modules", ro=True),
                      _mount("run-amd-validations", VALIDATIONS_HOST_DIR)], list(m.env), True, m.resources.model_dump())
    vols = [_hostpath("host-sys", "/sys", "Directory"), _hostpath("host-dev", "/dev", "Directory"),
            _hostpath("lib-modules", "/lib/modules", "Directory"), _hostpath("run-amd-validations", VALIDATIONS_HOST_DIR)]
    # reads its Node at exit: GPUs go back to amdgpu only when the node left vm-passthrough
    return [_sa(sa, ns, owner), _cluster_role(sa, PLUGIN_CONFIG_RULES[:1], owner), _cluster_binding(sa, sa, ns, owner),
            _daemonset(spec, ns, owner, name, "vfioManager", sa, [ctr], [], vols, host_pid=True)]


def state_sandbox_validator(spec: ClusterPolicySpec, ns: str, owner) -> list[dict]:
    """vm-passthrough nodes: every GPU on vfio-pci with its /dev/vfio group node."""
    v = spec.validator
    name, sa = "amd-sandbox-validator", "amd-sandbox-validator"
    image = v.ref("amd-operator-validator")
    init = _wait_init("vfio-pci-validation", image, v.imagePullPolicy, "vfio")
    ctr = _container("amd-sandbox-validator", image, v.imagePullPolicy, ["validate", "sandbox-complete"],
                     [_mount("run-amd-validations", VALIDATIONS_HOST_DIR)], list(v.env), True, v.resources.model_dump())
    vols = [_hostpath("run-amd-validations", VALIDATIONS_HOST_DIR)]
    return [_sa(sa, ns, owner), _cluster_role(sa, NODE_RW_RULES, owner), _cluster_binding(sa, sa, ns, owner),
            _daemonset(spec, ns, owner, name, "sandboxValidator", sa, [ctr], [init], vols, operand=v)]


def state_sandbox_device_plugin(spec: ClusterPolicySpec, ns: str, owner) -> list[dict]:
    """vm-passthrough nodes: vfio GPUs as amd.com/<product> (sandbox/plugin.py)."""
    p = spec.sandboxDevicePlugin
    name, sa = "amd-sandbox-device-plugin-daemonset", "amd-sandbox-device-plugin"
    image = p.ref("amd-sandbox-device-plugin")
    ctr = _container("amd-sandbox-device-plugin", image, p.imagePullPolicy,
                     ["sandbox-device-plugin", "--resource-prefix", p.resourcePrefix] + list(p.args),
                     [_mount("device-plugin", "/var/lib/kubelet/device-plugins"), *_host_view()],
                     list(p.env), True, p.resources.model_dump())
    init = _wait_init("vfio-pci-validation", image, p.imagePullPolicy, "vfio")
    vols = [_hostpath("device-plugin", "/var/lib/kubelet/device-plugins"), _hostpath("host-sys", "/sys", "Directory"),
            _hostpath("run-amd-validations", VALIDATIONS_HOST_DIR)]
    return [_sa(sa, ns, owner), _daemonset(spec, ns, owner, name, "sandboxDevicePlugin", sa, [ctr], [init], vols)]


KERNEL_LABEL = "feature.node.kubernetes.io/kernel-version.full"  # NFD's (discovery/labels.py nfd_labels)
KERNEL_DS_LABEL = "amd.com/driver-kernel"  # on the per-kernel driver DaemonSets and their pods


def kernel_suffix(kernel: str) -> str:
    """DNS-1123 form of a kernel release for object names and label values
    (``6.8.0-45-generic`` -> ``6-8-0-45-generic``); long ones keep a hash."""
    import hashlib
    import re

    x = re.sub(r"[^a-z0-9-]+", "-", kernel.lower()).strip("-")
    if len(x) > 40:
        x = x[:31].rstrip("-") + "-" + hashlib.sha1(kernel.encode()).hexdigest()[:8]
    return x


def state_driver_precompiled(spec: ClusterPolicySpec, ns: str, owner,
                             nodes: list[dict]) -> tuple[list[dict], list[str]]:
    """``driver.usePrecompiled``: one driver DaemonSet per kernel release among
    the driver nodes (NFD's ``kernel-version.full`` label), each running the
    image built for that kernel (``amd-driver:<driverVersion>-<kernel>``,
    deploy/images/amd-driver/Dockerfile.precompiled): no compiler, headers or
    network on the node.  Returns (objects, GPU nodes NFD has not labelled
    with their kernel yet)."""
    deploy = DEPLOY_LABEL.format(OPERAND_LABELS["driver"])
    kernels: set[str] = set()
    unlabelled = []
    for n in nodes:
        labels = n["metadata"].get("labels") or {}
        if labels.get(deploy) != "true":
            continue
        if labels.get(KERNEL_LABEL):
            kernels.add(labels[KERNEL_LABEL])
        else:
            unlabelled.append(n["metadata"]["name"])
    objs: list[dict] = []
    for k in sorted(kernels):
        for o in state_driver(spec, ns, owner, name=f"amd-driver-daemonset-{kernel_suffix(k)}", kernel=k):
            if o["kind"] == "DaemonSet" or not any(x["kind"] == o["kind"] and x["metadata"]["name"] == o["metadata"]["name"]
                                                   for x in objs):
                objs.append(o)
    return objs, sorted(unlabelled)


def state_driver_pools(spec: ClusterPolicySpec, ns: str, owner, drivers: list[dict],
                       nodes: list[dict]) -> tuple[list[dict], dict[str, dict]]:
    """``driver.useDriverCRD``: one driver DaemonSet per AMDGPUDriver object
    (api/driver_cr.py), owned by it.  Returns (objects, status per object);
    GPU nodes selected by more than one object are reported, not deployed."""
    from ..api.driver_cr import AMDGPUDriverSpec

    deploy = DEPLOY_LABEL.format(OPERAND_LABELS["driver"])
    gpu_nodes = [n for n in nodes if (n["metadata"].get("labels") or {}).get(deploy) == "true"]
    parsed, statuses = {}, {}
    for cr in drivers:
        name = cr["metadata"]["name"]
        try:
            parsed[name] = AMDGPUDriverSpec.model_validate(cr.get("spec") or {})
        except ValueError as e:
            statuses[name] = {"state": "error", "message": str(e).splitlines()[0], "nodeCount": 0, "nodes": []}
    matches: dict[str, list[str]] = {}
    for n in gpu_nodes:
        labels = n["metadata"].get("labels") or {}
        for name, dspec in parsed.items():
            if all(labels.get(k) == v for k, v in dspec.nodeSelector.items()):
                matches.setdefault(n["metadata"]["name"], []).append(name)
    conflicts = {node: crs for node, crs in matches.items() if len(crs) > 1}
    objs: list[dict] = []
    for cr in drivers:
        name = cr["metadata"]["name"]
        if name not in parsed:
            continue
        mine = sorted(node for node, crs in matches.items() if crs == [name])
        clash = sorted(node for node, crs in conflicts.items() if name in crs)
        if clash:
            statuses[name] = {"state": "error", "nodeCount": len(mine), "nodes": mine,
                              "message": f"nodes selected by more than one AMDGPUDriver: {clash}"}
            continue
        pool_spec = spec.model_copy(update={"driver": parsed[name]})
        pool_objs = state_driver(pool_spec, ns, owner, name=f"amd-driver-daemonset-{name}",
                                 node_selector=parsed[name].nodeSelector)
        for o in pool_objs:
            if o["kind"] == "DaemonSet":  # the pool's DaemonSet goes with its AMDGPUDriver
                o["metadata"]["ownerReferences"] = owner_ref({**cr, "apiVersion": cr.get("apiVersion", "amd.com/v1"),
                                                              "kind": "AMDGPUDriver"})
                objs.append(o)
            elif not any(x["kind"] == o["kind"] and x["metadata"]["name"] == o["metadata"]["name"] for x in objs):
                objs.append(o)  # shared RBAC, owned by the ClusterPolicy
        statuses[name] = {"state": "pending", "nodeCount": len(mine), "nodes": mine, "message": ""}
    return objs, statuses


STATE_BUILDERS = {
    "pre-requisites": state_prerequisites,
    "state-driver": state_driver,
    "state-container-toolkit": state_toolkit,
    "state-operator-validation": state_validator,
    "state-device-plugin": state_device_plugin,
    "state-dra-driver": state_dra_driver,
    "state-metrics-exporter": state_metrics_exporter,
    "state-node-feature-discovery": state_nfd,
    "state-gpu-feature-discovery": state_gfd,
    "state-partition-manager": state_partition_manager,
    "state-node-status-exporter": state_node_status_exporter,
    "state-vfio-manager": state_vfio_manager,
    "state-sandbox-validation": state_sandbox_validator,
    "state-sandbox-device-plugin": state_sandbox_device_plugin,
}
