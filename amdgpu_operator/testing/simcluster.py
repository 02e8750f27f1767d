"""Simulated Kubernetes cluster that runs the REAL operand code (C14).

SURVEY.md §4.2 / §7.4: without kind, kubectl, docker or root, the product is
exercised end to end in-process:

* :class:`~amdgpu_operator.kube.fakeapi.FakeApiServer` as the API server;
* a DaemonSet controller (pods per eligible node, rolling re-creation on
  template change, DaemonSet status);
* one simulated kubelet per node that runs pods: init containers in order,
  then the main containers, each mapped to the operand function its
  ``amdgpu-operator <subcommand>`` args name (the same functions the CLI runs
  inside the real images) - plus ``amdgpu-validator`` workload pods, which go
  through the device-plugin gRPC Allocate, the native OCI hook's precreate
  stage on a synthetic runtime spec, and the native validator binary on the
  allocated GPU;
* :class:`~amdgpu_operator.testing.fakekubelet.FakeKubelet` per node (device
  plugin registration / ListAndWatch / Allocate / pod-resources) feeding the
  node's Allocatable ``amd.com/gpu``.

Each node has its own host directories (validations, device-plugins, CDI,
containerd config) under ``workdir``; its sysfs root is a synthetic MI355X tree
(``fakesys``) or, on a GPU box, the real ``/``.  With ``fake_gpu=True`` GPU
processes are not started (CPU-only tests) and report a synthetic success.
"""

from __future__ import annotations

import hashlib
import json
import os
import shutil
import sys
import shlex
import tempfile
import threading
import time
import uuid
from dataclasses import dataclass, field

from .. import API_GROUP, API_VERSION, DEFAULT_NAMESPACE, RESOURCE_NAME
from ..api.clusterpolicy import cluster_policy, spec_from_values
from ..controller.reconciler import ClusterPolicyReconciler
from ..kube import resources as R
from ..kube.client import LocalClient, NotFound
from ..kube.fakeapi import FakeApiServer
from ..nodeenv import REPORT_EARLY_ENV, NodeEnv, ProcResult, run_local
from ..utils.logs import get_logger
from . import fakesys
from .fakekubelet import FakeKubelet

log = get_logger("amdgpu.sim")
CP_API = f"{API_GROUP}/{API_VERSION}"


@dataclass
class NodeSpec:
    name: str
    gpus: int = 8                     # 0 = CPU-only node
    compute_partition: str = "SPX"
    memory_partition: str = "NPS1"
    sysfs_root: str | None = None     # None = synthetic tree; "/" = this machine
    kernel: str = "6.8.0-45-generic"  # the node's kernel release (synthetic tree)
    rdma_nics: bool = False           # synthetic tree: one RDMA NIC per GPU on its PCIe switch


@dataclass
class SimNode:
    spec: NodeSpec
    dir: str
    env: NodeEnv
    kubelet: FakeKubelet
    pods: dict = field(default_factory=dict)  # pod name -> _PodRun
    terminating: set = field(default_factory=set)  # pods between graceful delete and removal
    dra: object = None  # the kubelet's DRA side (fakedra.FakeDraKubelet), created on first use
    # the DRA manager's claim cache lock: a shared claim's prepare, its pods'
    # use counts and its unprepare are one critical section
    dra_lock: threading.Lock = field(default_factory=threading.Lock)


class AdmissionError(RuntimeError):
    """The kubelet could not allocate a pod's devices (the pod fails with
    reason ``UnexpectedAdmissionError``, as on a real kubelet)."""


def fake_validator_result(argv: list[str], env: dict | None = None) -> ProcResult:
    """Synthetic ``amdgpu-validator`` output for CPU-only runs."""
    from .fake_validator import simulated_detail, visible_count

    def arg(name, default):
        return argv[argv.index(name) + 1] if name in argv else default

    expect = int(arg("--expect-devices", "-1"))
    seen = visible_count(env or {})
    if "--pod-check" in argv and expect >= 0 and seen is not None and seen != expect:
        rep = {"ok": False, "simulated": True, "error": f"{expect} GPU(s) allocated to the pod, {seen} visible",
               "steps": []}
        _write_result(argv, rep)
        return ProcResult(1, json.dumps(rep) + "\n", "", 0.0)
    steps = arg("--steps", "hip,vecadd,gemm,mfma,hbm,xgmi,rccl").split(",")
    rank, world = int(arg("--rank", "0")), int(arg("--world", "1"))
    recs = [{"name": s, "ok": True, "seconds": 0.0, "simulated": True, **simulated_detail(s, argv, rank, world)}
            for s in steps]
    ok = all(r["ok"] for r in recs)
    rep = {"ok": ok, "simulated": True, "rank": rank, "world": world, "device": int(arg("--device", "0")),
           "seconds": 0.0, "steps": recs, "rocr_visible_devices": (env or {}).get("ROCR_VISIBLE_DEVICES")}
    if not ok:
        rep["error"] = f"step {next(r['name'] for r in recs if not r['ok'])} failed"
    _write_result(argv, rep)
    return ProcResult(0 if ok else 1, json.dumps(rep) + "\n", "", 0.0)


def _write_result(argv: list[str], rep: dict) -> None:
    """The native checks' report file (--result-file always, --ready-file when ok)."""
    for flag, always in (("--result-file", True), ("--ready-file", False)):
        if flag in argv and (always or rep.get("ok")):
            path = argv[argv.index(flag) + 1]
            with open(path + ".tmp", "w") as f:
                f.write(json.dumps(rep))
            os.replace(path + ".tmp", path)


class _PodRun:
    def __init__(self, cluster: "SimCluster", node: SimNode, pod: dict):
        self.cluster = cluster
        self.node = node
        self.pod = pod
        self.name = pod["metadata"]["name"]
        self.ns = pod["metadata"].get("namespace", "default")
        self.stop = threading.Event()
        self.ready: dict[str, bool] = {}
        self.thread = threading.Thread(target=self._run, daemon=True, name=f"pod-{self.name}")
        self.cleanups: list = []
        self.dra_uids: list[str] = []  # ResourceClaims prepared for this pod
        self.restarts = 0
        self._status_lock = threading.Lock()

    # ------------------------------------------------------------- status
    def _status(self, phase: str, init_done: bool, reason: str = "", message: str = "") -> None:
        # containers report readiness from their own threads: compute and write
        # the status under one lock, or a slower writer's stale view of
        # self.ready overwrites a newer one (a container ready forever unseen)
        with self._status_lock:
            self._status_locked(phase, init_done, reason, message)

    def _status_locked(self, phase: str, init_done: bool, reason: str, message: str,
                       waiting: dict | None = None) -> None:
        spec = self.pod["spec"]
        ctrs = spec.get("containers", [])
        all_ready = init_done and bool(ctrs) and all(self.ready.get(c["name"]) for c in ctrs)

        def state(c):
            if waiting is not None:  # image pull failed: the kubelet's waiting state (ErrImagePull / ImagePullBackOff)
                return {"waiting": waiting}
            return {"running": {}} if phase == "Running" else {"terminated": {"reason": reason}}
        now = time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())
        st = {
            "phase": phase,
            "hostIP": "10.0.0.1",
            "conditions": [
                {"type": "PodScheduled", "status": "True"},
                {"type": "Initialized", "status": "True" if init_done else "False"},
                {"type": "ContainersReady", "status": "True" if all_ready else "False"},
                {"type": "Ready", "status": "True" if all_ready else "False", "lastTransitionTime": now},
            ],
            "containerStatuses": [{"name": c["name"], "ready": bool(self.ready.get(c["name"])),
                                   "restartCount": self.restarts, "image": c.get("image", ""), "state": state(c)}
                                  for c in ctrs],
        }
        if reason:
            st["reason"] = reason
        if message:
            st["message"] = message[:2000]
        try:
            cur = self.cluster.client.get("v1", "Pod", self.name, self.ns)
        except NotFound:
            return
        # fields of the pod's status other writers own (the resourceclaim controller's claim names)
        for k in ("resourceClaimStatuses",):
            if k in (cur.get("status") or {}):
                st[k] = cur["status"][k]
        if cur.get("status") == st:
            return
        cur["status"] = st
        try:
            self.cluster.client.update_status(cur)
        except Exception:  # noqa: BLE001 - pod deleted meanwhile / conflict: next update wins
            pass

    # ----------------------------------------------------------- lifecycle
    def _pull(self, attempt: int) -> bool:
        """The kubelet pulls every container's image before it starts any: an
        image the registry does not hold (SimCluster.known_images: the chart's
        and the ClusterPolicies' images, plus pushed ones) leaves the pod
        Pending with ``ErrImagePull``, then ``ImagePullBackOff`` - as a bare
        name pulled from Docker Hub does on a cluster."""
        spec = self.pod["spec"]
        want = [c.get("image", "") for c in spec.get("initContainers", []) + spec.get("containers", [])]
        known = self.cluster.known_images()
        missing = [i for i in want if i not in known]
        if not missing:
            return True
        msg = (f'Failed to pull image "{missing[0]}": rpc error: code = NotFound desc = failed to resolve reference '
               f'"{missing[0]}": not found')
        self.cluster.trace("image-pull-failed", f"{self.name} {missing[0]}")
        with self._status_lock:
            self._status_locked("Pending", False, "", "", waiting={
                "reason": "ErrImagePull" if attempt == 0 else "ImagePullBackOff",
                "message": msg if attempt == 0 else f'Back-off pulling image "{missing[0]}"'})
        return False

    def _run(self) -> None:
        restart = self.pod["spec"].get("restartPolicy", "Always") != "Never"
        backoff = self.cluster.poll_s * 10
        attempt = 0
        while not self._pull(attempt):
            attempt += 1
            if self.stop.wait(min(2.0, 0.1 * 2 ** attempt)):
                return
        while not self.stop.is_set():
            failed = self._run_once()
            if not failed or not restart:
                return
            self.restarts += 1
            if self.stop.wait(backoff):
                return
            backoff = min(backoff * 2, 2.0)

    def _run_once(self) -> bool:
        """One pass of init + main containers; True when something failed."""
        spec = self.pod["spec"]
        self.ready.clear()
        self._status("Pending", False)
        try:
            for c in spec.get("initContainers", []):
                if self.stop.is_set():
                    return False
                self.cluster.run_container(self, c, init=True)
            self._status("Running", True)
            threads = []
            errors = []
            reason = []
            for c in spec.get("containers", []):
                def body(c=c):
                    try:
                        self.cluster.run_container(self, c, init=False)
                    except Exception as e:  # noqa: BLE001
                        errors.append(f"{c['name']}: {e}")
                        reason.append("UnexpectedAdmissionError" if isinstance(e, AdmissionError) else "Error")
                th = threading.Thread(target=body, daemon=True, name=f"ctr-{self.name}-{c['name']}")
                th.start()
                threads.append(th)
            for th in threads:
                th.join()
            if self.stop.is_set():
                return False
            if errors:
                log.warning("pod %s failed: %s", self.name, "; ".join(errors))
                self._status("Failed", True, reason[0] if reason else "Error", "; ".join(errors))
                return True
            self._status("Succeeded", True, "Completed")
            return False
        except Exception as e:  # noqa: BLE001 - init container failure
            if not self.stop.is_set():
                log.warning("pod %s failed: %s", self.name, e)
                self._status("Failed", False, "Error", str(e))
            return True
        finally:
            for fn in reversed(self.cleanups):
                try:
                    fn()
                except Exception:  # noqa: BLE001
                    pass

    def set_ready(self, container: str) -> None:
        self.cluster.trace("container-ready", f"{self.name}/{container}")
        self.ready[container] = True
        self._status("Running", True)


class SimCluster:
    def __init__(self, workdir: str, nodes: list[NodeSpec], namespace: str = DEFAULT_NAMESPACE,
                 fake_gpu: bool = True, poll_s: float = 0.01, launcher=None,
                 termination_s: float | None = None, agent_poll_s: float | None = None,
                 node_status_s: float | None = None, operator_resync_s: float = 1.0,
                 operator_debounce_s: float = 0.005, http_api: bool = False, process_containers: bool = False,
                 rbac: bool = False):
        """``termination_s``: model graceful pod deletion - a deleted pod stays
        Terminating (listed, with ``deletionTimestamp``) for that many seconds
        (capped by its own grace period) before its kubelet removes it.
        ``poll_s`` paces the simulated kubelet / controllers; ``agent_poll_s``
        is the operands' own ``VALIDATION_POLL_S`` (default: ``poll_s``).
        ``node_status_s`` models the kubelet's ``nodeStatusUpdateFrequency``
        (10 s by default on a real kubelet): device-plugin capacity reaches
        ``Node.status`` only on that tick (default: every ``poll_s``).
        ``http_api``: the operator and every operand talk to the API server
        through :class:`~..kube.client.RestClient` over HTTP (real REST paths,
        chunked watches, merge-patch, gracePeriodSeconds), as in a cluster; the
        simulated kubelet and DaemonSet controller stay in-process.
        ``process_containers``: every operand container (init containers
        included) runs as its own ``python -m amdgpu_operator <args>``
        process - the production entry point of the operand images - with
        the node's host paths and the API server (over HTTP, so implies
        ``http_api``) in its environment, instead of as a thread of this
        process; readiness comes from the operand's ready file, a pod delete
        sends SIGTERM.  Interpreter and import start-up of every operand, and
        the device plugin's health-watcher start (on in this mode), are then
        inside the measured bring-up (:attr:`process_stats`)."""
        self.workdir = workdir
        self.process_containers = process_containers
        http_api = http_api or process_containers
        self.process_stats: list[dict] = []  # process_containers: one record per operand process
        self._kubeconfig = None
        self.termination_s = termination_s
        self.namespace = namespace
        self.fake_gpu = fake_gpu
        self.poll_s = poll_s
        self.agent_poll_s = poll_s if agent_poll_s is None else agent_poll_s
        self.node_status_s = poll_s if node_status_s is None else node_status_s
        self.operator_resync_s = operator_resync_s
        self.operator_debounce_s = operator_debounce_s
        self.launcher = launcher
        self.api = FakeApiServer()
        from ..kube import validation

        validation.install(self.api)  # objects kube-apiserver would reject fail here too
        self.api.graceful_pod_deletion = termination_s is not None
        self.api.hooks.append(self._trace_api)
        self.client = LocalClient(self.api)  # the simulated kubelets / controllers
        self._http = None
        self.agent_client = self.client  # what the operator and the operands use
        if http_api:
            from ..kube.client import RestClient
            from ..kube.httpapi import HttpApiServer

            self._http = HttpApiServer(self.api).start()
            self.agent_client = RestClient(self._http.url)
            if process_containers:  # what the operand processes read (main.py: KUBECONFIG)
                os.makedirs(workdir, exist_ok=True)
                self._kubeconfig = self._write_kubeconfig(os.path.join(workdir, "kubeconfig"))
            if rbac:
                if not process_containers:
                    raise ValueError("rbac=True needs process_containers=True (a ServiceAccount per process)")
                # every request authorized against the ClusterRoles the chart
                # and the operator create: the operator and each operand
                # process run as their own ServiceAccount (kube/rbac.py)
                self._http.enable_rbac()
        self.rbac = rbac
        self.nodes: dict[str, SimNode] = {}
        self.stop_event = threading.Event()
        self._threads: list[threading.Thread] = []
        self._lock = threading.RLock()
        self._ds_seq: dict[str, int] = {}  # DaemonSet uid -> the order its ADDED event came in
        self.reconciler: ClusterPolicyReconciler | None = None
        self._operator_proc = None  # process_containers: the operator as its own process (its Deployment's pod)
        # bring-up trace: (perf_counter, what, detail) - pods created/deleted,
        # containers started/finished (bench.py --detail prints it per step)
        self.events: list[tuple[float, str, str]] = []
        self._node_specs = nodes
        self._short_dirs: list[str] = []
        self._hashes: dict[tuple, str] = {}
        self.hook_drop_devices = 0  # fault injection: GPUs the runtime leaves out of a GPU container
        self.pod_reports: dict[str, dict] = {}  # GPU pod name -> its process's JSON report
        self.container_reports: dict[tuple[str, str], dict] = {}  # (pod, container) -> the same, per container
        # images "pushed" to the simulated registry besides the chart's and the policies' (known_images)
        self.pushed_images: set[str] = set()
        self._images_cache: tuple = (None, set())

    # -------------------------------------------------------------- setup
    # a unix socket path must fit sockaddr_un.sun_path (108 bytes); the node's
    # own directory can be deeper (pytest-xdist temp dirs), so its sockets
    # then live in a short private directory removed by stop()
    SOCKET_PATH_BUDGET = 40

    def _socket_dir(self, node_dir: str) -> str:
        if len(node_dir) <= self.SOCKET_PATH_BUDGET:
            return node_dir
        d = tempfile.mkdtemp(prefix="amdgpu-sock-")
        self._short_dirs.append(d)
        return d

    def _make_node(self, ns: NodeSpec) -> SimNode:
        d = os.path.join(self.workdir, ns.name)
        os.makedirs(d, exist_ok=True)
        if ns.sysfs_root is None:
            root = os.path.join(d, "host")
            if ns.gpus > 0:
                fake = fakesys.build_node(root, ns.gpus, ns.compute_partition, ns.memory_partition, kernel=ns.kernel,
                                          pcie_tree=ns.rdma_nics)
                if ns.rdma_nics:
                    fakesys.add_rdma_nics(root, fake, modules=False)  # the driver container loads the RDMA core
            else:
                os.makedirs(os.path.join(root, "sys/bus/pci/devices"), exist_ok=True)
                fakesys._w(os.path.join(root, "sys/bus/pci/devices/0000:00:01.0/vendor"), "0x1022\n")
                fakesys._w(os.path.join(root, "sys/bus/pci/devices/0000:00:01.0/class"), "0x060000\n")
        else:
            root = ns.sysfs_root
        sockets = self._socket_dir(d)
        dp_dir = os.path.join(sockets, "device-plugins")
        podres = os.path.join(sockets, "pod-resources", "kubelet.sock")
        kubelet = FakeKubelet(dp_dir, podres)
        env = NodeEnv(node_name=ns.name, client=self.agent_client, host_root=root,
                      validations_dir=os.path.join(d, "validations"), device_plugin_dir=dp_dir,
                      pod_resources_socket=podres, cdi_dir=os.path.join(d, "cdi"),
                      containerd_config=os.path.join(d, "etc/containerd/config.toml"),
                      crio_config_dir=os.path.join(d, "etc/crio/crio.conf.d"),
                      docker_config=os.path.join(d, "etc/docker/daemon.json"),
                      install_dir=os.path.join(d, "usr/local/amd"), namespace=self.namespace, poll_s=self.agent_poll_s,
                      launcher=self._launch)
        if ns.sysfs_root is None and ns.gpus > 0:  # driver installs / unloads act on the fake tree
            env.extra["kmod"] = fakesys.SimModule(root)
            env.extra["pci_backend"] = fakesys.FakePciKernel(root)  # vfio-manager binds act on the fake tree
        if self.fake_gpu:
            env.extra["metrics_fixture"] = os.path.join(fakesys.REAL_FIXTURE, "amd-smi-metric.json")
        os.makedirs(os.path.dirname(env.containerd_config), exist_ok=True)
        with open(env.containerd_config, "w") as f:  # the reference's own containerd edit (README.md:15-17)
            f.write('version = 2\n[plugins."io.containerd.grpc.v1.cri".containerd.runtimes.runc.options]\n'
                    "  SystemdCgroup = true\n")
        return SimNode(ns, d, env, kubelet)

    def _launch(self, argv, env, device, timeout) -> ProcResult:
        if self.fake_gpu and argv and os.path.basename(argv[0]) == "amdgpu-gpu-check":
            expect = ["--expect-devices", argv[argv.index("--expect-devices") + 1]] if "--expect-devices" in argv else []
            result = ["--result-file", argv[argv.index("--result-file") + 1]] if "--result-file" in argv else []
            argv = [argv[0], "--steps", "hsa,vecadd", "--pod-check", *expect, *result]  # the stand-in reports the check's steps
            if self.fake_gpu != "procs":
                return fake_validator_result(argv, env)
            import sys

            argv = [sys.executable, "-m", "amdgpu_operator.testing.fake_validator", *argv[1:]]
            return self.launcher(argv, env, device, timeout) if self.launcher is not None else run_local(argv, env,
                                                                                                        timeout)
        if self.fake_gpu and argv and os.path.basename(argv[0]) == "amdgpu-validator":
            if self.fake_gpu != "procs":
                from .fake_validator import wait_start_gate

                gate = argv[argv.index("--start-gate") + 1] if "--start-gate" in argv else None
                verdict = wait_start_gate(gate, timeout)
                if verdict != "go":
                    return ProcResult(3, json.dumps({"ok": False, "error": f"start gate: {verdict}"}) + "\n", "", 0.0)
                return fake_validator_result(argv)
            # run a stand-in process through the real launcher path (multi-rank rehearsal)
            import sys

            argv = [sys.executable, "-m", "amdgpu_operator.testing.fake_validator", *argv[1:]]
        if self.launcher is not None:
            return self.launcher(argv, env, device, timeout)
        return run_local(argv, env, timeout)

    def _write_kubeconfig(self, path: str, token: str | None = None) -> str:
        with open(path, "w") as f:
            json.dump({"apiVersion": "v1", "kind": "Config", "current-context": "sim",
                       "clusters": [{"name": "sim", "cluster": {"server": self._http.url}}],
                       "users": [{"name": "sim", "user": {"token": token} if token else {}}],
                       "contexts": [{"name": "sim", "context": {"cluster": "sim", "user": "sim"}}]}, f)
        return path

    def _kubeconfig_for(self, namespace: str, service_account: str) -> str:
        """rbac: the kubeconfig of a ServiceAccount (its token); else the shared one."""
        if not self.rbac:
            return self._kubeconfig
        path = os.path.join(self.workdir, f"kubeconfig-{namespace}-{service_account}")
        if not os.path.exists(path):
            self._write_kubeconfig(path, self._http.token_for(namespace, service_account))
        return path

    def install_chart_rbac(self) -> None:
        """The chart's own RBAC (the operator's ClusterRole and binding), as
        ``helm install`` creates it, for ``rbac`` runs."""
        from ..helm.render import render_chart

        for d in render_chart(set_flags=["operator.cleanupCRD=false"], namespace=self.namespace):
            if d.get("kind") in ("ClusterRole", "ClusterRoleBinding", "Role", "RoleBinding") \
                    and d["metadata"]["name"] == "amd-gpu-operator":
                try:
                    self.client.create(d)
                except Exception:  # noqa: BLE001 - already there
                    pass

    def start(self) -> "SimCluster":
        self.client.create(R.new("v1", "Namespace", self.namespace))
        if self.rbac:
            self.install_chart_rbac()
        for ns in self._node_specs:
            node = self._make_node(ns)
            node.kubelet.start()
            self.nodes[ns.name] = node
            self.client.create({"apiVersion": "v1", "kind": "Node",
                                "metadata": {"name": ns.name, "labels": {"kubernetes.io/hostname": ns.name}},
                                "status": {"capacity": {"cpu": "128"}, "allocatable": {"cpu": "128"},
                                           "conditions": [{"type": "Ready", "status": "True"}]}})
        self._spawn(self._ds_controller_loop, "sim-ds-controller")
        self._spawn(self._scheduler_loop, "sim-scheduler")
        for node in self.nodes.values():
            self._spawn(lambda n=node: self._kubelet_loop(n), f"sim-kubelet-{node.spec.name}")
            self._spawn(lambda n=node: self._node_status_loop(n), f"sim-nodestatus-{node.spec.name}")
        if self.process_containers:
            self._start_operator_process()
        return self

    def _start_operator_process(self, timeout: float = 120.0) -> None:
        """``process_containers``: the operator runs as its own process, as
        the chart's operator Deployment does, started (CRD installed, first
        pass done) before the ClusterPolicy appears - its own start-up is not
        part of a bring-up, as with the in-process reconciler, and its
        reconcile passes no longer share this process's interpreter lock with
        the simulated API server and kubelets."""
        import subprocess
        import sys

        from ..utils.fswait import wait_for_file

        try:
            self.install_crd()
        except Exception:  # noqa: BLE001 - already installed
            pass
        d = os.path.join(self.workdir, "operator")
        os.makedirs(d, exist_ok=True)
        ready = os.path.join(d, "ready")
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        penv = dict(os.environ)
        penv.update({"AMDGPU_READY_FILE": ready, "PYTHONPATH": os.pathsep.join(
            [root] + [x for x in os.environ.get("PYTHONPATH", "").split(os.pathsep) if x])})
        penv.pop("KUBERNETES_SERVICE_HOST", None)
        argv = [sys.executable, "-m", "amdgpu_operator", "operator", "--kubeconfig",
                self._kubeconfig_for(self.namespace, "amd-gpu-operator"),
                "--namespace", self.namespace, "--resync", str(self.operator_resync_s),
                "--debounce", str(self.operator_debounce_s), "--health-port", "0"]
        with open(os.path.join(d, "log"), "w") as log_f:
            self._operator_proc = subprocess.Popen(argv, env=penv, stdout=log_f, stderr=subprocess.STDOUT,
                                                   start_new_session=True)
        if not wait_for_file(ready, timeout, self.stop_event, 0.05) or self._operator_proc.poll() is not None:
            with open(os.path.join(d, "log")) as f:
                tail = f.read()[-2000:]
            raise RuntimeError(f"operator process did not come up: {tail}")

    def _spawn(self, fn, name: str) -> None:
        th = threading.Thread(target=fn, daemon=True, name=name)
        th.start()
        self._threads.append(th)

    def install_crd(self) -> None:
        from ..helm.render import load_crd

        self.client.create(load_crd())

    def install_operator(self, values: dict | None = None, name: str = "cluster-policy") -> dict:
        """``helm install`` equivalent: CRD + ClusterPolicy from values + operator loop."""
        try:
            self.install_crd()
        except Exception:  # noqa: BLE001 - already installed
            pass
        cp = self.client.create(cluster_policy(name, spec_from_values(values or {})))
        self.start_reconciler()
        return cp

    def start_reconciler(self) -> ClusterPolicyReconciler | None:
        if self._operator_proc is not None:
            return None  # the operator process (process_containers) reconciles
        if self.reconciler is None:
            self.reconciler = ClusterPolicyReconciler(self.agent_client, self.namespace)
            self._spawn(lambda: self.reconciler.run(self.stop_event, resync_s=self.operator_resync_s,
                                                    debounce_s=self.operator_debounce_s),
                        "sim-operator")
        return self.reconciler

    def stop(self) -> None:
        self.stop_event.set()
        if self._operator_proc is not None:  # SIGTERM, as the Deployment's pod gets it
            import signal
            import subprocess

            try:
                os.killpg(self._operator_proc.pid, signal.SIGTERM)
                self._operator_proc.wait(timeout=10)
            except (ProcessLookupError, subprocess.TimeoutExpired):
                try:
                    os.killpg(self._operator_proc.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
                self._operator_proc.wait()
            self._operator_proc = None
        for node in self.nodes.values():
            for run in list(node.pods.values()):
                run.stop.set()
        for node in self.nodes.values():
            for run in list(node.pods.values()):
                run.thread.join(timeout=5)
            node.kubelet.stop()
        for th in self._threads:
            th.join(timeout=5)
        for d in self._short_dirs:
            shutil.rmtree(d, ignore_errors=True)
        if self._http is not None:
            self._http.stop()

    # --------------------------------------------------- DaemonSet controller
    def _template_hash(self, ds: dict) -> str:
        """controller-revision-hash of the pod template (cached per spec generation)."""
        md = ds["metadata"]
        k = (md.get("uid"), md.get("generation"))
        h = self._hashes.get(k)
        if h is None:
            h = self._hashes[k] = hashlib.sha1(json.dumps(ds["spec"]["template"], sort_keys=True).encode()).hexdigest()[:10]
        return h

    def _eligible(self, ds: dict, node: dict) -> bool:
        tspec = ds["spec"]["template"]["spec"]
        return R.node_selector_matches(node, tspec.get("nodeSelector"), tspec.get("affinity"))

    def sync_daemonsets(self) -> None:
        with self._lock:
            nodes = self.client.list("v1", "Node")
            all_pods: dict[tuple, list] = {}  # (namespace, owner uid) -> pods: one list per sync
            for p in self.client.list("v1", "Pod"):
                for r in p["metadata"].get("ownerReferences") or []:
                    if r.get("kind") == "DaemonSet":
                        all_pods.setdefault((p["metadata"].get("namespace"), r.get("uid")), []).append(p)
            # in the order the DaemonSets were created, as the real controller's
            # work queue takes their ADDED events (the list is in name order)
            seq = {} if os.environ.get("AMDGPU_SIM_DS_NAME_ORDER") == "1" else self._ds_seq  # A/B: name order
            for ds in sorted(self.client.list("apps/v1", "DaemonSet"),
                             key=lambda d: (seq.get(d["metadata"]["uid"], float("inf")), d["metadata"]["name"])):
                ns = ds["metadata"]["namespace"]
                name = ds["metadata"]["name"]
                h = self._template_hash(ds)
                owned = all_pods.get((ns, ds["metadata"]["uid"]), [])
                pods = {p["spec"]["nodeName"]: p for p in owned}
                eligible = [n for n in nodes if self._eligible(ds, n)]
                want = {n["metadata"]["name"] for n in eligible}
                on_delete = (ds["spec"].get("updateStrategy") or {}).get("type") == "OnDelete"
                for node_name, p in pods.items():
                    stale = p["metadata"].get("labels", {}).get("controller-revision-hash") != h
                    if node_name not in want or (stale and not on_delete):
                        try:
                            self.client.delete("v1", "Pod", p["metadata"]["name"], ns)
                        except NotFound:
                            pass
                for node_name in want:
                    p = pods.get(node_name)
                    if p is not None and (on_delete or p["metadata"].get("labels", {}).get(
                            "controller-revision-hash") == h):
                        continue  # OnDelete: an outdated pod stays until someone deletes it
                    tmpl = R.deep(ds["spec"]["template"])
                    suffix = hashlib.sha1(f"{name}/{node_name}/{h}".encode()).hexdigest()[:5]
                    pod = {"apiVersion": "v1", "kind": "Pod",
                           "metadata": {"name": f"{name}-{suffix}", "namespace": ns,
                                        "labels": {**tmpl.get("metadata", {}).get("labels", {}),
                                                   "controller-revision-hash": h},
                                        "ownerReferences": [{"apiVersion": "apps/v1", "kind": "DaemonSet", "name": name,
                                                             "uid": ds["metadata"]["uid"], "controller": True}]},
                           "spec": {**tmpl["spec"], "nodeName": node_name}}
                    try:
                        owned.append(self.client.create(pod))
                    except Exception:  # noqa: BLE001 - AlreadyExists while the old one terminates
                        pass
                # status (pods deleted above drop out on the next sync, as with an informer cache)
                pods_now = [p for p in owned if p["spec"].get("nodeName") in want]
                ready = sum(1 for p in pods_now if R.condition(p, "Ready") and R.condition(p, "Ready")["status"] == "True"
                            and p["metadata"]["labels"].get("controller-revision-hash") == h)
                updated = sum(1 for p in pods_now if p["metadata"]["labels"].get("controller-revision-hash") == h)
                st = {"desiredNumberScheduled": len(want), "currentNumberScheduled": len(pods_now),
                      "numberReady": ready, "updatedNumberScheduled": updated, "numberAvailable": ready,
                      "numberMisscheduled": 0, "observedGeneration": ds["metadata"].get("generation", 1)}
                if ds.get("status") != st:
                    ds["status"] = st
                    try:
                        self.client.update_status(ds)
                    except Exception:  # noqa: BLE001
                        pass

    def _ds_controller_loop(self) -> None:
        import queue

        q: queue.Queue = queue.Queue()

        def pump(av, kind):
            while not self.stop_event.is_set():
                try:
                    for etype, obj in self.client.watch(av, kind, stop=self.stop_event):
                        if kind == "DaemonSet" and etype == "ADDED":
                            self._ds_seq.setdefault(obj["metadata"]["uid"], len(self._ds_seq))
                        q.put(kind)
                except Exception:  # noqa: BLE001
                    self.stop_event.wait(0.1)

        for av, kind in (("apps/v1", "DaemonSet"), ("v1", "Node"), ("v1", "Pod")):
            threading.Thread(target=pump, args=(av, kind), daemon=True, name=f"sim-ds-watch-{kind}").start()
        while not self.stop_event.is_set():
            try:
                q.get(timeout=0.5)
            except Exception:  # noqa: BLE001 - idle resync
                pass
            while not q.empty():
                q.get_nowait()
            try:
                self.sync_daemonsets()
            except Exception as e:  # noqa: BLE001
                log.warning("ds sync: %s", e)

    # ------------------------------------------------------------ scheduler
    def _scheduler_loop(self) -> None:
        """Pods without ``nodeName`` (those with ResourceClaims must go through
        the scheduler: it allocates the claims): bound to the node their
        ``kubernetes.io/hostname`` selector names once their claims are
        allocated there (testing/fakedra.py allocate, the structured-parameters
        allocator)."""
        while not self.stop_event.is_set():
            try:
                for etype, pod in self.client.watch("v1", "Pod", stop=self.stop_event):
                    if etype != "DELETED" and not pod["spec"].get("nodeName") \
                            and not pod["metadata"].get("deletionTimestamp"):
                        self._schedule(pod)
                    elif etype == "DELETED" or (pod.get("status") or {}).get("phase") in ("Succeeded", "Failed"):
                        # devices a pod held are free again: the pods waiting for them get another try
                        for waiting in self.client.list("v1", "Pod"):
                            if not waiting["spec"].get("nodeName") and not waiting["metadata"].get("deletionTimestamp") \
                                    and self._gpu_requests(waiting):
                                self._schedule(waiting)
            except Exception as e:  # noqa: BLE001
                log.debug("scheduler watch: %s", e)
                self.stop_event.wait(0.1)

    @staticmethod
    def _gpu_requests(pod: dict) -> dict[str, int]:
        """Extended-resource requests of the device plugin's resources (limits
        stand for requests, as for extended resources)."""
        out: dict[str, int] = {}
        for c in pod["spec"].get("containers") or []:
            for k, v in ((c.get("resources") or {}).get("limits") or {}).items():
                if k.startswith(RESOURCE_NAME):
                    out[k] = out.get(k, 0) + int(v)
        return out

    def _gpu_fits(self, pod: dict, node: str) -> str | None:
        """kube-scheduler's resource fit for the device plugin's resources: the
        requests of every pod bound to the node that has not finished -
        terminating ones included, until they are gone - plus this one's, within
        what the node's kubelet advertises.  None if it fits, else why not."""
        want = self._gpu_requests(pod)
        if not want:
            return None
        used: dict[str, int] = {}
        for p in self.client.list("v1", "Pod"):
            if p["spec"].get("nodeName") == node and (p.get("status") or {}).get("phase") not in ("Succeeded",
                                                                                                    "Failed"):
                for k, v in self._gpu_requests(p).items():
                    used[k] = used.get(k, 0) + v
        kubelet = self.nodes[node].kubelet
        for k, v in want.items():
            if used.get(k, 0) + v > kubelet.capacity(k):
                return f"Insufficient {k} on {node} ({used.get(k, 0)} in use of {kubelet.capacity(k)})"
        return None

    def _schedule(self, pod: dict) -> None:
        from . import fakedra

        md = pod["metadata"]
        want = dict(pod["spec"].get("nodeSelector") or {})
        host = want.pop("kubernetes.io/hostname", None)
        if host is not None and host not in self.nodes:
            return
        ns = md.get("namespace", "default")
        try:
            claims = [self.client.get("resource.k8s.io/v1beta1", "ResourceClaim", n, ns)
                      for n in self._pod_claims(pod).values()]
            # the nodes the pod may land on: its hostname selector, else every
            # GPU node whose labels match; a claim allocated earlier (shared by
            # several pods) pins the node it was allocated on
            pinned = {t["values"][0] for c in claims for term in ((((c.get("status") or {}).get("allocation") or {})
                                                                   .get("nodeSelector") or {}).get("nodeSelectorTerms") or [])
                      for t in term.get("matchFields") or [] if t.get("key") == "metadata.name"}
            cands = [host] if host else [n for n, sn in self.nodes.items() if sn.spec.gpus > 0 and all(
                (self.client.get("v1", "Node", n)["metadata"].get("labels") or {}).get(k) == v for k, v in want.items())]
            cands = [n for n in cands if not pinned or n in pinned]
            if not cands:
                raise ValueError(f"no node matches (selector {want}, claims allocated on {sorted(pinned)})")
            unfit = {n: self._gpu_fits(pod, n) for n in cands}
            cands = [n for n in cands if unfit[n] is None]
            if not cands:
                raise ValueError("; ".join(v for v in unfit.values() if v))
            err: Exception | None = None
            for node in cands:
                try:
                    for claim in claims:
                        if not (claim.get("status") or {}).get("allocation"):
                            fakedra.allocate(self.client, claim, node)
                    break
                except ValueError as e:  # this node cannot satisfy the claims: the next one
                    err = e
            else:
                raise err or ValueError("unschedulable")
            self.client.patch("v1", "Pod", md["name"], {"spec": {"nodeName": node}}, ns)
            self.trace("pod-scheduled", md["name"])
        except (ValueError, NotFound) as e:  # unschedulable for now: the next event tries again
            try:
                self.client.patch("v1", "Pod", md["name"], {"status": {"phase": "Pending", "conditions": [
                    {"type": "PodScheduled", "status": "False", "reason": "Unschedulable", "message": str(e)}]}}, ns)
            except NotFound:
                pass

    def _pod_claims(self, pod: dict) -> dict[str, str]:
        """The pod's resourceClaims entry name -> ResourceClaim name.  An entry
        naming a ResourceClaimTemplate gets its own claim the way
        kube-controller-manager's resourceclaim controller makes it: named
        ``<pod>-<entry>-<suffix>``, owned by the pod (deleted with it),
        annotated with the entry, and recorded in the pod's
        ``status.resourceClaimStatuses``."""
        md = pod["metadata"]
        ns = md.get("namespace", "default")
        done = {s["name"]: s.get("resourceClaimName") for s in (pod.get("status") or {}).get("resourceClaimStatuses") or []}
        out, new = {}, []
        for rc in pod["spec"].get("resourceClaims") or []:
            if rc.get("resourceClaimName"):
                out[rc["name"]] = rc["resourceClaimName"]
            elif rc.get("resourceClaimTemplateName"):
                if rc["name"] not in done:
                    tmpl = self.client.get("resource.k8s.io/v1beta1", "ResourceClaimTemplate",
                                           rc["resourceClaimTemplateName"], ns)
                    t_spec = tmpl.get("spec") or {}
                    name = f"{md['name']}-{rc['name']}-{os.urandom(3).hex()[:5]}"
                    self.client.create({
                        "apiVersion": "resource.k8s.io/v1beta1", "kind": "ResourceClaim",
                        "metadata": {"name": name, "namespace": ns,
                                     "labels": dict((t_spec.get("metadata") or {}).get("labels") or {}),
                                     "annotations": {"resource.kubernetes.io/pod-claim-name": rc["name"]},
                                     "ownerReferences": [{"apiVersion": "v1", "kind": "Pod", "name": md["name"],
                                                          "uid": md.get("uid"), "controller": True,
                                                          "blockOwnerDeletion": True}]},
                        "spec": t_spec.get("spec") or {}})
                    done[rc["name"]] = name
                    new.append({"name": rc["name"], "resourceClaimName": name})
                out[rc["name"]] = done[rc["name"]]
        if new:
            self.client.patch("v1", "Pod", md["name"], {"status": {"resourceClaimStatuses": [
                {"name": k, "resourceClaimName": v} for k, v in done.items()]}}, ns, subresource="status")
        return out

    def _prepare_claims(self, run: _PodRun, ctr: dict) -> tuple[list[int], dict[str, str], list[str]]:
        with run.node.dra_lock:
            devices, envs, uids = self._prepare_claims_locked(run, ctr)
            run.dra_uids = uids
            return devices, envs, uids

    def _prepare_claims_locked(self, run: _PodRun, ctr: dict) -> tuple[list[int], dict[str, str], list[str]]:
        """The kubelet's DRA manager for a pod's ResourceClaims: prepare all of
        them through the node's DRA driver (idempotent: once per pod in
        effect), then give container ``ctr`` the CDI devices of the claims -
        and requests - its ``resources.claims`` names, and only those, composed
        as a CDI runtime does (toolkit/cdi.py, strict: two claims setting one
        variable differently fail the container).  Returns (device indices
        the container sees, its env, the pod's prepared claim uids)."""
        from ..dra import api as dra_api
        from . import fakedra

        node = run.node
        try:  # the scheduler recorded template claims in the pod's status after the kubelet's copy was taken
            pod = self.client.get("v1", "Pod", run.name, run.ns)
        except NotFound:
            pod = run.pod
        by_ref = self._pod_claims(pod)
        claims = [self.client.get("resource.k8s.io/v1beta1", "ResourceClaim", n, run.ns) for n in by_ref.values()]
        try:
            out = self._dra_kubelet(node).prepare(dra_api.DRIVER_NAME, claims)
        except AdmissionError:
            raise
        except Exception:  # noqa: BLE001 - the driver restarted: the plugin watcher registers it again
            node.dra = None
            out = self._dra_kubelet(node).prepare(dra_api.DRIVER_NAME, claims)
        errors = [r.error for r in out.values() if r.error]
        if errors:
            raise AdmissionError("; ".join(errors))
        from ..discovery import topology

        by_minor = {f"/dev/dri/renderD{g.render_minor}": g.index for g in topology.enumerate_gpus(node.env.sysfs_root())}
        # pod-resources: each container holds the claims its resources.claims names
        held = {c["metadata"]["name"]: {"claim": (run.ns, c["metadata"]["name"]), "resources": [
            (dra_api.DRIVER_NAME, d.pool_name, d.device_name, list(d.cdi_device_ids)) for d in out[c["metadata"]["uid"]].devices]}
            for c in claims}
        for other in run.pod["spec"]["containers"]:
            refs = [by_ref.get(x.get("name")) for x in (other.get("resources") or {}).get("claims") or []]
            if any(r in held for r in refs):
                node.kubelet.record_claims(run.ns, run.name, other["name"], [held[r] for r in refs if r in held])
        from ..toolkit import cdi

        uid_of = {c["metadata"]["name"]: c["metadata"]["uid"] for c in claims}
        ids: list[str] = []
        for ref in (ctr.get("resources") or {}).get("claims") or []:
            claim_name = by_ref.get(ref.get("name"))
            if claim_name is None:
                raise AdmissionError(f"container {ctr['name']}: claim {ref.get('name')!r} is not in spec.resourceClaims")
            for dev in out[uid_of[claim_name]].devices:
                if ref.get("request") and ref["request"] not in dev.request_names:
                    continue  # a container may take one request of a shared claim
                ids += [i for i in dev.cdi_device_ids if i not in ids]
        try:
            edits = cdi.resolve(node.env.cdi_dir, ids, strict=True)
        except cdi.CDIError as e:
            raise RuntimeError(f"container {ctr['name']}: {e}") from e
        devices = [by_minor[dn["path"]] for dn in edits.device_nodes if dn.get("path") in by_minor]
        envs = dict(edits.env)
        return devices, envs, list(out)

    def _dra_kubelet(self, node: SimNode, timeout: float = 30.0):
        """The node's kubelet plugin watcher + DRA manager: the driver is
        registered once (GetInfo / NotifyRegistrationStatus) and its endpoint
        reused for every pod, as on a real kubelet."""
        from ..dra import api as dra_api
        from . import fakedra

        with self._lock:
            if node.dra is None:
                node.dra = fakedra.FakeDraKubelet(os.path.dirname(node.env.device_plugin_dir.rstrip("/")))
            k = node.dra
        deadline = time.monotonic() + timeout
        while dra_api.DRIVER_NAME not in k.plugins and dra_api.DRIVER_NAME not in k.discover():
            if time.monotonic() >= deadline:
                raise AdmissionError(f"DRA driver {dra_api.DRIVER_NAME} not registered on {node.spec.name}")
            time.sleep(0.05)
        return k

    def _unprepare_claims(self, run: _PodRun, uids: list[str]) -> None:
        """NodeUnprepareResources for the claims no other pod on the node
        still uses (the kubelet's DRA manager counts a shared claim's pods)."""
        with run.node.dra_lock:
            self._unprepare_claims_locked(run, uids)

    def _unprepare_claims_locked(self, run: _PodRun, uids: list[str]) -> None:
        from ..dra import api as dra_api

        with self._lock:
            run.dra_uids = []  # this pod's containers are done with them
            in_use = {u for r in run.node.pods.values() if r is not run for u in r.dra_uids}
        claims = [{"metadata": {"namespace": run.ns, "name": "", "uid": u}} for u in uids if u not in in_use]
        if not claims:
            return
        try:
            self._dra_kubelet(run.node, timeout=2.0).unprepare(dra_api.DRIVER_NAME, claims)
        except Exception:  # noqa: BLE001 - once more through a fresh registration
            run.node.dra = None
            try:
                self._dra_kubelet(run.node, timeout=2.0).unprepare(dra_api.DRIVER_NAME, claims)
            except Exception as e:  # noqa: BLE001 - the driver is gone: its checkpoint keeps the claim
                log.debug("unprepare %s: %s", uids, e)

    # -------------------------------------------------------------- kubelet
    def _kubelet_loop(self, node: SimNode) -> None:
        sel = f"spec.nodeName={node.spec.name}"
        threading.Thread(target=self._kubelet_resync, args=(node,), daemon=True,
                         name=f"sim-kubelet-resync-{node.spec.name}").start()
        while not self.stop_event.is_set():
            try:
                for etype, pod in self.client.watch("v1", "Pod", field_selector=sel, stop=self.stop_event):
                    self._on_pod(node, etype, pod)
            except Exception as e:  # noqa: BLE001
                log.debug("kubelet watch: %s", e)
                self.stop_event.wait(0.1)

    def _kubelet_resync(self, node: SimNode) -> None:
        """Periodic relist (like kubelet's sync loop): pods missed by the watch
        are started, pods deleted behind its back are stopped."""
        sel = f"spec.nodeName={node.spec.name}"
        while not self.stop_event.wait(0.5):
            try:
                live = {p["metadata"]["name"]: p for p in self.client.list("v1", "Pod", field_selector=sel)}
            except Exception:  # noqa: BLE001
                continue
            with self._lock:
                for name, pod in live.items():
                    if name not in node.pods or pod["metadata"].get("deletionTimestamp"):
                        try:  # listed before a delete the watch has handled since: do not run it again
                            pod = self.client.get("v1", "Pod", name, pod["metadata"].get("namespace"))
                        except NotFound:
                            continue
                        self._on_pod(node, "ADDED", pod)
                for name in [n for n in node.pods if n not in live]:
                    self._on_pod(node, "DELETED", {"metadata": {"name": name}})

    def _on_pod(self, node: SimNode, etype: str, pod: dict) -> None:
        with self._lock:
            self._on_pod_locked(node, etype, pod)

    def _on_pod_locked(self, node: SimNode, etype: str, pod: dict) -> None:
        name = pod["metadata"]["name"]
        if etype != "DELETED" and pod["metadata"].get("deletionTimestamp"):
            self._terminate(node, pod)
            return
        if etype == "DELETED":
            run = node.pods.pop(name, None)
            if run is not None:
                run.stop.set()
                node.kubelet.release(run.ns, name)
            return
        if etype == "ADDED" and name not in node.pods:
            run = _PodRun(self, node, pod)
            node.pods[name] = run
            run.thread.start()

    def _terminate(self, node: SimNode, pod: dict) -> None:
        """Graceful deletion: stop the containers, then confirm the delete once
        the termination time has passed (what the kubelet does)."""
        name, ns = pod["metadata"]["name"], pod["metadata"].get("namespace", "default")
        if name in node.terminating:
            return
        node.terminating.add(name)
        run = node.pods.get(name)
        if run is not None:
            run.stop.set()
        grace = float(pod["metadata"].get("deletionGracePeriodSeconds", 30))
        delay = min(grace, self.termination_s or 0.0)

        def finish():
            t0 = time.monotonic()
            if run is not None:  # like the kubelet: the delete is confirmed once the containers exited
                run.thread.join(grace)  # (their shutdown included), or the grace period ran out
            if not self.stop_event.wait(max(0.0, delay - (time.monotonic() - t0))):
                try:
                    self.client.delete("v1", "Pod", name, ns, grace_period_seconds=0)
                except NotFound:
                    pass
            node.terminating.discard(name)

        threading.Thread(target=finish, daemon=True, name=f"sim-terminate-{name}").start()

    def _node_status_loop(self, node: SimNode) -> None:
        """The kubelet's node-status sync: device-plugin capacity is published
        on every ``node_status_s`` tick (with client-go style 4% jitter when
        modelling a real period), not when a plugin registers."""
        import random

        last = None
        period = self.node_status_s
        modelled = period > self.poll_s
        delay = random.uniform(0, period) if modelled else period  # tick phase: the kubelet started long before
        while not self.stop_event.wait(delay):
            delay = period * (1 + 0.04 * random.random()) if modelled else period
            caps = {}
            for res in list(node.kubelet.resources):
                caps[res] = (node.kubelet.capacity(res), node.kubelet.allocatable(res))
            if caps == last:
                continue
            try:
                cur = self.client.get("v1", "Node", node.spec.name)
                st = cur.setdefault("status", {})
                cap = st.setdefault("capacity", {})
                alloc = st.setdefault("allocatable", {})
                for res, (c, a) in caps.items():
                    cap[res] = str(c)
                    alloc[res] = str(a)
                self.client.update_status(cur)
                last = caps
            except Exception:  # noqa: BLE001
                pass

    # --------------------------------------------------------------- trace
    def trace(self, what: str, detail: str) -> None:
        self.events.append((time.perf_counter(), what, detail))

    def _trace_api(self, etype: str, obj: dict) -> None:
        kind = obj.get("kind")
        if kind == "Pod" and etype in ("ADDED", "DELETED"):
            self.trace(f"pod-{etype.lower()}", obj["metadata"]["name"])
        elif kind == "DaemonSet" and etype == "MODIFIED":  # the status the operator's states read
            st = obj.get("status") or {}
            if st.get("desiredNumberScheduled") and st.get("numberReady") == st.get("desiredNumberScheduled"):
                self.trace("ds-ready", obj["metadata"]["name"])
        elif kind == "ClusterPolicy" and etype == "MODIFIED":
            self.trace("policy-status", (obj.get("status") or {}).get("state") or "")

    def trace_since(self, t0: float) -> list[tuple[float, str, str]]:
        """Events after ``t0`` (perf_counter), times relative to it."""
        return [(round(t - t0, 4), w, d) for t, w, d in list(self.events) if t >= t0]

    # ------------------------------------------------------------ containers
    def run_container(self, run: _PodRun, c: dict, init: bool) -> None:
        cmd = list(c.get("command") or []) + list(c.get("args") or [])
        if not cmd:
            raise RuntimeError(f"container {c['name']} has no command")
        prog = os.path.basename(cmd[0])
        label = f"{run.name}/{c['name']}"
        self.trace("container-start", label)
        try:
            if prog in ("amdgpu-operator", "amdgpu-nfd") and self.process_containers:
                self._run_process_container(run, c, cmd, init)
            elif prog == "amdgpu-operator":
                from ..cli import operands

                operands.run_in_sim(self, run, c, cmd[1:], init)
            elif prog == "amdgpu-nfd":  # in-process: the Python worker with the same labels and arguments
                from ..cli import operands

                operands.run_in_sim(self, run, c, ["nfd", *cmd[1:]], init)
            elif prog in ("amdgpu-validator", "amdgpu-gpu-check"):
                self._run_gpu_workload(run, c, cmd)
            else:
                raise RuntimeError(f"unknown program {prog}")
        finally:
            self.trace("container-end", label)

    def _process_env(self, run: _PodRun, c: dict, ready_file: str) -> dict:
        """Environment of an operand process: the container's env (downward
        API resolved) plus what the DaemonSet's host mounts give a real
        operand, pointed at this simulated node's directories."""
        from ..cli.operands import container_env

        env = run.node.env
        cenv = container_env(run.pod, c)
        if cenv.get("RUNTIME_PID_FILE"):  # never signal the machine's own container runtime
            cenv["RUNTIME_PID_FILE"] = os.path.join(run.node.dir, cenv["RUNTIME_PID_FILE"].lstrip("/"))
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        penv = dict(os.environ)
        penv.update(cenv)
        penv.update({
            "NODE_NAME": env.node_name, "HOST_ROOT": env.host_root, "VALIDATIONS_DIR": env.validations_dir,
            "DEVICE_PLUGIN_DIR": env.device_plugin_dir, "POD_RESOURCES_SOCKET": env.pod_resources_socket,
            "CDI_SPEC_DIR": env.cdi_dir, "CONTAINERD_CONFIG": env.containerd_config,
            "CRIO_CONFIG_DIR": env.crio_config_dir, "DOCKER_CONFIG": env.docker_config, "INSTALL_DIR": env.install_dir,
            "OPERATOR_NAMESPACE": env.namespace, "VALIDATION_POLL_S": str(env.poll_s),
            "KUBECONFIG": self._kubeconfig_for(run.ns, run.pod["spec"].get("serviceAccountName") or "default"),
            "AMDGPU_READY_FILE": ready_file, "AMDGPU_SIM_NODE": "1", "AMDGPU_STARTUP_TRACE": ready_file + ".trace",
            "PYTHONPATH": os.pathsep.join([root] + [x for x in os.environ.get("PYTHONPATH", "").split(os.pathsep) if x])})
        if "kmod" in env.extra:
            penv["AMDGPU_SIM_KMOD"] = "1"
        if env.extra.get("metrics_fixture"):
            penv["AMDGPU_SIM_METRICS_FIXTURE"] = env.extra["metrics_fixture"]
        if self.fake_gpu:
            penv["AMDGPU_SIM_FAKE_VALIDATOR"] = "1"
        penv.pop("KUBERNETES_SERVICE_HOST", None)  # the simulated API server, not a real cluster's
        return penv

    def _run_process_container(self, run: _PodRun, c: dict, cmd: list[str], init: bool) -> None:
        """``process_containers``: the operand as its own process (see __init__)."""
        import signal
        import subprocess

        from ..utils.fswait import wait_for_file

        d = os.path.join(run.node.dir, "containers", f"{run.name}.{c['name']}.{run.restarts}")
        os.makedirs(d, exist_ok=True)
        ready_file = os.path.join(d, "ready")
        for f in (ready_file, ready_file + ".started"):
            if os.path.exists(f):
                os.unlink(f)
        penv = self._process_env(run, c, ready_file)
        rec = {"pod": run.name, "container": c["name"], "init": init, "args": cmd[1:3]}
        t0 = time.perf_counter()
        rec["spawn"] = t0
        rec["spawn_wall"] = time.time()
        rec["trace_file"] = ready_file + ".trace"
        if os.path.basename(cmd[0]) == "amdgpu-nfd":  # the native worker (native/nfd)
            from .. import native

            argv = [str(native.binary("amdgpu-nfd")), *cmd[1:]]
        else:
            argv = [sys.executable, "-S", "-m", "amdgpu_operator", *cmd[1:]]  # as the images' entry point
        with open(os.path.join(d, "log"), "w") as log_f:
            p = subprocess.Popen(argv, env=penv, stdout=log_f, stderr=subprocess.STDOUT, start_new_session=True)
        self.process_stats.append(rec)

        def started_s():
            try:  # the operand's main began (interpreter + imports done): wall time in the file
                with open(ready_file + ".started") as f:
                    return round(float(f.read()) - (time.time() - (time.perf_counter() - t0)), 4)
            except (OSError, ValueError):
                return None

        def watch_ready():
            # inotify wakes this at the rename that publishes the file; the
            # period only bounds how late a stop is noticed (the harness
            # shares the GIL with the API server and the fake kubelet: no
            # tight polling here)
            if wait_for_file(ready_file, 600.0, run.stop, 0.05):
                rec["ready_s"] = round(time.perf_counter() - t0, 4)
                try:  # when the operand wrote it (wall clock), next to when the kubelet saw it
                    with open(ready_file) as f:
                        rec["ready_written_s"] = round(float(f.read()) - rec["spawn_wall"], 4)
                except (OSError, ValueError):
                    pass
                if started_s() is not None:
                    rec["started_s"] = started_s()
                run.set_ready(c["name"])

        if not init:
            threading.Thread(target=watch_ready, daemon=True, name=f"ready-{run.name}-{c['name']}").start()
        exited = threading.Event()

        def stop_on_delete():  # the kubelet's SIGTERM (then SIGKILL) when the pod goes
            while not exited.is_set():
                if run.stop.wait(0.25):
                    break
            if exited.is_set():
                return
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except ProcessLookupError:
                return
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass

        killer = threading.Thread(target=stop_on_delete, daemon=True, name=f"stop-{run.name}-{c['name']}")
        killer.start()
        p.wait()  # blocks without waking the interpreter
        exited.set()
        rec["exit_s"] = round(time.perf_counter() - t0, 4)
        rec["rc"] = p.returncode
        if "started_s" not in rec and started_s() is not None:
            rec["started_s"] = started_s()
        if p.returncode != 0 and not run.stop.is_set():
            with open(os.path.join(d, "log")) as f:
                tail = f.read()[-1500:]
            raise RuntimeError(f"{c['name']} exited {p.returncode}: {tail}")

    def _run_gpu_workload(self, run: _PodRun, c: dict, cmd: list[str]) -> None:
        """Non-operand pod with GPU limits: Allocate -> OCI hook -> validator."""
        from .. import native
        from ..validator.validate import REPORT_EARLY

        node = run.node
        limits = (c.get("resources") or {}).get("limits") or {}
        gpu_res = [(k, int(v)) for k, v in limits.items() if k.startswith(RESOURCE_NAME)]
        envs: dict[str, str] = {}
        devices: list[int] = []
        if run.pod["spec"].get("resourceClaims") and not gpu_res:  # DRA: the claims' CDI devices
            devices, envs, uids = self._prepare_claims(run, c)
            self.trace("gpu-pod-allocated", run.name)
            run.cleanups.append(lambda: self._unprepare_claims(run, uids))
        elif gpu_res:
            res, n = gpu_res[0]
            if not node.kubelet.wait_registered(res, timeout=30):
                raise AdmissionError(f"resource {res} not registered on {node.spec.name}")
            try:
                ids, resp = node.kubelet.allocate(res, n, run.ns, run.name, c["name"])
            except RuntimeError as e:
                raise AdmissionError(str(e)) from e
            self.trace("gpu-pod-allocated", run.name)
            envs = dict(resp.envs)
            devices = [int(x) for x in envs.get("AMD_VISIBLE_DEVICES", "").split(",") if x != ""]
            try:
                cur = self.client.get("v1", "Pod", run.name, run.ns)
                self.client.patch("v1", "Pod", run.name, {"metadata": {"annotations": {
                    "amd.com/gpu.allocated": ",".join(ids)}}}, run.ns)
            except NotFound:
                pass
            # OCI hook at the hooks.d precreate stage, exactly as CRI-O / podman
            # call it: the runtime spec on stdin, the edited spec on stdout
            spec = {"ociVersion": "1.1.0", "process": {"args": cmd, "env": [f"{k}={v}" for k, v in envs.items()]},
                    "root": {"path": "rootfs"}, "linux": {}}
            import subprocess

            p = subprocess.run([str(native.binary("amdgpu-oci-hook")), "precreate", "--root", node.env.sysfs_root()],
                               input=json.dumps(spec), capture_output=True, text=True, timeout=30)
            if p.returncode != 0:
                raise RuntimeError(f"OCI hook failed: {p.stderr.strip()}")
            spec = json.loads(p.stdout)
            paths = {d["path"] for d in spec.get("linux", {}).get("devices", [])}
            if "/dev/kfd" not in paths:
                raise RuntimeError("OCI hook did not inject /dev/kfd")
            # the container sees the GPUs whose render nodes the runtime put in
            # (fault injection: hook_drop_devices leaves the last ones out)
            from ..discovery import topology

            minors = {g.index: g.render_minor for g in topology.enumerate_gpus(node.env.sysfs_root())}
            injected = [d for d in devices if f"/dev/dri/renderD{minors.get(d)}" in paths]
            devices = injected[:max(0, len(injected) - self.hook_drop_devices)] if self.hook_drop_devices else injected
        self.trace("gpu-pod-hooked", run.name)
        argv = [str(native.binary(os.path.basename(cmd[0])))] + cmd[1:]
        proc_env = {e["name"]: e["value"] for e in c.get("env") or [] if "value" in e}  # the container's env
        if REPORT_EARLY:
            proc_env[REPORT_EARLY_ENV] = "1"
        dev = devices[0] if devices else None
        if devices:
            proc_env.update(container_device_env(node.env.sysfs_root(), devices))
        if run.pod["spec"].get("resourceClaims") and not gpu_res:
            proc_env.update(envs)  # the CDI edits' environment
            if not devices:  # a container of a claim-holding pod that names no claim: no GPU in it
                proc_env["ROCR_VISIBLE_DEVICES"] = ""
        self.trace("gpu-pod-launch", run.name)
        res = node.env.launch(argv, proc_env, device=dev, timeout=600)
        self.trace("gpu-pod-reported", run.name)
        try:  # the process's own step times, for the bring-up breakdown
            rep = json.loads(res.stdout.strip().splitlines()[-1])
            self.pod_reports[run.name] = rep
            self.container_reports[(run.name, c["name"])] = rep
            steps = " ".join(f"{x['name']}={x.get('seconds', 0):.4f}" for x in rep.get("steps", []))
            self.trace("gpu-pod-steps", f"{run.name} total={rep.get('seconds', 0):.4f} {steps}")
        except (ValueError, IndexError, KeyError, TypeError):
            pass
        if res.rc != 0:
            raise RuntimeError(f"workload failed rc={res.rc}: {res.stderr.strip()[-500:]} {res.stdout.strip()[-500:]}")

    def known_images(self) -> set[str]:
        """What the simulated registry holds: the chart's operator image, every
        image of every ClusterPolicy (api/clusterpolicy.py policy_images) and
        AMDGPUDriver, and :attr:`pushed_images`."""
        from ..api.clusterpolicy import policy_images
        from ..api.driver_cr import AMDGPUDriverSpec
        from ..helm.values import default_values

        try:
            cps = self.client.list(CP_API, "ClusterPolicy")
        except Exception:  # noqa: BLE001 - CRD not installed yet
            cps = []
        try:
            drvs = self.client.list(CP_API, "AMDGPUDriver")
        except Exception:  # noqa: BLE001
            drvs = []
        key = tuple((o["metadata"].get("name"), o["metadata"].get("resourceVersion")) for o in cps + drvs)
        if self._images_cache[0] != key:
            imgs = set()
            op = default_values().get("operator") or {}
            imgs.add(f"{op.get('repository')}/{op.get('image')}:{op.get('version')}")
            for cp in cps:
                try:
                    imgs.update(policy_images(cp.get("spec") or {}).values())
                except Exception:  # noqa: BLE001 - a spec the API would have rejected
                    continue
            for d in drvs:
                try:
                    spec = AMDGPUDriverSpec.model_validate(d.get("spec") or {})
                    imgs.add(spec.ref(spec.image))
                except Exception:  # noqa: BLE001
                    continue
            self._images_cache = (key, imgs)
        return self._images_cache[1] | self.pushed_images

    # -------------------------------------------------------------- queries
    def policy(self) -> dict | None:
        try:
            return self.client.get(CP_API, "ClusterPolicy", "cluster-policy")
        except NotFound:
            return None

    def is_ready(self, expect_allocatable: dict[str, int | dict] | None = None) -> bool:
        cp = self.policy()
        if not cp or (cp.get("status") or {}).get("state") != "ready":
            return False
        for node in self.nodes.values():
            if node.spec.gpus <= 0:
                continue
            n = self.client.get("v1", "Node", node.spec.name)
            if (n["metadata"].get("labels") or {}).get("amd.com/gpu.validated") != "true":
                return False
            want = (expect_allocatable or {}).get(node.spec.name)
            if want is not None:  # a count of amd.com/gpu, or {resource: count}
                alloc = (n.get("status") or {}).get("allocatable") or {}
                for res, count in (want.items() if isinstance(want, dict) else [(RESOURCE_NAME, want)]):
                    if int(alloc.get(res, "0")) != count:
                        return False
        return True

    def wait_for_state(self, state: str, timeout: float = 30.0) -> bool:
        """Wait until the ClusterPolicy reports ``state``."""
        deadline = time.perf_counter() + timeout
        while time.perf_counter() < deadline:
            if ((self.policy() or {}).get("status") or {}).get("state") == state:
                return True
            time.sleep(self.poll_s)
        return False

    def wait_ready(self, timeout: float = 60.0, expect_allocatable: dict[str, int | dict] | None = None) -> float:
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < timeout:
            if self.is_ready(expect_allocatable):
                return time.perf_counter() - t0
            time.sleep(self.poll_s)
        raise TimeoutError(f"cluster not ready after {timeout}s:\n{self.diagnostics()}")

    def diagnostics(self) -> str:
        """Policy status, node labels/allocatable and every pod's phase (debugging aid)."""
        out = {"policy": (self.policy() or {}).get("status"), "nodes": {}, "pods": {}}
        for n in self.client.list("v1", "Node"):
            out["nodes"][n["metadata"]["name"]] = {
                "labels": {k: v for k, v in (n["metadata"].get("labels") or {}).items() if k.startswith("amd.com")},
                "allocatable": (n.get("status") or {}).get("allocatable")}
        for p in self.client.list("v1", "Pod"):
            st = p.get("status") or {}
            out["pods"][p["metadata"]["name"]] = {"phase": st.get("phase"), "message": st.get("message", "")[:500],
                                                  "ready": [c.get("ready") for c in st.get("containerStatuses", [])]}
        for name, node in self.nodes.items():
            out["nodes"].setdefault(name, {})["validations"] = sorted(os.listdir(node.env.validations_dir)) \
                if os.path.isdir(node.env.validations_dir) else []
            kmod = node.env.extra.get("kmod")
            if kmod is not None:
                from ..driver.manager import read_state

                out["nodes"][name]["module"] = {"live": kmod._live(), "log": list(getattr(kmod, "log", []))[-6:],
                                                "state": read_state(node.env)}
        return json.dumps(out, indent=1, default=str)[:20000]

    def pods(self, namespace: str | None = None) -> list[dict]:
        return self.client.list("v1", "Pod", namespace or self.namespace)


def container_device_env(sysfs_root: str, devices: list[int]) -> dict:
    """What a GPU container's runtime sees: only its allocated devices.

    The hook / CDI give the container just the allocated render nodes, so its
    HSA runtime enumerates only those GPUs; a process on the host gets the
    same view from :func:`~..discovery.topology.visible_devices_env`."""
    from ..discovery import topology

    gpus = topology.enumerate_gpus(sysfs_root)
    by_index = {g.index: g for g in gpus}
    sel = [by_index.get(d) for d in devices]
    if any(g is None for g in sel):
        return {"HIP_VISIBLE_DEVICES": ",".join(str(d) for d in devices)}
    return topology.visible_devices_env(sel, gpus)


def new_id() -> str:
    return uuid.uuid4().hex[:8]


def _quote(argv) -> str:
    return " ".join(shlex.quote(a) for a in argv)

