"""Headline benchmark: validator time-to-Ready + allocatable amd.com/gpu.

Metric (BASELINE.json): "validator pod time-to-Ready (s) + allocatable
amd.com/gpu at 1/2/4/8 MI355X".  One step = one full operator bring-up on a
node with N MI355X GPUs, measured from ClusterPolicy creation (the moment
``helm install`` of /root/reference/README.md:101-110 creates it) until the
node is validated and advertises ``amd.com/gpu: N``:

  operator reconcile -> NFD labels -> operator GPU-node labels -> driver probe
  (N1) -> container toolkit (CDI spec + containerd drop-in, N2) -> validator
  workload: one native process per GPU (HIP vectorAdd, MFMA bf16 GEMM with
  rocprofiler counter gate, HBM stream, xGMI one-shot all-reduce, RCCL
  all-reduce across all N GPUs over xGMI) -> device plugin registers over
  kubelet gRPC (ListAndWatch: N healthy) -> plugin validation: N pods x 1 GPU,
  each GetPreferredAllocation/Allocate -> native OCI hook on an OCI bundle ->
  HIP workload on its GPU -> node labelled validated.

Kubernetes itself is simulated in-process (fake apiserver + kubelet, no
kind/kubectl on the box); every GPU-touching step runs for real on the
MI355X.  Under ``torch.distributed.run`` each rank owns one GPU and starts that
GPU's processes (gloo control channel); the node is the N GPUs of the job.

Reference number: no time-to-Ready is published; BASELINE.md gives <= ~600 s
(10 min pod AGE, README.md:202-206) and 1 allocatable GPU per node.
"""

from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# child processes (stand-in validators, operand helpers) import the package too
os.environ["PYTHONPATH"] = os.pathsep.join([ROOT] + [p for p in os.environ.get("PYTHONPATH", "").split(os.pathsep) if p])

BASELINE_TTR_S = 600.0
METRIC = "validator pod time-to-Ready (s) + allocatable amd.com/gpu at 1/2/4/8 MI355X"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--fake-gpu", action="store_true", help="CPU-only: synthetic sysfs, no GPU processes")
    ap.add_argument("--fake-gpu-procs", action="store_true",
                    help="CPU-only, but start stand-in validator processes through the rank launcher")
    ap.add_argument("--sysfs-root", default=None, help="default: / when a GPU is present, else synthetic")
    ap.add_argument("--quick-workload", action="store_true", help="small validator sizes (CI)")
    ap.add_argument("--operator-debounce", type=float, default=0.003,
                    help="the operator's reconcile debounce (s; the chart's default, cli/main.py --debounce)")
    ap.add_argument("--no-counter-gate", action="store_true", help="skip the rocprofiler counter gate (outer profiler)")
    ap.add_argument("--rccl-single-gpu", action="store_true",
                    help="rehearsal: run the RCCL validation process at N=1 too (multi-GPU critical path)")
    ap.add_argument("--rccl-process", choices=["separate", "shared"], default=None,
                    help="RCCL check in its own process per GPU or in the kernel-check process")
    ap.add_argument("--gate-mode", choices=["aql", "sdk"], default=None,
                    help="counter gate through AQL profiling packets (default) or the rocprofiler-sdk tool")
    ap.add_argument("--no-prespawn", action="store_true",
                    help="start the validator processes only after the driver validation (A/B of the start gate)")
    ap.add_argument("--kubelet-status-s", type=float, default=10.0,
                    help="simulated kubelet nodeStatusUpdateFrequency: Node.status.allocatable follows on that tick")
    ap.add_argument("--agent-poll-s", type=float, default=None,
                    help="operands' VALIDATION_POLL_S (default: the production default of NodeEnv)")
    ap.add_argument("--mode", choices=["process", "thread"], default="process",
                    help="operand containers as their own processes (python -m amdgpu_operator <operand>, the "
                         "operand images' entry point; device-plugin health watcher on) - the headline - or as "
                         "threads of the bench process (the round-1/2 lower bound)")
    ap.add_argument("--compare", type=int, default=2,
                    help="after the timed steps, this many bring-ups in the other --mode (reported, not timed)")
    ap.add_argument("--no-pod-workload", action="store_true",
                    help="skip the config-5 pod workload after the last timed bring-up")
    ap.add_argument("--pod-gemm", type=int, default=4096, help="GEMM size of the pod workload's pods")
    ap.add_argument("--no-sweep", action="store_true",
                    help="skip the collective sweep (RCCL all-reduce / all-gather / reduce-scatter, 8 B ... "
                         "--sweep-max-bytes, and every xGMI link on its own) after the last timed bring-up")
    ap.add_argument("--sweep-max-bytes", type=int, default=1 << 30)
    ap.add_argument("--settle-s", type=float, default=0.0,
                    help="start each bring-up this long after the previous one's cluster stopped (its GPU processes' "
                         "teardown in the kernel; 0: back to back)")
    ap.add_argument("--linger", action="store_true",
                    help="A/B: the workload validator processes stay until the plugin validation is done "
                         "(AMDGPU_VALIDATOR_LINGER=1) instead of exiting at their report")
    ap.add_argument("--no-tool-watch", action="store_true",
                    help="do not watch for GPU tools of other parties (amd-smi, rocm-smi, ...) during the bring-ups")
    ap.add_argument("--timeout", type=float, default=120.0)
    ap.add_argument("--detail", default=None, help="write per-step breakdown JSON here")
    ap.add_argument("--set", action="append", default=[], dest="extra_set",
                    help="experiments only: extra Helm --set flags on top of the reference's (the headline uses none)")
    return ap.parse_args()


def gpu_available(root: str = "/") -> bool:
    """GPUs from the KFD topology in sysfs (the N3 library), not from a HIP
    runtime: the harness never opens the device.  Every GPU process of a
    bring-up is a child (validator, plugin pod) that the step waits for, so
    there is no device work of the harness to synchronise, and a HIP context
    in each harness rank would hold /dev/kfd through every timed bring-up -
    at N = 8 eight GPU processes that a real control plane does not have."""
    if not os.path.exists(os.path.join(root, "dev/kfd")):
        return False
    try:
        from amdgpu_operator.discovery import topology

        return len(topology.enumerate_gpus(root)) > 0
    except Exception:  # noqa: BLE001 - no native library: no GPU path
        return False


def holds_kfd() -> bool:
    """Does this process have /dev/kfd open (a GPU context)?"""
    try:
        fds = os.listdir("/proc/self/fd")
    except OSError:
        return False
    for fd in fds:
        try:
            if os.readlink(f"/proc/self/fd/{fd}") == "/dev/kfd":
                return True
        except OSError:
            continue
    return False


def operand_breakdown(stats: list[dict], t0: float, t0_wall: float) -> dict:
    """Per operand container (process mode): when it was spawned (s after
    ClusterPolicy creation), when its main began (interpreter + imports),
    and when it was ready (long-running) or exited (init / run-to-completion)."""
    out = {}
    for r in stats:
        key = f"{r['pod'].rsplit('-', 1)[0]}/{r['container']}"
        e = {"spawn_at_s": round(r["spawn"] - t0, 4)}
        for k in ("started_s", "ready_written_s", "ready_s", "exit_s"):
            if k in r and not (k == "exit_s" and not r.get("init")):
                e[k] = r[k]
        # AMDGPU_STARTUP_TRACE: interpreter up (main), imports, API client, node env - s after spawn
        try:
            with open(r.get("trace_file", "")) as f:
                e["startup_s"] = {k: round(float(v) - r["spawn_wall"], 4) for k, v in (ln.split() for ln in f)}
        except (OSError, ValueError, KeyError):
            pass
        if r["container"] in ("amd-device-plugin", "amd-operator-validator"):
            # their JSON log lines, s after ClusterPolicy creation (critical-path operands)
            lines = []
            try:
                with open(os.path.join(os.path.dirname(r["trace_file"]), "log")) as f:
                    for ln in f:
                        try:
                            rec = json.loads(ln)
                            lines.append([round(rec["ts"] - t0_wall, 3), str(rec.get("msg", ""))[:120]])
                        except (ValueError, KeyError, TypeError):
                            continue
            except (OSError, KeyError):
                pass
            e["log"] = lines[:30]
        out.setdefault(key, e)
    return out


def cpu_throttle_stat() -> dict | None:
    """The job's cgroup CPU throttling counters (v2 ``cpu.stat`` or v1
    ``cpu/cpu.stat``), to tell a slow bring-up step that ran into the box's
    CPU quota (every thread of the job frozen until the next period) from
    one that was slow on its own."""
    try:
        with open("/proc/self/cgroup") as f:
            lines = [ln.strip().split(":", 2) for ln in f if ln.strip()]
    except OSError:
        return None
    cands = []
    for _, ctrl, path in lines:
        if ctrl == "":
            cands.append(f"/sys/fs/cgroup{path}/cpu.stat")
        elif "cpu" in ctrl.split(","):
            cands += [f"/sys/fs/cgroup/{ctrl}{path}/cpu.stat", f"/sys/fs/cgroup/cpu{path}/cpu.stat",
                      f"/sys/fs/cgroup/cpu,cpuacct{path}/cpu.stat"]
    for c in cands + ["/sys/fs/cgroup/cpu.stat", "/sys/fs/cgroup/cpu/cpu.stat"]:
        try:
            with open(c) as f:
                kv = dict(ln.split() for ln in f if len(ln.split()) == 2)
        except (OSError, ValueError):
            continue
        if "nr_throttled" in kv:
            ms = int(kv["throttled_usec"]) / 1e3 if "throttled_usec" in kv else int(kv.get("throttled_time", 0)) / 1e6
            return {"nr_periods": int(kv.get("nr_periods", 0)), "nr_throttled": int(kv["nr_throttled"]),
                    "throttled_ms": ms}
    return None


class GcMeter:
    """Collections of the bench process's garbage collector during a bring-up
    (each holds the interpreter lock, so it stalls the simulated cluster)."""

    def __init__(self):
        import gc

        self.pauses: list[tuple[int, float]] = []
        self._t = 0.0
        self._gc = gc
        gc.callbacks.append(self._cb)

    def _cb(self, phase, info):
        if phase == "start":
            self._t = time.perf_counter()
        else:
            self.pauses.append((info.get("generation", -1), time.perf_counter() - self._t))

    def stop(self) -> dict:
        self._gc.callbacks.remove(self._cb)
        longest = max((p for _, p in self.pauses), default=0.0)
        return {"collections": len(self.pauses), "gen2": sum(1 for g, _ in self.pauses if g == 2),
                "max_ms": round(longest * 1000, 1), "total_ms": round(sum(p for _, p in self.pauses) * 1000, 1)}


class StallMeter:
    """A thread of the bench process that wakes every 2 ms: its largest lateness
    is how long the simulated API server and kubelets (threads of this
    process) could not run - the interpreter lock held elsewhere, or the
    process not scheduled."""

    def __init__(self):
        self.max_s = 0.0
        self.max_cpu_s = 0.0  # this process's CPU time during the longest stall: ~the stall = a thread held the lock
        self._stop = threading.Event()
        self._th = threading.Thread(target=self._run, daemon=True, name="bench-stall-meter")
        self._th.start()

    def _run(self):
        period = 0.002
        while not self._stop.is_set():
            t, c = time.perf_counter(), time.process_time()
            time.sleep(period)
            late = time.perf_counter() - t - period
            if late > self.max_s:
                self.max_s, self.max_cpu_s = late, time.process_time() - c

    def stop(self) -> float:
        self._stop.set()
        self._th.join()
        return self.max_s


KFD_PROCS = "/sys/class/kfd/kfd/proc"
_LAST_STOP: list[float] = []  # perf_counter when the previous bring-up's cluster stopped


def settle_gpu(settle_s: float) -> dict | None:
    """Before a bring-up's clock starts: let the previous bring-up's GPU
    processes finish being torn down.  cluster.stop() ends the previous
    bring-up's operands (the device plugin's and the exporter's amd-smi
    sessions, the driver health container) right before the next clock
    starts; the kernel releases their KFD state afterwards, in a workqueue,
    and a new process's open of /dev/kfd waits for that work (BASELINE.md
    "what a fresh HIP process costs": ~0.14 s behind a just-exited process).
    A fresh node's GPUs have no such teardown in flight, so each bring-up
    starts ``settle_s`` after the previous one stopped.  Reports the wait and
    the KFD process count (every process on the host with /dev/kfd open)."""
    waited = 0.0
    if _LAST_STOP and settle_s > 0:
        waited = max(0.0, settle_s - (time.perf_counter() - _LAST_STOP[-1]))
        if waited:
            time.sleep(waited)
    try:
        kfd = len(os.listdir(KFD_PROCS))
    except OSError:
        kfd = None
    return {"waited_s": round(waited, 3), "kfd_procs": kfd}


def _proc_tree(root_pid: int) -> list[int]:
    """Every descendant of ``root_pid`` (from /proc/<pid>/stat's ppid)."""
    children: dict[int, list[int]] = {}
    try:
        pids = [int(p) for p in os.listdir("/proc") if p.isdigit()]
    except OSError:
        return []
    for pid in pids:
        try:
            with open(f"/proc/{pid}/stat", "rb") as f:
                st = f.read()
            ppid = int(st[st.rindex(b")") + 2:].split()[1])
        except (OSError, ValueError, IndexError):
            continue
        children.setdefault(ppid, []).append(pid)
    out, todo = [], [root_pid]
    while todo:
        p = todo.pop()
        for c in children.get(p, []):
            out.append(c)
            todo.append(c)
    return out


def tree_kfd_holders(root_pid: int | None = None) -> list[str]:
    """The processes of the bring-up's own tree (the harness's descendants;
    under torchrun the agent's, so every rank's children) holding /dev/kfd,
    as ``<pid>:<what>``: an operand container's ``python -m amdgpu_operator
    <operand>`` sub-command, or the executable's name (validator, pod check).
    Reading /proc/<pid>/fd of our own children sidesteps the PID namespace of
    the KFD process list in sysfs (it names host PIDs)."""
    if root_pid is None:
        root_pid = os.getppid() if int(os.environ.get("WORLD_SIZE", "1")) > 1 else os.getpid()
    out = []
    for pid in _proc_tree(root_pid):
        try:
            fds = os.listdir(f"/proc/{pid}/fd")
        except OSError:
            continue
        held = False
        for fd in fds:
            try:
                if os.readlink(f"/proc/{pid}/fd/{fd}") == "/dev/kfd":
                    held = True
                    break
            except OSError:
                continue
        if not held:
            continue
        try:
            with open(f"/proc/{pid}/cmdline", "rb") as f:
                argv = [a.decode(errors="replace") for a in f.read().split(b"\0") if a]
        except OSError:
            argv = []
        what = os.path.basename(argv[0]) if argv else "?"
        if "amdgpu_operator" in argv:
            i = argv.index("amdgpu_operator")
            what = " ".join(argv[i + 1:i + 3]) or what
        out.append(f"{pid}:{what[:40]}")
    return out


class BringUpFailed(RuntimeError):
    """A validation step of the bring-up failed: its host failure records
    (validate.py ``write_failure``) carry what failed and the rates measured
    against their floors."""

    def __init__(self, records: dict, elapsed_s: float):
        self.records = records
        self.elapsed_s = elapsed_s
        first = next(iter(records.values()), {})
        super().__init__(f"validation failed after {elapsed_s:.2f} s: {str(first.get('message', ''))[:400]}")


def failure_records(validations_dir: str, since_wall: float) -> dict:
    """``<step>-failed`` records written since ``since_wall`` (step -> record)."""
    out = {}
    try:
        names = os.listdir(validations_dir)
    except OSError:
        return out
    for name in names:
        if not name.endswith("-failed"):
            continue
        try:
            with open(os.path.join(validations_dir, name)) as f:
                rec = json.load(f)
        except (OSError, ValueError):
            continue
        if rec.get("time", 0) >= since_wall:
            out[name[:-len("-failed")]] = rec
    return out


def wait_ready_or_failed(cluster, node_env, timeout: float, t0_wall: float, expect=None) -> float:
    """cluster.wait_ready, but a validation that failed ends the wait at once
    with its records (:class:`BringUpFailed`) instead of at the timeout: the
    validator pod would restart and fail again, and the run would end with a
    bare timeout and none of the numbers that explain it."""
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < timeout:
        if cluster.is_ready(expect):
            return time.perf_counter() - t0
        recs = failure_records(node_env.validations_dir, t0_wall)
        if recs:
            time.sleep(0.05)  # the workload's detailed record is written just before the operand's own
            raise BringUpFailed(failure_records(node_env.validations_dir, t0_wall), time.perf_counter() - t0)
        time.sleep(cluster.poll_s)
    raise TimeoutError(f"cluster not ready after {timeout}s:\n{cluster.diagnostics()}")


def critical_path(r: dict) -> dict:
    """One bring-up's critical path, compact (s after ClusterPolicy creation
    unless named ``*_ms``): when each gate opened, the validator process's own
    steps, the plugin pod's HSA start, the gap from the validator's
    ``validated`` file to policy Ready, and what the harness or the machine
    did meanwhile (stall, GC, CPU throttling, GPU tools of other parties)."""
    tl = r.get("timeline_s") or {}
    cp: dict = {"ttr": round(r["time_to_ready_s"], 4)}
    at = {k: tl[k] for k in ("driver", "toolkit", "workload", "plugin", "complete") if k in tl}
    if r.get("kubelet_register_at_s"):
        at["registered"] = r["kubelet_register_at_s"][0]
    for k in ("plugin.devices_seen", "plugin.pods_created"):
        if k in tl:
            at[k.split(".", 1)[1]] = tl[k]
    for t, what, _ in r.get("trace") or []:
        if what in ("gpu-pod-hooked", "gpu-pod-reported") and what[8:] not in at and t < r["time_to_ready_s"]:
            at[what[8:]] = round(t, 4)
    cp["at"] = at
    if "complete" in tl:
        cp["ready_gap"] = round(r["time_to_ready_s"] - tl["complete"], 4)
    wl = {k: v for k, v in (r.get("rank0_step_seconds") or {}).items() if v is not None}
    if r.get("workload_process_seconds"):
        wl["proc"] = r["workload_process_seconds"][0]
    if r.get("rank0_gate_wait_s") is not None:
        wl["gate_wait"] = r["rank0_gate_wait_s"]
    cp["wl"] = {k: round(v, 4) for k, v in wl.items() if isinstance(v, (int, float))}
    pods = r.get("plugin_pod_reports") or []
    if pods:
        cp["pod"] = {k: v for k, v in pods[0].items() if v is not None}
    cp["stall_ms"] = r.get("harness_max_stall_ms")
    cp["gc_ms"] = (r.get("harness_gc") or {}).get("total_ms")
    cp["thr_ms"] = (r.get("cpu_throttled") or {}).get("ms")
    if r.get("foreign_gpu_tools"):
        cp["foreign_gpu_tools"] = r["foreign_gpu_tools"]
    if r.get("settle"):
        cp["settle"] = r["settle"]
    return cp


# the parts of a bring-up's critical path a slow step is measured on: (name,
# getter of the part's duration in s)
_CP_PARTS = (
    ("plugin pod HSA start-up (hsa_init)", lambda cp: (cp.get("pod") or {}).get("hsa_init")),
    ("plugin pod HSA set-up (queue, code object)", lambda cp: (cp.get("pod") or {}).get("hsa")),
    ("workload validator process", lambda cp: (cp.get("wl") or {}).get("proc")),
    ("driver validated", lambda cp: (cp.get("at") or {}).get("driver")),
    ("device plugin registered", lambda cp: (cp.get("at") or {}).get("registered")),
    ("plugin pod start (created -> main)", lambda cp: (((cp.get("pod") or {}).get("main_at") or 0)
                                                      - ((cp.get("at") or {}).get("pods_created") or 0)) or None),
    ("validated -> policy Ready", lambda cp: cp.get("ready_gap")),
    ("harness stall", lambda cp: (cp.get("stall_ms") or 0) / 1e3 or None),
)


def slow_steps(cps: list[dict], factor: float = 1.3) -> list[dict]:
    """Every timed bring-up above ``factor`` x the median time-to-Ready, with
    the critical-path part that grew the most against its own median (VERDICT
    r4: the record names the cause of any step above 1.3 x median)."""
    import statistics

    if len(cps) < 3:
        return []
    med = statistics.median(cp["ttr"] for cp in cps)
    meds = {}
    for name, get in _CP_PARTS:
        vals = [v for v in (get(cp) for cp in cps) if isinstance(v, (int, float))]
        if vals:
            meds[name] = statistics.median(vals)
    out = []
    for i, cp in enumerate(cps):
        if cp["ttr"] <= factor * med:
            continue
        growth = []
        for name, get in _CP_PARTS:
            v = get(cp)
            if isinstance(v, (int, float)) and name in meds:
                growth.append((v - meds[name], name, v))
        growth.sort(reverse=True)
        rec = {"step": i, "ttr": cp["ttr"], "median_ttr": round(med, 4)}
        if growth and growth[0][0] > 0:
            d, name, v = growth[0]
            rec["cause"] = name
            rec["cause_s"] = round(v, 4)
            rec["cause_median_s"] = round(meds[name], 4)
            rec["also"] = [{"part": n, "s": round(x, 4), "median_s": round(meds[n], 4)}
                           for dd, n, x in growth[1:3] if dd > 0.01]
        out.append(rec)
    return out


def one_bring_up(args, n_gpus: int, launcher, workdir: str, fake_gpu: bool, mode: str = "process",
                 pods: bool = False) -> dict:
    from amdgpu_operator.api.clusterpolicy import REFERENCE_SET_FLAGS, deep_merge, parse_set_flags
    from amdgpu_operator.testing.simcluster import NodeSpec, SimCluster

    root = None if fake_gpu else (args.sysfs_root or "/")
    node = NodeSpec("mi355x-node-0", gpus=n_gpus, sysfs_root=root)
    values = parse_set_flags(REFERENCE_SET_FLAGS + list(args.extra_set))
    if args.no_counter_gate:
        values = deep_merge(values, {"validator": {"workload": {"counterGate": False}}})
    if args.rccl_single_gpu:
        values = deep_merge(values, {"validator": {"workload": {"rcclSingleGpu": True}}})
    if args.rccl_process:
        values = deep_merge(values, {"validator": {"workload": {"rcclProcess": args.rccl_process}}})
    if args.gate_mode:
        values = deep_merge(values, {"validator": {"workload": {"counterGateMode": args.gate_mode}}})
    if args.no_prespawn:
        values = deep_merge(values, {"validator": {"workload": {"prespawn": False}}})
    if args.quick_workload:
        # small sizes fall outside the floors' calibration (gemmN 4096, 1 GiB copy): report only
        values = deep_merge(values, {"validator": {"workload": {"gemmN": 1024, "hbmBytes": 1 << 26,
                                                                "rcclElems": 1 << 20, "xgmiElems": 1 << 20,
                                                                "minGemmTflops": 0.0, "minHbmGbps": 0.0}}})
    from amdgpu_operator.nodeenv import NodeEnv

    d = tempfile.mkdtemp(prefix="step-", dir=workdir)
    agent_poll = NodeEnv.poll_s if args.agent_poll_s is None else args.agent_poll_s
    # termination_s=0: kubelet-confirmed pod deletes, as on a cluster
    cluster = SimCluster(d, [node], fake_gpu=fake_gpu, poll_s=0.005, launcher=launcher, agent_poll_s=agent_poll,
                         node_status_s=args.kubelet_status_s or None, termination_s=0.0,
                         operator_resync_s=30.0, operator_debounce_s=args.operator_debounce,  # cli/main.py defaults
                         process_containers=(mode == "process")).start()
    import gc

    try:
        # The simulated API server, kubelets and DaemonSet controller are
        # threads of this process; a collection of its garbage collector stops
        # them all (measured: up to ~0.1 s, the slowest bring-ups of a run,
        # harness_gc).  A cluster's control plane does not pause like that,
        # so the harness collects before the clock starts and not while it
        # runs.  The operator and the operands are processes of their own and
        # keep their collectors.
        gc.collect()
        settle = settle_gpu(args.settle_s)
        kfd_holders = {"start": tree_kfd_holders()}
        gc.disable()
        thr0 = cpu_throttle_stat()
        stall = StallMeter()
        gcm = GcMeter()
        t0 = time.perf_counter()
        t0_wall = time.time()
        nd = cluster.nodes["mi355x-node-0"]
        cluster.install_operator(values)
        try:
            # validator pod Ready: node validated, policy ready
            ttr = wait_ready_or_failed(cluster, nd.env, args.timeout, t0_wall)
        except BringUpFailed as e:
            e.partial = {"throttled": cpu_throttle_stat(), "stall_ms": round(stall.stop() * 1000, 1),
                         "gc": gcm.stop(), "t0_wall": t0_wall}
            raise
        thr1 = cpu_throttle_stat()
        max_stall = stall.stop()
        gc_stats = gcm.stop()
        gc.enable()
        # the operator's own GPU processes still open at Ready (operands' amd-smi sessions, ...)
        kfd_holders["ready"] = tree_kfd_holders()
        # the kubelet then publishes amd.com/gpu in Node.status on its own status tick
        # (experiments with the DRA driver instead of the device plugin: no amd.com/gpu)
        if (values.get("devicePlugin") or {}).get("enabled", True) is not False:
            cluster.wait_ready(args.timeout, {"mi355x-node-0": n_gpus})
        alloc_visible = time.perf_counter() - t0
        t_total = time.perf_counter() - t0
        pod_workload = None
        if pods:
            # BASELINE config 5 on the Ready node: user-shaped GEMM pods through
            # admission, GetPreferredAllocation, Allocate and the OCI hook
            # (reported next to the headline, not part of it)
            from amdgpu_operator.testing.podworkload import run_pod_workload

            pod_workload = run_pod_workload(cluster, "mi355x-node-0", n_gpus, gemm_n=args.pod_gemm,
                                            timeout=args.timeout,
                                            dra=(values.get("draDriver") or {}).get("enabled") is True)
        collectives = None
        if pods and not args.no_sweep:
            # SURVEY §5.8 on the Ready node: the RCCL curve and each xGMI link,
            # in validator processes the launcher starts on the GPUs' own ranks
            # (not part of `value`), with the Ready gate's floors next to them
            from amdgpu_operator.validator.sweep import collective_sweep

            w = ((cluster.policy() or {}).get("spec") or {}).get("validator", {}).get("workload", {}) or {}
            try:
                collectives = collective_sweep(nd.env, max_bytes=args.sweep_max_bytes,
                                               rccl_fraction=float(w.get("rcclBusbwLinkFraction", 0.2)),
                                               xgmi_fraction=float(w.get("xgmiReadLinkFraction", 0.25)),
                                               timeout=max(60.0, args.timeout))
            except Exception as e:  # noqa: BLE001 - reported, the headline stands
                collectives = {"ok": False, "error": f"{type(e).__name__}: {e}"[:1000]}
        cp = cluster.policy()
        nobj = cluster.client.get("v1", "Node", "mi355x-node-0")
        alloc = int(nobj["status"]["allocatable"].get("amd.com/gpu", "0"))
        from amdgpu_operator.validator.validate import read_ready

        wl = read_ready(nd.env, "workload") or {}
        plug = read_ready(nd.env, "plugin") or {}
        ranks = wl.get("ranks", [])
        steps = {}
        for r in ranks:
            for s in r.get("steps", []):
                steps.setdefault(s["name"], []).append(s)
        timeline = {}  # seconds after ClusterPolicy creation at which each ready file was written
        step_seconds = {}  # each step's own duration as its operand reported it
        for step in ("driver", "toolkit", "workload", "plugin", "complete"):
            r = read_ready(nd.env, step) or {}
            if "time" in r:
                timeline[step] = round(r["time"] - t0_wall, 4)
            if isinstance(r.get("seconds"), (int, float)):
                step_seconds[step] = round(r["seconds"], 4)
            for k, v in (r.get("marks") or {}).items():  # wall-clock marks inside a step
                timeline[f"{step}.{k}"] = round(v - t0_wall, 4)
        pod_reps = []  # the plugin-validation pods' own reports (their HSA start-up and check)
        for name, rep in cluster.pod_reports.items():
            if name.startswith("amd-validator-workload-") or name.startswith("amd-validator-dra-"):
                st = {}
                for x in rep.get("steps", []):
                    st[x["name"]] = round(st.get(x["name"], 0.0) + x.get("seconds", 0.0), 4)
                    for k in ("co_load_s", "queue_s"):  # the HSA set-up's parts (gpu_check.cpp)
                        if isinstance(x.get(k), (int, float)):
                            st[k[:-2]] = round(st.get(k[:-2], 0.0) + x[k], 4)
                main_at = None
                if isinstance(rep.get("t_main"), (int, float)):  # CLOCK_MONOTONIC at the pod process's main
                    main_at = round(rep["t_main"] - (time.monotonic() - time.perf_counter()) - t0, 4)
                pod_reps.append({"proc": rep.get("seconds"), "hsa_init": rep.get("hsa_init_s"), **st,
                                 "main_at": main_at,
                                 "done_at": round(main_at + rep["seconds"], 4) if main_at is not None
                                 and isinstance(rep.get("seconds"), (int, float)) else None})
        return {
            "mode": mode,
            "t0_wall": t0_wall,
            "settle": settle,
            "pod_workload": pod_workload,
            "collectives": collectives,
            "plugin_pod_reports": pod_reps,
            "rank0_gate_wait_s": ((ranks[0].get("start_gate") or {}).get("wait_s") if ranks else None),
            "operands": operand_breakdown(cluster.process_stats, t0, t0_wall) if mode == "process" else None,
            "time_to_ready_s": ttr,
            "allocatable_visible_s": alloc_visible,
            "allocatable_source": plug.get("allocatable_source"),
            "trace": cluster.trace_since(t0),
            "timeline_s": timeline,
            "step_seconds": step_seconds,
            "wall_s": t_total,
            "allocatable": alloc,
            "policy_state_seconds": (cp.get("status") or {}).get("stateReadySeconds"),
            "workload_seconds": wl.get("seconds"),
            "workload_process_seconds": [r.get("process_seconds") for r in ranks],
            "plugin_seconds": plug.get("seconds"),
            # the validator's pod-resources queries: (s after ClusterPolicy creation, duration, devices held)
            "plugin_kubelet_queries": [(round(q[0] - t0_wall, 4), q[1], q[2]) for q in plug.get("kubelet_queries", [])],
            "plugin_devices": plug.get("devices"),
            "kubelet_register_handler_s": [round(x, 4) for x in nd.kubelet.register_seconds],
            "harness_max_stall_ms": round(max_stall * 1000, 1),
            "harness_max_stall_cpu_ms": round(stall.max_cpu_s * 1000, 1),
            "harness_gc": gc_stats,
            # the job's cgroup CPU throttling during the timed bring-up (None: no cgroup stats)
            "cpu_throttled": None if not (thr0 and thr1) else {
                "periods": thr1["nr_throttled"] - thr0["nr_throttled"],
                "ms": round(thr1["throttled_ms"] - thr0["throttled_ms"], 2)},
            # s after ClusterPolicy creation: the plugin's Register arrived / its first device list arrived
            "kubelet_register_at_s": [round(x - t0_wall, 4) for x in nd.kubelet.register_walls],
            "kubelet_first_list_at_s": {r: round(x - t0_wall, 4) for r, x in nd.kubelet.first_list_walls.items()},
            "gemm_tflops": [s.get("tflops") for s in steps.get("gemm", [])],
            "gemm_counter_gate": [s.get("counter_gate") for s in steps.get("gemm", [])],
            "fp8_tflops": [s.get("tflops") for s in steps.get("gemm_fp8", [])],
            "fp8_counter_gate": [s.get("counter_gate") for s in steps.get("gemm_fp8", [])],
            "fp4_tflops": [s.get("tflops") for s in steps.get("gemm_fp4", [])],
            "fp4_counter_gate": [s.get("counter_gate") for s in steps.get("gemm_fp4", [])],
            "fp6_tflops": [s.get("tflops") for s in steps.get("gemm_fp6", [])],
            "fp6_counter_gate": [s.get("counter_gate") for s in steps.get("gemm_fp6", [])],
            "mxfp4_tflops": [s.get("tflops") for s in steps.get("gemm_mxfp4", [])],
            "mxfp4_counter_gate": [s.get("counter_gate") for s in steps.get("gemm_mxfp4", [])],
            "gate_attempts": [s.get("gate_attempts") for k in ("gemm", "gemm_fp8", "gemm_fp4", "gemm_fp6",
                                                                "gemm_mxfp4") for s in steps.get(k, [])],
            "kfd_holders": kfd_holders,
            # every counted dispatch of the bring-up: verdict, attempts, why a retry was needed, lock wait
            "gates": [{k: s.get(k) for k in ("name", "device", "counter_gate", "gate_attempts", "gate_retried_after",
                                             "gate_reason", "mfma_util", "mfma_util_floor", "gate_lock",
                                             "gate_lock_wait_s") if s.get(k) is not None}
                      for k2 in ("gemm", "gemm_fp8", "gemm_fp4", "gemm_fp6", "gemm_mxfp4") for s in steps.get(k2, [])],
            "hbm_gbps": [s.get("gbps") for s in steps.get("hbm", [])],
            "xgmi_read_gbps": [s.get("read_gbps") for s in steps.get("xgmi", [])],
            "rccl_busbw_gbps": [s.get("busbw_gbps") for s in steps.get("rccl", [])],
            "rccl_comm_init_s": [s.get("comm_init_s") for s in steps.get("rccl", [])],
            "rccl_library": [s.get("library") for s in steps.get("rccl", [])],
            "rccl_process_seconds": [r.get("rccl_process_seconds") for r in ranks],
            "rank0_step_seconds": {s["name"]: s.get("seconds") for s in (ranks[0].get("steps", []) if ranks else [])},
            "rank0_total_seconds": ranks[0].get("seconds") if ranks else None,
            "labels": {k: v for k, v in (nobj["metadata"].get("labels") or {}).items()
                       if k in ("amd.com/gpu.product", "amd.com/gpu.arch", "amd.com/gpu.family", "amd.com/gpu.memory",
                                "amd.com/gpu.xgmi.links", "amd.com/gpu.count", "amd.com/gpu.validated",
                                "amd.com/gpu.rdma.capable", "amd.com/gpu.rdma.nics", "amd.com/gpu.rdma.affinity")},
            "dmabuf": [s for s in steps.get("dmabuf", [])],  # driver.rdma (--set driver.rdma.enabled=true)
            "driver_rdma": (read_ready(nd.env, "driver") or {}).get("rdma"),
        }
    finally:
        gc.enable()
        cluster.stop()
        _LAST_STOP.append(time.perf_counter())
        shutil.rmtree(d, ignore_errors=True)


def standalone_sweep(args, launcher, fake_gpu, workdir: str) -> dict:
    """The collective sweep outside a cluster (after a failed bring-up): the
    node's GPUs, a scratch rendezvous directory and the run's launcher."""
    from amdgpu_operator.nodeenv import NodeEnv, run_local
    from amdgpu_operator.testing import fakesys
    from amdgpu_operator.validator.sweep import collective_sweep

    d = tempfile.mkdtemp(prefix="sweep-", dir=workdir)
    root = args.sysfs_root or "/"
    if fake_gpu:
        root = os.path.join(d, "host")
        fakesys.build_node(root, args.gpus)

    def launch(argv, env, device, timeout):
        if fake_gpu and os.path.basename(argv[0]) == "amdgpu-validator":
            argv = [sys.executable, "-m", "amdgpu_operator.testing.fake_validator", *argv[1:]]
        return launcher(argv, env, device, timeout) if launcher is not None else run_local(argv, env, timeout)

    env = NodeEnv("mi355x-node-0", None, host_root=root, validations_dir=os.path.join(d, "validations"),
                  launcher=launch)
    try:
        return collective_sweep(env, max_bytes=args.sweep_max_bytes, timeout=max(60.0, args.timeout))
    finally:
        shutil.rmtree(d, ignore_errors=True)


# The driver keeps a ~9 KB tail of the run's stdout + stderr and parses the JSON
# line out of it (BENCH_r05: a 22 KB line with every step's critical path did
# not parse).  The line carries the headline and summaries only; everything
# per step, per rank, per size or per link goes to the detail file it names.
LINE_BUDGET = 3000
MODEL = "amd-gpu-operator ClusterPolicy bring-up (reference --set flags) + HIP/MFMA/RCCL validator"


def default_detail_path(n_gpus: int) -> str:
    """``gpurun_out/bench_detail_n<N>.json`` in the tree (merged back from a GPU
    box), or the temp dir when the tree is read-only."""
    d = os.path.join(ROOT, "gpurun_out")
    try:
        os.makedirs(d, exist_ok=True)
        if os.access(d, os.W_OK):
            return os.path.join(d, f"bench_detail_n{n_gpus}.json")
    except OSError:
        pass
    return os.path.join(tempfile.gettempdir(), f"amdgpu_bench_detail_n{n_gpus}.json")


def write_detail(path: str, obj: dict) -> str | None:
    try:
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        tmp = f"{path}.tmp.{os.getpid()}"
        with open(tmp, "w") as f:
            json.dump(obj, f, indent=1, default=str)
        os.replace(tmp, path)
        return path
    except OSError:
        return None


def _r(x, nd=4):
    return round(x, nd) if isinstance(x, (int, float)) and not isinstance(x, bool) else x


def dist_summary(xs: list, nd: int = 4) -> dict | None:
    """min / median / p90 / max / mean of a list of numbers (nearest rank)."""
    v = sorted(x for x in xs if isinstance(x, (int, float)) and not isinstance(x, bool))
    if not v:
        return None
    n = len(v)

    def q(p):
        return v[min(n - 1, max(0, int(round(p * (n - 1)))))]

    return {"min": round(v[0], nd), "med": round(q(0.5), nd), "p90": round(q(0.9), nd), "max": round(v[-1], nd),
            "mean": round(sum(v) / n, nd)}


def per_gpu_range(xs: list, nd: int = 1):
    """A per-GPU list as [min, max] (one value at N = 1), None entries dropped."""
    v = [x for x in (xs or []) if isinstance(x, (int, float)) and not isinstance(x, bool)]
    if not v:
        return None
    return [round(min(v), nd)] if len(set(v)) == 1 or len(v) == 1 else [round(min(v), nd), round(max(v), nd)]


def gate_verdict(xs: list):
    """Per-GPU counter-gate verdicts, as one word when they agree."""
    v = [x for x in (xs or []) if x is not None]
    if not v:
        return None
    return v[0] if len(set(v)) == 1 else {k: v.count(k) for k in sorted(set(v))}


def collectives_summary(col: dict | None) -> dict | None:
    """The sweep (validator/sweep.py) as peak busBW, busBW at 1 MiB / 256 MiB,
    the Ready gate's worst ratio and the slowest link; the rows stay in the
    detail file."""
    if not col:
        return None
    out = {k: col[k] for k in ("ok", "world", "sizes", "simulated", "seconds") if k in col}
    if col.get("error"):
        out["error"] = str(col["error"])[:200]
    ar = (col.get("ops") or {}).get("allreduce") or []
    if ar:
        out["peak_busbw_gbps"] = max(r.get("busbw_gbps", 0.0) for r in ar)
        out["peak_algbw_gbps"] = max(r.get("algbw_gbps", 0.0) for r in ar)
        for label, b in (("1MiB", 1 << 20), ("256MiB", 256 << 20)):
            row = min(ar, key=lambda r: abs(r["bytes"] - b))
            if row["bytes"] == b or abs(row["bytes"] - b) <= b // 2:
                out[f"busbw_{label}_gbps"] = row.get("busbw_gbps")
        out["small_latency_us"] = ar[0].get("latency_us")
    ff = col.get("fabric_floors") or {}
    if ff:
        out["min_allreduce_ratio"] = ff.get("min_allreduce_ratio")
        below = ff.get("links_below_floor") or []
        out["links_below_floor"] = len(below)
        if below:
            out["links_below_floor_first"] = below[:4]
    lm = col.get("xgmi_links") or {}
    if lm:
        out["min_read_gbps"] = lm.get("min_read_gbps")
        out["links_intact"] = lm.get("intact")
    return out


def pod_workload_summary(pw: dict | None) -> dict | None:
    if not pw:
        return None
    out = {"ok": bool(pw.get("all_succeeded")) and pw.get("gemm_correct", True) is not False}
    for k, name in (("pods", "pods"), ("allocation", "allocation"), ("admission_to_kernel_done_p50_s", "p50_s"),
                    ("admission_to_kernel_done_p99_s", "p99_s"), ("single_gpu_pods_distinct_devices", "distinct"),
                    ("error", "error")):
        if k in pw:
            out[name] = str(pw[k])[:200] if k == "error" else pw[k]
    return out


def slow_summary(slow: list[dict]) -> dict:
    causes: dict[str, int] = {}
    for s in slow:
        if s.get("cause"):
            causes[s["cause"]] = causes.get(s["cause"], 0) + 1
    out: dict = {"count": len(slow), "factor": 1.3, "steps": [s["step"] for s in slow][:20]}
    if causes:
        top = max(causes.items(), key=lambda kv: kv[1])
        out["top_cause"] = top[0]
        out["top_cause_count"] = top[1]
    return out


def rates_summary(r: dict) -> dict:
    """The last timed bring-up's per-GPU validator rates, as [min, max]."""
    out = {}
    for k, name in (("gemm_tflops", "bf16_tflops"), ("fp8_tflops", "fp8_tflops"), ("fp4_tflops", "fp4_tflops"),
                    ("fp6_tflops", "fp6_tflops"), ("mxfp4_tflops", "mxfp4_tflops"), ("hbm_gbps", "hbm_gbps"),
                    ("xgmi_read_gbps", "xgmi_read_gbps"), ("rccl_busbw_gbps", "rccl_busbw_gbps"),
                    ("rccl_comm_init_s", "rccl_comm_init_s")):
        v = per_gpu_range(r.get(k) or [], 4 if k.endswith("_s") else 1)
        if v is not None:
            out[name] = v
    gates = {}
    for k, name in (("gemm_counter_gate", "bf16"), ("fp8_counter_gate", "fp8"), ("fp4_counter_gate", "fp4"),
                    ("fp6_counter_gate", "fp6"), ("mxfp4_counter_gate", "mxfp4")):
        g = gate_verdict(r.get(k) or [])
        if g is not None:
            gates[name] = g
    if gates:
        out["counter_gate"] = gates
    att = [a for a in (r.get("gate_attempts") or []) if isinstance(a, int)]
    if att:
        out["gate_attempts_max"] = max(att)
    return out


def gate_retry_summary(results: list) -> dict | None:
    """Every timed bring-up's counted dispatches: how many were counted again
    (another process's work in the window, gate_policy.h gate_retry_kind)
    and the most attempts any took."""
    att = [a for r in results for a in (r.get("gate_attempts") or []) if isinstance(a, int)]
    if not att:
        return None
    return {"gates": len(att), "retried": sum(1 for a in att if a > 1), "max_attempts": max(att)}


# the order optional summary fields leave the line if it is still over budget
# (a safety net: the summaries are sized to fit well below it at N = 8)
_SHED = ("warmup_time_to_ready_s", "other_mode_time_to_ready_s", "gate_retries", "kfd_holders", "pod_workload", "rates",
         "allocatable_visible_s", "collectives", "time_to_ready_s", "slow_steps", "settle")


def fit_line(out: dict, budget: int = LINE_BUDGET) -> str:
    """The JSON line, at most ``budget`` bytes: the headline fields first,
    optional summaries shed (and named in ``config.shed``) if it is over."""
    line = json.dumps(out, separators=(",", ":"))
    cfg = out.get("config") or {}
    shed = []
    for k in _SHED:
        if len(line) <= budget:
            break
        if k in cfg:
            cfg.pop(k)
            shed.append(k)
            cfg["shed"] = shed
            line = json.dumps(out, separators=(",", ":"))
    if len(line) > budget and isinstance(out.get("error"), dict):
        out["error"] = {k: out["error"][k] for k in ("phase", "bring_up", "type", "failed_steps") if k in out["error"]}
        line = json.dumps(out, separators=(",", ":"))
    return line


def error_summary(err: dict) -> dict:
    """A failed run's ``error`` object, <= ~1 KB: which bring-up, which
    validation step, which ranks, the floors it was held to; the ranks'
    steps, the messages in full and any traceback are in the detail file."""
    recs = err.get("records") or {}
    e = {k: err[k] for k in ("phase", "bring_up", "type", "elapsed_s") if k in err}
    e["message"] = str(err.get("message", ""))[:300]
    e["failed_steps"] = sorted(recs)
    wl = recs.get("workload")
    if wl:
        e["world"] = wl.get("world")
        e["failed_ranks"] = (wl.get("failed_ranks") or [])[:16]
        fl = wl.get("floors") or {}
        mins = {k: v for k, v in fl.items() if k.startswith("min_") and isinstance(v, (int, float))}
        if mins:
            e["floors"] = mins
        # the first failing step of the first failed rank, measured vs floor
        for r in wl.get("ranks") or []:
            bad = next((s for s in r.get("steps", []) if s.get("ok") is False), None)
            if bad:
                e["first_failed"] = {"rank": r.get("rank"), **{k: bad[k] for k in
                                     ("name", "tflops", "min_tflops", "gbps", "min_gbps", "busbw_gbps",
                                      "min_busbw_gbps", "peer_read_gbps", "min_peer_read_gbps", "counter_gate",
                                      "error") if k in bad}}
                if "error" in e["first_failed"]:
                    e["first_failed"]["error"] = str(e["first_failed"]["error"])[:160]
                break
        fp = wl.get("fabric_problems") or []
        if fp:
            e["fabric_problems"] = len(fp)
            e["fabric_problem_first"] = str(fp[0])[:160]
        cp = wl.get("coverage_problems") or []
        if cp:
            e["coverage_problems"] = len(cp)
    msgs = {step: str(rec.get("message", ""))[:120] for step, rec in recs.items() if step != "workload"}
    if msgs:
        e["step_messages"] = dict(list(msgs.items())[:3])
    return e


def failure_line(args, n_gpus: int, fake_gpu, err: dict, results: list, warm: list, elapsed: float,
                 detail: str | None = None) -> dict:
    """The JSON line of a run whose bring-up failed: ``value`` null, a compact
    ``error`` object (:func:`error_summary`) and the summaries of what the run
    measured before and after it; the records, the traceback and every step's
    critical path are in the detail file."""
    ttr = [r["time_to_ready_s"] for r in results]
    cps = [critical_path(r) for r in results]
    cfg = {
        "model": MODEL, "global_batch": n_gpus, "seq_len": 0, "parallelism": f"dp{n_gpus}",
        "detail": detail,
        "ttr_s": dist_summary(ttr),
        "time_to_ready_s": [round(x, 3) for x in ttr][:40],
        "warmup_time_to_ready_s": [round(r["time_to_ready_s"], 3) for r in warm][:10],
        "slow_steps": slow_summary(slow_steps(cps)),
        "collectives": collectives_summary(err.get("collectives")),
    }
    return {
        "metric": METRIC, "value": None, "unit": "s", "n_gpus": n_gpus, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / max(1, len(results)) * 1000, 2) if results else None,
        "higher_is_better": False, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
        "data": "synthetic" + (" (simulated GPUs: no GPU present)" if fake_gpu else ""),
        "error": error_summary(err),
        "config": {k: v for k, v in cfg.items() if v is not None},
    }


def success_line(args, n_gpus: int, fake_gpu, results: list, warm: list, compare: list, other: str,
                 elapsed: float, kfd_held: bool, detail: str | None) -> dict:
    """The headline JSON line (module docstring): value = mean time-to-Ready of
    the timed bring-ups; config = summaries only (LINE_BUDGET)."""
    from amdgpu_operator.nodeenv import NodeEnv

    ttr = [r["time_to_ready_s"] for r in results]
    mean_ttr = sum(ttr) / len(ttr)
    vis = [r["allocatable_visible_s"] for r in results]
    cps = [critical_path(r) for r in results]
    last = results[-1]
    holders = [r["kfd_holders"] for r in results if r.get("kfd_holders")]
    cfg = {
        "model": MODEL, "global_batch": n_gpus, "seq_len": 0, "parallelism": f"dp{n_gpus}",
        "allocatable_amd_com_gpu": last["allocatable"],
        "detail": detail,
        # the validator's Ready (`value`) over the timed bring-ups
        "ttr_s": dist_summary(ttr),
        "time_to_ready_s": [round(x, 3) for x in ttr] if len(ttr) <= 40 else None,
        # the other half of the metric: allocatable amd.com/gpu in Node.status
        # (README.md:122), on the kubelet's status tick
        "allocatable_visible_s": {"mean": round(sum(vis) / len(vis), 3),
                                  "p95": round(sorted(vis)[min(len(vis) - 1, int(0.95 * len(vis)))], 3)},
        "kubelet_node_status_s": args.kubelet_status_s,
        "validation_poll_s": NodeEnv.poll_s if args.agent_poll_s is None else args.agent_poll_s,
        "slow_steps": slow_summary(slow_steps(cps)),
        # processes of the bring-up's own tree holding /dev/kfd at each timed step's start and at its
        # Ready (max over steps; who they were: the detail file), and the host's KFD process count
        "kfd_holders": {"start_max": max(len(h.get("start") or []) for h in holders),
                        "ready_max": max(len(h.get("ready") or []) for h in holders),
                        "host_procs_max": max((r.get("settle") or {}).get("kfd_procs") or 0 for r in results)}
        if holders else None,
        "rates": rates_summary(last),
        "gate_retries": gate_retry_summary(results),
        "operand_mode": args.mode,
        # the harness itself never held a GPU context (no /dev/kfd descriptor)
        "harness_holds_kfd": kfd_held,
        # BASELINE config 5 after the last timed bring-up (not part of `value`)
        "pod_workload": pod_workload_summary(last.get("pod_workload")),
        # SURVEY §5.8 after the last timed bring-up (not part of `value`)
        "collectives": collectives_summary(last.get("collectives")),
        "other_mode_time_to_ready_s": {"mode": other, "s": [round(r["time_to_ready_s"], 3) for r in compare]}
        if compare else None,
    }
    return {
        "metric": METRIC,
        "value": round(mean_ttr, 4),
        "unit": "s",
        "n_gpus": n_gpus,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1000, 2),
        "higher_is_better": False,
        "scaling": "weak",
        "vs_baseline": round(mean_ttr / BASELINE_TTR_S, 6),
        "dtype": "bf16",
        "data": "synthetic" + (" (simulated GPUs: no GPU present)" if fake_gpu else ""),
        "config": {k: v for k, v in cfg.items() if v is not None},
    }


def route_logs(detail_path: str, rank: int) -> str | None:
    """The ``amdgpu`` loggers of this process (the simulated cluster's pod
    failures with their operands' tracebacks, ...) into
    ``<detail>.rank<r>.log``."""
    import logging

    path = f"{os.path.splitext(detail_path)[0]}.rank{rank}.log"
    try:
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        h = logging.FileHandler(path, mode="w")
    except OSError:
        return None
    h.setFormatter(logging.Formatter("%(asctime)s %(levelname)s %(name)s %(message)s"))
    root = logging.getLogger("amdgpu")
    root.handlers[:] = [h]
    root.setLevel(logging.INFO)
    root.propagate = False
    return path


class Progress:
    """A few stderr lines per run: one at each phase's end and at most one a
    minute within a phase (the caller's silence watchdog), so the JSON line
    stays inside the driver's tail."""

    def __init__(self, every_s: float = 60.0):
        self.every_s = every_s
        self.last = time.monotonic()

    def step(self, phase: str, i: int, n: int, force: bool = False) -> None:
        now = time.monotonic()
        if force or i == n or now - self.last >= self.every_s:
            self.last = now
            print(f"bench: {phase} {i}/{n}", file=sys.stderr, flush=True)


def main():
    args = parse()
    if args.linger:  # read by the validator operand processes (validate.py LINGER)
        os.environ["AMDGPU_VALIDATOR_LINGER"] = "1"
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and args.gpus != world:
        args.gpus = world
    # the operator's and the simulated cluster's log records go to a file next to
    # the detail file: on stderr they would push the JSON line out of the driver's tail
    detail_path = args.detail or default_detail_path(args.gpus)
    log_path = route_logs(detail_path, rank)
    os.environ.setdefault("TORCH_CPP_LOG_LEVEL", "ERROR")  # c10d's per-rank socket warnings
    has_gpu = gpu_available(args.sysfs_root or "/")
    fake_gpu = args.fake_gpu or args.fake_gpu_procs or not has_gpu
    if fake_gpu and args.fake_gpu_procs:
        fake_gpu = "procs"

    dist = None
    group = None
    if world > 1:  # the ranks' control channel only (gloo): no rank opens a GPU
        import torch.distributed as dist

        dist.init_process_group("gloo", rank=rank, world_size=world)
        group = dist.group.WORLD
    del local_rank  # GPU d's processes run on rank d % world (launcher), children of the harness

    from amdgpu_operator.parallel.launcher import DistributedLauncher

    launcher =DistributedLauncher(rank, world, group) if world > 1 else None
    n_gpus = args.gpus
    if not fake_gpu and rank == 0:
        from amdgpu_operator.discovery import topology

        present = len(topology.enumerate_gpus(args.sysfs_root or "/"))
        if present > n_gpus:
            os.environ["AMDGPU_VISIBLE_GPUS"] = ",".join(str(i) for i in range(n_gpus))
        elif present < n_gpus:
            raise RuntimeError(f"requested {n_gpus} GPUs, node exposes {present}")

    workdir = tempfile.mkdtemp(prefix="amdgpu-bench-")
    results: list[dict] = []
    warm: list = []
    errors: list[dict] = []
    tools = None
    if rank == 0 and not args.no_tool_watch:
        from amdgpu_operator.utils.procwatch import ToolWatch

        tools = ToolWatch(os.path.join(workdir, "gpu-tools.jsonl"))

    progress = Progress()

    def driver_thread(n_steps: int, out: list, mode: str):
        import faulthandler

        faulthandler.dump_traceback_later(args.timeout + 60, exit=False)  # stacks if a step wedges
        i = 0
        label = "timed" if out is results else "warm-up" if out is warm else "compare"
        try:
            for i in range(n_steps):
                pods = out is results and i == n_steps - 1 and not args.no_pod_workload
                out.append(one_bring_up(args, n_gpus, launcher, workdir, fake_gpu, mode, pods))
                # progress on stderr: a run that prints nothing for minutes looks hung to its
                # caller, and every line also takes room from the JSON line in the driver's tail
                progress.step(label, i + 1, n_steps)
        except Exception as e:  # noqa: BLE001
            import traceback

            err = {"phase": label, "bring_up": i + 1, "type": type(e).__name__, "message": str(e)[:2000],
                   "traceback": traceback.format_exc()[-6000:]}
            if isinstance(e, BringUpFailed):
                err.update(records=e.records, elapsed_s=round(e.elapsed_s, 4), harness=getattr(e, "partial", None))
            print(f"bench: {label} bring-up {i + 1} failed: {type(e).__name__}: {str(e)[:200]}", file=sys.stderr,
                  flush=True)
            if not args.no_sweep:
                # what the fabric does, measured, next to the failure (the floors it failed are in the records)
                try:
                    err["collectives"] = standalone_sweep(args, launcher, fake_gpu, workdir)
                except Exception as se:  # noqa: BLE001
                    err["collectives"] = {"ok": False, "error": f"{type(se).__name__}: {se}"[:1000]}
            errors.append(err)
        finally:
            faulthandler.cancel_dump_traceback_later()
            if launcher is not None:
                launcher.request_stop()

    def phase(n_steps: int, out: list, mode: str = args.mode) -> None:
        if world == 1:
            driver_thread(n_steps, out, mode)
            return
        if rank == 0:
            th = threading.Thread(target=driver_thread, args=(n_steps, out, mode), daemon=True)
            th.start()
            launcher._stop_requested.clear()
            th_started = th
            launcher.serve()
            th_started.join()
        else:
            launcher.serve()

    def sync():
        # every GPU process of a step is a child that the step has waited for:
        # the barrier is the whole synchronisation (see gpu_available)
        if world > 1:
            dist.barrier()

    # warmup (page-in, first HIP/RCCL init of the box)
    if args.warmup > 0:
        phase(args.warmup, warm)
        if world > 1:
            launcher = DistributedLauncher(rank, world, group)
    run_timed = [not errors]
    if world > 1:
        dist.broadcast_object_list(run_timed, src=0)  # a failed warm-up ends the run on every rank
    sync()
    t0 = time.perf_counter()
    if run_timed[0]:
        phase(args.steps, results)
    sync()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    kfd_held = holds_kfd()  # after the timed bring-ups, before the other-mode comparison
    # the other mode, untimed: in-process (lower bound) next to per-process
    other = "thread" if args.mode == "process" else "process"
    compare: list = []
    do_compare = [args.compare > 0 and not errors]
    if world > 1:
        dist.broadcast_object_list(do_compare, src=0)  # every rank takes part in the launcher's loop, or none
    if do_compare[0]:
        if world > 1:
            launcher = DistributedLauncher(rank, world, group)
        phase(args.compare, compare, other)
    if world > 1:
        box = [elapsed]
        all_el = [None] * world
        dist.all_gather_object(all_el, elapsed)
        elapsed = max(all_el)
        err_box = [errors]
        dist.broadcast_object_list(err_box, src=0)
        errors = err_box[0]
    if tools is not None:
        tools.stop()
        for r in results + warm:  # GPU tools of other parties alive during each timed bring-up
            r["foreign_gpu_tools"] = tools.overlapping(r["t0_wall"], r["t0_wall"] + r["time_to_ready_s"])
    rc = 1 if errors else 0  # every rank: the run failed
    if rank == 0:
        # everything per step / rank / size / link goes to the detail file, the
        # line names it; the line is the last thing this process prints
        cps = [critical_path(r) for r in results]
        if errors:
            out = failure_line(args, n_gpus, fake_gpu, errors[0], results, warm, elapsed, detail_path)
            detail = {"summary": out, "errors": errors, "critical_path": cps, "steps": results, "warmup": warm}
        else:
            out = success_line(args, n_gpus, fake_gpu, results, warm, compare, other, elapsed, kfd_held, detail_path)
            detail = {"summary": out, "critical_path": cps, "slow_steps": slow_steps(cps),
                      "collectives": results[-1].get("collectives"), "pod_workload": results[-1].get("pod_workload"),
                      "operands": results[-1].get("operands"),
                      "kfd_holders": [r.get("kfd_holders") for r in results],
                      "steps": results, "warmup": warm, "compare": compare}
        detail["log"] = log_path
        if write_detail(detail_path, detail) is None:
            out["config"]["detail"] = None
        sys.stderr.flush()
        print(fit_line(out), flush=True)
    shutil.rmtree(workdir, ignore_errors=True)
    if world > 1:
        dist.barrier()  # rank 0 has printed the line
        dist.destroy_process_group()
    if rc and rank == 0:
        # the other ranks exit 0 first: torchrun then reports one failed rank
        # (not eight, nor SIGTERMs to the rest) after the line
        if world > 1:
            time.sleep(1.0)
        raise SystemExit(rc)


def setup_failure_line(e: BaseException) -> dict:
    """The line of a run that failed before its first bring-up (the node has
    fewer GPUs than asked for, the ranks' rendezvous, an import): the same
    shape as :func:`failure_line`, phase ``setup``."""
    import traceback

    try:
        args = parse()
    except BaseException:  # noqa: BLE001 - the arguments themselves: the contract's defaults
        args = argparse.Namespace(steps=None, warmup=None, gpus=int(os.environ.get("WORLD_SIZE", "1")))
    n = int(os.environ.get("WORLD_SIZE", "0")) or args.gpus
    err = {"phase": "setup", "type": type(e).__name__, "message": str(e)[:2000],
           "traceback": traceback.format_exc()[-6000:]}
    return failure_line(args, n, False, err, [], [], 0.0, None)


if __name__ == "__main__":
    try:
        main()
    except (SystemExit, KeyboardInterrupt):
        raise
    except BaseException as exc:  # noqa: BLE001 - one parseable line, then the failure
        if int(os.environ.get("RANK", "0")) == 0:
            print(fit_line(setup_failure_line(exc)), flush=True)
        raise SystemExit(1) from exc
