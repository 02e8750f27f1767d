"""Operator-validator steps (init containers of ``amd-operator-validator``).

Reference parity: validator pods that end ``Completed`` (/root/reference/
README.md:199).  The steps and the host files they produce, in order:

==================  =====================================================  =================
step                what it checks                                         ready file
==================  =====================================================  =================
driver              N1 probe: amdgpu live, /dev/kfd, KFD GPU nodes, render  driver-ready
toolkit             toolkit installed (CDI spec + runtime config)           toolkit-ready
workload            one native ``amdgpu-validator`` process per GPU: HIP    workload-ready
                    vectorAdd, MFMA GEMM + counter gate, one exact MFMA tile
                    per CDNA4 data type, HBM, xGMI one-shot all-reduce,
                    RCCL all-reduce across ALL GPUs over xGMI
plugin              node Allocatable ``amd.com/gpu`` == GPUs found, then    plugin-ready
                    one pod per GPU requesting ``amd.com/gpu: 1`` (device
                    plugin Allocate -> OCI hook -> HIP workload) Succeeded
complete            node labelled ``amd.com/gpu.validated=true`` with the    validated
                    per-step durations (time-to-Ready breakdown)
==================  =====================================================  =================

Other operands gate on these files (their init containers run
``amdgpu-operator validate <step>`` in wait mode).
"""

from __future__ import annotations

import json
import os
import shutil
import threading
import time

from .. import RESOURCE_NAME, native
from ..kube.client import wait_for
from ..nodeenv import REPORT_EARLY_ENV, NodeEnv, report_rc
from ..utils.logs import get_logger

log = get_logger("amdgpu.validator")

READY_FILES = {
    "driver": "driver-ready",
    "toolkit": "toolkit-ready",
    "workload": "workload-ready",
    "plugin": "plugin-ready",
    "complete": "validated",
    "vfio": "vfio-ready",          # sandbox workloads: GPUs bound to vfio-pci
    "sandbox": "sandbox-validated",
}
VALIDATED_LABEL = "amd.com/gpu.validated"
MFMA_LABEL = "amd.com/gpu.validated.mfma"  # data types whose MFMA tile checked out on every GPU
# data types whose GEMM held its TF/s floor (and counter gate) on every GPU:
# bf16 (the gemm step), fp8 (gemm_fp8, e4m3), fp4 (gemm_fp4, e2m1), fp6
# (gemm_fp6, e2m3) and block-scaled mxfp4 (gemm_mxfp4, E8M0 scales) on the
# f8f6f4 MFMA, e.g. "bf16.fp8.fp4.fp6.mxfp4"
MFMA_RATE_LABEL = "amd.com/gpu.validated.mfma-rate"
WORKLOAD_POD_LABEL = "amd.com/validator-workload"
# take a validator process's result at its report, not at its exit (A/B: =0)
REPORT_EARLY = os.environ.get("AMDGPU_VALIDATOR_REPORT_EARLY", "1") == "1"


class StepFailed(RuntimeError):
    pass


def write_ready(env: NodeEnv, step: str, payload: dict) -> str:
    os.makedirs(env.validations_dir, exist_ok=True)
    path = env.validation_file(READY_FILES[step])
    tmp = f"{path}.tmp.{os.getpid()}.{threading.get_ident()}"
    with open(tmp, "w") as f:
        json.dump({"step": step, "node": env.node_name, "time": time.time(), **payload}, f)
    os.replace(tmp, path)
    return path


def read_ready(env: NodeEnv, step: str) -> dict | None:
    try:
        with open(env.validation_file(READY_FILES[step])) as f:
            txt = f.read()
    except OSError:
        return None
    try:
        return json.loads(txt)
    except ValueError:
        return {"raw": txt.strip()}


def clear_ready(env: NodeEnv, steps=READY_FILES) -> None:
    for s in steps:
        try:
            os.unlink(env.validation_file(READY_FILES[s]))
        except OSError:
            pass


def wait_ready(env: NodeEnv, step: str, timeout: float = 600.0, stop: threading.Event | None = None) -> dict:
    from ..utils import logs
    from ..utils.fswait import wait_for_file

    got = read_ready(env, step)
    if got is not None:
        return got
    # logging loads during the wait, not at the first log call after it (and
    # not when there is no wait: the import would hold the interpreter lock
    # beside what follows)
    logs.preload_async()
    path = env.validation_file(READY_FILES[step])
    if wait_for_file(path, timeout, stop, env.poll_s, check=lambda p: read_ready(env, step) is not None):
        return read_ready(env, step)
    if stop is not None and stop.is_set():
        raise StepFailed("stopped")
    raise StepFailed(f"timed out waiting for {READY_FILES[step]}")


# -------------------------------------------------------------------- steps --

def validate_driver(env: NodeEnv, timeout: float = 600.0, stop=None) -> dict:
    """N1 probe of the host, retried until ``timeout`` (driver still loading)."""
    from ..discovery import topology

    t0 = time.perf_counter()
    deadline = time.monotonic() + timeout
    for delay in env.waits():
        ok, msg = topology.probe(env.sysfs_root())
        if ok:
            gpus = topology.enumerate_gpus(env.sysfs_root())
            out = {"ok": True, "message": msg, "gpus": len(gpus), "seconds": time.perf_counter() - t0}
            prev = read_ready(env, "driver") or {}
            if "rdma" in prev:  # the driver container's driver.rdma record (driver/manager.py ensure_rdma)
                out["rdma"] = prev["rdma"]
            write_ready(env, "driver", out)
            return out
        if time.monotonic() >= deadline:
            raise StepFailed(f"driver not ready: {msg}")
        if stop is not None:
            if stop.wait(delay):
                raise StepFailed("stopped")
        else:
            time.sleep(delay)


def gate_env() -> dict:
    """Environment of a counter-gated validator process: the N7 tool library
    and its four-counter definitions.  Both must be in place before the
    process starts (the SDK loads with the HIP runtime and must see ONE
    counter set: a definition path changed after it loaded leaves the
    dispatch records unnamed and the gate fails closed)."""
    return {"AMDGPU_VALIDATOR_COUNTERS": "1",
            "ROCP_TOOL_LIBRARIES": str(native.artefact("libamdgpu_counter_gate.so")),
            "ROCPROFILER_METRICS_PATH": str(native.artefact("gate-metrics"))}


def thp_malloc_env() -> dict:
    """glibc's malloc on transparent huge pages (``glibc.malloc.hugetlb=1``,
    glibc >= 2.35; an older glibc ignores the tunable) for the processes that
    set up an RCCL communicator.  Most of ``ncclCommInitRank`` is the HIP
    runtime loading RCCL's ~108 MB of gfx950 device code through freshly
    allocated host buffers, and most of that was page faults (system time):
    0.35 s -> 0.22 s per communicator on MI355X, process wall 450 -> 320 ms
    (tools/rccl_thp_probe.sh, profiles/r3_thp).  The kernel-check and
    plugin-pod processes showed no change and keep the default."""
    cur = os.environ.get("GLIBC_TUNABLES", "")
    if "glibc.malloc.hugetlb" in cur:
        return {}
    return {"GLIBC_TUNABLES": f"{cur}:glibc.malloc.hugetlb=1" if cur else "glibc.malloc.hugetlb=1"}


def _arg_value(args: list[str], flag: str) -> str | None:
    return args[args.index(flag) + 1] if flag in args and args.index(flag) + 1 < len(args) else None


def workload_argv(args: list[str], rank: int, world: int, rendezvous: str, run_id: str, device: int) -> list[str]:
    return [str(native.binary("amdgpu-validator")), "--device", str(device), "--rank", str(rank), "--world",
            str(world), "--rendezvous", rendezvous, "--run-id", run_id, *args]


# Written into a run's rendezvous directory when any rank failed: every
# sibling still waiting on a peer (RCCL set-up, IPC handles, barriers, its
# start gate) stops within milliseconds (validator_main.cpp Rendezvous).
ABORT_FILE = "abort"


def abort_run(rdv: str, reason: str) -> None:
    path = os.path.join(rdv, ABORT_FILE)
    if os.path.exists(path):
        return
    tmp = f"{path}.tmp.{os.getpid()}.{threading.get_ident()}"
    try:
        with open(tmp, "w") as f:
            f.write(reason[:400])
        os.replace(tmp, path)
    except OSError:
        pass


# The xGMI link model the multi-GPU gates are derived from.  KFD reports every
# XGMI io_link's bandwidth per direction: 76,000 MB/s on MI355X (16 lanes x
# 38 Gb/s; amd-smi shows the same link as bit_rate 38 Gb/s, max_bandwidth
# 608 Gb/s - tests/fixtures/mi355x).  A rank's collective traffic leaves it
# over the links to its N-1 peers (one per peer in a full mesh), so the sum
# of those links' bandwidth bounds what one rank can move per direction.
#
#   K4 one-shot (every rank reads all N-1 peer buffers at once, one per link):
#     floor = xgmiReadLinkFraction x sum(link GB/s)
#   RCCL fp32 all-reduce busBW at B bytes (bus bandwidth per rank, striped
#   over the links; the per-launch start-up gives the alpha-beta shape
#   busBW(B) = peak x B / (B + B_half), B_half = RCCL_HALF_BW_BYTES):
#     floor = rcclBusbwLinkFraction x sum(link GB/s) x B / (B + B_half)
#
# A mesh whose links are all "up" but trained to half their rate halves both
# measured rates: the link-rate check in check_fabric (amd-smi rate x width
# against KFD's nominal) names it outright, and the throughput floors catch
# what the status does not show.  Both fractions sit below the efficiency a
# healthy mesh delivers so that run-to-run noise never fails a good node;
# they are model-derived, not yet calibrated on an 8-GPU MI355X run (the
# builder's box has one GPU) - the driver's scaling run records the measured
# rates next to the floors (bench.py config.rccl_busbw_gbps / xgmi).
RCCL_HALF_BW_BYTES = 16 << 20  # ~30 us of launch + sync at ~500 GB/s


def _xgmi_link_gbps(env: NodeEnv, gpus: list) -> dict[tuple[int, int], float]:
    """GB/s per direction of the KFD XGMI link between GPU indices (a, b)."""
    from ..discovery import topology

    idx = {g.index for g in gpus}
    out = {}
    for lk in topology.links(env.sysfs_root()):
        if lk.is_xgmi and lk.src in idx and lk.dst in idx:
            out[(lk.src, lk.dst)] = lk.max_bandwidth_mbps / 1000.0
    return out


# The per-peer rate the floors assume where KFD reports no XGMI link
# bandwidth between two GPUs of a multi-GPU node (PCIe-routed peers, or a
# driver that reports max_bandwidth 0): the MI355X xGMI nominal.  Without it
# such a node summed to 0 and its floors to "no floor"; with it the node is
# held to the xGMI rate it should have and a PCIe-routed node fails, as the
# ClusterPolicy's derivation says (api/clusterpolicy.py WorkloadSpec).
NOMINAL_XGMI_LINK_GBPS = 76.0


def rccl_busbw_floor(link_sum_gbps: float, fraction: float, nbytes: int) -> float:
    """The all-reduce busBW floor at ``nbytes`` (the alpha-beta shape above)."""
    if nbytes <= 0:
        return 0.0
    return fraction * link_sum_gbps * nbytes / (nbytes + RCCL_HALF_BW_BYTES)


def fabric_floors(env: NodeEnv, plan: list[list], gpus: list, rccl_fraction: float, xgmi_fraction: float,
                  rccl_bytes: int) -> dict:
    """Throughput floors of the multi-GPU steps, from the KFD link model above:
    per rank the sum of the links from its first device to every peer GPU's
    first device; the floors use the smallest such sum of the node.  A peer
    pair with no KFD XGMI bandwidth counts at :data:`NOMINAL_XGMI_LINK_GBPS`
    (``nominal_pairs`` says how many), so such a node is never left without a
    floor."""
    links = _xgmi_link_gbps(env, gpus)
    sums, nominal = [], 0
    for r, devs in enumerate(plan):
        me = devs[0].index
        total = 0.0
        for q, p in enumerate(plan):
            if q == r:
                continue
            bw = links.get((me, p[0].index)) or links.get((p[0].index, me)) or 0.0
            if bw <= 0:
                bw = NOMINAL_XGMI_LINK_GBPS
                nominal += 1
            total += bw
        sums.append(total)
    link_sum = min(sums) if sums else 0.0
    out = {"link_gbps_per_rank": [round(x, 1) for x in sums],
           "min_rccl_busbw_gbps": round(rccl_busbw_floor(link_sum, rccl_fraction, rccl_bytes), 1),
           "min_xgmi_peer_read_gbps": round(xgmi_fraction * link_sum, 1)}
    if nominal:
        out["nominal_pairs"] = nominal  # peer pairs without KFD XGMI bandwidth, held to the xGMI nominal
    return out


def check_fabric(env: NodeEnv, gpus: list, smi_metrics: list | None = None, min_link_fraction: float = 0.9) -> dict:
    """The xGMI fabric between the validated GPUs is whole and at speed.

    Every pair of distinct physical GPUs must share one xGMI hive and be
    joined by an XGMI link in the KFD topology (``io_links``); where amd-smi
    answers, each GPU must report at least one link up per physical peer, no
    link in error, and its links trained to at least ``min_link_fraction`` of
    the KFD nominal rate (amd-smi rate x width, e.g. 38 Gb/s x 16 = 76 GB/s,
    against io_link max_bandwidth; a link that retrained to a lower rate or
    width is "up" and slow).  Partitions of one physical GPU are not peers of
    each other.  A dead or slow link leaves RCCL routing around it at a
    fraction of the bandwidth; this check names the GPU."""
    from ..discovery import topology

    phys: dict[str, object] = {}
    for g in gpus:
        phys.setdefault(g.bdf, g)
    out: dict = {"ok": True, "physical_gpus": len(phys), "problems": []}
    if len(phys) < 2:
        out["skipped"] = "one physical GPU: no xGMI peer"
        return out
    problems = out["problems"]
    hives = {g.hive_id for g in phys.values()}
    if 0 in hives or len(hives) != 1:
        problems.append(f"GPUs are not in one xGMI hive (hive ids {sorted(hives)})")
    idx = {g.index: g.bdf for g in gpus}
    linked: set[tuple[str, str]] = set()
    nominal: dict[str, float] = {}  # bdf -> slowest nominal KFD XGMI link (GB/s per direction)
    for lk in topology.links(env.sysfs_root()):
        if lk.is_xgmi and lk.src in idx and lk.dst in idx and idx[lk.src] != idx[lk.dst]:
            linked.add(tuple(sorted((idx[lk.src], idx[lk.dst]))))
            if lk.max_bandwidth_mbps:
                b = idx[lk.src]
                nominal[b] = min(nominal.get(b, float("inf")), lk.max_bandwidth_mbps / 1000.0)
    bdfs = sorted(phys)
    missing = [(a, b) for i, a in enumerate(bdfs) for b in bdfs[i + 1:] if (a, b) not in linked]
    if missing:
        problems.append(f"no XGMI link between {missing[:8]}" + (f" (+{len(missing) - 8})" if len(missing) > 8 else ""))
    out["kfd_xgmi_pairs"] = len(linked)
    if smi_metrics is None:
        try:
            with topology.Smi() as smi:
                smi_metrics = smi.collect()
        except Exception as e:  # noqa: BLE001 - amd-smi absent (sim, minimal image): KFD view only
            out["smi"] = f"unavailable: {e}"
            smi_metrics = []
    peers = len(phys) - 1
    live = {}
    lower = {b.lower(): b for b in phys}
    for m in smi_metrics:
        if m.bdf.lower() not in lower or "xgmi_links_up" not in m.values:
            continue
        bdf = lower[m.bdf.lower()]
        up, err = m.values.get("xgmi_links_up", 0), m.values.get("xgmi_links_error", 0)
        rec = {"up": up, "total": m.values.get("xgmi_links_total", 0), "error": err}
        speed, width = m.values.get("xgmi_link_speed_gbps", 0), m.values.get("xgmi_link_width", 0)
        if speed and width:
            rec["link_gbps"] = speed * width / 8.0
            want = nominal.get(bdf)
            if want and rec["link_gbps"] < min_link_fraction * want:
                problems.append(f"{m.bdf}: xGMI links at {rec['link_gbps']:g} GB/s ({speed} Gb/s x{width}), "
                                f"nominal {want:g} GB/s")
        live[m.bdf] = rec
        if up < peers:
            problems.append(f"{m.bdf}: {up} xGMI links up, {peers} physical peers")
        if err:
            problems.append(f"{m.bdf}: {err} xGMI links in error")
    if live:
        out["links"] = live
    out["ok"] = not problems
    return out


def rank_plan(gpus: list) -> list[list]:
    """The workload's ranks: one per physical GPU, in enumeration order, each
    with the schedulable devices it validates - the GPU itself in SPX, its
    compute partitions in DPX/QPX/CPX (they share the GPU's PCI address)."""
    groups: dict[str, list] = {}
    for g in gpus:
        groups.setdefault(g.bdf, []).append(g)
    return list(groups.values())


# Concurrent GPU processes one node's validation may start: the workload
# processes plus the plugin-validation pods running beside them.  A GPU box
# caps the processes holding its devices (16 on the MI355X pool this was
# measured on, tools/storm_probe.py), and the HIP runtime start-up that a
# crowd of processes stretches is the longest term of the bring-up
# (BASELINE.md "the N = 8 start-up storm").
DEFAULT_MAX_GPU_PROCESSES = 16


def workload_processes(world: int, run_rccl: bool, separate: bool, budget: int) -> tuple[int, bool]:
    """(processes, separate) for ``world`` ranks: one process per physical GPU
    (kernel checks, xGMI and RCCL together), or, when ``separate`` is asked
    for and fits ``budget``, a second RCCL process per GPU."""
    if run_rccl and separate and 2 * world <= budget:
        return 2 * world, True
    return world, False


def planned_workload_processes(env: NodeEnv, args: list[str], budget: int) -> int:
    """How many processes :func:`validate_workload` would start on this node."""
    from ..discovery import topology

    world = len(rank_plan(topology.enumerate_gpus(env.sysfs_root())))
    run_rccl = "rccl" in _steps_of(args) and (world > 1 or "--rccl-single-gpu" in args)
    return workload_processes(world, run_rccl, "--rccl-separate-process" in args, budget)[0]


# AMDGPU_VALIDATOR_LINGER=1: the workload validator processes stay until the
# plugin validation is done (``--linger-until`` its ready file, at most
# LINGER_MAX_S), so their teardown cannot overlap the plugin pod's HSA
# set-up (validator_main.cpp, end of main).  Off by default: interleaved A/B
# on the MI355X found no gain, before (profiles/r5_ttr/linger) and after the
# HBM step kept its buffers to the process's end (profiles/r5_init/wipe).
LINGER = os.environ.get("AMDGPU_VALIDATOR_LINGER", "0") == "1"
LINGER_MAX_S = 3.0


def validate_workload(env: NodeEnv, args: list[str] | None = None, timeout: float = 600.0,
                      start_gate: str | None = None, budget: int | None = None,
                      linger_until: str | None = None) -> dict:
    """One native validator process per physical GPU, all in one RCCL
    communicator.

    Each process validates every schedulable device of its GPU - the whole
    GPU in SPX, each compute partition otherwise, concurrently on threads
    (``amdgpu-validator --local-bdf``) - then runs the xGMI one-shot and the
    RCCL collectives on its first device, across the physical GPUs.  An 8-GPU
    node therefore starts 8 processes whatever its partitioning; one process
    per partition made an 8 x CPX node start 128 and a 64-rank communicator.
    At N >= 2 each process sees its own devices plus the first device of every
    peer GPU (``ROCR_VISIBLE_DEVICES``): RCCL's and the IPC step's peer access
    needs the peers visible, the runtime need not set up the rest.

    ``start_gate``: a file the processes wait on before their first HIP call
    (``amdgpu-validator --start-gate``): "init" lets the runtime start (the
    driver container has the module loaded), "go" releases the kernel steps,
    anything else aborts them.  The caller spawns them before the driver is validated and
    writes the verdict afterwards (:func:`validate_gpu`).

    Bounded failure at N >= 2: every rank keeps a liveness record in the
    run's rendezvous directory and watches its peers' while it waits on them
    (RCCL's non-blocking set-up included), so a rank that never started, died
    or failed ends the run within milliseconds of being seen - or after
    ``--peer-timeout`` for one that never appears - with the rank named in the
    error.  As soon as any process reports a failure this function writes the
    run's abort file, so siblings that are not waiting on that rank stop too
    instead of running out their own timeouts.

    validate.py's own flags (not passed to the binary): ``--rccl-single-gpu``,
    ``--rccl-separate-process`` (RCCL in a second process per GPU, when that
    fits ``budget``; ``--rccl-shared-process`` is the default and accepted),
    ``--rccl-busbw-link-fraction F`` and ``--xgmi-read-link-fraction F``
    (the throughput floors of :func:`fabric_floors`, passed to the binary as
    ``--min-rccl-busbw-gbps`` / ``--min-xgmi-read-gbps``),
    ``--max-gpu-processes N`` (the budget), ``--require-xgmi-links`` and
    ``--min-xgmi-link-fraction F`` (:func:`check_fabric` on multi-GPU nodes),
    ``--dmabuf`` (driver.rdma: every device exports HBM as a dma-buf and
    imports it back, the step an RDMA NIC's access rests on)."""
    from ..discovery import topology

    t0 = time.perf_counter()
    gpus = topology.enumerate_gpus(env.sysfs_root())
    if not gpus:
        raise StepFailed("no GPUs to validate")
    plan = rank_plan(gpus)
    world = len(plan)
    args = list(args or [])
    if budget is None:
        budget = int(_arg_value(args, "--max-gpu-processes") or DEFAULT_MAX_GPU_PROCESSES)
    if world > 8:  # the xGMI one-shot kernel takes <= 8 peers; RCCL still spans all
        args = _drop_step(args, "xgmi")
    run_id = os.urandom(6).hex()
    rdv = os.path.join(env.validations_dir, "rendezvous", run_id)
    os.makedirs(rdv, exist_ok=True)
    # N7: the counter gate is a rocprofiler-sdk tool library loaded only into
    # the gated kernel processes (the binary does not link the SDK)
    # (the default AQL-packet gate needs no tool library: only --gate-mode sdk)
    sdk_gate = "--counter-gate" in args and _arg_value(args, "--gate-mode") == "sdk"
    if "--no-gate-lock" in args:
        env.extra["no_gate_lock"] = True
    counter_env = {**(gate_env() if sdk_gate else {}), **gate_lock_env(env)}
    rccl_single = "--rccl-single-gpu" in args  # validate.py's own flags, not the binary's
    separate = "--rccl-separate-process" in args
    require_links = "--require-xgmi-links" in args
    dmabuf = "--dmabuf" in args  # driver.rdma: HBM exported as a dma-buf on every device
    if "--no-mfma-rate" in args:  # validator.workload.mfmaRateCheck off
        for st in ("gemm_fp8", "gemm_fp4", "gemm_fp6", "gemm_mxfp4"):
            args = _drop_step(args, st)
    rccl_frac = float(_arg_value(args, "--rccl-busbw-link-fraction") or 0.0)
    xgmi_frac = float(_arg_value(args, "--xgmi-read-link-fraction") or 0.0)
    link_frac = float(_arg_value(args, "--min-xgmi-link-fraction") or 0.9)
    args = _drop_flag(args, "--rccl-single-gpu", "--rccl-shared-process", "--rccl-separate-process",
                      "--require-xgmi-links", "--dmabuf", "--no-mfma-rate", "--no-gate-lock")
    args = _drop_value(args, "--rccl-busbw-link-fraction", "--xgmi-read-link-fraction", "--min-xgmi-link-fraction",
                       "--max-gpu-processes")
    steps = _steps_of(args)
    # A single-GPU node has no collective to validate (no xGMI peer) unless
    # rcclSingleGpu asks for the rehearsal.
    run_rccl = "rccl" in steps and (world > 1 or rccl_single)
    floors = None
    if world > 1 and (rccl_frac > 0 or xgmi_frac > 0):
        rccl_bytes = 4 * int(_arg_value(args, "--rccl-elems") or (1 << 24))
        floors = fabric_floors(env, plan, gpus, rccl_frac, xgmi_frac, rccl_bytes)
        if rccl_frac > 0:
            args += ["--min-rccl-busbw-gbps", f"{floors['min_rccl_busbw_gbps']:g}"]
        if xgmi_frac > 0:
            args += ["--min-xgmi-read-gbps", f"{floors['min_xgmi_peer_read_gbps']:g}"]
    kernel_steps = [s for s in steps if s not in ("xgmi", "rccl")] + ["dmabuf"] * (dmabuf and "dmabuf" not in steps)
    xgmi = "xgmi" in steps  # real peers at N >= 2, emulated peers on one device otherwise
    nproc, separate = workload_processes(world, run_rccl, separate, budget)
    jobs = []  # (rank, binary flags, run id, env)
    for r, devs in enumerate(plan):
        others = [plan[q][0] for q in range(world) if q != r]
        local = ["--local-bdf", devs[0].bdf]
        if separate:  # kernel checks of the GPU's devices; xGMI + RCCL in a process of their own
            jobs.append((r, _with_steps(args, kernel_steps) + local + ["--expect-devices", str(len(devs))], run_id,
                         {**counter_env, **topology.visible_devices_env(devs, gpus)}))
            jobs.append((r, _with_steps(_drop_flag(args, "--counter-gate"), ["hip"] + ["xgmi"] * xgmi + ["rccl"])
                         + local + ["--expect-devices", "1"], run_id + "-rccl",
                         {**thp_malloc_env(), **gate_lock_env(env),
                          **topology.visible_devices_env([devs[0], *others], gpus)}))
            continue
        jenv = dict(counter_env)
        if run_rccl:
            jenv.update(thp_malloc_env())
        if world > 1:
            jenv.update(topology.visible_devices_env([*devs, *others], gpus))
        jobs.append((r, _with_steps(args, kernel_steps + ["xgmi"] * xgmi + ["rccl"] * run_rccl) + local
                     + ["--expect-devices", str(len(devs))], run_id, jenv))

    def failed(res) -> bool:
        return res.rc != 0 or report_rc(res.stdout) != 0

    def one(job):
        rank, jargs, rid, jenv = job
        # the report (pipes closed) is the result: the process exit and the
        # kernel's teardown of its GPU state do not hold up the node
        if REPORT_EARLY:
            jenv = {**jenv, REPORT_EARLY_ENV: "1"}
        argv = workload_argv(jargs, rank, world, rdv, rid, 0)
        _startup_mark(f"spawn{rank}")
        if start_gate:
            argv += ["--start-gate", start_gate]
        if linger_until and LINGER:
            argv += ["--linger-until", linger_until, "--linger-max-s", f"{LINGER_MAX_S:g}"]
        # the launcher runs the process on the rank that owns physical GPU `rank`
        res = env.launch(argv, jenv, device=rank, timeout=timeout)
        if world > 1 and failed(res):
            abort_run(rdv, f"{rid} rank {rank} failed (rc {res.rc})")
        return res

    fabric = None
    try:
        if len(jobs) == 1 and not (require_links and world > 1):
            results = [one(jobs[0])]  # one GPU: no pool (its import is on the spawn's path)
        else:
            from concurrent.futures import ThreadPoolExecutor

            with ThreadPoolExecutor(max_workers=len(jobs) + 1) as ex:
                fabric_f = (ex.submit(check_fabric, env, gpus, None, link_frac) if require_links and world > 1
                            else None)
                results = list(ex.map(one, jobs))
                fabric = fabric_f.result() if fabric_f is not None else None
    finally:
        shutil.rmtree(rdv, ignore_errors=True)
    reports = []
    for (rank, _, rid, _), res in zip(jobs, results):
        try:
            rep = json.loads(res.stdout.strip().splitlines()[-1]) if res.stdout.strip() else {}
        except ValueError:
            rep = {"raw": res.stdout[-2000:]}
        rep["rc"] = res.rc
        rep["process_seconds"] = round(res.seconds, 4)
        if res.rc != 0:
            rep["stderr"] = res.stderr[-2000:]
        if rid.endswith("-rccl"):
            main = reports[rank]
            # the peer process's checks (xgmi, rccl); its own hip step is not one
            main["steps"] = main.get("steps", []) + [s for s in rep.get("steps", []) if s.get("name") != "hip"]
            main["ok"] = bool(main.get("ok")) and bool(rep.get("ok"))
            main["rc"] = main.get("rc", 0) or rep["rc"]
            main["rccl_process_seconds"] = rep["process_seconds"]
            if rep.get("error"):
                main["error"] = rep["error"]
            for k in ("failed_peer", "peer_state"):
                if k in rep:
                    main[k] = rep[k]
            if res.rc != 0:
                main["stderr"] = rep.get("stderr", "")
        else:
            reports.append(rep)
    if run_rccl and not separate:
        for rep in reports:
            rep["rccl_process_seconds"] = rep.get("process_seconds")
    if "rccl" in steps and not run_rccl:
        for rep in reports:
            rep.setdefault("steps", []).append({"name": "rccl", "ok": True, "skipped": "single GPU: no xGMI peer"})
    problems = device_coverage(plan, reports)
    ok = all(r.get("rc") == 0 and r.get("ok") for r in reports) and not problems
    summary = {"ok": ok, "world": world, "devices": len(gpus), "processes": len(jobs),
               "process_mode": "separate" if separate else "shared", "seconds": time.perf_counter() - t0,
               "ranks": reports}
    if problems:
        summary["coverage_problems"] = problems
    if floors is not None:
        summary["floors"] = floors
    if fabric is not None:
        summary["fabric"] = fabric
        if not fabric["ok"]:
            ok = summary["ok"] = False
    if not ok:
        msg = f"workload validation failed: {failure_summary(reports, fabric, problems)}"
        write_failure(env, "workload", failure_record(summary, msg))
        raise StepFailed(msg)
    clear_failure(env, "workload")
    write_ready(env, "workload", summary)
    return summary


# A failed step leaves ``<step>-failed`` next to the ready files: what failed
# and every rate the run measured against the floor it was held to, so a node
# that will not validate can be diagnosed from the host (must-gather collects
# the directory) and a harness can stop at the first failure instead of
# waiting out its timeout (bench.py).  The next pass of the step clears it.
FAILED_SUFFIX = "-failed"
_RATE_KEYS = ("tflops", "min_tflops", "gbps", "min_gbps", "busbw_gbps", "min_busbw_gbps", "algbw_gbps", "bytes",
              "peer_read_gbps", "min_peer_read_gbps", "perf_ok", "counter_gate", "mismatches", "max_abs_err",
              "freivalds_rel_err", "comm_init_s", "world", "device", "error", "failed", "gate_reason",
              "gate_retried_after", "gate_attempts", "mfma_util", "mfma_util_floor", "n")


def write_failure(env: NodeEnv, step: str, payload: dict) -> str:
    os.makedirs(env.validations_dir, exist_ok=True)
    path = env.validation_file(step + FAILED_SUFFIX)
    tmp = f"{path}.tmp.{os.getpid()}.{threading.get_ident()}"
    with open(tmp, "w") as f:
        json.dump({"step": step, "node": env.node_name, "time": time.time(), **payload}, f)
    os.replace(tmp, path)
    return path


def read_failure(env: NodeEnv, step: str) -> dict | None:
    try:
        with open(env.validation_file(step + FAILED_SUFFIX)) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def clear_failure(env: NodeEnv, step: str) -> None:
    try:
        os.unlink(env.validation_file(step + FAILED_SUFFIX))
    except OSError:
        pass


def failure_record(summary: dict, message: str) -> dict:
    """The compact record of a failed workload run: per rank its error (or the
    peer it found gone), and per step the measured rates next to the floors
    (``min_*``), the fabric check's problems and the floors the node was held
    to (:func:`fabric_floors`)."""
    ranks = []
    for i, r in enumerate(summary.get("ranks", [])):
        steps = [{"name": s.get("name"), "ok": s.get("ok"), **{k: s[k] for k in _RATE_KEYS if k in s}}
                 for s in r.get("steps", [])]
        ranks.append({"rank": i, "ok": bool(r.get("ok")) and r.get("rc") == 0, "rc": r.get("rc"),
                      **{k: r[k] for k in ("error", "failed_peer", "peer_state") if r.get(k) is not None},
                      "steps": steps})
    fabric = summary.get("fabric")
    return {"message": message[:2000], "world": summary.get("world"), "floors": summary.get("floors"),
            "fabric_problems": (fabric or {}).get("problems", []) if fabric else [],
            "coverage_problems": summary.get("coverage_problems", []), "ranks": ranks,
            "failed_ranks": [r["rank"] for r in ranks if not r["ok"]]}


def device_coverage(plan: list[list], reports: list[dict]) -> list[str]:
    """Every device of every rank reported its kernel steps: a partition
    the process did not see (wrong visibility, a partition switch under way)
    fails the run instead of passing on the devices that were there."""
    problems = []
    for r, (devs, rep) in enumerate(zip(plan, reports)):
        if not rep.get("ok"):
            continue
        seen = rep.get("local_devices")
        if seen is not None and len(seen) != len(devs):
            problems.append(f"rank {r}: {len(seen)} of {len(devs)} devices validated")
    return problems


def failure_summary(reports: list[dict], fabric: dict | None = None, problems: list[str] | None = None) -> str:
    """The causes of a failed run first: a rank's own failure, or a peer it
    found missing/dead; ranks that only stopped because of another's failure
    (peer state ``failed`` / ``aborted``) come last, as consequences."""
    causes, consequences = [], []
    for i, r in enumerate(reports):
        if r.get("ok") and r.get("rc") == 0:
            continue
        msg = r.get("error") or (r.get("stderr") or "")[-300:] or f"rc {r.get('rc')}"
        bad_steps = [s.get("name") for s in r.get("steps", []) if s.get("ok") is False]
        item = f"rank {i}: {msg}" + (f" (steps {bad_steps})" if bad_steps else "")
        (consequences if r.get("peer_state") in ("failed", "aborted") else causes).append(item)
    parts = list(problems or [])
    if fabric is not None and not fabric.get("ok"):
        parts.append("xGMI fabric: " + "; ".join(fabric.get("problems", [])))
    parts += causes
    if consequences:
        parts.append("then " + "; ".join(consequences))
    return "; ".join(parts) or "no report"


ALL_STEPS = ("hip", "vecadd", "gemm", "gemm_fp8", "gemm_fp4", "gemm_fp6", "gemm_mxfp4", "mfma", "hbm", "xgmi", "rccl")  # + "dmabuf" with driver.rdma


def _steps_of(args: list[str]) -> list[str]:
    if "--steps" in args:
        return [s for s in args[args.index("--steps") + 1].split(",") if s]
    return list(ALL_STEPS)


def _with_steps(args: list[str], steps: list[str]) -> list[str]:
    out = list(args)
    if "--steps" in out:
        i = out.index("--steps")
        del out[i:i + 2]
    return out + ["--steps", ",".join(steps if "hip" in steps else ["hip", *steps])]


def _drop_flag(args: list[str], *flags: str) -> list[str]:
    return [a for a in args if a not in flags]


def _drop_value(args: list[str], *flags: str) -> list[str]:
    """Remove ``flag VALUE`` pairs."""
    out, i = [], 0
    while i < len(args):
        if args[i] in flags:
            i += 2
            continue
        out.append(args[i])
        i += 1
    return out


def _drop_step(args: list[str], step: str) -> list[str]:
    out = list(args)
    if "--steps" in out:
        i = out.index("--steps")
        out[i + 1] = ",".join(s for s in out[i + 1].split(",") if s != step)
    else:
        out += ["--steps", ",".join(s for s in ALL_STEPS if s != step)]
    return out


def _node(env: NodeEnv) -> dict:
    return env.client.get("v1", "Node", env.node_name)


def allocatable(node: dict, resource: str) -> int:
    try:
        return int(((node.get("status") or {}).get("allocatable") or {}).get(resource, "0"))
    except ValueError:
        return 0


# The plugin-validation pod proves its allocated GPU runs a kernel from inside
# a container; its few small copies go through blit kernels instead of the
# SDMA engines, whose first use costs a fresh process ~8 ms of queue set-up
# (tools/plugin_pod_probe.sh, profiles/r2_ttr/plugin_pod_probe.txt).  The
# node's workload validation keeps SDMA on, so the copy engines are exercised.
PLUGIN_POD_ENV = [{"name": "HSA_ENABLE_SDMA", "value": "0"}]


def expected_devices(env: NodeEnv, resource: str = RESOURCE_NAME, partition_strategy: str = "single") -> dict:
    """Devices the device plugin advertises on this node, per resource name:
    every GPU (or partition) under ``resource``, except that under the
    ``mixed`` strategy partitioned GPUs are ``<resource>-<mode>``
    (discovery/topology.py partition_resource, which the plugin uses too)."""
    from ..discovery import topology

    out: dict[str, int] = {}
    for dev in topology.enumerate_gpus(env.sysfs_root()):
        r = topology.partition_resource(dev, resource, partition_strategy)
        out[r] = out.get(r, 0) + 1
    return out


def _device_plan(expected: dict, held: dict[str, list[str]]) -> dict | None:
    """Pods to run per resource, from the kubelet's devices, or None while
    the plugin's devices are not all there.

    The ``expected`` resources, once each holds its count of distinct GPUs
    (time-sliced replicas ``<id>::<n>`` count once).  A device-plugin config
    file can rename them (time-slicing ``rename`` / ``renameByDefault``,
    deviceplugin/config.py), which the validator's flags do not know: then
    every resource of the vendor domain (``amd.com/``) counts, one pod per
    distinct GPU it holds."""
    from ..deviceplugin.api import REPLICA_SEP

    def gpus(ids):
        return len({i.split(REPLICA_SEP, 1)[0] for i in ids})

    if all(gpus(held.get(r, ())) >= n for r, n in expected.items()):
        return dict(expected)
    domain = next(iter(expected)).split("/", 1)[0] + "/"
    plan = {r: gpus(ids) for r, ids in held.items() if r.startswith(domain) and ids}
    return plan if sum(plan.values()) >= sum(expected.values()) else None


def _wait_kubelet_devices(env: NodeEnv, expected: dict, deadline: float, stop, kd=None,
                          shared: set | None = None, log_queries: list | None = None) -> dict | None:
    """Wait until the kubelet's device manager holds the ``expected`` devices
    (pod-resources ``GetAllocatableResources``, deviceplugin/podresources.py;
    :func:`_device_plan`).  Returns the pods to run per resource, or None when
    that API is not reachable (the caller falls back to ``Node.status``)."""
    from ..deviceplugin.podresources import KubeletDevices

    from ..utils.fswait import DirWatch

    kd = kd or KubeletDevices(env.pod_resources_socket)
    if not kd.available():
        return None
    # the kubelet checkpoints every device-list update into the device-plugins
    # directory (and the plugin's socket appears there first): an inotify event
    # there triggers a look at once, so registration is seen within ~1 ms
    # instead of at the next backed-off poll
    w = DirWatch(env.device_plugin_dir) if os.path.isdir(env.device_plugin_dir) else None
    try:
        waits = env.waits()
        while True:
            tq = time.time()
            held = kd.allocatable()
            if log_queries is not None and len(log_queries) < 40:  # (wall start, seconds, devices held)
                log_queries.append((round(tq, 4), round(time.time() - tq, 4),
                                    sum(len(v) for v in (held or {}).values())))
            if held is None:
                return None
            plan = _device_plan(expected, held)
            if plan is not None:
                if shared is not None:  # time-sliced resources: replicas <id>::<k>
                    from ..deviceplugin.api import REPLICA_SEP

                    shared.update(r for r, ids in held.items() if any(REPLICA_SEP in i for i in ids))
                return plan
            if time.monotonic() >= deadline:
                raise StepFailed(f"kubelet holds {({r: len(v) for r, v in held.items()})} devices, "
                                 f"expected {expected}")
            if stop is not None and stop.is_set():
                raise StepFailed("stopped")
            delay = next(waits)
            if w is not None and w.active:
                w.wait(delay)  # an event (checkpoint written, socket created) means: look now
            elif stop is not None:
                stop.wait(delay)
            else:
                time.sleep(delay)
    finally:
        kd.close()
        if w is not None:
            w.close()


def _startup_mark(what: str) -> None:
    """AMDGPU_STARTUP_TRACE (the simulated kubelet's operand processes): the
    wall time of a point on the validator's path, next to cli/main.py's
    start-up phases (bench.py operand_breakdown)."""
    trace = os.environ.get("AMDGPU_STARTUP_TRACE")
    if trace:
        with open(trace, "a") as f:
            f.write(f"{what} {time.time():.4f}\n")


POD_RESULTS = "pod-results"  # validations_dir/<this>: the plugin pods' reports (hostPath in the pods)


def _pod_results_dir(env: NodeEnv) -> str:
    d = os.path.join(env.validations_dir, POD_RESULTS)
    os.makedirs(d, exist_ok=True)
    return d


# The counter gate's per-GPU lock files (native/include/gate_lock.h): the
# validator holds a GPU's lock exclusively around each counted dispatch, and
# the operator's other GPU work on it - the plugin-validation pod's check, the
# validator's RCCL processes - holds it shared, so none of it lands in a
# counted window.  They live in the pod-results hostPath, which the
# plugin-validation pods already mount.
GATE_LOCK_ENV = "AMDGPU_GATE_LOCK_DIR"


def gate_lock_env(env: NodeEnv) -> dict:
    """The lock directory for the node's GPU processes (none with
    ``validator.workload.gateLock`` off: ``--no-gate-lock``)."""
    if env.extra.get("no_gate_lock"):
        return {}
    return {GATE_LOCK_ENV: _pod_results_dir(env)}


def _with_result_file(env: NodeEnv, pod: dict, flag: str) -> dict:
    """The pod writes its report into the node's validation directory too
    (``flag``: the check's option for it, published by rename): the
    validator has the result as soon as the check is done, while the kernel
    is still releasing the pod process's GPU state (~50 ms, BASELINE.md
    pod_exit_probe), which the pod's Succeeded waits for.  The directory is
    a hostPath on the node, at the same path in the pod as in the validator's
    container."""
    d = _pod_results_dir(env)
    name = pod["metadata"]["name"]
    ctr = pod["spec"]["containers"][0]
    ctr["args"] = list(ctr.get("args") or []) + [flag, os.path.join(d, f"{name}.json")]
    if gate_lock_env(env):
        ctr.setdefault("env", []).append({"name": GATE_LOCK_ENV, "value": d})  # the gate locks (gate_lock_env)
    ctr.setdefault("volumeMounts", []).append({"name": "pod-results", "mountPath": d})
    pod["spec"].setdefault("volumes", []).append({"name": "pod-results",
                                                   "hostPath": {"path": d, "type": "DirectoryOrCreate"}})
    return pod


def _await_pods(env: NodeEnv, names, run_id: str, deadline: float, stop=None) -> tuple[dict, dict]:
    """Wait for the pods ``names`` (label ``run_id``): -> (pods by name,
    {name: report}) once every pod has written an ``ok`` report to its result
    file, or once every pod has ended (Succeeded / Failed).  A pod that
    reports a failure, or ends without a result file (not admitted, an image
    without the option), is judged by its phase as before."""
    from ..kube.client import wait_for
    from ..utils.fswait import wait_for_file

    halt = threading.Event()
    box: dict = {}

    def phases():
        try:
            box["live"], box["ended"] = wait_for(
                env.client, "v1", "Pod", lambda objs: all(
                    n in objs and ((objs[n].get("status") or {}).get("phase") in ("Succeeded", "Failed"))
                    for n in names),
                namespace=env.namespace, label_selector=f"{WORKLOAD_POD_LABEL}={run_id}",
                timeout=max(0.0, deadline - time.monotonic()), stop=halt, poll_s=env.poll_s)
        finally:
            halt.set()

    th = threading.Thread(target=phases, name="validate-pod-phases", daemon=True)
    th.start()
    d = _pod_results_dir(env)
    stopped = (lambda: False) if stop is None else stop.is_set
    reports: dict = {}
    for n in names:
        path = os.path.join(d, f"{n}.json")
        if not wait_for_file(path, max(0.0, deadline - time.monotonic()), halt, 0.5,
                             check=lambda p: os.path.exists(p) or stopped()) or stopped():
            halt.set()  # a stop ends the phase wait too
            break
        try:
            with open(path) as f:
                reports[n] = json.loads(f.read())
        except (OSError, ValueError):
            break
        if not reports[n].get("ok"):
            break
    for n in names:
        try:
            os.unlink(os.path.join(d, f"{n}.json"))
        except OSError:
            pass
    if len(reports) == len(names) and all(r.get("ok") for r in reports.values()):
        # the phase wait notices ``halt`` at its next watch event (the pods'
        # deletion below at the latest): not joined, it would hold the result
        # until the pod processes have exited after all
        halt.set()
        live = {}
        for n in names:  # the allocation the kubelet recorded; the pod may still be exiting
            try:
                live[n] = env.client.get("v1", "Pod", n, env.namespace)
            except Exception:  # noqa: BLE001
                live[n] = {}
        return live, reports
    th.join()
    return box.get("live") or {}, {}


def validate_plugin(env: NodeEnv, resource: str = RESOURCE_NAME, expect: int | None = None,
                    pod_args: list[str] | None = None, timeout: float = 600.0, stop=None,
                    image: str | None = None, pull_policy: str = "IfNotPresent",
                    pull_secrets: list[str] | None = None, kubelet=None,
                    partition_strategy: str = "single", pod_check: str = "hsa", per_device: bool = False,
                    max_concurrent: int | None = None) -> dict:
    """Wait until the kubelet holds one device per GPU (or partition), then
    prove the device-plugin path with pods: by default one pod per resource
    holding all of its devices (every device still goes through Allocate, the
    OCI hook and a kernel launch, from one process - at N = 8, 8 fewer process
    and HIP starts in the node's start-up storm, profiles/r3_storm); with
    ``per_device`` one 1-device pod per device (N pods x 1 GPU, each its own
    GetPreferredAllocation / Allocate / hook), at most ``max_concurrent``
    running at a time.  Each pod requests the resource its device is
    advertised under (:func:`expected_devices`; ``expect`` overrides the
    count of ``resource``) and is told how many devices it was allocated
    (``--expect-devices``): a device the runtime left out of the container
    fails the pod instead of passing on the ones that are there.

    The pods run the validator's own image (``VALIDATOR_IMAGE`` in the
    validator container's env, with its pull policy and secrets, which
    cli/operands.py puts in ``env.extra["validator_image"]``)."""
    pod_image = env.extra.get("validator_image") or {}  # from the container env (cli/operands.py)
    image = image or pod_image.get("image") or "amd-operator-validator"
    pull_policy = pod_image.get("pull_policy") or pull_policy
    if pull_secrets is None:
        pull_secrets = list(pod_image.get("pull_secrets") or [])
    t0 = time.perf_counter()
    expected = {resource: expect} if expect is not None else expected_devices(env, resource, partition_strategy)
    deadline = time.monotonic() + timeout
    shared: set = set()
    queries: list = []
    plan = _wait_kubelet_devices(env, expected, deadline, stop, kubelet, shared, queries)
    source = "kubelet"
    if plan is None:  # no pod-resources API: wait for the kubelet to publish Node.status.allocatable
        source = "node-status"
        shared = set(expected) | {"*"}  # replicas cannot be told apart here: one device per pod

        def node_plan(node: dict):
            # counts only: replicas are not told apart here, so a renamed
            # resource gets as many pods as there are GPUs, not replicas
            alloc = (node.get("status") or {}).get("allocatable") or {}
            plan = _device_plan(expected, {r: [f"{r}#{i}" for i in range(allocatable(node, r))] for r in alloc})
            if plan is None or plan == expected:
                return plan
            left, capped = sum(expected.values()), {}
            for r, n in sorted(plan.items()):
                if left > 0:
                    capped[r] = min(n, left)
                    left -= capped[r]
            return capped

        nodes, ok = wait_for(env.client, "v1", "Node", lambda o: node_plan(o.get(env.node_name) or {}) is not None,
                             name=env.node_name, timeout=max(0.0, deadline - time.monotonic()), stop=stop,
                             poll_s=env.poll_s)
        node = nodes.get(env.node_name) or {}
        if not ok:
            if stop is not None and stop.is_set():
                raise StepFailed("stopped")
            raise StepFailed(f"allocatable {({r: allocatable(node, r) for r in expected})}, expected {expected}")
        plan = node_plan(node)
    t_alloc = time.perf_counter() - t0
    marks = {"start": time.time() - (time.perf_counter() - t0), "devices_seen": time.time()}
    pod_args = list(pod_args or ["--steps", "hip,vecadd,gemm", "--gemm", "1024"])

    def make_pod(name: str, run_id: str, res: str, count: int = 1) -> dict:
        expect = ["--expect-devices", str(count)]
        if pod_check == "hsa":  # a kernel per allocated GPU on the HSA runtime (native/validator/gpu_check.cpp)
            command, args = "amdgpu-gpu-check", ["--timeout", "30", *expect]
        else:
            command, args = "amdgpu-validator", pod_args + ["--all-devices", *expect]
        pod = {
            "apiVersion": "v1", "kind": "Pod",
            "metadata": {"name": name, "namespace": env.namespace,
                         "labels": {"app": "amd-validator-workload", WORKLOAD_POD_LABEL: run_id}},
            "spec": {
                "nodeName": env.node_name,
                "restartPolicy": "Never",
                "tolerations": [{"key": resource, "operator": "Exists", "effect": "NoSchedule"}],
                "containers": [{"name": "workload", "image": image, "imagePullPolicy": pull_policy,
                                "command": [command], "args": args, "env": PLUGIN_POD_ENV,
                                "resources": {"limits": {res: str(count)}, "requests": {res: str(count)}}}],
            },
        }
        if pull_secrets:
            pod["spec"]["imagePullSecrets"] = [{"name": x} for x in pull_secrets]
        return _with_result_file(env, pod, "--result-file" if pod_check == "hsa" else "--ready-file")

    def phase(o):
        return (o.get("status") or {}).get("phase", "Pending")

    # a pod the kubelet could not admit (UnexpectedAdmissionError: the device
    # list it planned from was stale, e.g. a re-registering plugin's devices
    # still unhealthy) is run again; any other failure fails the step.
    # Time-sliced resources keep one 1-replica pod per GPU: a multi-replica
    # request may land twice on one GPU.
    def pods_for(one_each: bool) -> list[tuple[str, int]]:
        single = lambda r: one_each or r in shared or "*" in shared  # noqa: E731
        return ([(r, 1) for r, n in sorted(plan.items()) if single(r) for _ in range(n)]
                + [(r, n) for r, n in sorted(plan.items()) if not single(r)])

    todo = pods_for(per_device)
    fallback = None
    if per_device and max_concurrent is not None and len(todo) > max(1, max_concurrent):
        # every 1-device pod must hold its device while the others are admitted
        # (a finished pod's device goes back to the kubelet and the next pod may
        # get it again), so they all run at once - or, past the process budget,
        # one pod per resource instead
        fallback = f"{len(todo)} 1-device pods exceed the {max_concurrent} GPU processes left: one pod per resource"
        log.info("plugin validation: %s", fallback)
        todo = pods_for(False)
    devices: list[str] = []
    attempts, backoff, pods_run = 0, 0.05, 0
    while todo:
        attempts += 1
        run_id = os.urandom(4).hex()
        names = {}
        for i, (res, count) in enumerate(todo):
            name = f"amd-validator-workload-{run_id}-{i}"
            env.client.create(make_pod(name, run_id, res, count))
            names[name] = (res, count)
        marks.setdefault("pods_created", time.time())
        live, reports = _await_pods(env, list(names), run_id, deadline, stop)
        if reports:
            marks.setdefault("pods_reported", time.time())
        for n in names:
            try:
                env.client.delete("v1", "Pod", n, env.namespace)
            except Exception:  # noqa: BLE001
                pass
        phases = {n: "Succeeded" if n in reports else phase(live[n]) if n in live else "Missing" for n in names}
        retry = [n for n in names if phases[n] == "Failed"
                 and (live[n].get("status") or {}).get("reason") == "UnexpectedAdmissionError"]
        hard = {n: p for n, p in phases.items() if p != "Succeeded" and n not in retry}
        if hard:
            why = "; ".join(f"{n}: {((live.get(n) or {}).get('status') or {}).get('message', '')[-300:]}"
                            for n in hard if n in live)
            raise StepFailed(f"plugin validation pods did not succeed: {phases}" + (f" ({why})" if why else ""))
        for n in names:
            if phases[n] == "Succeeded":
                alloc = (live[n].get("metadata", {}).get("annotations") or {}).get("amd.com/gpu.allocated", "")
                devices += alloc.split(",") if alloc else [""] * names[n][1]
        pods_run += sum(1 for n in names if phases[n] == "Succeeded")
        todo = [names[n] for n in retry]
        if todo:
            if time.monotonic() + backoff >= deadline or (stop is not None and stop.is_set()):
                raise StepFailed(f"plugin validation pods not admitted: {phases}")
            log.info("%d plugin validation pod(s) not admitted, retrying in %.2f s", len(todo), backoff)
            (stop.wait if stop is not None else time.sleep)(backoff)
            backoff = min(backoff * 2, 2.0)
    summary = {"ok": True, "pods": pods_run, "devices_validated": len(devices), "resources": plan, "devices": devices,
               "attempts": attempts, "pod_mode": "perDevice" if per_device and not fallback else "perResource",
               "allocatable_wait_s": round(t_alloc, 4),
               "allocatable_source": source, "marks": {k: round(v, 4) for k, v in marks.items()},
               "kubelet_queries": queries,
               "seconds": time.perf_counter() - t0}
    if fallback:
        summary["pod_mode_fallback"] = fallback
    write_ready(env, "plugin", summary)
    return summary


def validate_dra(env: NodeEnv, timeout: float = 600.0, stop=None, image: str | None = None,
                 pull_policy: str = "IfNotPresent", pull_secrets: list[str] | None = None,
                 device_class: str | None = None) -> dict:
    """The DRA counterpart of :func:`validate_plugin` (``draDriver.enabled``,
    device plugin off): once the node's ResourceSlice lists every device, a
    ResourceClaim for all of them (``allocationMode: All``) and one pod that
    uses it and runs the pod check with ``--expect-devices`` - the scheduler
    allocates the claim, the kubelet has the DRA driver prepare it, the
    runtime injects the claim's CDI devices.  The pod goes through the
    scheduler (``kubernetes.io/hostname`` selector, no ``nodeName``): a pod
    bound directly would skip the claim's allocation."""
    from ..discovery import topology
    from ..dra.api import DRIVER_NAME
    from ..kube.client import wait_for

    pod_image = env.extra.get("validator_image") or {}
    image = image or pod_image.get("image") or "amd-operator-validator"
    pull_policy = pod_image.get("pull_policy") or pull_policy
    pull_secrets = list(pod_image.get("pull_secrets") or []) if pull_secrets is None else pull_secrets
    t0 = time.perf_counter()
    n = len(topology.enumerate_gpus(env.sysfs_root()))
    deadline = time.monotonic() + timeout
    slice_name = f"{env.node_name}-{DRIVER_NAME}"
    _, ok = wait_for(env.client, "resource.k8s.io/v1beta1", "ResourceSlice",
                     lambda objs: len(((objs.get(slice_name) or {}).get("spec") or {}).get("devices") or []) == n,
                     name=slice_name, timeout=timeout, stop=stop, poll_s=env.poll_s)
    if not ok:
        raise StepFailed(f"ResourceSlice {slice_name} does not list the node's {n} device(s)")
    marks = {"start": time.time() - (time.perf_counter() - t0), "devices_seen": time.time()}
    run_id = os.urandom(4).hex()
    name = f"amd-validator-dra-{run_id}"
    claim = {"apiVersion": "resource.k8s.io/v1beta1", "kind": "ResourceClaim",
             "metadata": {"name": name, "namespace": env.namespace, "labels": {WORKLOAD_POD_LABEL: run_id}},
             "spec": {"devices": {"requests": [{"name": "gpus", "deviceClassName": device_class or DRIVER_NAME,
                                                "allocationMode": "All"}]}}}
    pod = {"apiVersion": "v1", "kind": "Pod",
           "metadata": {"name": name, "namespace": env.namespace,
                        "labels": {"app": "amd-validator-workload", WORKLOAD_POD_LABEL: run_id}},
           "spec": {"nodeSelector": {"kubernetes.io/hostname": env.node_name}, "restartPolicy": "Never",
                    "resourceClaims": [{"name": "gpus", "resourceClaimName": name}],
                    "containers": [{"name": "workload", "image": image, "imagePullPolicy": pull_policy,
                                    "command": ["amdgpu-gpu-check"], "args": ["--timeout", "30", "--expect-devices",
                                                                              str(n)],
                                    "env": PLUGIN_POD_ENV, "resources": {"claims": [{"name": "gpus"}]}}]}}
    if pull_secrets:
        pod["spec"]["imagePullSecrets"] = [{"name": x} for x in pull_secrets]
    pod = _with_result_file(env, pod, "--result-file")
    env.client.create(claim)
    try:
        env.client.create(pod)
        marks["pods_created"] = time.time()
        objs, reports = _await_pods(env, [name], run_id, deadline, stop)
        st = (objs.get(name) or {}).get("status") or {}
        if name in reports:
            st = {"phase": "Succeeded"}
            marks["pods_reported"] = time.time()
        if st.get("phase") != "Succeeded":
            raise StepFailed(f"DRA validation pod {st.get('phase', 'Missing')}: {st.get('message', '')[-300:]}")
        got = env.client.get("resource.k8s.io/v1beta1", "ResourceClaim", name, env.namespace)
        devices = [r["device"] for r in (((got.get("status") or {}).get("allocation") or {}).get("devices") or {})
                   .get("results", [])]
    finally:
        for kind, api_version in (("Pod", "v1"), ("ResourceClaim", "resource.k8s.io/v1beta1")):
            try:
                env.client.delete(api_version, kind, name, env.namespace)
            except Exception:  # noqa: BLE001
                pass
    summary = {"ok": True, "pods": 1, "devices_validated": len(devices), "devices": devices, "pod_mode": "dra",
               "claim": name, "marks": {k: round(v, 4) for k, v in marks.items()}, "seconds": time.perf_counter() - t0}
    write_ready(env, "plugin", summary)
    return summary


START_GATE_PREFIX = ".start-gate-"


def prespawn_safe(env: NodeEnv, sdk_gate: bool = False) -> bool:
    """May validator processes start before the driver validation?

    Without a profiler tool a process touches no device before its start
    gate (``kfd_open_at_gate`` false), so it may always start early.  With
    the rocprofiler-sdk gate (``--gate-mode sdk``) the tool initialises the
    HSA runtime as the process loads and opens ``/dev/kfd`` before the gate:
    such a process is spawned early only when the kernel driver is already
    live and no driver upgrade is under way on the node.  Either way the
    driver manager aborts pending gates before it unloads a module
    (driver/manager.py), so an early process never holds the device against
    a driver replacement."""
    from ..wellknown import ACTIVE, UPGRADE_STATE_LABEL as STATE_LABEL
    from ..discovery import topology

    if not sdk_gate:
        return True
    if not topology.probe(env.sysfs_root())[0]:
        return False
    try:
        node = env.client.get("v1", "Node", env.node_name)
    except Exception:  # noqa: BLE001 - no API answer: take the safe path
        return False
    return (node["metadata"].get("labels") or {}).get(STATE_LABEL) not in ACTIVE


def abort_start_gates(env: NodeEnv) -> list[str]:
    """Release every validator process still waiting at its start gate with
    "abort" (they exit without touching the GPU further); returns the gates."""
    out = []
    try:
        names = os.listdir(env.validations_dir)
    except FileNotFoundError:
        return out
    for name in names:
        if not name.startswith(START_GATE_PREFIX) or name.endswith((".tmp", ".held")):
            continue
        path = os.path.join(env.validations_dir, name)
        try:
            with open(path) as f:
                if f.read().strip() not in ("", "init"):
                    continue  # final verdict already given ("init": the runtime may be starting, abort it too)
        except FileNotFoundError:
            continue
        tmp = f"{path}.abort.tmp"
        with open(tmp, "w") as f:
            f.write("abort")
        os.replace(tmp, path)
        out.append(name)
    return out


def validate_gpu(env: NodeEnv, workload_args: list[str], resource: str = RESOURCE_NAME,
                 pod_args: list[str] | None = None, timeout: float = 600.0, stop=None,
                 wait_toolkit: bool = False, with_driver: bool = False, partition_strategy: str = "single",
                 pod_check: str = "hsa", per_device: bool = False, dra: bool = False,
                 dra_device_class: str | None = None) -> dict:
    """Workload and plugin validation concurrently (each skipped if already done).
    ``dra``: the plugin step validates the DRA driver instead (:func:`validate_dra`).

    Only the driver gates the workload: its processes run in this privileged
    pod, not through the container runtime, so they start while the toolkit
    is still being installed.  The plugin pods go through the runtime hook
    and therefore wait for the toolkit (``wait_toolkit``) before running.

    ``with_driver``: this step also validates the driver (instead of a
    separate init container before it).  When :func:`prespawn_safe`, the
    workload processes are spawned right away behind a start gate, so their
    exec and library loading overlap the driver wait; the gate opens only once
    :func:`validate_driver` passed (and aborts them if it failed), so none of
    the validator's own GPU work precedes the driver validation."""
    t0 = time.perf_counter()
    results: dict = {}
    errors: list[str] = []
    gate = None
    driver_done = threading.Event()
    # the node's GPU-process budget: the workload keeps one process for the
    # plugin pods, which get what the workload leaves
    budget = int(_arg_value(workload_args, "--max-gpu-processes") or DEFAULT_MAX_GPU_PROCESSES)
    wl_procs = 0 if read_ready(env, "workload") is not None else planned_workload_processes(env, workload_args,
                                                                                             budget - 1)
    sdk_gate = "--counter-gate" in workload_args and _arg_value(workload_args, "--gate-mode") == "sdk"
    if "--no-gate-lock" in workload_args:  # before the plugin thread creates its pods
        env.extra["no_gate_lock"] = True
    prespawn = with_driver and prespawn_safe(env, sdk_gate)
    if with_driver:
        os.makedirs(env.validations_dir, exist_ok=True)
        gate = os.path.join(env.validations_dir, f"{START_GATE_PREFIX}{os.urandom(6).hex()}")
        open(gate, "w").close()  # empty = no verdict yet (driver/manager.py may abort it)

    def publish(verdict: str) -> None:
        tmp = f"{gate}.tmp"
        with open(tmp, "w") as f:
            f.write(verdict)
        os.replace(tmp, gate)

    _startup_mark("validate_gpu")

    def driver():
        verdict = "abort"
        try:
            wait_ready(env, "driver", timeout, stop)
            if gate:  # the module is loaded: the runtime may start while the N1 check runs (validator_main.cpp)
                publish("init")
                _startup_mark("gate_init")
            results["driver"] = validate_driver(env, timeout, stop)
            verdict = "go"
        except Exception as e:  # noqa: BLE001
            errors.append(f"driver: {e}")
        finally:
            if gate:
                publish(verdict)
            driver_done.set()

    def workload():
        try:
            if with_driver and not prespawn:  # spawn only once the driver passed
                driver_done.wait()
                if "driver" not in results:
                    return
            if read_ready(env, "workload") is None:
                # the plugin validation runs beside it: the processes leave once it is done
                linger = env.validation_file(READY_FILES["plugin"]) if read_ready(env, "plugin") is None else None
                results["workload"] = validate_workload(env, workload_args, timeout, start_gate=gate, budget=budget - 1,
                                                        linger_until=linger)
        except Exception as e:  # noqa: BLE001
            errors.append(f"workload: {e}")

    def plugin():
        from ..deviceplugin.podresources import KubeletDevices

        # the channel opens at the first query: connecting it up front
        # (grpc.channel_ready_future) cost the bring-up 0.2 s on the MI355X
        # box, interleaved A/B in profiles/r2_ttr/preconnect_ab.json
        kubelet = KubeletDevices(env.pod_resources_socket)
        try:
            if with_driver:
                driver_done.wait()
                if "driver" not in results:
                    return
            if wait_toolkit:
                wait_ready(env, "toolkit", timeout, stop)
            if os.environ.get("AMDGPU_EXPERIMENT_PLUGIN_AFTER_WORKLOAD"):  # start-up contention experiment
                wait_ready(env, "workload", timeout, stop)
            if read_ready(env, "plugin") is None and dra:
                results["plugin"] = validate_dra(env, timeout, stop, device_class=dra_device_class)
            elif read_ready(env, "plugin") is None:
                results["plugin"] = validate_plugin(env, resource, pod_args=pod_args, timeout=timeout, stop=stop,
                                                    kubelet=kubelet, partition_strategy=partition_strategy,
                                                    pod_check=pod_check, per_device=per_device,
                                                    max_concurrent=max(1, budget - wl_procs))
        except Exception as e:  # noqa: BLE001
            errors.append(f"plugin: {e}")
        finally:
            kubelet.close()

    threads = [threading.Thread(target=workload, name="validate-workload"),
               threading.Thread(target=plugin, name="validate-plugin")]
    if with_driver:
        threads.insert(0, threading.Thread(target=driver, name="validate-driver"))
    try:
        for th in threads:
            th.start()
        for th in threads:
            th.join()
    finally:
        if gate:
            for path in (gate, gate + ".held"):  # .held: the processes' lifetime lock (driver/manager.py)
                try:
                    os.unlink(path)
                except FileNotFoundError:
                    pass
    if errors:
        raise StepFailed("; ".join(errors))
    return {"ok": True, "seconds": time.perf_counter() - t0, **results}


def validated_mfma_dtypes(workload: dict | None) -> list[str]:
    """MFMA data types that passed the K5 probe on every rank of the workload
    report (empty when the step did not run, e.g. simulated GPUs)."""
    ranks = (workload or {}).get("ranks") or []
    sets = []
    for r in ranks:
        step = next((s for s in r.get("steps", []) if s.get("name") == "mfma"), None)
        if not step or not isinstance(step.get("dtypes"), dict):
            return []
        sets.append([k for k, ok in step["dtypes"].items() if ok is True])
    if not sets:
        return []
    common = set(sets[0]).intersection(*sets[1:])
    return [d for d in sets[0] if d in common]


RATE_STEPS = (("bf16", "gemm"), ("fp8", "gemm_fp8"), ("fp4", "gemm_fp4"), ("fp6", "gemm_fp6"),
              ("mxfp4", "gemm_mxfp4"))


def validated_rate_dtypes(workload: dict | None) -> list[str]:
    """Data types whose GEMM step passed on every device of every rank of the
    workload report with a TF/s floor applied (``min_tflops`` > 0: a
    report-only run proves no rate) and, where the counter gate was asked
    for, counted by it (``counter_gate`` "pass"; "not_counted": the sdk-mode
    gate counts only the bf16 GEMM, so that rate is not claimed)."""
    reports = (workload or {}).get("ranks") or []
    out = []
    for dtype, name in RATE_STEPS:
        recs = [s for r in reports for s in r.get("steps", []) if s.get("name") == name]
        if recs and all(s.get("ok") is True and (s.get("min_tflops") or 0) > 0
                        and s.get("counter_gate", "off") in ("pass", "off") for s in recs):
            out.append(dtype)
    return out


def complete(env: NodeEnv) -> dict:
    """Mark the node validated: label, the MFMA data types the probe confirmed
    (``amd.com/gpu.validated.mfma=f16.bf16.fp8...``, next to GFD's per-arch
    ``amd.com/gpu.mfma.*`` claims) and an annotation with the step durations."""
    drv_time = (read_ready(env, "driver") or {}).get("time")
    steps = {s: (read_ready(env, s) or {}).get("seconds") for s in ("driver", "workload", "plugin")}
    ann = {"amd.com/gpu.validation": json.dumps({k: round(v, 4) for k, v in steps.items() if v is not None})}
    labels = {VALIDATED_LABEL: "true"}
    dtypes = validated_mfma_dtypes(read_ready(env, "workload"))
    if dtypes:
        labels[MFMA_LABEL] = ".".join(dtypes)[:63]
    rates = validated_rate_dtypes(read_ready(env, "workload"))
    labels[MFMA_RATE_LABEL] = ".".join(rates) if rates else None  # a stale claim goes
    env.client.patch("v1", "Node", env.node_name, {"metadata": {"labels": labels, "annotations": ann}})
    write_ready(env, "complete", {"steps": steps, "mfma_dtypes": dtypes, "mfma_rate_dtypes": rates})
    # The driver can go while this runs: the driver container's health
    # monitor then leaves its loss marker, removes every ready file and these
    # labels (driver/manager.py _withdraw_validation).  Had that happened
    # between the label patch and the file above, the node would stay
    # marked validated on a driver that is gone; so, with a marker newer
    # than the driver validation this completes, or with no driver
    # validation left (the marker stays until the driver is back and the
    # validator restarted; an older one is a loss that a later driver
    # validation already followed), the node's validation goes again.
    from ..driver.manager import LOST_MARKER

    try:
        lost_at = os.stat(env.validation_file(LOST_MARKER)).st_mtime
    except FileNotFoundError:
        lost_at = None
    if lost_at is not None and (drv_time is None or lost_at >= drv_time):
        clear_ready(env, ("complete",))
        env.client.patch("v1", "Node", env.node_name, {"metadata": {"labels": {
            VALIDATED_LABEL: None, MFMA_LABEL: None, MFMA_RATE_LABEL: None}}})
        return {"ok": False, "reason": "driver withdrawn during completion", "steps": steps}
    return {"ok": True, "steps": steps, "mfma_dtypes": dtypes, "mfma_rate_dtypes": rates}


# ------------------------------------------------------- sandbox workloads --

def validate_vfio(env: NodeEnv, pci, timeout: float = 600.0, stop=None) -> dict:
    """vm-passthrough node: the vfio-manager has run and every AMD GPU sits on
    vfio-pci with its ``/dev/vfio/<group>`` node (retried until ``timeout``)."""
    from ..sandbox.vfio import check_bound

    t0 = time.perf_counter()
    wait_ready(env, "vfio", timeout, stop)
    deadline = time.monotonic() + timeout
    for delay in env.waits():
        ok, msg, detail = check_bound(pci)
        if ok:
            return {"ok": True, "message": msg, "gpus": detail, "seconds": time.perf_counter() - t0}
        if time.monotonic() >= deadline or (stop is not None and stop.is_set()):
            raise StepFailed(msg)
        time.sleep(delay)


def complete_sandbox(env: NodeEnv) -> dict:
    """Mark a vm-passthrough node validated (same label as the container path)."""
    vf = read_ready(env, "vfio") or {}
    gpus = sum(len(g.get("gpus", [])) for g in vf.get("groups", []))
    ann = {"amd.com/gpu.validation": json.dumps({"vfio": round(vf.get("seconds", 0.0), 4), "workload": "vm-passthrough"})}
    env.client.patch("v1", "Node", env.node_name, {"metadata": {"labels": {VALIDATED_LABEL: "true"}, "annotations": ann}})
    write_ready(env, "sandbox", {"gpus": gpus})
    return {"ok": True, "gpus": gpus}
