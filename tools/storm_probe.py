"""The N = 8 validator start-up storm, rehearsed on the GPUs of this machine.

At N = 8 a node's validation starts, within a few milliseconds:

* 8 kernel-check processes (validate.py validate_workload: hip, vecadd,
  gemm + counter gate, mfma, hbm; one per GPU),
* 8 RCCL processes (hip + rccl, one per GPU),
* 8 plugin-validation pods (hip, vecadd, 1024^3 gemm; one per GPU).

This probe starts the same processes, for N GPUs, through the same code
(``validate_workload`` for the first two groups, the plugin pods' argv and
environment for the third) against the GPUs present - on a 1-GPU box all 3N
land on device 0 (N = 5 by default: the box allows 16 GPU processes of one
user at a time), a worst case for per-device contention and a faithful one
for the host side (process start, KFD open, driver locks).  The RCCL
processes run ``hip`` only: 8 ranks of one communicator cannot share a GPU.

Variants (each repeated ``--reps`` times):

  single     one kernel-check process alone (the N = 1 reference point)
  storm      all 3N at once (the current design)
  merged     RCCL folded into the kernel-check process (rcclProcess=shared):
             2N processes
  staggered  the plugin pods start only after the 2N workload processes reported
  onepod     the round-3 design: the plugin check is one pod holding every GPU
             (amdgpu-validator --all-devices), 2N + 1 processes

Per process: ``hip`` step (runtime + context init), ``vecadd`` (first kernel
launch), the process's own total, and spawn-to-report as the orchestrator saw
it.  Prints one JSON object.
"""

from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import tempfile
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from amdgpu_operator import native  # noqa: E402
from amdgpu_operator.nodeenv import REPORT_EARLY_ENV, NodeEnv, run_local  # noqa: E402
from amdgpu_operator.testing import fakesys  # noqa: E402
from amdgpu_operator.validator import validate as V  # noqa: E402

# no counter gate: PMC counters are per device, and concurrent counted
# dispatches of several processes on one GPU would read each other's work
# (on a real node each process counts its own GPU)
KERNEL_ARGS = ["--steps", "hip,vecadd,gemm,mfma,hbm,rccl"]
POD_ARGS = ["--steps", "hip,vecadd,gemm", "--gemm", "1024"]


def _rewrite(argv: list[str], real_gpus: int) -> list[str]:
    out = list(argv)
    i = out.index("--device")
    out[i + 1] = str(int(out[i + 1]) % real_gpus)  # the fake node's GPU d -> a real one
    if "--steps" in out:
        j = out.index("--steps")
        steps = out[j + 1].split(",")
        if "rccl" in steps:  # ranks of one communicator cannot share a device: HIP start-up only
            out[j + 1] = ",".join(s for s in steps if s != "rccl") or "hip"
    return out


def _summ(reports: list[dict]) -> dict:
    def col(f):
        xs = [f(r) for r in reports if f(r) is not None]
        return {"median": round(statistics.median(xs), 4), "max": round(max(xs), 4)} if xs else None

    def step(name):
        return lambda r: next((s.get("seconds") for s in r.get("steps", []) if s.get("name") == name), None)

    return {"n": len(reports), "hip_s": col(step("hip")), "vecadd_s": col(step("vecadd")), "gemm_s": col(step("gemm")),
            "process_total_s": col(lambda r: r.get("seconds")), "spawn_to_report_s": col(lambda r: r.get("process_seconds"))}


def run_variant(variant: str, n: int, real_gpus: int, tmp: str) -> dict:
    root = os.path.join(tmp, f"node-{variant}-{time.monotonic_ns()}")
    fakesys.build_node(root, n)
    env = NodeEnv("storm", None, host_root=root, validations_dir=os.path.join(root, "val"), poll_s=0.01)
    # the fake node's KFD unique ids mean nothing to this machine's runtime:
    # the kernel-check processes see the real GPUs
    env.launcher = lambda argv, e, d, t: run_local(_rewrite(argv, real_gpus),
                                                   {k: v for k, v in e.items() if k != "ROCR_VISIBLE_DEVICES"}, t)
    args = list(KERNEL_ARGS)
    if variant == "merged":
        args.append("--rccl-shared-process")
    if variant == "single":
        t0 = time.perf_counter()
        p = run_local([str(native.binary("amdgpu-validator")), "--device", "0", "--rendezvous", env.validations_dir,
                       "--steps", "hip,vecadd,gemm,mfma,hbm"], {REPORT_EARLY_ENV: "1"}, 120)
        rep = json.loads(p.stdout.strip().splitlines()[-1])
        rep["process_seconds"] = p.seconds
        return {"wall_s": round(time.perf_counter() - t0, 4), "workload": _summ([rep]), "pods": None}

    def workload():
        return V.validate_workload(env, args, timeout=300)

    def pods():
        jobs = [[str(native.binary("amdgpu-validator")), "--device", str(i % real_gpus), "--rendezvous",
                 env.validations_dir, "--run-id", f"pod{i}", *POD_ARGS] for i in range(n)]
        if variant == "onepod":
            jobs = [[str(native.binary("amdgpu-validator")), "--all-devices", "--rendezvous", env.validations_dir,
                     "--run-id", "pod", *POD_ARGS]]
        penv = {REPORT_EARLY_ENV: "1", **{e["name"]: e["value"] for e in V.PLUGIN_POD_ENV}}
        with ThreadPoolExecutor(max_workers=len(jobs)) as ex:
            res = list(ex.map(lambda a: run_local(a, penv, 300), jobs))
        out = []
        for r in res:
            rep = json.loads(r.stdout.strip().splitlines()[-1])
            rep["process_seconds"] = r.seconds
            out.append(rep)
        return out

    t0 = time.perf_counter()
    with ThreadPoolExecutor(max_workers=2) as ex:
        fw = ex.submit(workload)
        if variant == "staggered":
            wl = fw.result()
            t_wl = time.perf_counter() - t0
            pod_reps = pods()
        else:
            fp = ex.submit(pods)
            wl = fw.result()
            t_wl = time.perf_counter() - t0
            pod_reps = fp.result()
    wall = time.perf_counter() - t0
    return {"wall_s": round(wall, 4), "workload_s": round(t_wl, 4), "workload": _summ(wl["ranks"]),
            "pods": _summ(pod_reps), "processes": len(wl["ranks"]) * (1 if variant == "merged" else 2) + len(pod_reps)}


def main() -> int:
    ap = argparse.ArgumentParser()
    # the GPU box allows 16 GPU processes of one user at a time: 5 GPUs x 3
    # processes is the largest storm of this shape that fits on one device
    ap.add_argument("--gpus", type=int, default=5, help="GPUs of the rehearsed node (3 processes each)")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--variants", default="single,storm,onepod,merged,staggered")
    a = ap.parse_args()
    from amdgpu_operator.discovery import topology

    real = max(1, len(topology.enumerate_gpus("/")))
    out = {"node_gpus": a.gpus, "real_gpus": real, "variants": {}}
    with tempfile.TemporaryDirectory() as tmp:
        run_variant("single", a.gpus, real, tmp)  # page-in / first HIP init of the box, not reported
        for v in a.variants.split(","):
            reps = [run_variant(v, a.gpus, real, tmp) for _ in range(a.reps)]
            out["variants"][v] = {"wall_s": [r["wall_s"] for r in reps], "runs": reps}
            print(json.dumps({"variant": v, "wall_s": [r["wall_s"] for r in reps]}), file=sys.stderr, flush=True)
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
