"""Where the plugin-validation pod's wall time goes: exec -> main -> report -> exit.

The pod's check (amdgpu-gpu-check) reports in ~0.07-0.10 s of its own clock,
but the bring-up sees the pod done 0.16-0.18 s after its OCI hook ran.  The
kubelet reports a pod Succeeded only once its process has exited, so both the
exec (dynamic loading of the HSA runtime) and the exit (the kernel releasing
the process's GPU memory and queues) are on the critical path.  This probe
times each part on one GPU, with the GPU idle and with the node's workload
validator (HIP) starting at the same moment, as in a bring-up:

  main_lag   spawn -> main (exec, ld.so, static initialisers)   [t_main in the report]
  report     spawn -> report line on stdout
  exit       report line -> process reaped (waitpid)

Prints one JSON object; medians per arm.
"""

from __future__ import annotations

import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE = os.path.join(ROOT, "amdgpu_operator", "_native")
CHECK = [os.path.join(NATIVE, "amdgpu-gpu-check"), "--timeout", "30"]
WORKLOAD = [os.path.join(NATIVE, "amdgpu-validator"), "--steps", "hip,vecadd,gemm,mfma,hbm", "--rendezvous",
            "/tmp/pod-exit-probe"]
ENV = {**os.environ, "HSA_ENABLE_SDMA": "0"}


def once(with_workload: bool, env: dict | None = None) -> dict:
    wl = None
    if with_workload:
        wl = subprocess.Popen(WORKLOAD, env={**ENV, "AMDGPU_REPORT_EARLY": "1"}, stdout=subprocess.PIPE,
                              stderr=subprocess.DEVNULL)
    t0 = time.monotonic()
    p = subprocess.Popen(CHECK, env={**ENV, **(env or {})}, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL)
    line = p.stdout.readline()
    t_rep = time.monotonic()
    rest = p.stdout.read()
    t_eof = time.monotonic()
    rc = p.wait()
    t_exit = time.monotonic()
    rep = json.loads(line or rest.splitlines()[-1])
    out = {"rc": rc, "ok": rep.get("ok"), "main_lag_s": round(rep["t_main"] - t0, 4),
           "report_s": round(t_rep - t0, 4), "eof_after_report_s": round(t_eof - t_rep, 4),
           "exit_after_report_s": round(t_exit - t_rep, 4), "wall_s": round(t_exit - t0, 4),
           "process_s": rep.get("seconds"), "steps": {s["name"]: s.get("seconds") for s in rep.get("steps", [])},
           "hsa_detail": next(({k: s.get(k) for k in ("co_load_s", "queue_s")} for s in rep.get("steps", [])
                               if s.get("name") == "hsa"), None)}
    if wl is not None:
        wl.stdout.read()
        out["workload_rc"] = wl.wait()
    return out


KNOBS = {  # --knobs: ROCr settings that might shorten the check's start or its exit
    "sdma_on": {"HSA_ENABLE_SDMA": "1"},
    "interrupt_off": {"HSA_ENABLE_INTERRUPT": "0"},
    "no_scratch_reclaim": {"HSA_NO_SCRATCH_RECLAIM": "1"},
    "signal_pool_16": {"ROC_SIGNAL_POOL_SIZE": "16"},
}


def knobs(rounds: int) -> int:
    """Idle GPU, baseline against each ROCr knob, interleaved round by round."""
    once(False)
    arms = {"baseline": {}, **KNOBS}
    runs = {k: [] for k in arms}
    for _ in range(rounds):
        for k, env in arms.items():
            runs[k].append(once(False, env))
            time.sleep(0.3)
    keys = ("main_lag_s", "report_s", "exit_after_report_s", "wall_s", "process_s")
    out = {arm: {"median": {k: round(statistics.median(r[k] for r in v), 4) for k in keys},
                 "all_ok": all(r["ok"] and r["rc"] == 0 for r in v)} for arm, v in runs.items()}
    print(json.dumps(out))
    return 0 if all(v["all_ok"] for v in out.values()) else 1


def main() -> int:
    if len(sys.argv) > 1 and sys.argv[1] == "--knobs":
        return knobs(int(sys.argv[2]) if len(sys.argv) > 2 else 6)
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    once(False)  # page-in
    runs = {"idle": [], "with_workload": [], "idle_hsa_shut_down": []}
    for _ in range(rounds):
        runs["idle"].append(once(False))
        time.sleep(0.3)  # let the previous processes' teardown finish
        runs["with_workload"].append(once(True))
        time.sleep(0.3)
        runs["idle_hsa_shut_down"].append(once(False, {"AMDGPU_GPU_CHECK_SHUTDOWN": "1"}))
        time.sleep(0.3)
    keys = ("main_lag_s", "report_s", "exit_after_report_s", "wall_s", "process_s")
    out = {arm: {"median": {k: round(statistics.median(r[k] for r in v), 4) for k in keys},
                 "all_ok": all(r["ok"] and r["rc"] == 0 for r in v), "runs": v} for arm, v in runs.items()}
    print(json.dumps(out))
    return 0 if all(v["all_ok"] for v in out.values()) else 1


if __name__ == "__main__":
    sys.exit(main())
