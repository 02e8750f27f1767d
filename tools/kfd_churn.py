"""Which KFD processes come and go during a bring-up (the second mode).

A fresh process's HSA start-up on this box takes ~0.07 s, or 0.15-0.25 s
right behind another KFD process's exit (the kernel releases the exiting
process's GPU state in a workqueue; BASELINE.md "What a fresh HIP process
costs").  The bench's slow bring-ups are slow HSA start-ups of the plugin pod
or the workload validator.  This tool runs ``--steps`` bring-ups at driver
settings (bench.one_bring_up) with a sampler thread that lists
/sys/class/kfd/kfd/proc every ``--period-ms`` and records every KFD process
that appears or disappears, with its time relative to the step's start
(host PIDs: the list is not in this PID namespace).  Per step it writes the
critical path and those events; the summary counts, for slow and for normal
plugin-pod HSA start-ups, the KFD exits that fell inside that start-up.

  python tools/kfd_churn.py --steps 40 --out gpurun_out/kfd_churn.json
"""

from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


class Sampler:
    def __init__(self, period_s: float):
        self.period_s = period_s
        self.events: list[tuple[float, str, int]] = []  # (wall time, "+" / "-", host pid)
        self.names: dict[int, str] = {}  # pid -> what /proc says at first sight ("?" outside this PID namespace)
        self._stop = threading.Event()
        self._th = threading.Thread(target=self._run, daemon=True, name="kfd-churn")

    def _list(self) -> set[int]:
        try:
            return {int(p) for p in os.listdir(bench.KFD_PROCS) if p.isdigit()}
        except OSError:
            return set()

    def _run(self) -> None:
        prev = self._list()
        while not self._stop.wait(self.period_s):
            cur = self._list()
            if cur != prev:
                t = time.time()
                self.events += [(t, "+", p) for p in sorted(cur - prev)] + [(t, "-", p) for p in sorted(prev - cur)]
                for p in cur - prev:
                    self.names[p] = self._name(p)
                prev = cur

    @staticmethod
    def _name(pid: int) -> str:
        try:
            with open(f"/proc/{pid}/cmdline", "rb") as f:
                argv = f.read().split(b"\0")
            exe = os.path.basename(argv[0].decode(errors="replace"))
            rest = " ".join(a.decode(errors="replace") for a in argv[1:4] if a)
            return f"{exe} {rest}".strip()[:80]
        except OSError:
            return "?"

    def start(self) -> "Sampler":
        self._th.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        self._th.join()

    def window(self, t0: float, lo: float, hi: float) -> list[tuple[float, str, int]]:
        """Events from t0 + lo to t0 + hi, timed from t0."""
        return [(round(t - t0, 4), s, p) for t, s, p in self.events if t0 + lo <= t <= t0 + hi]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--period-ms", type=float, default=1.0)
    ap.add_argument("--kubelet-status-s", type=float, default=0.5)
    ap.add_argument("--out", default="gpurun_out/kfd_churn.json")
    ap.add_argument("--idle-s", type=float, default=0.0,
                    help="first sample this long with no bring-up running: the host's own KFD churn")
    a = ap.parse_args()
    sys.argv = [sys.argv[0], "--kubelet-status-s", str(a.kubelet_status_s), "--no-sweep", "--no-pod-workload"]
    args = bench.parse()
    fake = not bench.gpu_available("/")
    workdir = tempfile.mkdtemp(prefix="kfd-churn-")
    sampler = Sampler(a.period_ms / 1000.0).start()
    idle = None
    if a.idle_s > 0:
        t_idle = time.time()
        time.sleep(a.idle_s)
        ev = sampler.window(t_idle, 0.0, a.idle_s)
        idle = {"seconds": a.idle_s, "appeared": sum(1 for e in ev if e[1] == "+"),
                "exited": sum(1 for e in ev if e[1] == "-"), "events": ev}
    rows = []
    t_print = time.monotonic()
    try:
        for i in range(a.warmup + a.steps):
            r = bench.one_bring_up(args, 1, None, workdir, fake, "process", False)
            if i < a.warmup:
                continue
            cp = bench.critical_path(r)
            t0 = r["t0_wall"]
            pod = cp.get("pod") or {}
            rows.append({"ttr": cp["ttr"], "pod_main_at": pod.get("main_at"), "pod_hsa_init": pod.get("hsa_init"),
                         "wl_proc": (cp.get("wl") or {}).get("proc"), "at": cp.get("at"),
                         "kfd_procs_at_start": (r.get("settle") or {}).get("kfd_procs"),
                         "events": [(t, sg, p, sampler.names.get(p, "?"))
                                    for t, sg, p in sampler.window(t0, -0.5, cp["ttr"] + 0.05)]})
            if time.monotonic() - t_print > 50:
                print(f"kfd_churn: {len(rows)}/{a.steps}", file=sys.stderr, flush=True)
                t_print = time.monotonic()
    finally:
        sampler.stop()
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump({"idle": idle, "steps": rows} if idle is not None else rows, f, indent=1)
    hsa = [r["pod_hsa_init"] for r in rows if isinstance(r["pod_hsa_init"], (int, float))]
    med = statistics.median(hsa) if hsa else 0.0

    def exits_inside(r):
        lo, hi = r["pod_main_at"], r["pod_main_at"] + r["pod_hsa_init"]
        return [e for e in r["events"] if e[1] == "-" and lo <= e[0] <= hi]

    ok = [r for r in rows if isinstance(r["pod_hsa_init"], (int, float)) and isinstance(r["pod_main_at"], (int, float))]
    slow = [r for r in ok if r["pod_hsa_init"] > 1.5 * med]
    fast = [r for r in ok if r["pod_hsa_init"] <= 1.5 * med]
    summary = {
        "steps": len(rows), "pod_hsa_init_median_s": round(med, 4),
        "slow_pod_hsa_init": len(slow),
        "slow_with_a_kfd_exit_inside": sum(1 for r in slow if exits_inside(r)),
        "normal_with_a_kfd_exit_inside": sum(1 for r in fast if exits_inside(r)),
        "normal": len(fast),
        "kfd_exits_per_step_median": statistics.median(
            [sum(1 for e in r["events"] if e[1] == "-" and e[0] >= 0) for r in rows]) if rows else None,
        "ttr": bench.dist_summary([r["ttr"] for r in rows]),
    }
    if idle is not None:
        summary["idle"] = {k: idle[k] for k in ("seconds", "appeared", "exited")}
    print(json.dumps(summary))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
