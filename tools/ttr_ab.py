"""Interleaved A/B of the bring-up's time-to-Ready (VERDICT r5 task 2).

Runs ``--pairs`` rounds of one bring-up per arm, alternating the arms in every
round (ABAB..., the arm order flipped every other round), so a mode that hits
a quarter of the steps lands in both arms alike instead of in whichever arm
ran while the box was noisy.  Each arm is a list of Helm ``--set`` flags on
top of the reference's (bench.py ``--set``).  Prints one JSON line per arm
(mean / median / p90 / max TTR, steps above 1.3 x the run's median, and the
medians of the critical-path parts) and writes every step to ``--out``.

  python tools/ttr_ab.py --pairs 40 --arm after= \\
      --arm immediate=devicePlugin.healthStart=immediate
"""

from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--arm", action="append", required=True,
                    help="NAME=SET[,SET...] (Helm --set flags of this arm, or env:VAR=VALUE for the environment "
                         "its processes inherit; empty: the defaults)")
    ap.add_argument("--kubelet-status-s", type=float, default=0.5,
                    help="the simulated kubelet's status tick (time-to-Ready does not wait for it)")
    ap.add_argument("--out", default="gpurun_out/ttr_ab.json")
    a = ap.parse_args()
    arms = []
    for spec in a.arm:
        name, _, sets = spec.partition("=")
        arms.append((name, [s for s in sets.split(",") if s]))
    sys.argv = [sys.argv[0], "--kubelet-status-s", str(a.kubelet_status_s), "--no-sweep", "--no-pod-workload"]
    args = bench.parse()
    fake = not bench.gpu_available("/")
    workdir = tempfile.mkdtemp(prefix="ttr-ab-")
    steps: dict[str, list[dict]] = {n: [] for n, _ in arms}

    def one(name, sets):
        # "env:NAME=VALUE" entries set the environment the bring-up's processes inherit
        envs = dict(x[4:].split("=", 1) for x in sets if x.startswith("env:"))
        args.extra_set = [x for x in sets if not x.startswith("env:")]
        saved = {k: os.environ.get(k) for k in envs}
        os.environ.update(envs)
        try:
            r = bench.one_bring_up(args, 1, None, workdir, fake, "process", False)
        finally:
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        cp = bench.critical_path(r)
        cp["kfd_holders"] = r.get("kfd_holders")
        cp["gates"] = [{k: g.get(k) for k in ("name", "gate_attempts", "gate_lock_wait_s", "gate_retried_after")}
                       for g in (r.get("gates") or [])]
        return cp

    for i in range(a.warmup):
        for name, sets in arms:
            one(name, sets)
    t0 = time.monotonic()
    for i in range(a.pairs):
        order = arms if i % 2 == 0 else arms[::-1]
        for name, sets in order:
            steps[name].append(one(name, sets))
        if time.monotonic() - t0 > 50:
            print(f"ttr_ab: {i + 1}/{a.pairs}", file=sys.stderr, flush=True)
            t0 = time.monotonic()
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump({"arms": {n: s for n, s in arms}, "steps": steps}, f, indent=1, default=str)
    for name, sets in arms:
        cps = steps[name]
        ttr = [c["ttr"] for c in cps]
        med = statistics.median(ttr)
        parts = {}
        for pname, get in bench._CP_PARTS:
            v = [x for x in (get(c) for c in cps) if isinstance(x, (int, float))]
            if v:
                parts[pname] = round(statistics.median(v), 4)
        slow = bench.slow_steps(cps)
        print(json.dumps({"arm": name, "set": sets, "n": len(ttr), "ttr": bench.dist_summary(ttr),
                          "p90_over_median": round(sorted(ttr)[int(0.9 * (len(ttr) - 1))] / med, 3),
                          "above_1.3x_median": len(slow), "slow": bench.slow_summary(slow),
                          "part_medians": parts,
                          "gate_retries": sum(max(0, (g.get("gate_attempts") or 1) - 1) for c in cps for g in c["gates"]),
                          "first_gate_lock_wait_median_s": statistics.median(
                              [c["gates"][0]["gate_lock_wait_s"] or 0.0 for c in cps if c["gates"]] or [0.0])}))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
