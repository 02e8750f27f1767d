"""Counter gates beside a continuously dispatching second process, with and
without the gate lock (native/include/gate_lock.h; VERDICT r5 task 3).

Each trial starts ``amdgpu-gpu-check --loop-seconds`` (the plugin-validation
pod's check, looping its kernel) and runs the validator's three counted GEMMs
(bf16, fp8, fp4) while it dispatches.  Arm ``locked``: both get
AMDGPU_GATE_LOCK_DIR (production).  Arm ``unlocked``: neither does (round 5).
Prints one JSON line per arm: gates passed on the first attempt, passed after
a retry, failed, and the lock waits.

  python tools/gate_lock_ab.py --trials 10 --out gpurun_out/gate_lock_ab.json
"""

from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from amdgpu_operator import native  # noqa: E402


def trial(locked: bool, loop_s: float) -> dict:
    d = tempfile.mkdtemp(prefix="gate-ab-")
    env = dict(os.environ)
    env.pop("AMDGPU_GATE_LOCK_DIR", None)
    if locked:
        env["AMDGPU_GATE_LOCK_DIR"] = d
    bg = subprocess.Popen([str(native.binary("amdgpu-gpu-check")), "--loop-seconds", str(loop_s), "--elems",
                           str(1 << 22), "--timeout", "30"], env=env, stdout=subprocess.PIPE, text=True)
    time.sleep(0.3)  # its HSA start-up: dispatching by now
    p = subprocess.run([str(native.binary("amdgpu-validator")), "--rendezvous", d, "--steps",
                        "hip,gemm,gemm_fp8,gemm_fp4", "--counter-gate"], env=env, capture_output=True, text=True,
                       timeout=120)
    alive = bg.poll() is None
    out = bg.communicate(timeout=60)[0]
    rep = json.loads(p.stdout.strip().splitlines()[-1])
    bgrep = json.loads(out.strip().splitlines()[-1]) if out.strip() else {}
    gates = [{k: s.get(k) for k in ("name", "counter_gate", "gate_attempts", "gate_lock", "gate_lock_wait_s",
                                     "gate_retried_after", "gate_reason")}
             for s in rep.get("steps", []) if s.get("name", "").startswith("gemm")]
    vec = next((s for s in bgrep.get("steps", []) if s.get("name") == "vecadd"), {})
    return {"locked": locked, "ok": rep.get("ok"), "gates": gates, "bg_alive_after": alive,
            "bg_dispatches": vec.get("dispatches")}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=10)
    ap.add_argument("--loop-seconds", type=float, default=3.0)
    ap.add_argument("--out", default="gpurun_out/gate_lock_ab.json")
    a = ap.parse_args()
    rows = []
    for i in range(a.trials):
        for locked in ((True, False) if i % 2 == 0 else (False, True)):
            rows.append(trial(locked, a.loop_seconds))
        print(f"gate_lock_ab: {i + 1}/{a.trials}", file=sys.stderr, flush=True)
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(rows, f, indent=1)
    for locked in (True, False):
        g = [x for r in rows if r["locked"] == locked for x in r["gates"]]
        print(json.dumps({
            "arm": "locked" if locked else "unlocked", "trials": sum(r["locked"] == locked for r in rows),
            "gates": len(g), "first_attempt_pass": sum(x["counter_gate"] == "pass" and x["gate_attempts"] == 1 for x in g),
            "pass_after_retry": sum(x["counter_gate"] == "pass" and (x["gate_attempts"] or 0) > 1 for x in g),
            "fail": sum(x["counter_gate"] != "pass" for x in g),
            "max_lock_wait_s": max((x["gate_lock_wait_s"] or 0 for x in g), default=None),
            "bg_alive_after_all": all(r["bg_alive_after"] for r in rows if r["locked"] == locked),
            "bg_dispatches_min": min((r["bg_dispatches"] or 0 for r in rows if r["locked"] == locked), default=None),
            "reasons": sorted({x["gate_reason"] or x["gate_retried_after"] for x in g
                               if x["gate_reason"] or x["gate_retried_after"]})[:3]}))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
