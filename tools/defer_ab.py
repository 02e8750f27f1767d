"""A/B of the validator's deferred counter gates (--defer-gates, PendingGate) against
counting each GEMM inside its step (the default): the arms alternate,
one validator process per trial with the default kernel steps and the
counter gate; per trial the steps' rates, gate attempts and the process's
step time.

  python tools/defer_ab.py --trials 10 --out gpurun_out/defer_ab.jsonl
"""

from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from amdgpu_operator import native  # noqa: E402

STEPS = "hip,vecadd,gemm,gemm_fp8,gemm_fp4,gemm_fp6,gemm_mxfp4,mfma,hbm"


def one(defer: bool) -> dict:
    with tempfile.TemporaryDirectory() as d:
        argv = [str(native.binary("amdgpu-validator")), "--rendezvous", d, "--steps", STEPS, "--counter-gate"]
        if defer:
            argv.append("--defer-gates")
        p = subprocess.run(argv, capture_output=True, text=True, timeout=60)
    rep = json.loads(p.stdout.strip().splitlines()[-1])
    out = {"defer": defer, "ok": rep.get("ok"), "seconds": rep.get("seconds")}
    for s in rep.get("steps", []):
        out[s["name"]] = {k: s.get(k) for k in ("seconds", "tflops", "gbps", "counter_gate", "gate_attempts",
                                                "gate_lock_wait_s", "mfma_util") if s.get(k) is not None}
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=10)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    f = open(a.out, "w") if a.out else None
    for i in range(a.trials):
        for defer in ((True, False) if i % 2 == 0 else (False, True)):
            r = one(defer)
            r["trial"] = i
            line = json.dumps(r)
            print(line, flush=True)
            if f:
                f.write(line + "\n")
                f.flush()
    return 0


if __name__ == "__main__":
    sys.exit(main())
