"""Plugin-validation pod check: HIP validator vs the HSA-only gpu-check.

Times, from exec to the report (the pod's critical path), both ways of
proving that the pod's GPU runs a kernel, interleaved round by round:

  hip   amdgpu-validator --steps hip,vecadd (HIP runtime + context, 1 Mi floats)
  hsa   amdgpu-gpu-check (HSA runtime only, the validator's code object)

Prints one JSON object with per-arm wall times and medians.
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
ENV = {**os.environ, "HSA_ENABLE_SDMA": "0", "AMDGPU_REPORT_EARLY": "1"}
ARMS = {
    "hip": [os.path.join(NATIVE, "amdgpu-validator"), "--steps", "hip,vecadd", "--rendezvous", "/tmp/pod-probe"],
    "hsa": [os.path.join(NATIVE, "amdgpu-gpu-check")],
}


def once(argv):
    t = time.perf_counter()
    p = subprocess.run(argv, env=ENV, capture_output=True, text=True, timeout=60)
    wall = time.perf_counter() - t
    rep = json.loads(p.stdout.strip().splitlines()[-1])
    return {"rc": p.returncode, "wall_s": round(wall, 4), "ok": rep.get("ok"), "seconds": rep.get("seconds"),
            "steps": {s["name"]: s.get("seconds") for s in rep.get("steps", [])}}


def main() -> int:
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    for argv in ARMS.values():  # page-in
        once(argv)
    runs = {k: [] for k in ARMS}
    for _ in range(rounds):
        for k, argv in ARMS.items():
            runs[k].append(once(argv))
    out = {k: {"median_wall_s": round(statistics.median(r["wall_s"] for r in v), 4),
               "min_wall_s": min(r["wall_s"] for r in v), "all_ok": all(r["ok"] and r["rc"] == 0 for r in v),
               "runs": v} for k, v in runs.items()}
    print(json.dumps(out))
    return 0 if all(v["all_ok"] for v in out.values()) else 1


if __name__ == "__main__":
    sys.exit(main())
