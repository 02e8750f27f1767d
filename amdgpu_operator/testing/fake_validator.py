"""Stand-in for the native ``amdgpu-validator`` on machines without a GPU.

Accepts the same arguments, rendezvous with its peer ranks through the same
directory protocol (so multi-rank orchestration is exercised for real) and
prints the same JSON report shape with ``"simulated": true``.
"""

from __future__ import annotations

import json
import os
import sys
import time


def wait_start_gate(path: str | None, timeout: float = 120.0) -> str:
    """The native validator's ``--start-gate``: block until the file has a
    verdict; "go" releases the process (same protocol as validator_main.cpp)."""
    if not path:
        return "go"
    deadline = time.time() + timeout
    while time.time() < deadline:
        try:
            with open(path) as f:
                text = f.read().strip()
            if text:
                return text
        except FileNotFoundError:
            pass
        time.sleep(0.001)
    return "timeout"


def main(argv: list[str]) -> int:
    def arg(name, default):
        return argv[argv.index(name) + 1] if name in argv else default

    verdict = wait_start_gate(arg("--start-gate", None))
    if verdict != "go":
        print(json.dumps({"ok": False, "error": f"start gate: {verdict}", "steps": []}))
        return 3

    rank, world = int(arg("--rank", "0")), int(arg("--world", "1"))
    rdv, run_id = arg("--rendezvous", "/tmp/amdgpu-validator"), arg("--run-id", "run")
    steps = arg("--steps", "hip,vecadd,gemm,mfma,hbm,xgmi,rccl").split(",")
    t0 = time.perf_counter()
    os.makedirs(rdv, exist_ok=True)
    if "rccl" in steps and world > 1:  # barrier like the RCCL unique-id exchange
        open(os.path.join(rdv, f"{run_id}-fake-{rank}"), "w").close()
        deadline = time.time() + 60
        while any(not os.path.exists(os.path.join(rdv, f"{run_id}-fake-{r}")) for r in range(world)):
            if time.time() > deadline:
                print(json.dumps({"ok": False, "error": "rendezvous timeout"}))
                return 1
            time.sleep(0.002)
    rep = {"ok": True, "simulated": True, "rank": rank, "world": world, "device": int(arg("--device", "0")),
           "owner_rank_env": os.environ.get("RANK"), "hip_visible_devices": os.environ.get("HIP_VISIBLE_DEVICES"),
           "seconds": time.perf_counter() - t0,
           "steps": [{"name": s, "ok": True, "seconds": 0.0, "simulated": True} for s in steps]}
    print(json.dumps(rep))
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
