"""Counter gates beside a co-tenant that takes no gate lock: a PyTorch
process running bf16 GEMMs (hipBLASLt), either back to back (``busy``) or in
bursts with idle gaps (``bursty``: 8 GEMMs, then ``--gap-ms`` idle).  Per
trial the validator runs its gated steps once; one JSON line per trial with
each gate's verdict, attempts and the retried windows' signatures
(gate_policy.h gate_retry_kind).

  python tools/cotenant_gate.py --trials 5 --out gpurun_out/cotenant.jsonl
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

LOOP = ("import sys, time, torch\n"
        "a = torch.randn(4096, 4096, device='cuda', dtype=torch.bfloat16)\n"
        "b = torch.randn(4096, 4096, device='cuda', dtype=torch.bfloat16)\n"
        "(a @ b).sum().item()\n"
        "print('ready', flush=True)\n"
        "t, gap = time.monotonic(), float(sys.argv[2]) / 1000.0\n"
        "while time.monotonic() - t < float(sys.argv[1]):\n"
        "    for _ in range(8):\n"
        "        c = a @ b\n"
        "    torch.cuda.synchronize()\n"
        "    if gap > 0:\n"
        "        time.sleep(gap)\n")

GATED = ("gemm", "gemm_fp8", "gemm_fp4", "gemm_fp6", "gemm_mxfp4")


def trial(mode: str, gap_ms: float, steps: str) -> dict:
    bg = None
    if mode != "quiet":
        bg = subprocess.Popen([sys.executable, "-c", LOOP, "20", str(gap_ms if mode == "bursty" else 0)],
                              stdout=subprocess.PIPE, text=True)
        if bg.stdout.readline().strip() != "ready":
            raise RuntimeError("co-tenant did not start")
    try:
        with tempfile.TemporaryDirectory() as d:
            p = subprocess.run([str(native.binary("amdgpu-validator")), "--rendezvous", d, "--steps", steps,
                                "--counter-gate"], capture_output=True, text=True, timeout=60)
        rep = json.loads(p.stdout.strip().splitlines()[-1])
    finally:
        if bg is not None:
            bg.kill()
            bg.communicate(timeout=30)
    out = {"mode": mode, "gap_ms": gap_ms if mode == "bursty" else None, "ok": rep.get("ok"), "gates": {}}
    for s in rep.get("steps", []):
        if s["name"] in GATED:
            tries = [r for r in str(s.get("gate_retried_after", "")).split("; ") if r]
            out["gates"][s["name"]] = {
                "verdict": s.get("counter_gate"), "attempts": s.get("gate_attempts"),
                "kinds": [r[r.rfind(", ") + 2:-1] if r.endswith(")") and ", " in r else "final" for r in tries],
                "retried_after": tries,
                "tflops": s.get("tflops"), "mfma_util": s.get("mfma_util")}
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=5)
    ap.add_argument("--gap-ms", type=float, default=20.0)
    ap.add_argument("--steps", default="hip,gemm,gemm_fp8,gemm_fp4,gemm_fp6,gemm_mxfp4")
    ap.add_argument("--modes", default="quiet,bursty,busy")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    f = open(a.out, "w") if a.out else None
    for i in range(a.trials):
        for mode in a.modes.split(","):
            t0 = time.monotonic()
            r = trial(mode, a.gap_ms, a.steps)
            r["trial"] = i
            r["seconds"] = round(time.monotonic() - t0, 2)
            line = json.dumps(r)
            print(line, flush=True)
            if f:
                f.write(line + "\n")
                f.flush()
    return 0


if __name__ == "__main__":
    sys.exit(main())
