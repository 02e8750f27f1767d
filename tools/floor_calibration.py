"""Ready-gate floor calibration from repeated validator runs (VERDICT r5 task 5).

Runs the native validator ``--runs`` times on the GPU at the shipped sizes
(4096^3 GEMMs, 1 GiB HBM copy) with the counter gate and NO floors, one
process per run like a bring-up's validator, and records per run the rates
(bf16 / fp8 / fp4 / fp6 / mxfp4 TF/s, HBM GB/s) and the gate's MFMA
utilisation per data type.  Prints one JSON line with, per quantity, min /
p5 / median / max and the floor this derivation proposes:

  floor = min(FRACTION x median, DVFS x min)     (rounded down)

FRACTION 0.72 puts the floor at ~70-75 % of the typical rate (a GPU at half
its peers' rate - power-capped, a stuck DPM state - fails); DVFS 0.90 keeps it
10 % under the slowest healthy run seen, for clock and thermal variation the
runs here did not reach.  The shipped floors (api/clusterpolicy.py
WorkloadSpec) are set from this table; BASELINE.md carries it.

  python tools/floor_calibration.py --runs 60 --out gpurun_out/floors.json
"""

from __future__ import annotations

import argparse
import json
import math
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from amdgpu_operator import native  # noqa: E402

FRACTION = 0.72
DVFS = 0.90
RATE_STEPS = {"gemm": "bf16", "gemm_fp8": "fp8", "gemm_fp4": "fp4", "gemm_fp6": "fp6", "gemm_mxfp4": "mxfp4"}


def q(v: list[float], p: float) -> float:
    v = sorted(v)
    return v[min(len(v) - 1, max(0, int(round(p * (len(v) - 1)))))]


def derive(vals: list[float], step: float) -> dict:
    med, lo = q(vals, 0.5), min(vals)
    floor = math.floor(min(FRACTION * med, DVFS * lo) / step) * step
    return {"n": len(vals), "min": round(lo, 4), "p5": round(q(vals, 0.05), 4), "median": round(med, 4),
            "max": round(max(vals), 4), "floor": round(floor, 4), "floor_over_median": round(floor / med, 3)}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=60)
    ap.add_argument("--out", default="gpurun_out/floor_calibration.json")
    a = ap.parse_args()
    binary = str(native.binary("amdgpu-validator"))
    rows = []
    for i in range(a.runs):
        d = tempfile.mkdtemp(prefix="floors-")
        p = subprocess.run([binary, "--rendezvous", d, "--steps", "hip,gemm,gemm_fp8,gemm_fp4,gemm_fp6,gemm_mxfp4,hbm",
                            "--counter-gate"], capture_output=True, text=True, timeout=120)
        rep = json.loads(p.stdout.strip().splitlines()[-1])
        row = {"ok": rep.get("ok")}
        for s in rep.get("steps", []):
            dt = RATE_STEPS.get(s.get("name"))
            if dt:
                row[f"{dt}_tflops"] = s.get("tflops")
                row[f"{dt}_mfma_util"] = s.get("mfma_util")
                row[f"{dt}_gate"] = s.get("counter_gate")
            elif s.get("name") == "hbm":
                row["hbm_gbps"] = s.get("gbps")
        rows.append(row)
        if (i + 1) % 10 == 0:
            print(f"floor_calibration: {i + 1}/{a.runs}", file=sys.stderr, flush=True)
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    table = {}
    for key, step in ([(f"{dt}_tflops", 10.0) for dt in RATE_STEPS.values()] + [("hbm_gbps", 10.0)]
                      + [(f"{dt}_mfma_util", 0.01) for dt in RATE_STEPS.values()]):
        vals = [r[key] for r in rows if isinstance(r.get(key), (int, float))]
        if vals:
            table[key] = derive(vals, step)
    gates = {dt: sum(1 for r in rows if r.get(f"{dt}_gate") == "pass") for dt in RATE_STEPS.values()}
    out = {"runs": len(rows), "all_ok": all(r["ok"] for r in rows), "gates_passed": gates,
           "fraction": FRACTION, "dvfs": DVFS, "table": table}
    with open(a.out, "w") as f:
        json.dump({**out, "rows": rows}, f, indent=1)
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
