"""Validator process wall time with and without the N7 counter gate, and the
gate's start-up options (symbol tracing, lazy counter config), interleaved.

Run on the GPU box: python3 tools/gate_startup.py [reps] > out.json
"""
import json
import os
import random
import statistics
import subprocess
import sys
import time

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
V = os.path.join(R, "amdgpu_operator/_native/amdgpu-validator")
STEPS = "hip,vecadd,gemm,hbm,xgmi"
MODES = {
    "no_gate": ([], {}),
    "gate": (["--counter-gate"], {"AMDGPU_VALIDATOR_COUNTERS": "1"}),
    "gate_symbols": (["--counter-gate"], {"AMDGPU_VALIDATOR_COUNTERS": "1", "AMDGPU_GATE_KERNEL_NAMES": "1"}),
    "gate_sdk_metrics": (["--counter-gate"], {"AMDGPU_VALIDATOR_COUNTERS": "1",
                                              "ROCPROFILER_METRICS_PATH": "/opt/rocm/share/rocprofiler-sdk"}),
    "gate_lazy": (["--counter-gate"], {"AMDGPU_VALIDATOR_COUNTERS": "1", "AMDGPU_GATE_LAZY_CONFIG": "1"}),
    "gate_symbols_lazy": (["--counter-gate"], {"AMDGPU_VALIDATOR_COUNTERS": "1", "AMDGPU_GATE_KERNEL_NAMES": "1",
                                               "AMDGPU_GATE_LAZY_CONFIG": "1"}),
}


def one(mode: str) -> dict:
    args, env = MODES[mode]
    t0 = time.perf_counter()
    p = subprocess.run([V, "--rendezvous", f"/tmp/gs-{os.getpid()}", "--steps", STEPS, *args], capture_output=True,
                       text=True, timeout=60, env={**os.environ, **env})
    wall = time.perf_counter() - t0
    rep = json.loads(p.stdout.strip().splitlines()[-1]) if p.stdout.strip() else {}
    steps = {s["name"]: s for s in rep.get("steps", [])}
    g = steps.get("gemm", {})
    return {"wall": wall, "rc": p.returncode, "ok": rep.get("ok"), "in_process": rep.get("seconds"),
            "hip": steps.get("hip", {}).get("seconds"), "gemm": g.get("seconds"),
            "gate": g.get("counter_gate"), "gate_seconds": g.get("gate_seconds"),
            "gate_config_seconds": g.get("gate_config_seconds")}


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    runs = {m: [] for m in MODES}
    for m in MODES:  # page-in of every path
        one(m)
    rng = random.Random(7)
    for _ in range(reps):
        order = list(MODES)
        rng.shuffle(order)  # no mode always follows the same predecessor
        for m in order:
            time.sleep(0.2)  # let the previous process's teardown finish
            runs[m].append(one(m))
    out = {}
    for m, rs in runs.items():
        med = lambda k: statistics.median([r[k] for r in rs if isinstance(r.get(k), (int, float))] or [float("nan")])
        out[m] = {"wall_median": med("wall"), "in_process_median": med("in_process"), "hip_median": med("hip"),
                  "gemm_median": med("gemm"), "gate_seconds_median": med("gate_seconds"),
                  "gate_config_seconds_median": med("gate_config_seconds"),
                  "gates": sorted({str(r["gate"]) for r in rs}), "rcs": sorted({r["rc"] for r in rs}),
                  "walls": [round(r["wall"], 4) for r in rs]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
