"""Where a validator process's start-up time goes (run on the GPU box).

Times the native validator from spawn to its start gate (no HIP call: exec,
dynamic linking, library constructors, rocprofiler-sdk tool registration)
and through its steps, with and without the counter-gate tool, and with a
do-nothing rocprofiler-sdk tool (tools/native/sdk_noop_tool.cpp, T2_MODE=0..3)
to separate the SDK's own start-up from the gate's.  Prints JSON.
"""
import json
import os
import resource
import statistics
import subprocess
import sys
import time

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N = os.path.join(R, "amdgpu_operator/_native")
V = os.path.join(N, "amdgpu-validator")
GATE = {"AMDGPU_VALIDATOR_COUNTERS": "1", "ROCP_TOOL_LIBRARIES": os.path.join(N, "libamdgpu_counter_gate.so"),
        "ROCPROFILER_METRICS_PATH": os.path.join(N, "gate-metrics")}
NOOP = sys.argv[1] if len(sys.argv) > 1 else None


def run(args, env, reps):
    walls, sys_s, flt, inproc = [], [], [], []
    for _ in range(reps):
        r0 = resource.getrusage(resource.RUSAGE_CHILDREN)
        t = time.perf_counter()
        p = subprocess.run([V, "--rendezvous", "/tmp/rv-probe", *args], capture_output=True, text=True,
                           env={**os.environ, **env}, timeout=60)
        walls.append(time.perf_counter() - t)
        r1 = resource.getrusage(resource.RUSAGE_CHILDREN)
        sys_s.append(r1.ru_stime - r0.ru_stime)
        flt.append(r1.ru_minflt - r0.ru_minflt)
        try:
            inproc.append(json.loads(p.stdout.strip().splitlines()[-1]).get("seconds"))
        except (ValueError, IndexError):
            inproc.append(None)
    med = statistics.median
    return {"wall_median": round(med(walls), 4), "walls": [round(w, 4) for w in walls], "sys_median": round(med(sys_s), 4),
            "minflt_median": med(flt), "in_process": inproc[-1], "rc": p.returncode}


with open("/tmp/gate-abort", "w") as f:
    f.write("abort")
out = {}
to_gate = ["--steps", "hip", "--start-gate", "/tmp/gate-abort"]
out["to_gate_plain"] = run(to_gate, {}, 5)
out["to_gate_counter_gate"] = run(to_gate, GATE, 5)
if NOOP:
    for m in ("0", "3"):
        out[f"to_gate_noop_tool_mode{m}"] = run(to_gate, {"ROCP_TOOL_LIBRARIES": NOOP, "T2_MODE": m}, 5)
out["hip_plain"] = run(["--steps", "hip"], {}, 5)
out["hip_counter_gate"] = run(["--steps", "hip", "--counter-gate"], GATE, 5)
full = ["--steps", "hip,vecadd,gemm,mfma,hbm,xgmi"]
out["full_plain"] = run(full, {}, 5)
out["full_counter_gate"] = run(full + ["--counter-gate"], GATE, 5)
print(json.dumps(out, indent=1))
