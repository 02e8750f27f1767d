"""Wall-clock of process start-up paths on the GPU box (validator cold start)."""
import json
import os
import subprocess
import sys
import time

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
V = os.path.join(R, "amdgpu_operator/_native/amdgpu-validator")


def wall(argv, reps, env=None):
    out = []
    for i in range(reps):
        t0 = time.perf_counter()
        p = subprocess.run(argv, capture_output=True, text=True, timeout=60, env={**os.environ, **(env or {})})
        out.append({"wall": round(time.perf_counter() - t0, 4), "rc": p.returncode, "out": p.stdout.strip()[-300:]})
    return out


res = {}
for name in sys.argv[1:]:
    pass
res["sp_plain"] = wall([os.path.join(R, "build/sp/sp_plain")], 4)
res["sp_prof"] = wall([os.path.join(R, "build/sp/sp_prof")], 4)
res["validator_hip"] = wall([V, "--rendezvous", "/tmp/rvh", "--steps", "hip"], 4)
res["validator_hip_vecadd"] = wall([V, "--rendezvous", "/tmp/rvv", "--steps", "hip,vecadd"], 3)
res["validator_full_gate"] = wall([V, "--rendezvous", "/tmp/rvg", "--steps", "hip,vecadd,gemm,hbm,xgmi", "--counter-gate"],
                                  3, {"AMDGPU_VALIDATOR_COUNTERS": "1"})
print(json.dumps(res, indent=1))
