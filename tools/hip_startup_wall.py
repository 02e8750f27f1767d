"""Spawn-to-report wall time of fresh HIP processes under runtime settings
(interleaved, 7 reps): the probe binary and the plugin-pod validator
(`--steps hip,vecadd`).  Prints JSON medians."""
import json
import os
import statistics
import subprocess
import sys
import time

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
V = os.path.join(R, "amdgpu_operator/_native/amdgpu-validator")
P = os.path.join(R, "tools/native/hip_init_probe")
settings = {"default": {}, "deferred0": {"HIP_ENABLE_DEFERRED_LOADING": "0"}}
progs = {"probe": [P], "plugin_pod": [V, "--rendezvous", "/tmp/rv-wall", "--steps", "hip,vecadd"],
         "workload": [V, "--rendezvous", "/tmp/rv-wall2", "--steps", "hip,vecadd,gemm,mfma,hbm,xgmi", "--counter-gate"]}
res = {f"{p}/{s}": [] for p in progs for s in settings}
inproc = {k: [] for k in res}
for _ in range(7):
    for p, argv in progs.items():
        for s, env in settings.items():
            t = time.perf_counter()
            out = subprocess.run(argv, capture_output=True, text=True, env={**os.environ, **env}, timeout=120)
            res[f"{p}/{s}"].append(time.perf_counter() - t)
            try:
                inproc[f"{p}/{s}"].append(json.loads(out.stdout.strip().splitlines()[-1]).get("seconds"))
            except (ValueError, IndexError):
                pass
print(json.dumps({k: {"wall_median": round(statistics.median(v), 4), "walls": [round(x, 4) for x in v],
                      "in_process_median": (round(statistics.median([x for x in inproc[k] if x is not None]), 4)
                                            if any(x is not None for x in inproc[k]) else None)}
                  for k, v in res.items()}, indent=1))
