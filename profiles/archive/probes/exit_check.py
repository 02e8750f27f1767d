"""Run the native validator repeatedly and record exit codes (teardown crash hunt)."""
import collections, json, os, subprocess, sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
V = os.path.join(R, "amdgpu_operator/_native/amdgpu-validator")
for tag, args, env in [("gate", ["--steps", "hip,vecadd,gemm,hbm,xgmi", "--counter-gate"], {"AMDGPU_VALIDATOR_COUNTERS": "1"}),
                       ("plain", ["--steps", "hip,vecadd,gemm,hbm,xgmi"], {})]:
    rcs = collections.Counter()
    errs = []
    for i in range(12):
        p = subprocess.run([V, "--rendezvous", f"/tmp/rvx-{tag}-{i}", *args], capture_output=True, text=True,
                           env={**os.environ, **env}, timeout=60)
        ok = '"ok": true' in p.stdout
        rcs[(p.returncode, ok)] += 1
        if p.returncode != 0:
            errs.append(p.stderr[-1500:])
    print(json.dumps({"tag": tag, "rcs": {str(k): v for k, v in rcs.items()}, "errs": errs[:2]}), flush=True)
