"""Time the native validator process under different configurations (GPU box)."""
import json, os, subprocess, sys, time
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
V = os.path.join(R, "amdgpu_operator/_native/amdgpu-validator")

def run(args, env_extra, tag, reps=2):
    out = []
    for i in range(reps):
        env = dict(os.environ); env.update(env_extra)
        t0 = time.perf_counter()
        p = subprocess.run([V, "--rendezvous", f"/tmp/rv-{tag}-{i}", "--run-id", f"{tag}{i}", *args], capture_output=True, text=True, env=env, timeout=120)
        wall = time.perf_counter() - t0
        try:
            rep = json.loads(p.stdout.strip().splitlines()[-1])
        except Exception:
            rep = {"raw": p.stdout[-500:], "err": p.stderr[-1500:]}
        steps = {s["name"]: round(s["seconds"], 4) for s in rep.get("steps", [])}
        extra = {k: v for s in rep.get("steps", []) for k, v in s.items() if k in ("comm_init_s", "tflops", "gbps", "counter_gate", "read_gbps")}
        out.append({"wall": round(wall, 4), "in_process": rep.get("seconds"), "ok": rep.get("ok"), "steps": steps, **extra})
    print(json.dumps({"tag": tag, "args": args, "env": env_extra, "runs": out}), flush=True)

run(["--steps", "hip"], {}, "hip-only")
run(["--steps", "hip,rccl"], {}, "rccl-default")
run(["--steps", "hip,rccl"], {"NCCL_IB_DISABLE": "1"}, "rccl-noib")


run([], {}, "full-default")
run(["--counter-gate"], {"AMDGPU_VALIDATOR_COUNTERS": "1"}, "full-gate")
run(["--steps", "hip,gemm", "--counter-gate"], {"AMDGPU_VALIDATOR_COUNTERS": "1"}, "gemm-gate")
env = {"NCCL_DEBUG": "INFO", "NCCL_DEBUG_SUBSYS": "INIT,ENV"}
p = subprocess.run([V, "--steps", "hip,rccl", "--rendezvous", "/tmp/rv-dbg"], capture_output=True, text=True, env={**os.environ, **env}, timeout=120)
open(os.path.join(R, "gpurun_out/s6/rccl_debug.txt"), "w").write(p.stdout + "\n----\n" + p.stderr)
