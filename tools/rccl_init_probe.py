"""RCCL communicator start-up on the GPU box: where ncclCommInitRank's time
goes and which environment knobs shorten it (the rccl step sits on the
time-to-Ready critical path for N >= 2).

Runs ``amdgpu-validator --steps hip,rccl`` at world 1 under each variant,
interleaved over rounds (one process per run), and once with NCCL_DEBUG=INFO
to capture RCCL's own "Init timings" breakdown.  Output: one JSON document.
"""
import json
import os
import re
import subprocess
import sys
import time

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
V = os.path.join(R, "amdgpu_operator/_native/amdgpu-validator")
OUT = sys.argv[1] if len(sys.argv) > 1 else os.path.join(R, "gpurun_out/rccl_init")
ROUNDS = int(sys.argv[2]) if len(sys.argv) > 2 else 3
os.makedirs(OUT, exist_ok=True)

VARIANTS = {
    "system-rccl": {"AMDGPU_RCCL_LIBRARY": ""},  # ROCm's librccl: 13-arch bundle, 5.3 GB uncompressed
    "gfx950-rccl": {},  # the validator's default on an all-gfx950 node: native/Makefile RCCL_SLIM
}
TIMING = re.compile(r"Init timings.*total ([\d.]+) \(kernels ([\d.]+), alloc ([\d.]+), bootstrap ([\d.]+), "
                    r"allgathers ([\d.]+), topo ([\d.]+), graphs ([\d.]+), connections ([\d.]+), rest ([\d.]+)\)")


def run(tag, env_extra, i, debug=False):
    env = dict(os.environ, **env_extra)
    if debug:
        env.update({"NCCL_DEBUG": "INFO", "NCCL_DEBUG_SUBSYS": "INIT,ENV,GRAPH"})
    argv = [V, "--steps", "hip,rccl", "--rccl-elems", str(1 << 24), "--rendezvous", f"/tmp/rip-{tag}-{i}",
            "--run-id", f"{tag}{i}"]
    t0 = time.perf_counter()
    if debug:  # straight to a file, so a stalled run still leaves its log
        log = os.path.join(OUT, f"debug_{tag}.log")
        with open(log, "w") as f:
            try:
                rc = subprocess.run(argv, stdout=f, stderr=subprocess.STDOUT, env=env, timeout=45).returncode
            except subprocess.TimeoutExpired:
                rc = "timeout"
        text = open(log).read()
        p = subprocess.CompletedProcess(argv, rc, text, "")
    else:
        p = subprocess.run(argv, capture_output=True, text=True, env=env, timeout=90)
    wall = time.perf_counter() - t0
    rec = {"variant": tag, "round": i, "wall_s": round(wall, 4), "rc": p.returncode}
    try:
        rep = json.loads(p.stdout.strip().splitlines()[-1])
        st = next(s for s in rep["steps"] if s["name"] == "rccl")
        rec.update({k: st.get(k) for k in ("lib_load_s", "comm_init_s", "init_wait_s", "first_allreduce_s", "checks_s",
                                       "finish_s", "seconds", "ok", "library")})
        rec["hip_s"] = next(s["seconds"] for s in rep["steps"] if s["name"] == "hip")
        rec["process_in_s"] = rep.get("seconds")
    except Exception:  # noqa: BLE001
        rec["stdout"] = p.stdout[-800:]
        rec["stderr"] = p.stderr[-800:]
    if debug:
        m = TIMING.search(p.stdout + p.stderr)
        if m:
            keys = ("total", "kernels", "alloc", "bootstrap", "allgathers", "topo", "graphs", "connections", "rest")
            rec["rccl_init_timings"] = dict(zip(keys, map(float, m.groups())))
    print(json.dumps(rec), flush=True)
    return rec


def page_in(path="/opt/rocm/lib/librccl.so.1"):
    """Read the library once (a fresh box pages its image in lazily)."""
    t0 = time.perf_counter()
    n = 0
    with open(os.path.realpath(path), "rb") as f:
        while True:
            b = f.read(1 << 24)
            if not b:
                break
            n += len(b)
    rec = {"page_in_bytes": n, "page_in_s": round(time.perf_counter() - t0, 3)}
    print(json.dumps(rec), flush=True)
    return rec


runs = [page_in(), page_in()]
for i in range(ROUNDS):
    for tag, env in VARIANTS.items():
        runs.append(run(tag, env, i))
for tag in ("system-rccl", "gfx950-rccl"):  # RCCL's own breakdown, after the timed rounds
    runs.append(run(tag, VARIANTS[tag], 99, debug=True))
    if runs[-1]["rc"] == "timeout":  # a stalled GPU process: run nothing more on the GPU
        break
summary = {}
for tag in VARIANTS:
    xs = sorted(r["comm_init_s"] for r in runs if r.get("variant") == tag and r.get("round") != 99
                and r.get("comm_init_s") is not None)
    ws = sorted(r["wall_s"] for r in runs if r.get("variant") == tag and r.get("round") != 99)
    summary[tag] = {"comm_init_median_s": xs[len(xs) // 2] if xs else None,
                    "wall_median_s": ws[len(ws) // 2] if ws else None,
                    "breakdown": next((r.get("rccl_init_timings") for r in runs
                                       if r.get("variant") == tag and r.get("round") == 99), None)}
json.dump({"summary": summary, "runs": runs}, open(os.path.join(OUT, "rccl_init_probe.json"), "w"), indent=1)
print(json.dumps(summary, indent=1))
