"""Cost of starting a child process from the bench process.

Every GPU step of a bring-up (validator processes, the OCI hook, the CDI
generator) is a child of the bench process, which imports torch and holds a
HIP context (the bench contract's ``torch.cuda.synchronize``).  This times
``subprocess.run(["/bin/true"])`` after each of those stages: medians of
``--reps`` spawns, in ms.

``python tools/spawn_cost_probe.py [--reps 20]`` -> JSON on stdout.
"""

from __future__ import annotations

import argparse
import json
import statistics
import subprocess
import time


def spawn_ms(reps: int, **kw) -> float:
    xs = []
    for _ in range(reps):
        t0 = time.perf_counter()
        subprocess.run(["/bin/true"], **kw)
        xs.append(time.perf_counter() - t0)
    return round(1e3 * statistics.median(xs), 3)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    out = {"plain": spawn_ms(a.reps), "plain_close_fds_false": spawn_ms(a.reps, close_fds=False)}
    import torch

    out["torch_imported"] = spawn_ms(a.reps)
    if torch.cuda.is_available():
        torch.cuda.set_device(0)
        x = torch.ones(1 << 20, device="cuda")
        torch.cuda.synchronize()
        out["hip_context"] = spawn_ms(a.reps)
        out["hip_context_close_fds_false"] = spawn_ms(a.reps, close_fds=False)
        del x
    try:
        import resource

        out["maxrss_mib"] = round(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1024, 1)
    except Exception:  # noqa: BLE001
        pass
    with open("/proc/self/status") as f:
        out["vm"] = {k: v.strip() for k, v in (line.split(":", 1) for line in f) if k in ("VmSize", "VmRSS", "VmPTE")}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
