"""What each operand's start-up work costs on this machine (wall and CPU).

In the bench every operand runs as threads of one Python process, so CPU
spent by one operand (GFD labels, the exporter's amd-smi start, the toolkit's
CDI generation) delays the others that are on the time-to-Ready path.  This
times each piece alone against the real sysfs: medians of ``--reps`` runs.

``python tools/operand_cost_probe.py [--root /] [--reps 5]`` -> JSON on stdout.
"""

from __future__ import annotations

import argparse
import json
import os
import shutil
import statistics
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps: int) -> dict:
    walls, cpus = [], []
    for _ in range(reps):
        c0, t0 = time.process_time(), time.perf_counter()
        fn()
        walls.append(time.perf_counter() - t0)
        cpus.append(time.process_time() - c0)
    return {"wall_ms": round(1e3 * statistics.median(walls), 2), "cpu_ms": round(1e3 * statistics.median(cpus), 2),
            "first_wall_ms": round(1e3 * walls[0], 2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--root", default="/")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    from amdgpu_operator.discovery import labels as L
    from amdgpu_operator.discovery import topology
    from amdgpu_operator.nodeenv import NodeEnv
    from amdgpu_operator.toolkit import install as tk

    work = tempfile.mkdtemp(prefix="opcost-")
    env = NodeEnv("probe", None, host_root=a.root, validations_dir=os.path.join(work, "val"),
                  cdi_dir=os.path.join(work, "cdi"), containerd_config=os.path.join(work, "containerd/config.toml"),
                  install_dir=os.path.join(work, "amd"))
    os.makedirs(os.path.dirname(env.containerd_config), exist_ok=True)
    with open(env.containerd_config, "w") as f:
        f.write("version = 2\n")
    out: dict = {"root": a.root, "gpus": len(topology.enumerate_gpus(a.root))}
    out["probe"] = timed(lambda: topology.probe(a.root), a.reps)
    out["enumerate_gpus"] = timed(lambda: topology.enumerate_gpus(a.root), a.reps)
    out["links"] = timed(lambda: topology.links(a.root), a.reps)
    out["nfd_labels"] = timed(lambda: L.nfd_labels(a.root), a.reps)
    out["gfd_labels"] = timed(lambda: L.gfd_labels(topology.enumerate_gpus(a.root), a.root), a.reps)
    out["generate_cdi"] = timed(lambda: tk.generate_cdi(env, os.path.join(env.cdi_dir, "amd.com-gpu.json")), a.reps)
    out["toolkit_install"] = timed(lambda: tk.install(env), a.reps)
    try:
        from amdgpu_operator.exporter.metrics import SmiSource

        def smi():
            s = SmiSource()
            s.close()

        out["smi_source_open_close"] = timed(smi, a.reps)
    except Exception as e:  # noqa: BLE001 - no amd-smi here
        out["smi_source_open_close"] = {"error": str(e)[:200]}
    shutil.rmtree(work, ignore_errors=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
