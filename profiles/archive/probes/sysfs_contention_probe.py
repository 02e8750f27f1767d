"""Do KFD sysfs reads stall while another process starts the HIP runtime?

Operands read the KFD topology (N1 probe, GPU enumeration, CDI generation)
while the prespawned validator process initialises HIP.  This loops
``topology.enumerate_gpus`` / ``topology.probe`` / a plain-file read in one
thread, starts ``amdgpu-validator --steps hip`` 100 ms in, and reports the
call latencies before, during and after that start (ms).

``python tools/sysfs_contention_probe.py [--root /] [--runs 3]`` -> JSON.
"""

from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--root", default="/")
    ap.add_argument("--runs", type=int, default=3)
    a = ap.parse_args()
    from amdgpu_operator import native
    from amdgpu_operator.discovery import topology

    ops = {"enumerate_gpus": lambda: topology.enumerate_gpus(a.root), "probe": lambda: topology.probe(a.root),
           "read_file": lambda: open("/proc/self/stat").read()}
    runs = []
    for _ in range(a.runs):
        for name, fn in ops.items():
            samples: list[tuple[float, float]] = []
            stop = threading.Event()
            t0 = time.perf_counter()

            def loop():
                while not stop.is_set():
                    s = time.perf_counter()
                    fn()
                    samples.append((s - t0, time.perf_counter() - s))

            th = threading.Thread(target=loop)
            th.start()
            time.sleep(0.1)
            ts = time.perf_counter() - t0
            p = subprocess.run([str(native.binary("amdgpu-validator")), "--steps", "hip"], capture_output=True)
            te = time.perf_counter() - t0
            time.sleep(0.1)
            stop.set()
            th.join()

            def stat(xs):
                xs = [d for _, d in xs]
                return {"n": len(xs), "p50_ms": round(1e3 * statistics.median(xs), 3) if xs else None,
                        "max_ms": round(1e3 * max(xs), 2) if xs else None}

            runs.append({"op": name, "hip_process_s": round(te - ts, 3), "rc": p.returncode,
                         "before": stat([x for x in samples if x[0] < ts]),
                         "during": stat([x for x in samples if ts <= x[0] < te]),
                         "after": stat([x for x in samples if x[0] >= te])})
    print(json.dumps(runs, indent=1))


if __name__ == "__main__":
    main()
