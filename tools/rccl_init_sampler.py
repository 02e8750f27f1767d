"""Where the validator's ncclCommInitRank time goes (no perf / root on the box).

Runs ``amdgpu-validator --steps hip,rccl`` (1 rank) ``--reps`` times and
samples, every millisecond, each thread's current syscall and kernel wait
channel (``/proc/<pid>/task/<tid>/{syscall,wchan}``).  Prints the child's
user/sys CPU, the validator's own RCCL timings, and the sample histogram:
user-space running, ioctl on /dev/kfd (allocations, queues), futex waits,
file I/O.

``python tools/rccl_init_sampler.py [--reps 3]`` -> JSON.
"""

from __future__ import annotations

import argparse
import collections
import json
import os
import resource
import subprocess
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SYSCALLS = {"0": "read", "1": "write", "3": "close", "7": "poll", "9": "mmap", "10": "mprotect", "11": "munmap",
            "16": "ioctl", "17": "pread64", "202": "futex", "232": "epoll_wait", "257": "openat",
            "230": "clock_nanosleep", "35": "nanosleep", "4": "stat", "5": "fstat", "262": "newfstatat",
            "running": "running(user)", "28": "madvise", "12": "brk", "25": "mremap", "281": "epoll_pwait",
            "271": "ppoll", "7 ": "poll"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    from amdgpu_operator import native

    argv = [str(native.binary("amdgpu-validator")), "--steps", "hip,rccl", "--rccl-elems", str(1 << 20),
            "--rendezvous", tempfile.mkdtemp(prefix="ris-")]
    runs = []
    for rep in range(a.reps):
        r0 = resource.getrusage(resource.RUSAGE_CHILDREN)
        t0 = time.perf_counter()
        p = subprocess.Popen(argv + ["--run-id", f"r{rep}"], stdout=subprocess.PIPE, stderr=subprocess.DEVNULL,
                             text=True)
        by_state: collections.Counter = collections.Counter()
        by_wchan: collections.Counter = collections.Counter()
        threads_seen = set()
        n = 0
        while p.poll() is None:
            try:
                for tid in os.listdir(f"/proc/{p.pid}/task"):
                    try:
                        sc = open(f"/proc/{p.pid}/task/{tid}/syscall").read().split()[0]
                        wc = open(f"/proc/{p.pid}/task/{tid}/wchan").read().strip() or "-"
                    except OSError:
                        continue
                    threads_seen.add(tid)
                    by_state[SYSCALLS.get(sc, "sys" + sc)] += 1
                    if sc != "running":
                        by_wchan[wc] += 1
                n += 1
            except OSError:
                pass
            time.sleep(0.001)
        out = p.stdout.read()
        wall = time.perf_counter() - t0
        r1 = resource.getrusage(resource.RUSAGE_CHILDREN)
        rccl = {}
        try:
            rep_j = json.loads(out.strip().splitlines()[-1])
            rccl = next((s for s in rep_j["steps"] if s["name"] == "rccl"), {})
        except (ValueError, IndexError, KeyError, StopIteration):
            pass
        runs.append({"wall_s": round(wall, 3), "user_s": round(r1.ru_utime - r0.ru_utime, 3),
                     "sys_s": round(r1.ru_stime - r0.ru_stime, 3), "samples": n, "threads": len(threads_seen),
                     "comm_init_s": rccl.get("comm_init_s"), "lib_load_s": rccl.get("lib_load_s"),
                     "thread_samples_by_syscall": dict(by_state.most_common(12)),
                     "blocked_wchan": dict(by_wchan.most_common(12))})
    print(json.dumps(runs, indent=1))


if __name__ == "__main__":
    main()
