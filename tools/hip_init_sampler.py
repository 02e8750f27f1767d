"""Poor man's profiler of a fresh HIP process's start-up (no perf / root on the
box): sample every thread's current syscall and wchan each millisecond, and
report the child's user/sys CPU.  Answers: is HIP start-up CPU work, or time
spent blocked in the kernel driver (ioctl on /dev/kfd)?"""
import collections
import json
import os
import resource
import subprocess
import sys
import time

P = sys.argv[1]
SYSCALLS = {"0": "read", "1": "write", "3": "close", "7": "poll", "9": "mmap", "10": "mprotect", "11": "munmap",
            "16": "ioctl", "17": "pread64", "202": "futex", "232": "epoll_wait", "257": "openat", "230": "clock_nanosleep",
            "35": "nanosleep", "4": "stat", "5": "fstat", "262": "newfstatat", "running": "running(user)"}
out = []
for rep in range(3):
    r0 = resource.getrusage(resource.RUSAGE_CHILDREN)
    t0 = time.perf_counter()
    p = subprocess.Popen([P], stdout=subprocess.PIPE, stderr=subprocess.DEVNULL)
    samples = collections.Counter()
    wchans = collections.Counter()
    n = 0
    while p.poll() is None:
        try:
            for tid in os.listdir(f"/proc/{p.pid}/task"):
                try:
                    sc = open(f"/proc/{p.pid}/task/{tid}/syscall").read().split()[0]
                    wc = open(f"/proc/{p.pid}/task/{tid}/wchan").read().strip() or "-"
                except OSError:
                    continue
                samples[SYSCALLS.get(sc, sc)] += 1
                wchans[wc] += 1
            n += 1
        except OSError:
            pass
        time.sleep(0.001)
    wall = time.perf_counter() - t0
    r1 = resource.getrusage(resource.RUSAGE_CHILDREN)
    out.append({"wall": round(wall, 4), "user": round(r1.ru_utime - r0.ru_utime, 4),
                "sys": round(r1.ru_stime - r0.ru_stime, 4), "sample_rounds": n,
                "syscalls": samples.most_common(8), "wchan": wchans.most_common(8),
                "stdout": p.stdout.read().decode()[:400]})
print(json.dumps(out, indent=1))
