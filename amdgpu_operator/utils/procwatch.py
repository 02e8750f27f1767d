"""Which GPU tools outside the bring-up ran while it was being timed.

A node's time-to-Ready is the time of its GPU processes' start-up, and those
serialise in the kernel driver with anything else that opens the GPU at the
same moment: an ``amd-smi`` / ``rocm-smi`` poll of a monitoring agent takes
the driver's locks and reads the SMU for hundreds of milliseconds.  Such a
poll is not part of the operator, so a bring-up it overlapped is slow for a
reason the bring-up's own record cannot show.  This watcher lists the
processes of those tools while the bench runs, from a process of its own
(a /proc scan every 20 ms would cost the harness's interpreter lock, which
the simulated API server and kubelets share), and reports per process
``[name, pid, first seen, last seen]`` in ``time.time()`` seconds, so each
timed bring-up can be checked for overlap.

``python -m amdgpu_operator.utils.procwatch OUT [PERIOD_S]``: append one JSON
line per finished process to OUT until SIGTERM.
"""

from __future__ import annotations

import json
import os
import signal
import subprocess
import sys
import time

# process names (``/proc/<pid>/comm``, 15 characters) of GPU tools that open
# the device or the SMU; python entry points show as their script name
TOOLS = ("amd-smi", "amdsmi", "rocm-smi", "rocm_smi.py", "rocminfo", "rocprofv3", "rocprof", "rdc", "rdcd",
         "amd-metrics-exp", "gpuagent")


def scan(own: set[int]) -> dict[int, str]:
    out = {}
    try:
        pids = [int(p) for p in os.listdir("/proc") if p.isdigit()]
    except OSError:
        return out
    for pid in pids:
        if pid in own:
            continue
        try:
            with open(f"/proc/{pid}/comm") as f:
                comm = f.read().strip()
        except OSError:
            continue
        if comm.startswith(TOOLS) or comm in TOOLS:
            out[pid] = comm
            continue
        if comm.startswith("python"):
            try:
                with open(f"/proc/{pid}/cmdline", "rb") as f:
                    argv = f.read().split(b"\0")
            except OSError:
                continue
            for a in argv[1:3]:
                base = os.path.basename(a.decode(errors="replace"))
                if base.startswith(("amd-smi", "amdsmi", "rocm-smi", "rocm_smi")):
                    out[pid] = base
                    break
    return out


def main(argv: list[str]) -> int:
    out_path = argv[0]
    period = float(argv[1]) if len(argv) > 1 else 0.02
    own = {os.getpid(), os.getppid()}
    live: dict[int, list] = {}
    stop = []
    signal.signal(signal.SIGTERM, lambda *_: stop.append(1))

    def flush(items):
        if not items:
            return
        with open(out_path, "a") as f:
            for rec in items:
                f.write(json.dumps(rec) + "\n")

    while not stop:
        now = time.time()
        seen = scan(own)
        for pid, name in seen.items():
            if pid in live:
                live[pid][3] = now
            else:
                live[pid] = [name, pid, now, now]
        flush([live.pop(pid) for pid in [p for p in live if p not in seen]])
        time.sleep(period)
    flush(list(live.values()))
    return 0


class ToolWatch:
    """The watcher as a child process of the bench (start / intervals / stop)."""

    def __init__(self, path: str, period_s: float = 0.02):
        self.path = path
        open(path, "w").close()
        self.proc = subprocess.Popen([sys.executable, "-m", "amdgpu_operator.utils.procwatch", path, str(period_s)],
                                     stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)

    def intervals(self) -> list[list]:
        out = []
        try:
            with open(self.path) as f:
                for ln in f:
                    try:
                        out.append(json.loads(ln))
                    except ValueError:
                        continue
        except OSError:
            pass
        return out

    def overlapping(self, t0: float, t1: float, slack_s: float = 0.05) -> list[dict]:
        """Tool processes alive within [t0 - slack, t1] (time.time()); a process
        still running is not in the file yet, so a finished-first read of a
        step is completed by :meth:`stop`."""
        return [{"tool": n, "pid": p, "from_s": round(a - t0, 3), "to_s": round(b - t0, 3)}
                for n, p, a, b in self.intervals() if b >= t0 - slack_s and a <= t1]

    def stop(self) -> None:
        if self.proc.poll() is None:
            self.proc.terminate()
            try:
                self.proc.wait(5)
            except subprocess.TimeoutExpired:
                self.proc.kill()


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
