"""Find what holds the GIL for long stretches during a bring-up.

A probe thread sleeps 1 ms in a loop and records how late it wakes.  A late
wake-up means another thread held the GIL (or the process was descheduled);
at that moment the probe snapshots every thread's innermost frames, so the
holder's code is in the snapshot.  Runs ``--steps`` bring-ups as bench.py
does and prints the stalls longer than ``--min-ms`` with the stacks seen.

``python tools/gil_probe.py [--steps 3] [--min-ms 8] [bench.py flags]``
"""

from __future__ import annotations

import collections
import json
import os
import sys
import threading
import time
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class Probe:
    def __init__(self, min_ms: float):
        self.min_s = min_ms / 1e3
        self.stalls: list[dict] = []
        self.stop = threading.Event()
        self.t0 = time.perf_counter()
        self.th = threading.Thread(target=self.run, daemon=True, name="gil-probe")

    def run(self):
        me = threading.get_ident()
        names = {}
        while not self.stop.is_set():
            t = time.perf_counter()
            time.sleep(0.001)
            late = time.perf_counter() - t - 0.001
            if late < self.min_s:
                continue
            for th in threading.enumerate():
                names[th.ident] = th.name
            frames = {}
            for ident, fr in sys._current_frames().items():
                if ident == me:
                    continue
                st = traceback.extract_stack(fr, limit=6)
                frames[names.get(ident, str(ident))] = [f"{os.path.basename(f.filename)}:{f.lineno} {f.name}"
                                                        for f in st[-4:]]
            self.stalls.append({"at_s": round(t - self.t0, 4), "late_ms": round(late * 1e3, 1), "threads": frames})


def main():
    import bench

    steps, min_ms = 3, 8.0
    argv = sys.argv[1:]
    for flag in ("--steps", "--min-ms"):
        if flag in argv:
            i = argv.index(flag)
            v = argv[i + 1]
            del argv[i:i + 2]
            if flag == "--steps":
                steps = int(v)
            else:
                min_ms = float(v)
    sys.argv = ["bench.py", *argv]
    args = bench.parse()
    import tempfile

    has_gpu = bench.gpu_available()
    fake = args.fake_gpu or not has_gpu
    if has_gpu:
        import torch

        torch.cuda.set_device(0)
    work = tempfile.mkdtemp(prefix="gp-")
    bench.one_bring_up(args, 1, None, work, fake)  # warm-up
    out = []
    hot: collections.Counter = collections.Counter()
    for _ in range(steps):
        p = Probe(min_ms)
        p.th.start()
        r = bench.one_bring_up(args, 1, None, work, fake)
        p.stop.set()
        p.th.join()
        ttr = r["time_to_ready_s"]
        stalls = [s for s in p.stalls if s["at_s"] <= ttr + 0.05]
        for s in stalls:
            for name, fr in s["threads"].items():
                if fr and not any(w in fr[-1] for w in (" wait", " sleep", " select", " _wait", " get", " accept",
                                                        "readinto", " read", "recv", "serve_forever", " poll")):
                    hot[f"{name.split('-')[0]}: {fr[-1]}"] += s["late_ms"]
        out.append({"ttr_s": round(ttr, 4), "stall_ms_total": round(sum(s["late_ms"] for s in stalls), 1),
                    "stalls": stalls[:40]})
    print(json.dumps({"steps": out, "hot_frames_ms": dict(hot.most_common(30))}, indent=1))


if __name__ == "__main__":
    main()
