"""Which threads of the bench process burn CPU during a bring-up.

In bench.py every operand of the simulated cluster is a thread of one Python
process, so a busy operand delays the others through the GIL.  This runs
``--steps`` bring-ups exactly as bench.py does and samples
``/proc/self/task/<tid>/schedstat`` (CPU ns per thread) every 5 ms,
naming threads through ``threading.enumerate()``.  Prints per-thread-group
CPU ms per bring-up (group = thread name without its pod/node suffix).

``python tools/bringup_threads.py [--steps 5] [bench.py flags]``
"""

from __future__ import annotations

import collections
import json
import os
import re
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def group(name: str) -> str:
    name = re.sub(r"-[0-9a-f]{5}\b", "", name)            # DaemonSet pod suffix
    name = re.sub(r"-[0-9a-f]{8}-\d+", "", name)         # validation pod run id
    name = re.sub(r"mi355x-node-0", "node", name)
    name = re.sub(r"_\d+$", "", name)                     # ThreadPoolExecutor workers
    name = re.sub(r"Thread-\d+.*", "Thread-N", name)
    return name


class Sampler:
    def __init__(self, period_s: float = 0.005):
        self.period = period_s
        self.names: dict[int, str] = {}
        self.cpu: dict[int, int] = {}
        self.first: dict[int, int] = {}
        self.stop = threading.Event()
        self.th = threading.Thread(target=self.run, daemon=True, name="sampler")

    def run(self):
        task_dir = "/proc/self/task"
        while not self.stop.wait(self.period):
            for t in threading.enumerate():
                if t.native_id is not None:
                    self.names[t.native_id] = t.name
            for tid in os.listdir(task_dir):
                try:
                    with open(f"{task_dir}/{tid}/schedstat") as f:
                        ns = int(f.read().split()[0])
                except (OSError, ValueError, IndexError):
                    continue
                tid_i = int(tid)
                self.first.setdefault(tid_i, ns)
                self.cpu[tid_i] = ns

    def totals(self) -> dict[str, float]:
        out: dict[str, float] = collections.Counter()
        for tid, ns in self.cpu.items():
            out[group(self.names.get(tid, f"native-{tid}"))] += (ns - self.first.get(tid, ns)) / 1e6
        return dict(out)


def main():
    import bench

    steps = 5
    argv = sys.argv[1:]
    if "--steps" in argv:
        i = argv.index("--steps")
        steps = int(argv[i + 1])
        del argv[i:i + 2]
    sys.argv = ["bench.py", *argv]
    args = bench.parse()
    import tempfile

    has_gpu = bench.gpu_available()
    fake = args.fake_gpu or not has_gpu
    if has_gpu:
        import torch

        torch.cuda.set_device(0)
    work = tempfile.mkdtemp(prefix="bt-")
    bench.one_bring_up(args, 1, None, work, fake)  # warm-up (page-in)
    rows = []
    for _ in range(steps):
        s = Sampler()
        s.th.start()
        t0 = time.perf_counter()
        r = bench.one_bring_up(args, 1, None, work, fake)
        s.stop.set()
        s.th.join()
        tot = s.totals()
        rows.append({"ttr_s": round(r["time_to_ready_s"], 4), "wall_s": round(time.perf_counter() - t0, 3),
                     "cpu_ms": {k: round(v, 1) for k, v in sorted(tot.items(), key=lambda kv: -kv[1]) if v >= 1.0}})
    agg: dict[str, list[float]] = collections.defaultdict(list)
    for r in rows:
        for k, v in r["cpu_ms"].items():
            agg[k].append(v)
    summary = {k: round(sum(v) / steps, 1) for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))}
    print(json.dumps({"steps": rows, "mean_cpu_ms_per_bringup": summary}, indent=1))


if __name__ == "__main__":
    main()
