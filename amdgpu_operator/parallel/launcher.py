"""GPU process placement across the ranks of a multi-GPU job.

One process per GPU: under ``torch.distributed.run`` every rank owns one
MI355X (``LOCAL_RANK``).  The simulated cluster (rank 0) decides *when* a GPU
process must start (a validator pod's container, a workload rank); this
launcher makes the rank that owns that GPU start it as a child process and
return its result, using CPU-side ``gloo`` object collectives for the control
messages (GPU data never moves through them - the validator processes talk
RCCL over xGMI among themselves).

Protocol (all ranks loop in :meth:`DistributedLauncher.serve`):
  1. rank 0 broadcasts the batch of new requests (or ``stop``);
  2. each rank spawns the requests whose device it owns (``device % world``)
     without waiting for them - ranks of one validator run must be alive at the
     same time to rendezvous;
  3. ranks gather the results of processes that finished since the last round
     to rank 0, which completes the waiting callers.
"""

from __future__ import annotations

import os
import queue
import subprocess
import threading
import time
from concurrent.futures import Future

from ..nodeenv import REPORT_EARLY_ENV, PipeReader, ProcResult


class _Running:
    def __init__(self, rid: int, proc: subprocess.Popen, t0: float, early: bool):
        self.rid = rid
        self.proc = proc
        self.t0 = t0
        self.reader = PipeReader(proc)
        self.early = early  # done at the report (pipes closed), not at the exit

    def done(self) -> bool:
        return self.reader.eof() and (self.early or self.proc.poll() is not None)

    def result(self) -> ProcResult:
        if not self.early:
            self.proc.wait()
        return self.reader.result(self.t0)


def _spawn(argv: list[str], env: dict) -> subprocess.Popen:
    full = dict(os.environ)
    full.update(env or {})
    return subprocess.Popen(argv, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=full)


class DistributedLauncher:
    def __init__(self, rank: int, world: int, group=None, tick_s: float = 0.002):
        self.rank = rank
        self.world = world
        self.group = group
        self.tick_s = tick_s
        self._requests: queue.Queue = queue.Queue()
        self._futures: dict[int, Future] = {}
        self._next = 0
        self._lock = threading.Lock()
        self._stop_requested = threading.Event()
        self.rounds = 0

    # ----------------------------------------------------------- rank 0 API
    def __call__(self, argv, env, device, timeout) -> ProcResult:
        """Launcher callable for :class:`~amdgpu_operator.nodeenv.NodeEnv`."""
        if self.world == 1 or device is None:
            from ..nodeenv import run_local

            return run_local(argv, env, timeout)
        fut: Future = Future()
        with self._lock:
            rid = self._next
            self._next += 1
            self._futures[rid] = fut
        self._requests.put((rid, list(argv), dict(env or {}), int(device)))
        return fut.result(timeout=timeout + 30)

    def request_stop(self) -> None:
        self._stop_requested.set()

    # ------------------------------------------------------------ all ranks
    def serve(self) -> None:
        import torch.distributed as dist

        running: list[_Running] = []
        while True:
            batch: object = []
            if self.rank == 0:
                items = []
                while True:
                    try:
                        items.append(self._requests.get_nowait())
                    except queue.Empty:
                        break
                batch = "stop" if (self._stop_requested.is_set() and not items and not self._futures) else items
            box = [batch]
            dist.broadcast_object_list(box, src=0, group=self.group)
            batch = box[0]
            if batch == "stop":
                for r in running:
                    r.proc.kill()
                return
            for rid, argv, env, device in batch:
                if device % self.world == self.rank:
                    running.append(_Running(rid, _spawn(argv, env), time.perf_counter(),
                                            (env or {}).get(REPORT_EARLY_ENV) == "1"))
            done = []
            still = []
            for r in running:
                if not r.done():
                    still.append(r)
                    continue
                done.append((r.rid, r.result()))
            running = still
            gathered = [None] * self.world if self.rank == 0 else None
            dist.gather_object(done, gathered, dst=0, group=self.group)
            if self.rank == 0:
                for lst in gathered:
                    for rid, res in lst:
                        with self._lock:
                            fut = self._futures.pop(rid, None)
                        if fut is not None:
                            fut.set_result(res)
            self.rounds += 1
            if not batch and not running:
                time.sleep(self.tick_s)
