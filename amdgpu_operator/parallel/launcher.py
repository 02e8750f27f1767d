"""GPU process placement across the ranks of a multi-GPU job.

One process per GPU: under ``torch.distributed.run`` every rank owns one
MI355X (``LOCAL_RANK``).  The simulated cluster (rank 0) decides *when* a GPU
process must start (a validator pod's container, a workload rank); this
launcher makes the rank that owns that GPU start it as a child process and
return its result.  GPU data never moves through it - the validator
processes talk RCCL over xGMI among themselves.

Control messages go through the job's TCP key-value store (the one
``torch.distributed`` rendezvoused on), not through collectives, so nothing
polls: round 2's loop ran a gloo broadcast + gather every 2 ms on every rank,
rank 0 - the process hosting the whole simulated cluster - included.

  * rank 0 runs processes for its own GPUs directly, and publishes any other
    request as ``req/<n>`` (sequence number n);
  * every other rank blocks in the store on the next ``req/<n>`` and starts
    the process if it owns the device (``device % world``) - without waiting
    for it: ranks of one validator run must be alive at the same time;
  * a per-process thread publishes the result as ``res/<id>`` once the child
    reported (``AMDGPU_REPORT_EARLY``) or exited; the caller on rank 0 blocks
    on that key.

Every blocking call uses a store connection of its own thread.
"""

from __future__ import annotations

import os
import pickle
import secrets
import subprocess
import threading
import time
from datetime import timedelta

from ..nodeenv import REPORT_EARLY_ENV, PipeReader, ProcResult

STOP = b"stop"


class _Running:
    def __init__(self, rid: int, proc: subprocess.Popen, t0: float, early: bool):
        self.rid = rid
        self.proc = proc
        self.t0 = t0
        self.reader = PipeReader(proc)
        self.early = early  # done at the report (pipes closed), not at the exit

    def wait(self) -> None:
        """Until the report (pipes closed) when ``early``, else the exit."""
        self.reader.join(None)
        if not self.early:
            self.proc.wait()

    def result(self) -> ProcResult:
        if not self.early:
            self.proc.wait()
        return self.reader.result(self.t0)


def _spawn(argv: list[str], env: dict) -> subprocess.Popen:
    full = dict(os.environ)
    full.update(env or {})
    return subprocess.Popen(argv, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=full)


class DistributedLauncher:
    _generation = 0  # constructed in lockstep on every rank: one key namespace per instance

    def __init__(self, rank: int, world: int, group=None, store_addr: tuple[str, int] | None = None):
        self.rank = rank
        self.world = world
        DistributedLauncher._generation += 1
        nonce = [secrets.token_hex(4) if rank == 0 else None]
        if world > 1:
            import torch.distributed as dist

            dist.broadcast_object_list(nonce, src=0, group=group)
        self.prefix = f"amdgpu-launch/{nonce[0]}/{DistributedLauncher._generation}/"
        self.addr = store_addr or (os.environ.get("MASTER_ADDR", "127.0.0.1"), int(os.environ.get("MASTER_PORT", "0")))
        self._local = threading.local()
        self._seq = 0
        self._lock = threading.Lock()
        self._stop_requested = threading.Event()
        self._stop_published = False
        self.rounds = 0  # requests this rank served

    def _store(self):
        """This thread's own connection to the job's store (blocking gets
        must not share a socket with other threads' calls)."""
        st = getattr(self._local, "store", None)
        if st is None:
            import torch.distributed as dist

            st = dist.TCPStore(self.addr[0], self.addr[1], is_master=False, timeout=timedelta(hours=2))
            self._local.store = st
        return st

    # ----------------------------------------------------------- rank 0 API
    def __call__(self, argv, env, device, timeout) -> ProcResult:
        """Launcher callable for :class:`~amdgpu_operator.nodeenv.NodeEnv`."""
        if self.world == 1 or device is None or int(device) % self.world == self.rank:
            from ..nodeenv import run_local

            return run_local(argv, env, timeout)
        with self._lock:
            n = self._seq
            self._seq += 1
        st = self._store()
        st.set(f"{self.prefix}req/{n}", pickle.dumps((n, list(argv), dict(env or {}), int(device))))
        key = f"{self.prefix}res/{n}"
        try:
            st.wait([key], timedelta(seconds=timeout + 30))
        except Exception as e:  # noqa: BLE001 - the store's timeout (DistStoreError / RuntimeError)
            return ProcResult(124, "", f"no result from rank {int(device) % self.world}: {e}", float(timeout))
        return pickle.loads(st.get(key))

    def request_stop(self) -> None:
        self._stop_requested.set()

    def _publish_stop(self) -> None:
        with self._lock:
            if self._stop_published:
                return
            self._stop_published = True
            n = self._seq
            self._seq += 1
        self._store().set(f"{self.prefix}req/{n}", STOP)

    # ------------------------------------------------------------ all ranks
    def serve(self) -> None:
        """Rank 0: until :meth:`request_stop`.  Other ranks: run the requests
        for their GPUs until rank 0 publishes the stop record."""
        if self.world == 1:
            return
        if self.rank == 0:
            self._stop_requested.wait()
            self._publish_stop()
            return
        st = self._store()
        running: list[subprocess.Popen] = []
        n = 0
        while True:
            data = st.get(f"{self.prefix}req/{n}")  # blocks in the store until rank 0 writes it
            n += 1
            if data == STOP:
                for p in running:
                    if p.poll() is None:
                        p.kill()
                return
            rid, argv, env, device = pickle.loads(data)
            if device % self.world != self.rank:
                continue
            self.rounds += 1
            r = _Running(rid, _spawn(argv, env), time.perf_counter(), (env or {}).get(REPORT_EARLY_ENV) == "1")
            running.append(r.proc)
            threading.Thread(target=self._finish, args=(r,), daemon=True, name=f"launch-{rid}").start()

    def _finish(self, r: "_Running") -> None:
        r.wait()
        self._store().set(f"{self.prefix}res/{r.rid}", pickle.dumps(r.result()))
