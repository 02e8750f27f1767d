"""Hold-off between the node's amd-smi clients and a partition change.

A GPU's compute/memory partition can only be switched while nothing holds the
device: amd-smi answers ``AMDSMI_STATUS_BUSY`` to ``amdsmi_set_gpu_compute_
partition`` while another client has the GPU's DRM node open (the rule the
partition manager cites, partition/manager.py).  The operands that keep an
amd-smi session for their lifetime (device plugin, metrics exporter) are
paused off the node for a change; the driver container's health agent
(``amd-driver-health``, driver/manager.py ``publish_smi``) is not - it must
keep watching the driver through the reload a memory-partition change needs -
and opens amd-smi for a moment every minute.  Without a hand-off that poll
can land on the apply and fail it.

The hand-off, over files in the node's validations directory:

* a client writes its lease ``.smi-clients/<pid>.<thread>`` FIRST, then looks
  for ``.smi-hold``: present -> it drops the lease and skips this poll;
* the partition manager writes ``.smi-hold`` FIRST, then waits until no lease
  of a live process is left, applies, and removes the hold.

Whatever the interleaving, either the client sees the hold or the manager
sees the lease (each writes before it reads), so no poll overlaps an apply.
A lease whose process is gone is stale and ignored.
"""

from __future__ import annotations

import os
import threading
import time
from contextlib import contextmanager

HOLD = ".smi-hold"
CLIENTS = ".smi-clients"


def _dir(validations_dir: str) -> str:
    return os.path.join(validations_dir, CLIENTS)


def held(validations_dir: str) -> bool:
    return os.path.exists(os.path.join(validations_dir, HOLD))


@contextmanager
def client(validations_dir: str):
    """``with client(dir) as allowed:`` - open amd-smi only when ``allowed``."""
    d = _dir(validations_dir)
    os.makedirs(d, exist_ok=True)
    lease = os.path.join(d, f"{os.getpid()}.{threading.get_ident()}")
    with open(lease, "w") as f:
        f.write(str(time.time()))
    try:
        yield not held(validations_dir)
    finally:
        try:
            os.unlink(lease)
        except FileNotFoundError:
            pass


def _alive(pid: int) -> bool:
    try:
        with open(f"/proc/{pid}/stat") as f:
            return f.read().rsplit(")", 1)[1].split()[0] not in ("Z", "X")
    except (OSError, IndexError):
        return False


def live_clients(validations_dir: str) -> list[str]:
    """Leases of processes still running (stale ones are removed)."""
    d = _dir(validations_dir)
    try:
        names = os.listdir(d)
    except FileNotFoundError:
        return []
    out = []
    for n in names:
        try:
            pid = int(n.split(".", 1)[0])
        except ValueError:
            continue
        if _alive(pid):
            out.append(n)
        else:
            try:
                os.unlink(os.path.join(d, n))
            except FileNotFoundError:
                pass
    return out


def hold(validations_dir: str, reason: str) -> None:
    os.makedirs(validations_dir, exist_ok=True)
    path = os.path.join(validations_dir, HOLD)
    with open(path + ".tmp", "w") as f:
        f.write(reason)
    os.replace(path + ".tmp", path)


def release(validations_dir: str) -> None:
    try:
        os.unlink(os.path.join(validations_dir, HOLD))
    except FileNotFoundError:
        pass


def wait_clients_gone(validations_dir: str, timeout: float, poll_s: float = 0.01) -> list[str]:
    """After :func:`hold`: wait until no amd-smi client is in a poll; returns
    the leases left at ``timeout``."""
    deadline = time.monotonic() + timeout
    while True:
        left = live_clients(validations_dir)
        if not left or time.monotonic() >= deadline:
            return left
        time.sleep(poll_s)
