"""Wait for a file to appear: inotify on its directory, polling as a backstop.

The operands hand readiness to each other through files in the validations
directory (``/run/amd/validations`` on the host, mounted into every operand
pod with HostToContainer propagation).  A ready file is written as a temp
file and renamed into place (validator/validate.py ``write_ready``), which
inotify reports on the directory as IN_MOVED_TO, so a waiter wakes when the
file lands instead of at its next poll.  inotify sees writes from every
container because they all share the host directory's inode.  The directory
is re-checked every ``poll_s`` anyway (a directory created after the watch
started, filesystems without inotify).
"""

from __future__ import annotations

import ctypes
import ctypes.util
import os
import select
import threading
import time

IN_CLOSE_WRITE = 0x00000008
IN_MOVED_TO = 0x00000080
IN_CREATE = 0x00000100
IN_NONBLOCK = 0o4000
IN_CLOEXEC = 0o2000000

_libc = None

# Closing an inotify instance waits for an SRCU grace period in the kernel
# (fsnotify group teardown): 15-40 ms, measured here and on the MI355X box.
# Every wait below ends with a close, so a waiter that found its file would
# sit that long before acting on it (the validator saw the kubelet's devices
# ~40 ms after its query returned them).  Closes are therefore handed to one
# background thread per process; os.close releases the interpreter lock.
_closer_lock = threading.Lock()
_closer_q = None


def _closer(q) -> None:
    while True:
        fd = q.get()
        try:
            os.close(fd)
        except OSError:
            pass


def _close_later(fd: int) -> None:
    global _closer_q
    with _closer_lock:
        if _closer_q is None:
            import queue

            _closer_q = queue.SimpleQueue()
            threading.Thread(target=_closer, args=(_closer_q,), daemon=True, name="inotify-closer").start()
        _closer_q.put(fd)


def _reset_closer_in_child() -> None:  # a forked child has no closer thread: it starts its own
    global _closer_q, _closer_lock
    _closer_q = None
    _closer_lock = threading.Lock()


os.register_at_fork(after_in_child=_reset_closer_in_child)


def _lib():
    global _libc
    if _libc is None:
        lib = ctypes.CDLL(ctypes.util.find_library("c") or "libc.so.6", use_errno=True)
        lib.inotify_init1.argtypes = [ctypes.c_int]
        lib.inotify_add_watch.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_uint32]
        _libc = lib
    return _libc


class DirWatch:
    """inotify watch on one directory (entries created, written or moved in)."""

    def __init__(self, directory: str):
        self.fd = -1
        try:
            lib = _lib()
            fd = lib.inotify_init1(IN_NONBLOCK | IN_CLOEXEC)
            if fd < 0:
                return
            if lib.inotify_add_watch(fd, os.fsencode(directory), IN_CREATE | IN_MOVED_TO | IN_CLOSE_WRITE) < 0:
                os.close(fd)
                return
            self.fd = fd
        except (OSError, AttributeError):
            self.fd = -1

    @property
    def active(self) -> bool:
        return self.fd >= 0

    def wait(self, timeout: float) -> bool:
        """Block up to ``timeout`` for an event; drain it.  True on an event."""
        if self.fd < 0:
            time.sleep(max(0.0, timeout))
            return False
        r, _, _ = select.select([self.fd], [], [], max(0.0, timeout))
        if not r:
            return False
        try:
            while os.read(self.fd, 65536):
                pass
        except BlockingIOError:
            pass
        return True

    def close(self) -> None:
        if self.fd >= 0:
            _close_later(self.fd)  # not on the caller's time (see _close_later)
            self.fd = -1


def wait_for_file(path: str, timeout: float, stop: threading.Event | None = None, poll_s: float = 1.0,
                  check=os.path.exists) -> bool:
    """True once ``check(path)`` holds (default: the file exists); False on
    timeout or ``stop``.  Wakes on inotify events in the file's directory and
    re-checks at least every ``poll_s`` (every 50 ms when a ``stop`` event is
    given, to notice it; every 10 ms without inotify)."""
    deadline = time.monotonic() + timeout
    if check(path):
        return True
    directory = os.path.dirname(path) or "."
    os.makedirs(directory, exist_ok=True)
    w = DirWatch(directory)
    period = poll_s if w.active else min(poll_s, 0.01)
    if stop is not None:
        period = min(period, 0.05)
    try:
        while True:
            if check(path):  # checked after the watch is armed: a file landing in between is not missed
                return True
            left = deadline - time.monotonic()
            if left <= 0 or (stop is not None and stop.is_set()):
                return False
            w.wait(min(left, period))
    finally:
        w.close()
