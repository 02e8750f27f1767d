"""utils/fswait.py: ready-file waits wake on inotify, not on the next poll."""

import os
import threading
import time

from amdgpu_operator.utils import fswait


def _later(delay, fn):
    t = threading.Timer(delay, fn)
    t.start()
    return t


def test_wakes_on_rename_into_place(tmp_path):
    path = str(tmp_path / "toolkit-ready")
    stamp = {}

    def write():
        with open(path + ".tmp", "w") as f:
            f.write("{}")
        stamp["t"] = time.perf_counter()
        os.replace(path + ".tmp", path)

    _later(0.2, write)
    assert fswait.wait_for_file(path, 5, poll_s=10.0)  # a 10 s poll would miss it: the event wakes it
    assert time.perf_counter() - stamp["t"] < 0.05


def test_existing_file_and_timeout(tmp_path):
    path = str(tmp_path / "x")
    open(path, "w").close()
    assert fswait.wait_for_file(path, 0.01)
    t0 = time.monotonic()
    assert not fswait.wait_for_file(str(tmp_path / "never"), 0.2, poll_s=0.05)
    assert 0.15 < time.monotonic() - t0 < 2.0


def test_stop_event_ends_the_wait(tmp_path):
    stop = threading.Event()
    _later(0.1, stop.set)
    t0 = time.monotonic()
    assert not fswait.wait_for_file(str(tmp_path / "never"), 30, stop=stop, poll_s=10.0)
    assert time.monotonic() - t0 < 1.0


def test_check_predicate_and_missing_directory(tmp_path):
    path = str(tmp_path / "sub" / "ready")  # the directory does not exist yet
    _later(0.1, lambda: open(path, "w").write("partial"))
    _later(0.2, lambda: open(path, "w").write("done"))
    assert fswait.wait_for_file(path, 5, poll_s=10.0, check=lambda p: os.path.exists(p) and open(p).read() == "done")


def test_polls_without_inotify(tmp_path, monkeypatch):
    monkeypatch.setattr(fswait.DirWatch, "__init__", lambda self, d: setattr(self, "fd", -1))
    path = str(tmp_path / "f")
    _later(0.1, lambda: open(path, "w").close())
    assert fswait.wait_for_file(path, 5, poll_s=10.0)  # falls back to a 10 ms poll


def test_dir_watch_sees_create(tmp_path):
    w = fswait.DirWatch(str(tmp_path))
    try:
        assert w.active
        assert not w.wait(0.05)
        _later(0.05, lambda: open(str(tmp_path / "a"), "w").close())
        assert w.wait(2.0)
    finally:
        w.close()


def test_close_does_not_wait_for_the_kernel(tmp_path):
    """Closing an inotify instance waits for an SRCU grace period (15-40 ms);
    DirWatch.close hands it to a background thread, and the fd is closed."""
    import os
    import time

    from amdgpu_operator.utils.fswait import DirWatch

    fds, t = [], []
    for _ in range(5):
        w = DirWatch(str(tmp_path))
        assert w.active
        fds.append(w.fd)
        t0 = time.perf_counter()
        w.close()
        t.append(time.perf_counter() - t0)
        assert w.fd == -1
    assert max(t) < 0.01

    def inotify_open(fd: int) -> bool:  # the background close may win between any two looks
        try:
            return "inotify" in os.readlink(f"/proc/self/fd/{fd}")
        except OSError:
            return False

    deadline = time.monotonic() + 5
    while time.monotonic() < deadline and any(inotify_open(fd) for fd in fds):
        time.sleep(0.05)
    assert not any(inotify_open(fd) for fd in fds)
