"""Structured JSON logging for every operand.

``logging`` is imported when a logger is first used, not when a module
asks for one.  It costs a fresh interpreter 9.5 ms on the MI355X box
(``profiles/r5_ttr/startup``), and an operand's start (``python3 -S -m
amdgpu_operator <cmd>``) is on the bring-up's critical path.  The operands
that log nothing before they are ready no longer pay it there.
:func:`setup` is likewise applied when ``logging`` is first used.
"""

from __future__ import annotations

import os
import sys
import threading
import time

_pending: tuple | None = None  # setup()'s arguments, applied when logging is first used
_lock = threading.Lock()
_preloading = False


def _logging():
    import logging

    global _pending
    if _pending is not None or _preloading:  # a preload may be applying setup: wait for it
        with _lock:
            args, _pending = _pending, None
            if args is not None:
                _apply(logging, *args)
    return logging


def load() -> None:
    """Import ``logging`` (and apply setup) now."""
    _logging()


def preload_async() -> None:
    """Import ``logging`` (and apply setup) on a daemon thread.  An operand
    calls this before it waits (for a gate, another operand's ready file),
    so its first log call after the wait finds logging loaded: otherwise the
    import would move from its start onto its path after the wait (the
    device plugin's registration, profiles/r5_ttr/startup)."""
    global _preloading
    if _preloading or ("logging" in sys.modules and _pending is None):
        return
    _preloading = True
    threading.Thread(target=_logging, name="logging-preload", daemon=True).start()


def _json_formatter(logging):
    import json

    class JsonFormatter(logging.Formatter):
        def format(self, record):
            d = {"ts": round(record.created, 3), "level": record.levelname.lower(), "logger": record.name,
                 "msg": record.getMessage()}
            for k in ("node", "state", "span", "seconds", "device"):
                if hasattr(record, k):
                    d[k] = getattr(record, k)
            if record.exc_info:
                d["exc"] = self.formatException(record.exc_info)
            return json.dumps(d, default=str)

    return JsonFormatter()


def _stderr_handler(logging):
    """A StreamHandler on whatever ``sys.stderr`` is at each record (like
    logging's last-resort handler), not on the stream it was created with: a
    replaced stderr (a test's capture, a daemon's redirect) that was since
    closed would otherwise fail every later record of a long-lived thread."""

    class StderrHandler(logging.StreamHandler):
        def __init__(self):
            logging.Handler.__init__(self)

        @property
        def stream(self):
            return sys.stderr

    return StderrHandler()


def _apply(logging, level: str | None, json_logs: bool | None) -> None:
    level = (level or os.environ.get("LOG_LEVEL", "info")).upper()
    json_logs = json_logs if json_logs is not None else os.environ.get("LOG_FORMAT", "json") == "json"
    h = _stderr_handler(logging)
    h.setFormatter(_json_formatter(logging) if json_logs
                   else logging.Formatter("%(asctime)s %(levelname)s %(name)s %(message)s"))
    root = logging.getLogger("amdgpu")
    root.handlers[:] = [h]
    root.setLevel(level)
    root.propagate = False


def setup(level: str | None = None, json_logs: bool | None = None) -> None:
    """The ``amdgpu`` loggers write to stderr, JSON by default (``LOG_FORMAT``,
    ``LOG_LEVEL``); applied now if ``logging`` is loaded, else at its first use."""
    global _pending
    if "logging" in sys.modules:
        _pending = None
        _apply(sys.modules["logging"], level, json_logs)
    else:
        _pending = (level, json_logs)


class _LazyLogger:
    """A ``logging.Logger`` that is looked up (and ``logging`` imported) at
    its first attribute access; from then on every attribute is the real
    logger's."""

    __slots__ = ("_name", "_real")

    def __init__(self, name: str) -> None:
        self._name = name
        self._real = None

    def __getattr__(self, attr):
        real = self._real
        if real is None:
            real = self._real = _logging().getLogger(self._name)
        return getattr(real, attr)

    def __repr__(self) -> str:
        return f"<logger {self._name} (lazy)>"


def get_logger(name: str):
    return _LazyLogger(name)


class Span:
    """Timing span logged as one JSON record (time-to-Ready breakdown)."""

    def __init__(self, logger, name: str, **fields):
        self.logger, self.name, self.fields = logger, name, fields

    def __enter__(self):
        self.t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        self.seconds = time.perf_counter() - self.t0
        self.logger.info("span %s", self.name, extra={"span": self.name, "seconds": round(self.seconds, 6), **self.fields})
        return False
