"""Structured JSON logging for every operand."""

from __future__ import annotations

import json
import logging
import os
import sys
import time


class JsonFormatter(logging.Formatter):
    def format(self, record: logging.LogRecord) -> str:
        d = {"ts": round(record.created, 3), "level": record.levelname.lower(), "logger": record.name,
             "msg": record.getMessage()}
        for k in ("node", "state", "span", "seconds", "device"):
            if hasattr(record, k):
                d[k] = getattr(record, k)
        if record.exc_info:
            d["exc"] = self.formatException(record.exc_info)
        return json.dumps(d, default=str)


def setup(level: str | None = None, json_logs: bool | None = None) -> None:
    level = (level or os.environ.get("LOG_LEVEL", "info")).upper()
    json_logs = json_logs if json_logs is not None else os.environ.get("LOG_FORMAT", "json") == "json"
    h = logging.StreamHandler(sys.stderr)
    h.setFormatter(JsonFormatter() if json_logs else logging.Formatter("%(asctime)s %(levelname)s %(name)s %(message)s"))
    root = logging.getLogger("amdgpu")
    root.handlers[:] = [h]
    root.setLevel(level)
    root.propagate = False


def get_logger(name: str) -> logging.Logger:
    return logging.getLogger(name)


class Span:
    """Timing span logged as one JSON record (time-to-Ready breakdown)."""

    def __init__(self, logger: logging.Logger, name: str, **fields):
        self.logger, self.name, self.fields = logger, name, fields

    def __enter__(self):
        self.t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        self.seconds = time.perf_counter() - self.t0
        self.logger.info("span %s", self.name, extra={"span": self.name, "seconds": round(self.seconds, 6), **self.fields})
        return False
