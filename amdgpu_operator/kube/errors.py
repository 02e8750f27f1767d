"""Kubernetes API errors shared by the REST client and the in-memory API server.

Kept apart from kube/fakeapi.py so that an operand process, which only needs
the client, does not import the simulated API server (its queues, pickling
and uuid/platform imports were ~13 ms of every operand's start-up).
"""

from __future__ import annotations


class ApiError(Exception):
    def __init__(self, code: int, reason: str, message: str = ""):
        super().__init__(f"{code} {reason}: {message}")
        self.code = code
        self.reason = reason
        self.message = message


class NotFound(ApiError):
    def __init__(self, msg=""):
        super().__init__(404, "NotFound", msg)


class AlreadyExists(ApiError):
    def __init__(self, msg=""):
        super().__init__(409, "AlreadyExists", msg)


class Conflict(ApiError):
    def __init__(self, msg=""):
        super().__init__(409, "Conflict", msg)
