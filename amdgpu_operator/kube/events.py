"""Kubernetes Events from the operator and its operands (``v1`` Event).

The reference troubleshoots with ``kubectl describe pod`` and
``kubectl logs`` (/root/reference/README.md:172-184): ``describe`` shows the
Events of an object, so the operator reports what it does to the objects an
admin looks at - the ClusterPolicy (ready / not ready / error), each GPU
Node (driver upgrade steps, validation passed or failed).

Like client-go's recorder, repeats of the same (object, type, reason,
message) within ``aggregate_s`` update one Event's ``count`` and
``lastTimestamp`` instead of creating a new object.  Recording is best
effort: an API error is logged and never fails the caller.
"""

from __future__ import annotations

import os
import threading
import time

from .errors import NotFound
from ..utils.logs import get_logger

log = get_logger("amdgpu.events")
NORMAL, WARNING = "Normal", "Warning"


def _ts(t: float) -> str:
    return time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime(t))


class EventRecorder:
    def __init__(self, client, component: str, host: str = "", aggregate_s: float = 600.0, clock=time.time):
        self.client = client
        self.component = component
        self.host = host
        self.aggregate_s = aggregate_s
        self.clock = clock
        self._lock = threading.Lock()
        self._seen: dict[tuple, tuple[str, str, int, float]] = {}  # key -> (namespace, name, count, first)

    def record(self, obj: dict, etype: str, reason: str, message: str) -> None:
        if self.client is None:
            return
        md = obj.get("metadata") or {}
        ns = md.get("namespace") or "default"  # cluster-scoped objects: events live in "default"
        key = (obj.get("kind"), ns, md.get("name"), md.get("uid"), etype, reason, message)
        now = self.clock()
        try:
            with self._lock:
                prev = self._seen.get(key)
                if prev and now - prev[3] <= self.aggregate_s:
                    ev_ns, ev_name, count, first = prev
                    self.client.patch("v1", "Event", ev_name, {"count": count + 1, "lastTimestamp": _ts(now)}, ev_ns)
                    self._seen[key] = (ev_ns, ev_name, count + 1, first)
                    return
                name = f"{md.get('name', 'object')}.{os.urandom(8).hex()}"
                ev = {"apiVersion": "v1", "kind": "Event",
                      "metadata": {"name": name, "namespace": ns},
                      "involvedObject": {"apiVersion": obj.get("apiVersion"), "kind": obj.get("kind"),
                                         "name": md.get("name"), "namespace": md.get("namespace"),
                                         "uid": md.get("uid")},
                      "reason": reason, "message": message[:1024], "type": etype,
                      "source": {"component": self.component, **({"host": self.host} if self.host else {})},
                      "reportingComponent": self.component, "reportingInstance": self.host or self.component,
                      "firstTimestamp": _ts(now), "lastTimestamp": _ts(now), "count": 1}
                self.client.create(ev)
                self._seen[key] = (ns, name, 1, now)
        except NotFound:
            with self._lock:  # the aggregated event was deleted (TTL): start a new one next time
                self._seen.pop(key, None)
        except Exception as e:  # noqa: BLE001 - events are best effort
            log.debug("event %s/%s not recorded: %s", reason, md.get("name"), e)


def events_for(client, kind: str, name: str) -> list[dict]:
    """Events whose involvedObject is ``kind/name`` (``kubectl describe``'s list)."""
    out = []
    for ev in client.list("v1", "Event"):
        io = ev.get("involvedObject") or {}
        if io.get("kind") == kind and io.get("name") == name:
            out.append(ev)
    out.sort(key=lambda e: e.get("lastTimestamp", ""))
    return out
