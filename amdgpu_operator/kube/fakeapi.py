"""In-memory Kubernetes API server (CRUD + watch + label selectors + GC).

SURVEY.md §4.2: the build environment has no kind, kubectl or apiserver, so
the operator is exercised against this fake.  It implements the semantics the
operator and the simulated kubelet depend on:

* resourceVersion (global, monotonically increasing), uid, generation bump on
  spec change, creationTimestamp;
* ``watch`` streams (ADDED / MODIFIED / DELETED) from a resourceVersion;
* label-selector / field-selector (``spec.nodeName``, ``metadata.name``) lists;
* status subresource updates that do not bump generation;
* JSON merge-patch;
* garbage collection of dependents through ``ownerReferences``;
* cascading namespace deletion.

An HTTP front end (:mod:`.httpapi`) serves the same store with the real REST
paths, so :class:`amdgpu_operator.kube.client.RestClient` is tested over HTTP.
"""

from __future__ import annotations

import itertools
import pickle
import queue
import threading
import time
import uuid

from . import resources as R
from .errors import AlreadyExists, ApiError, Conflict, NotFound  # noqa: F401 - re-exported (kube.fakeapi.NotFound)


def _now() -> str:
    return time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())


def _field_ok(obj: dict, field_selector: str | None) -> bool:
    if not field_selector:
        return True
    for part in field_selector.split(","):
        if "=" not in part:
            continue
        neg = "!=" in part
        k, v = part.split("!=" if neg else "=", 1)
        cur = obj
        for seg in k.strip().split("."):
            cur = cur.get(seg) if isinstance(cur, dict) else None
        if (str(cur) == v.strip()) == neg:
            return False
    return True


def _pack(obj: dict) -> bytes:
    return pickle.dumps(obj, pickle.HIGHEST_PROTOCOL)


def _copy(obj: dict) -> dict:
    """Deep copy of a JSON-shaped object through pickle (C speed)."""
    return pickle.loads(_pack(obj))


class _Watch:
    def __init__(self, t: R.ResourceType, namespace, label_selector, field_selector):
        self.t = t
        self.namespace = namespace
        self.reqs = R.parse_selector(label_selector)
        self.field_selector = field_selector
        self.q: queue.Queue = queue.Queue()
        self.closed = False

    def _passes(self, obj: dict) -> bool:
        return R.matches(R.labels_of(obj), self.reqs) and _field_ok(obj, self.field_selector)

    def offer(self, etype: str, obj: dict, blob: bytes | None = None, old: dict | None = None,
              old_blob: bytes | None = None) -> None:
        """``blob``: the object pickled once by the server for every watcher;
        each consumer unpickles its own copy (3x cheaper than a deep copy).

        A modification that moves an object into or out of this watch's
        selectors arrives as ADDED or DELETED, as kube-apiserver's watch cache
        sends it (the DELETED carrying the object as it last matched): a
        kubelet watching ``spec.nodeName=<node>`` sees a pod the scheduler
        binds as ADDED."""
        if self.closed or R.rtype_of(obj) != self.t:
            return
        if self.t.namespaced and self.namespace and R.ns_of(obj) != self.namespace:
            return
        now = self._passes(obj)
        if etype == "MODIFIED" and old is not None:
            before = self._passes(old)
            if now and not before:
                etype = "ADDED"
            elif before and not now:
                self.q.put(("DELETED", old_blob if old_blob is not None else _pack(old)))
                return
        if not now:
            return
        self.q.put((etype, blob if blob is not None else _pack(obj)))

    def stream(self, timeout: float | None = None, stop: threading.Event | None = None):
        """Yield (type, obj) until closed, ``stop`` is set or ``timeout`` passes idle."""
        deadline = None if timeout is None else time.monotonic() + timeout
        while not self.closed and not (stop is not None and stop.is_set()):
            wait = 0.2 if deadline is None else max(0.0, min(0.2, deadline - time.monotonic()))
            try:
                item = self.q.get(timeout=wait)
            except queue.Empty:
                if deadline is not None and time.monotonic() >= deadline:
                    return
                continue
            if item is None:
                return
            yield item[0], pickle.loads(item[1])

    def close(self) -> None:
        self.closed = True
        self.q.put(None)


class FakeApiServer:
    def __init__(self):
        self._lock = threading.RLock()
        self._store: dict[tuple, dict] = {}
        self._rv = itertools.count(1)
        self._last_rv = 0
        self._watches: list[_Watch] = []
        self._history: list[tuple[int, str, bytes]] = []  # for watch-from-resourceVersion
        # every stored object, pickled at its last write: reads hand out
        # pickle.loads copies (the store itself is never handed out)
        self._blobs: dict[tuple, bytes] = {}
        self.request_count = 0
        self.hooks: list = []  # callables(event_type, obj) run synchronously after commit
        self.validators: list = []  # callables(obj) -> [errors], before a create/update commits (kube/validation.py)
        # Pods on a node stay Terminating until a zero-grace delete (see delete())
        self.graceful_pod_deletion = False

    # ------------------------------------------------------------------ core
    def _bump(self, obj: dict) -> None:
        rv = next(self._rv)
        self._last_rv = rv
        obj["metadata"]["resourceVersion"] = str(rv)

    def _emit(self, etype: str, obj: dict, old: dict | None = None) -> None:
        blob = _pack(obj)
        k = R.key_of(obj)
        old_blob = self._blobs.get(k) if old is not None else None
        if etype == "DELETED":
            self._blobs.pop(k, None)
        else:
            self._blobs[k] = blob
        self._history.append((int(obj["metadata"]["resourceVersion"]), etype, blob, old_blob))
        if len(self._history) > 20000:
            del self._history[:5000]
        for w in list(self._watches):
            w.offer(etype, obj, blob, old, old_blob)
        for h in list(self.hooks):
            h(etype, pickle.loads(blob))

    def _out(self, k: tuple, o: dict) -> dict:
        """A caller's copy of the stored object ``o`` at key ``k``."""
        b = self._blobs.get(k)
        return pickle.loads(b) if b is not None else R.deep(o)

    def _validate(self, obj: dict) -> None:
        errs = [e for v in self.validators for e in v(obj)]
        if errs:
            raise ApiError(422, "Invalid", f"{obj.get('kind')} {R.name_of(obj)!r} is invalid: " + "; ".join(errs))

    def _key(self, t: R.ResourceType, namespace, name) -> tuple:
        return (t.api_version, t.kind, namespace if t.namespaced else None, name)

    # ------------------------------------------------------------------ verbs
    def create(self, obj: dict) -> dict:
        self.request_count += 1
        obj = _copy(obj)
        t = R.rtype_of(obj)
        md = R.meta(obj)
        if not md.get("name"):
            if md.get("generateName"):
                md["name"] = md["generateName"] + uuid.uuid4().hex[:5]
            else:
                raise ApiError(422, "Invalid", "metadata.name required")
        if t.namespaced and not md.get("namespace"):
            md["namespace"] = "default"
        if not t.namespaced:
            md.pop("namespace", None)
        self._validate(obj)
        with self._lock:
            k = self._key(t, md.get("namespace"), md["name"])
            if k in self._store:
                raise AlreadyExists(f"{t.kind} {md['name']}")
            if t.namespaced and md["namespace"] != "default":
                nsk = ("v1", "Namespace", None, md["namespace"])
                if nsk not in self._store:
                    raise NotFound(f"namespace {md['namespace']}")
            md["uid"] = str(uuid.uuid4())
            md["creationTimestamp"] = _now()
            md["generation"] = 1
            md.pop("deletionTimestamp", None)
            self._bump(obj)
            self._store[k] = obj
            self._emit("ADDED", obj)
            return self._out(k, obj)

    def get(self, api_version: str, kind: str, name: str, namespace: str | None = None) -> dict:
        self.request_count += 1
        t = R.rtype(api_version, kind)
        with self._lock:
            k = self._key(t, namespace, name)
            o = self._store.get(k)
            if o is None:
                raise NotFound(f"{kind} {namespace}/{name}")
            return self._out(k, o)

    def list(self, api_version: str, kind: str, namespace: str | None = None, label_selector=None,
             field_selector: str | None = None) -> list[dict]:
        self.request_count += 1
        t = R.rtype(api_version, kind)
        reqs = R.parse_selector(label_selector)
        with self._lock:
            out = []
            for k, o in self._store.items():
                av, kd, ns, _ = k
                if av != t.api_version or kd != t.kind:
                    continue
                if t.namespaced and namespace and ns != namespace:
                    continue
                if R.matches(R.labels_of(o), reqs) and _field_ok(o, field_selector):
                    out.append(self._out(k, o))
            out.sort(key=lambda o: (R.ns_of(o) or "", R.name_of(o)))
            return out

    def resource_version(self) -> int:
        return self._last_rv

    def update(self, obj: dict, subresource: str | None = None) -> dict:
        self.request_count += 1
        obj = _copy(obj)
        t = R.rtype_of(obj)
        md = R.meta(obj)
        with self._lock:
            k = self._key(t, md.get("namespace"), md.get("name"))
            cur = self._store.get(k)
            if cur is None:
                raise NotFound(f"{t.kind} {md.get('name')}")
            rv = md.get("resourceVersion")
            if rv and rv != cur["metadata"]["resourceVersion"]:
                raise Conflict(f"{t.kind} {md.get('name')}: resourceVersion {rv} != {cur['metadata']['resourceVersion']}")
            if subresource == "status":
                new = self._out(k, cur)
                new["status"] = obj.get("status", {})
            else:
                new = obj
                self._validate(new)
                # the main endpoint never changes status (status subresource semantics)
                if "status" in cur:
                    new["status"] = self._out(k, cur)["status"]
                else:
                    new.pop("status", None)
                for f in ("uid", "creationTimestamp", "generation"):
                    new["metadata"][f] = cur["metadata"].get(f)
                if {kk: v for kk, v in obj.items() if kk not in ("metadata", "status")} != \
                        {kk: v for kk, v in cur.items() if kk not in ("metadata", "status")}:
                    new["metadata"]["generation"] = cur["metadata"].get("generation", 1) + 1
            self._bump(new)
            self._store[k] = new
            self._emit("MODIFIED", new, cur)
            return self._out(k, new)

    def patch(self, api_version: str, kind: str, name: str, patch: dict, namespace: str | None = None,
              subresource: str | None = None) -> dict:
        with self._lock:
            cur = self.get(api_version, kind, name, namespace)
            merged = R.merge_patch(cur, patch)
            merged["metadata"]["resourceVersion"] = cur["metadata"]["resourceVersion"]
            return self.update(merged, subresource=subresource)

    def delete(self, api_version: str, kind: str, name: str, namespace: str | None = None,
               grace_period_seconds: int | None = None) -> None:
        """Delete an object.  With :attr:`graceful_pod_deletion` a Pod bound to
        a node is only marked Terminating (``deletionTimestamp``) and stays
        listed until its kubelet confirms with a zero-grace delete, as on a
        real API server; ``grace_period_seconds=0`` removes it at once."""
        self.request_count += 1
        t = R.rtype(api_version, kind)
        with self._lock:
            k = self._key(t, namespace, name)
            cur = self._store.get(k)
            if cur is None:
                raise NotFound(f"{kind} {namespace}/{name}")
            if (self.graceful_pod_deletion and kind == "Pod" and grace_period_seconds != 0
                    and (cur.get("spec") or {}).get("nodeName")):
                if not cur["metadata"].get("deletionTimestamp"):
                    grace = grace_period_seconds
                    if grace is None:
                        grace = int((cur.get("spec") or {}).get("terminationGracePeriodSeconds", 30))
                    cur["metadata"]["deletionTimestamp"] = _now()
                    cur["metadata"]["deletionGracePeriodSeconds"] = grace
                    self._bump(cur)
                    self._emit("MODIFIED", cur)
                return
            o = self._store.pop(k)
            self._bump(o)
            self._emit("DELETED", o)
            uid = o["metadata"]["uid"]
            # cascading GC of dependents (foreground semantics, synchronously)
            deps = [v for v in self._store.values()
                    if any(ref.get("uid") == uid for ref in v.get("metadata", {}).get("ownerReferences") or [])]
            if kind == "Namespace":
                deps += [v for (av, kd, ns, _), v in self._store.items() if ns == name]
            if kind == "CustomResourceDefinition":
                spec = o.get("spec", {})
                grp = spec.get("group")
                knd = (spec.get("names") or {}).get("kind")
                for ver in spec.get("versions", []):
                    av = f"{grp}/{ver.get('name')}"
                    deps += [v for (a, kd, ns, _), v in self._store.items() if a == av and kd == knd]
            seen = set()
            for d in deps:
                dk = R.key_of(d)
                if dk in seen:
                    continue
                seen.add(dk)
                try:
                    dt = R.rtype_of(d)
                    self.delete(dt.api_version, dt.kind, R.name_of(d), R.ns_of(d))
                except NotFound:
                    pass

    def watch(self, api_version: str, kind: str, namespace: str | None = None, label_selector=None,
              field_selector: str | None = None, resource_version: int | str | None = None) -> _Watch:
        t = R.rtype(api_version, kind)
        w = _Watch(t, namespace, label_selector, field_selector)
        with self._lock:
            if resource_version not in (None, "", "0", 0):
                rv = int(resource_version)
                for erv, etype, blob, old_blob in self._history:
                    if erv > rv:
                        w.offer(etype, pickle.loads(blob), blob,
                                pickle.loads(old_blob) if old_blob is not None else None, old_blob)
            else:  # like kube-apiserver: the current state as synthetic ADDED events first
                for k, obj in self._store.items():
                    w.offer("ADDED", obj, self._blobs.get(k))
            self._watches.append(w)
        return w

    def stop_watch(self, w: _Watch) -> None:
        w.close()
        with self._lock:
            if w in self._watches:
                self._watches.remove(w)

    # ------------------------------------------------------------ conveniences
    def apply(self, obj: dict) -> dict:
        """Create or replace (keeps status), like ``kubectl apply`` for tests."""
        t = R.rtype_of(obj)
        try:
            cur = self.get(t.api_version, t.kind, R.name_of(obj), R.ns_of(obj))
        except NotFound:
            return self.create(obj)
        o = R.deep(obj)
        o["metadata"]["resourceVersion"] = cur["metadata"]["resourceVersion"]
        return self.update(o)
