"""Watch-backed object caches for the operator (client-go informers).

A reconcile pass reads every object it owns (27 GETs per pass for the
reference's ``--set`` flags, plus Node and ClusterPolicy lists).  Against a
real API server each GET is a round trip, so a pass costs tens to hundreds of
milliseconds and the API load grows with the resync rate.
:class:`CachedClient` serves those reads from per-kind caches kept current by
list-then-watch (:class:`Informer`), and passes every write through to the
server:

* a write's response is put into the cache at once (write-through), so the
  next pass sees the operator's own writes even before the watch event
  arrives;
* a watch event never replaces a newer object (resourceVersions compared as
  integers when both parse, as etcd's do);
* a kind whose informer has not synced (initial list pending, or a kind the
  server does not serve, such as ServiceMonitor without the Prometheus
  operator) is read from the server;
* conflicts are resolved against the server (``uncached()``): see
  :func:`.client.apply_object`.
"""

from __future__ import annotations

import pickle
import threading
import time

from . import resources as R
from .fakeapi import ApiError, _field_ok
from ..utils.logs import get_logger

log = get_logger("amdgpu.informer")


def _rv(obj: dict) -> int | None:
    try:
        return int((obj.get("metadata") or {}).get("resourceVersion"))
    except (TypeError, ValueError):
        return None


class Informer:
    """List-then-watch cache of one kind (optionally one namespace)."""

    def __init__(self, client, api_version: str, kind: str, namespace: str | None = None, on_event=None,
                 relist_wait_s: float = 1.0, watch_timeout_s: float = 300.0, is_echo=None):
        """``is_echo(obj)``: True for the watch event of a write the owner
        made itself (its own resourceVersion): cached, but ``on_event`` is not
        called for it."""
        self.is_echo = is_echo
        self.client = client
        self.watch_timeout_s = watch_timeout_s
        self.api_version = api_version
        self.kind = kind
        self.namespace = namespace
        self.on_event = on_event
        self.relist_wait_s = relist_wait_s
        self.synced = threading.Event()
        self.failed = threading.Event()  # the server does not serve this kind (404 on list)
        self._lock = threading.Lock()
        self._store: dict[tuple, bytes] = {}  # (namespace, name) -> pickled object
        self._rvs: dict[tuple, int | None] = {}
        self._thread: threading.Thread | None = None

    # ------------------------------------------------------------ store
    @staticmethod
    def _key(obj: dict) -> tuple:
        md = obj.get("metadata") or {}
        return (md.get("namespace"), md.get("name"))

    def put(self, obj: dict) -> None:
        """Insert ``obj`` unless the cache holds a newer version."""
        k = self._key(obj)
        rv = _rv(obj)
        with self._lock:
            cur = self._rvs.get(k)
            if cur is not None and rv is not None and rv < cur:
                return
            self._store[k] = pickle.dumps(obj, pickle.HIGHEST_PROTOCOL)
            self._rvs[k] = rv

    def remove(self, namespace: str | None, name: str, rv: int | None = None) -> None:
        k = (namespace, name)
        with self._lock:
            cur = self._rvs.get(k)
            if rv is not None and cur is not None and rv < cur:
                return  # a delete older than the object we hold (re-created since)
            self._store.pop(k, None)
            self._rvs.pop(k, None)

    def get(self, name: str, namespace: str | None = None) -> dict | None:
        with self._lock:
            b = self._store.get((namespace, name))
        return pickle.loads(b) if b is not None else None

    def list(self, namespace: str | None = None, label_selector=None, field_selector: str | None = None) -> list[dict]:
        reqs = R.parse_selector(label_selector)
        with self._lock:
            blobs = [b for (ns, _), b in self._store.items() if namespace is None or ns == namespace]
        out = []
        for b in blobs:
            o = pickle.loads(b)
            if R.matches(R.labels_of(o), reqs) and _field_ok(o, field_selector):
                out.append(o)
        out.sort(key=lambda o: (R.ns_of(o) or "", R.name_of(o)))
        return out

    # ------------------------------------------------------------- loop
    def start(self, stop: threading.Event) -> "Informer":
        self._thread = threading.Thread(target=self._run, args=(stop,), daemon=True,
                                        name=f"informer-{self.kind}")
        self._thread.start()
        return self

    def _relist(self):
        items, rv = self.client.list_rv(self.api_version, self.kind, self.namespace)
        fresh = {}
        for o in items:
            fresh[self._key(o)] = (pickle.dumps(o, pickle.HIGHEST_PROTOCOL), _rv(o))
        with self._lock:
            self._store = {k: b for k, (b, _) in fresh.items()}
            self._rvs = {k: r for k, (_, r) in fresh.items()}
        return rv

    def _run(self, stop: threading.Event) -> None:
        while not stop.is_set():
            try:
                rv = self._relist()
            except ApiError as e:
                if e.code == 404:  # kind not served (CRD absent): reads go to the server
                    self.failed.set()
                    return
                log.debug("informer %s list: %s", self.kind, e)
                stop.wait(self.relist_wait_s)
                continue
            except Exception as e:  # noqa: BLE001 - API unavailable: retry
                log.debug("informer %s list: %s", self.kind, e)
                stop.wait(self.relist_wait_s)
                continue
            self.synced.set()
            if self.on_event is not None:
                self.on_event(self.kind)
            # a watch that times out is resumed from the last version seen;
            # only an error (410 Gone, network) costs a relist
            try:
                while not stop.is_set():
                    began, events = time.monotonic(), 0
                    for etype, obj in self.client.watch(self.api_version, self.kind, self.namespace,
                                                        resource_version=rv, stop=stop,
                                                        timeout=self.watch_timeout_s):
                        rv = (obj.get("metadata") or {}).get("resourceVersion") or rv
                        events += 1
                        if etype == "DELETED":
                            self.remove(R.ns_of(obj) if obj.get("metadata", {}).get("namespace") else None,
                                        R.name_of(obj), _rv(obj))
                        elif etype in ("ADDED", "MODIFIED"):
                            self.put(obj)
                        else:
                            continue  # BOOKMARK: only the version moves
                        if self.on_event is not None and not (etype != "DELETED" and self.is_echo is not None
                                                              and self.is_echo(obj)):
                            self.on_event(self.kind)
                    if not events and time.monotonic() - began < 1.0:
                        stop.wait(self.relist_wait_s)  # closed at once: do not spin on a failing server
            except Exception as e:  # noqa: BLE001 - watch failed (410 Gone, network): relist
                log.debug("informer %s watch: %s", self.kind, e)


class CachedClient:
    """A client whose reads of the informed kinds come from the caches."""

    def __init__(self, client, kinds: list[tuple], stop: threading.Event, on_event=None):
        """``kinds``: (api_version, kind, namespace or None[, trigger]); ``on_event(kind)``
        is called for every change of a kind whose ``trigger`` is true."""
        self._client = client
        self._stop = stop
        # resourceVersions of this client's own writes: their watch events are
        # echoes, which update the caches but trigger nothing (bounded)
        self._own: dict[tuple, bool] = {}
        self.informers: dict[tuple[str, str], Informer] = {}
        for spec in kinds:
            av, kind, ns = spec[:3]
            trigger = spec[3] if len(spec) > 3 else False
            self.informers[(av, kind)] = Informer(client, av, kind, ns, on_event=on_event if trigger else None,
                                                  is_echo=self._is_echo).start(stop)

    OWN_WRITES_KEPT = 4096

    @staticmethod
    def _ident(obj: dict) -> tuple:
        md = obj.get("metadata") or {}
        return (obj.get("apiVersion"), obj.get("kind"), md.get("namespace"), md.get("name"))

    def _is_echo(self, obj: dict) -> bool:
        rv = (obj.get("metadata") or {}).get("resourceVersion")
        return rv is not None and (self._ident(obj), rv) in self._own

    def uncached(self):
        return self._client

    def wait_synced(self, timeout: float = 10.0) -> bool:
        deadline = time.monotonic() + timeout
        for inf in self.informers.values():
            while not (inf.synced.is_set() or inf.failed.is_set()):
                if time.monotonic() >= deadline or self._stop.is_set():
                    return False
                inf.synced.wait(0.01)
        return True

    def _informer(self, api_version: str, kind: str, namespace: str | None) -> Informer | None:
        inf = self.informers.get((api_version, kind))
        if inf is None or not inf.synced.is_set():
            return None
        if inf.namespace is not None and namespace != inf.namespace:
            return None  # outside the informer's scope
        return inf

    # ------------------------------------------------------------ reads
    def get(self, api_version, kind, name, namespace=None):
        inf = self._informer(api_version, kind, namespace)
        if inf is None:
            return self._client.get(api_version, kind, name, namespace)
        t = R.rtype(api_version, kind)
        o = inf.get(name, namespace if t.namespaced else None)
        if o is None:
            from .fakeapi import NotFound

            raise NotFound(f"{kind} {namespace}/{name}")
        return o

    def list(self, api_version, kind, namespace=None, label_selector=None, field_selector=None):
        inf = self._informer(api_version, kind, namespace) if namespace or not self._namespaced(api_version, kind) \
            else self._cluster_wide(api_version, kind)
        if inf is None:
            return self._client.list(api_version, kind, namespace, label_selector, field_selector)
        return inf.list(namespace, label_selector, field_selector)

    def _namespaced(self, api_version, kind) -> bool:
        return R.rtype(api_version, kind).namespaced

    def _cluster_wide(self, api_version, kind):
        inf = self.informers.get((api_version, kind))
        return inf if inf is not None and inf.synced.is_set() and inf.namespace is None else None

    # ----------------------------------------------------------- writes
    def _remember(self, obj: dict) -> dict:
        inf = self.informers.get((obj.get("apiVersion"), obj.get("kind")))
        if inf is not None and isinstance(obj, dict) and obj.get("metadata"):
            inf.put(obj)
            rv = obj["metadata"].get("resourceVersion")
            if rv is not None:  # every version this client wrote (a write's event may come after the next write)
                if len(self._own) >= self.OWN_WRITES_KEPT:
                    self._own.pop(next(iter(self._own)))
                self._own[(self._ident(obj), rv)] = True
        return obj

    def create(self, obj):
        return self._remember(self._client.create(obj))

    def update(self, obj):
        return self._remember(self._client.update(obj))

    def update_status(self, obj):
        return self._remember(self._client.update_status(obj))

    def patch(self, api_version, kind, name, patch, namespace=None, subresource=None):
        return self._remember(self._client.patch(api_version, kind, name, patch, namespace, subresource))

    def delete(self, api_version, kind, name, namespace=None, grace_period_seconds=None):
        out = self._client.delete(api_version, kind, name, namespace, grace_period_seconds)
        inf = self.informers.get((api_version, kind))
        if inf is not None:
            inf.remove(namespace if R.rtype(api_version, kind).namespaced else None, name)
        return out

    def __getattr__(self, name):  # watch, list_rv, ... go to the server
        return getattr(self._client, name)
