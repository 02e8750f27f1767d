"""Kubernetes client interface used by every component of the operator.

Two implementations with the same methods:

* :class:`LocalClient` - direct calls into :class:`~.fakeapi.FakeApiServer`
  (unit / integration tests, bench);
* :class:`RestClient` - the Kubernetes REST API over HTTP(S) (in-cluster
  service-account config or a kubeconfig), including streaming watches.  It is
  exercised in tests against the fake server's HTTP front end
  (:mod:`.httpapi`).
"""

from __future__ import annotations

import json
import os
import threading
from typing import TYPE_CHECKING
from urllib.parse import quote, urlencode

from . import resources as R
from .errors import AlreadyExists, ApiError, Conflict, NotFound

if TYPE_CHECKING:
    from .fakeapi import FakeApiServer

__all__ = ["LocalClient", "RestClient", "ApiError", "NotFound", "AlreadyExists", "Conflict", "apply_object", "wait_for"]


class LocalClient:
    def __init__(self, server: FakeApiServer):
        self.server = server

    def create(self, obj):
        return self.server.create(obj)

    def get(self, api_version, kind, name, namespace=None):
        return self.server.get(api_version, kind, name, namespace)

    def list(self, api_version, kind, namespace=None, label_selector=None, field_selector=None):
        return self.server.list(api_version, kind, namespace, label_selector, field_selector)

    def list_rv(self, api_version, kind, namespace=None, label_selector=None, field_selector=None):
        """Items plus a resourceVersion to watch from (changes after it are replayed)."""
        rv = self.server.resource_version()
        return self.server.list(api_version, kind, namespace, label_selector, field_selector), str(rv)

    def update(self, obj):
        return self.server.update(obj)

    def update_status(self, obj):
        return self.server.update(obj, subresource="status")

    def patch(self, api_version, kind, name, patch, namespace=None, subresource=None):
        return self.server.patch(api_version, kind, name, patch, namespace, subresource)

    def delete(self, api_version, kind, name, namespace=None, grace_period_seconds=None):
        return self.server.delete(api_version, kind, name, namespace, grace_period_seconds)

    def watch(self, api_version, kind, namespace=None, label_selector=None, field_selector=None,
              resource_version=None, stop: threading.Event | None = None, timeout=None):
        w = self.server.watch(api_version, kind, namespace, label_selector, field_selector, resource_version)
        try:
            yield from w.stream(timeout=timeout, stop=stop)
        finally:
            self.server.stop_watch(w)


def _raise_for(resp) -> None:
    if resp.status_code < 400:
        return
    try:
        body = resp.json()
        reason, msg = body.get("reason", ""), body.get("message", "")
    except ValueError:
        reason, msg = "", resp.text[:500]
    if resp.status_code == 404:
        raise NotFound(msg)
    if resp.status_code == 409:
        raise AlreadyExists(msg) if reason == "AlreadyExists" else Conflict(msg)
    raise ApiError(resp.status_code, reason or "Error", msg)


class TokenFileAuth:
    """Bearer token read from a file and re-read as it rotates.

    The kubelet refreshes a pod's projected service-account token (valid for
    an hour where the API server does not extend it) well before expiry; like
    client-go, the client re-reads the file at most every ``reload_s`` so a
    long-running operator keeps authenticating."""

    def __init__(self, path: str, reload_s: float = 60.0, clock=None):
        import time

        self.path = path
        self.reload_s = reload_s
        self.clock = clock or time.monotonic
        self._token = ""
        self._read_at = None
        self._lock = threading.Lock()

    def token(self) -> str:
        with self._lock:
            now = self.clock()
            if self._read_at is None or now - self._read_at >= self.reload_s:
                try:
                    with open(self.path) as f:
                        self._token = f.read().strip()
                except OSError:
                    pass  # keep the last token; the API server says whether it still works
                self._read_at = now
            return self._token

    def __call__(self, request):  # the session's auth hook (kube/transport.py)
        request.headers["Authorization"] = f"Bearer {self.token()}"
        return request


class RestClient:
    """Minimal Kubernetes REST client (JSON, merge-patch, streaming watch)."""

    SA_DIR = "/var/run/secrets/kubernetes.io/serviceaccount"

    def __init__(self, base_url: str, token: str | None = None, verify=True, cert=None, timeout: float = 30.0,
                 token_file: str | None = None):
        from .transport import Session

        self.base = base_url.rstrip("/")
        self.session = Session()  # standard-library HTTP(S) (kube/transport.py: operand start-up cost)
        self.session.verify = verify
        if cert:
            self.session.cert = cert
        if token_file:
            self.session.auth = TokenFileAuth(token_file)
        elif token:
            self.session.headers["Authorization"] = f"Bearer {token}"
        self.session.headers["Accept"] = "application/json"
        self.timeout = timeout

    RETRIES = 4

    def _call(self, method: str, url: str, **kw):
        """One request, retried like client-go: on 429 / 503 (the server did
        not process it; honour Retry-After, else back off), and on connection
        errors for reads only (a write may have landed)."""
        import time

        delay = 0.1
        for attempt in range(self.RETRIES + 1):
            try:
                r = self.session.request(method, url, timeout=self.timeout, **kw)
            except ConnectionError:
                if method != "GET" or attempt == self.RETRIES:
                    raise
                time.sleep(delay)
                delay = min(delay * 2, 2.0)
                continue
            if r.status_code in (429, 503) and attempt < self.RETRIES:
                try:
                    wait = float(r.headers.get("Retry-After", ""))
                except ValueError:
                    wait = delay
                time.sleep(min(max(wait, 0.0), 10.0))
                delay = min(delay * 2, 2.0)
                continue
            return r
        return r

    @classmethod
    def from_incluster(cls) -> "RestClient":
        host = os.environ["KUBERNETES_SERVICE_HOST"]
        port = os.environ.get("KUBERNETES_SERVICE_PORT", "443")
        return cls(f"https://{host}:{port}", token_file=os.path.join(cls.SA_DIR, "token"),
                   verify=os.path.join(cls.SA_DIR, "ca.crt"))

    @classmethod
    def from_kubeconfig(cls, path: str | None = None, context: str | None = None) -> "RestClient":
        import base64
        import tempfile

        path = path or os.environ.get("KUBECONFIG") or os.path.expanduser("~/.kube/config")
        with open(path) as f:
            text = f.read()
        try:  # a JSON kubeconfig needs no YAML parser (operand start-up: kube/transport.py)
            cfg = json.loads(text)
        except ValueError:
            import yaml

            cfg = yaml.safe_load(text)
        ctx_name = context or cfg.get("current-context")
        ctx = next(c["context"] for c in cfg["contexts"] if c["name"] == ctx_name)
        cluster = next(c["cluster"] for c in cfg["clusters"] if c["name"] == ctx["cluster"])
        user = next(u["user"] for u in cfg["users"] if u["name"] == ctx["user"])

        def materialise(data_key, file_key, src):
            if src.get(file_key):
                return src[file_key]
            if src.get(data_key):
                fd, p = tempfile.mkstemp(prefix="kube-")
                with os.fdopen(fd, "wb") as fh:
                    fh.write(base64.b64decode(src[data_key]))
                return p
            return None

        verify = materialise("certificate-authority-data", "certificate-authority", cluster) or True
        if cluster.get("insecure-skip-tls-verify"):
            verify = False
        cert = None
        cc = materialise("client-certificate-data", "client-certificate", user)
        ck = materialise("client-key-data", "client-key", user)
        if cc and ck:
            cert = (cc, ck)
        return cls(cluster["server"], token=user.get("token"), verify=verify, cert=cert,
                   token_file=user.get("tokenFile"))

    # -------------------------------------------------------------- helpers
    def _url(self, t: R.ResourceType, namespace=None, name=None, sub=None, query=None) -> str:
        u = self.base + t.path(namespace, quote(name) if name else None)
        if sub:
            u += "/" + sub
        if query:
            u += "?" + urlencode({k: v for k, v in query.items() if v not in (None, "")})
        return u

    def create(self, obj):
        t = R.rtype_of(obj)
        r = self._call("POST", self._url(t, R.ns_of(obj) if t.namespaced else None), data=json.dumps(obj),
                       headers={"Content-Type": "application/json"})
        _raise_for(r)
        return r.json()

    def get(self, api_version, kind, name, namespace=None):
        t = R.rtype(api_version, kind)
        r = self._call("GET", self._url(t, namespace, name))
        _raise_for(r)
        return r.json()

    def list(self, api_version, kind, namespace=None, label_selector=None, field_selector=None):
        return self.list_rv(api_version, kind, namespace, label_selector, field_selector)[0]

    def list_rv(self, api_version, kind, namespace=None, label_selector=None, field_selector=None):
        t = R.rtype(api_version, kind)
        if isinstance(label_selector, dict):
            label_selector = ",".join(f"{k}={v}" for k, v in label_selector.items())
        r = self._call("GET", self._url(t, namespace, query={"labelSelector": label_selector,
                                                            "fieldSelector": field_selector}))
        _raise_for(r)
        body = r.json()
        return body.get("items", []), (body.get("metadata") or {}).get("resourceVersion")

    def update(self, obj):
        t = R.rtype_of(obj)
        r = self._call("PUT", self._url(t, R.ns_of(obj), R.name_of(obj)), data=json.dumps(obj),
                       headers={"Content-Type": "application/json"})
        _raise_for(r)
        return r.json()

    def update_status(self, obj):
        t = R.rtype_of(obj)
        r = self._call("PUT", self._url(t, R.ns_of(obj), R.name_of(obj), "status"), data=json.dumps(obj),
                       headers={"Content-Type": "application/json"})
        _raise_for(r)
        return r.json()

    def patch(self, api_version, kind, name, patch, namespace=None, subresource=None):
        t = R.rtype(api_version, kind)
        r = self._call("PATCH", self._url(t, namespace, name, subresource), data=json.dumps(patch),
                       headers={"Content-Type": "application/merge-patch+json"})
        _raise_for(r)
        return r.json()

    def delete(self, api_version, kind, name, namespace=None, grace_period_seconds=None):
        t = R.rtype(api_version, kind)
        q = None if grace_period_seconds is None else {"gracePeriodSeconds": str(int(grace_period_seconds))}
        r = self._call("DELETE", self._url(t, namespace, name, query=q))
        _raise_for(r)

    def watch(self, api_version, kind, namespace=None, label_selector=None, field_selector=None,
              resource_version=None, stop: threading.Event | None = None, timeout=None):
        t = R.rtype(api_version, kind)
        if isinstance(label_selector, dict):
            label_selector = ",".join(f"{k}={v}" for k, v in label_selector.items())
        q = {"watch": "1", "labelSelector": label_selector, "fieldSelector": field_selector,
             "resourceVersion": resource_version, "timeoutSeconds": int(timeout) if timeout else None}
        with self.session.get(self._url(t, namespace, query=q), stream=True,
                              timeout=(self.timeout, None)) as r:
            _raise_for(r)
            # chunk_size=None: hand over each chunk as it arrives (the default
            # 512-byte reads hold a small event until more bytes follow)
            for line in r.iter_lines(chunk_size=None):
                if stop is not None and stop.is_set():
                    return
                if not line:
                    continue
                ev = json.loads(line)
                if ev.get("type") == "ERROR":
                    raise ApiError(int(ev["object"].get("code", 500)), ev["object"].get("reason", ""),
                                   ev["object"].get("message", ""))
                yield ev["type"], ev["object"]


def wait_for(client, api_version: str, kind: str, done, namespace=None, name: str | None = None,
             label_selector=None, field_selector: str | None = None, timeout: float = 60.0,
             stop: threading.Event | None = None, poll_s: float = 1.0) -> tuple[dict, bool]:
    """Block until ``done(objects)`` holds for the ``kind`` objects named
    ``name`` (and/or matching the selectors); ``objects`` maps name -> object.

    List, then watch from the list's resourceVersion (client-go's
    list-watch): the condition is checked on the listed state (an empty one
    included) and again on every change, so it is seen as soon as it holds,
    and waiting costs one open request instead of a GET per object per poll.
    The list-watch restarts when the server ends the watch (timeout, 410
    Gone); if watching fails altogether (RBAC, proxy) it lists every
    ``poll_s``.  Returns ``(objects, True)``, or the last state and False on
    timeout / ``stop``.
    """
    import time

    fields = ",".join(f for f in (f"metadata.name={name}" if name else None, field_selector) if f) or None
    deadline = time.monotonic() + timeout
    objs: dict = {}
    watch_ok = True
    while True:
        try:
            items, rv = client.list_rv(api_version, kind, namespace, label_selector, fields)
            objs = {o["metadata"]["name"]: o for o in items}
        except (ApiError, OSError, ValueError):
            rv = None
        if done(objs):
            return objs, True
        remaining = deadline - time.monotonic()
        if remaining <= 0 or (stop is not None and stop.is_set()):
            return objs, False
        if watch_ok and rv is not None:
            try:
                for etype, obj in client.watch(api_version, kind, namespace, label_selector, fields,
                                               resource_version=rv, stop=stop,
                                               timeout=max(1.0, min(remaining, 30.0))):
                    n = obj["metadata"]["name"]
                    if etype == "DELETED":
                        objs.pop(n, None)
                    elif etype in ("ADDED", "MODIFIED"):
                        objs[n] = obj
                    else:
                        continue  # BOOKMARK
                    if done(objs):
                        return objs, True
                    if time.monotonic() >= deadline:
                        return objs, False
                continue  # watch ended: list again
            except ApiError as e:
                if e.code != 410:  # 410 Gone: resourceVersion too old, list again
                    watch_ok = False
            except (OSError, ValueError):
                watch_ok = False
        wait = min(poll_s, max(0.0, deadline - time.monotonic()))
        if stop is not None:
            stop.wait(wait)
        else:
            time.sleep(wait)


# maps the operator owns completely: an extra key on the live object is drift
# (e.g. a nodeSelector key would move operand pods), not a server default
EXACT_KEYS = ("nodeSelector", "matchLabels", "args", "command")


def contains(live, desired, key: str = "") -> bool:
    """True when every field of ``desired`` is present with the same value in
    ``live`` (server-side defaults on ``live`` are ignored, except under the
    fully-owned :data:`EXACT_KEYS`)."""
    if key in EXACT_KEYS:
        return live == desired
    if isinstance(desired, dict):
        if not isinstance(live, dict):
            return False
        return all(k in live and contains(live[k], v, k) for k, v in desired.items())
    if isinstance(desired, list):
        if not isinstance(live, list) or len(live) != len(desired):
            return False
        return all(contains(a, b) for a, b in zip(live, desired))
    return live == desired


def apply_object(client, obj: dict, field_owner: str = "amd-gpu-operator",
                 verified: dict | None = None) -> tuple[dict, str]:
    """Create or update ``obj`` when the live object no longer contains it.

    Returns ``(object, action)`` with action in {"created", "updated", "unchanged"}.
    Drift made by someone else (a changed or removed field we own) is reverted:
    reconcile is level-triggered.  Server-added defaults do not count as drift.

    ``verified`` (a dict the caller keeps across passes) remembers, per object,
    the resourceVersion at which the live object was last found to contain
    the desired state with a given hash: while neither changed, the field-by-
    field comparison is skipped (any write by anyone bumps resourceVersion).
    """
    t = R.rtype_of(obj)
    md = dict(R.meta(obj))  # copy the levels this function writes; the rest is only read
    md["annotations"] = dict(md.get("annotations") or {})
    obj = {**obj, "metadata": md}
    ann = md["annotations"]
    ann.setdefault("amd.com/managed-by", field_owner)
    ann["amd.com/last-applied-hash"] = want = R.spec_hash(obj)
    key = (t.api_version, t.kind, R.ns_of(obj), R.name_of(obj))
    server = client.uncached() if hasattr(client, "uncached") else client  # past a read cache (kube/informer.py)
    try:
        cur = client.get(t.api_version, t.kind, R.name_of(obj), R.ns_of(obj))
    except NotFound:
        try:
            return client.create(obj), "created"
        except AlreadyExists:  # created meanwhile by someone else: the cache may not have it yet
            cur = server.get(t.api_version, t.kind, R.name_of(obj), R.ns_of(obj))
    rv = (cur.get("metadata") or {}).get("resourceVersion")
    if verified is not None and rv and verified.get(key) == (rv, want):
        return cur, "unchanged"
    desired = {k: v for k, v in obj.items() if k != "status"}
    if contains(cur, desired):
        if verified is not None and rv:
            verified[key] = (rv, want)
        return cur, "unchanged"
    obj["metadata"]["resourceVersion"] = cur["metadata"]["resourceVersion"]
    # keep fields other controllers own on the live object
    for k in ("ownerReferences", "finalizers"):
        if k in cur["metadata"] and k not in obj["metadata"]:
            obj["metadata"][k] = cur["metadata"][k]
    try:
        return client.update(obj), "updated"
    except Conflict:  # our copy was stale: re-read from the server, not from a cache
        cur = server.get(t.api_version, t.kind, R.name_of(obj), R.ns_of(obj))
        obj["metadata"]["resourceVersion"] = cur["metadata"]["resourceVersion"]
        return client.update(obj), "updated"
