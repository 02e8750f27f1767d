"""Fake API server semantics and the REST client over HTTP."""

import threading
import time

import pytest

from amdgpu_operator.kube import resources as R
from amdgpu_operator.kube.client import AlreadyExists, Conflict, LocalClient, NotFound, RestClient, apply_object
from amdgpu_operator.kube.fakeapi import FakeApiServer
from amdgpu_operator.kube.httpapi import HttpApiServer


@pytest.fixture(params=["local", "rest"])
def client(request):
    api = FakeApiServer()
    if request.param == "local":
        yield LocalClient(api)
        return
    srv = HttpApiServer(api).start()
    try:
        yield RestClient(srv.url)
    finally:
        srv.stop()


def test_crud_and_selectors(client):
    client.create(R.new("v1", "Namespace", "ns"))
    client.create(R.new("v1", "Node", "a", labels={"gpu": "yes", "zone": "z1"}))
    client.create(R.new("v1", "Node", "b", labels={"zone": "z2"}))
    assert [n["metadata"]["name"] for n in client.list("v1", "Node", label_selector="gpu=yes")] == ["a"]
    assert len(client.list("v1", "Node", label_selector="zone in (z1,z2)")) == 2
    assert [n["metadata"]["name"] for n in client.list("v1", "Node", label_selector="!gpu")] == ["b"]
    assert [n["metadata"]["name"] for n in client.list("v1", "Node", label_selector="zone!=z1")] == ["b"]
    with pytest.raises(AlreadyExists):
        client.create(R.new("v1", "Node", "a"))
    with pytest.raises(NotFound):
        client.get("v1", "Node", "zz")
    p = client.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "p", "namespace": "ns"},
                       "spec": {"nodeName": "a"}})
    assert client.list("v1", "Pod", "ns", field_selector="spec.nodeName=a")[0]["metadata"]["uid"] == p["metadata"]["uid"]
    assert client.list("v1", "Pod", "ns", field_selector="spec.nodeName=b") == []


def test_conflict_and_status_subresource(client):
    n = client.create(R.new("v1", "Node", "a"))
    stale = dict(n)
    n["metadata"]["labels"] = {"x": "1"}
    n2 = client.update(n)
    assert int(n2["metadata"]["generation"]) == 1  # metadata-only change
    with pytest.raises(Conflict):
        client.update(stale)
    n2["status"] = {"allocatable": {"amd.com/gpu": "8"}}
    client.update_status(n2)
    cur = client.get("v1", "Node", "a")
    assert cur["status"]["allocatable"]["amd.com/gpu"] == "8"
    cur["status"] = {}
    cur["spec"] = {"unschedulable": True}
    cur = client.update(cur)  # main endpoint ignores status
    assert cur["status"]["allocatable"]["amd.com/gpu"] == "8" and cur["metadata"]["generation"] == 2


def test_merge_patch_removes_keys(client):
    client.create(R.new("v1", "Node", "a", labels={"x": "1", "y": "2"}))
    client.patch("v1", "Node", "a", {"metadata": {"labels": {"x": None, "z": "3"}}})
    assert client.get("v1", "Node", "a")["metadata"]["labels"] == {"y": "2", "z": "3"}


def test_watch_stream(client):
    client.create(R.new("v1", "Namespace", "ns"))
    events = []
    stop = threading.Event()

    def w():
        for et, obj in client.watch("apps/v1", "DaemonSet", namespace="ns", stop=stop, timeout=5):
            events.append((et, obj["metadata"]["name"]))
            if len(events) == 3:
                return

    th = threading.Thread(target=w)
    th.start()
    time.sleep(0.3)
    client.create(R.new("apps/v1", "DaemonSet", "d", "ns", spec={"a": 1}))
    client.patch("apps/v1", "DaemonSet", "d", {"spec": {"a": 2}}, "ns")
    client.delete("apps/v1", "DaemonSet", "d", "ns")
    th.join(timeout=10)
    stop.set()
    assert events == [("ADDED", "d"), ("MODIFIED", "d"), ("DELETED", "d")]


def test_watch_from_resource_version():
    api = FakeApiServer()
    c = LocalClient(api)
    c.create(R.new("v1", "Node", "a"))
    rv = api.resource_version()
    c.create(R.new("v1", "Node", "b"))
    got = [o["metadata"]["name"] for _, o in c.watch("v1", "Node", resource_version=rv, timeout=0.3)]
    assert got == ["b"]


def test_watch_selector_transitions_are_added_and_deleted(client):
    """kube-apiserver's watch cache: a modification that moves an object into
    a watch's label/field selector is ADDED, one that moves it out is DELETED
    (with the object as it last matched) - how a kubelet watching
    spec.nodeName sees the pod the scheduler just bound.  Also on a replay
    from a resourceVersion."""
    c = client
    c.create(R.new("v1", "Namespace", "ns"))
    _, rv = c.list_rv("v1", "Namespace")
    c.create(R.new("v1", "Pod", "p", "ns", spec={"containers": []}))
    c.patch("v1", "Pod", "p", {"spec": {"nodeName": "n1"}}, "ns")
    c.patch("v1", "Pod", "p", {"metadata": {"labels": {"x": "1"}}}, "ns")
    c.patch("v1", "Pod", "p", {"spec": {"nodeName": "n2"}}, "ns")
    got = [(et, o["spec"].get("nodeName")) for et, o in
           c.watch("v1", "Pod", "ns", field_selector="spec.nodeName=n1", resource_version=rv, timeout=0.3)]
    assert got == [("ADDED", "n1"), ("MODIFIED", "n1"), ("DELETED", "n1")]
    got = [et for et, _ in c.watch("v1", "Pod", "ns", label_selector="x=1", resource_version=rv, timeout=0.3)]
    assert got == ["ADDED", "MODIFIED"]


def test_owner_reference_gc_and_namespace_delete(client):
    client.create(R.new("v1", "Namespace", "ns"))
    owner = client.create(R.new("amd.com/v1", "ClusterPolicy", "cp"))
    ds = R.new("apps/v1", "DaemonSet", "d", "ns")
    ds["metadata"]["ownerReferences"] = [{"uid": owner["metadata"]["uid"], "kind": "ClusterPolicy", "name": "cp"}]
    client.create(ds)
    client.create(R.new("v1", "ConfigMap", "c", "ns"))
    client.delete("amd.com/v1", "ClusterPolicy", "cp")
    with pytest.raises(NotFound):
        client.get("apps/v1", "DaemonSet", "d", "ns")
    client.delete("v1", "Namespace", "ns")
    with pytest.raises(NotFound):
        client.get("v1", "ConfigMap", "c", "ns")


@pytest.mark.parametrize("cached", [False, True])
def test_apply_object_reverts_drift(client, cached):
    verified = {} if cached else None  # the reconciler's fast path must not hide drift
    client.create(R.new("v1", "Namespace", "ns"))
    ds = R.new("apps/v1", "DaemonSet", "d", "ns", spec={"template": {"spec": {"containers": [{"name": "x"}]}}})
    before = R.deep(ds)
    assert apply_object(client, ds, verified=verified)[1] == "created"
    assert apply_object(client, ds, verified=verified)[1] == "unchanged"
    assert apply_object(client, ds, verified=verified)[1] == "unchanged"
    client.patch("apps/v1", "DaemonSet", "d", {"spec": {"template": {"spec": {"containers": [{"name": "hacked"}]}}}},
                 "ns")
    assert apply_object(client, ds, verified=verified)[1] == "updated"
    assert client.get("apps/v1", "DaemonSet", "d", "ns")["spec"]["template"]["spec"]["containers"][0]["name"] == "x"
    # server-side defaults on the live object are not drift
    client.patch("apps/v1", "DaemonSet", "d", {"spec": {"revisionHistoryLimit": 10}}, "ns")
    assert apply_object(client, ds, verified=verified)[1] == "unchanged"
    # a changed desired object is applied even when the live one is unchanged
    ds2 = R.deep(ds)
    ds2["spec"]["template"]["spec"]["containers"][0]["name"] = "y"
    assert apply_object(client, ds2, verified=verified)[1] == "updated"
    assert ds == before  # the caller's object is not modified


def test_selector_parser_edge_cases():
    reqs = R.parse_selector("a=b, c in (x, y),!d,e")
    assert R.matches({"a": "b", "c": "y", "e": "1"}, reqs)
    assert not R.matches({"a": "b", "c": "z", "e": "1"}, reqs)
    assert not R.matches({"a": "b", "c": "x", "d": "1", "e": "1"}, reqs)
    assert R.matches({"k": "v"}, R.parse_selector({"matchLabels": {"k": "v"}}))
    node = {"metadata": {"labels": {"gpu": "true", "zone": "a"}}}
    aff = {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {"nodeSelectorTerms": [
        {"matchExpressions": [{"key": "zone", "operator": "In", "values": ["a"]}]}]}}}
    assert R.node_selector_matches(node, {"gpu": "true"}, aff)
    assert not R.node_selector_matches(node, {"gpu": "false"})


def test_unversioned_watch_starts_with_current_state(client):
    """kube-apiserver semantics: a watch without resourceVersion first
    replays the current objects as ADDED."""
    client.create(R.new("v1", "Node", "a"))
    client.create(R.new("v1", "Node", "b"))
    got = [(et, o["metadata"]["name"]) for et, o in client.watch("v1", "Node", timeout=0.3)]
    assert sorted(got) == [("ADDED", "a"), ("ADDED", "b")]


def test_wait_for_list_then_watch(client):
    from amdgpu_operator.kube.client import wait_for

    client.create(R.new("v1", "Namespace", "ns"))
    # an empty state can satisfy the condition at once (no event ever comes)
    objs, ok = wait_for(client, "v1", "Pod", lambda o: not o, namespace="ns", timeout=2)
    assert ok and objs == {}
    for i in range(3):
        client.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": f"p{i}", "namespace": "ns",
                                                                       "labels": {"run": "x"}}, "spec": {}})

    def finish():
        time.sleep(0.2)
        for i in range(3):
            p = client.get("v1", "Pod", f"p{i}", "ns")
            p["status"] = {"phase": "Succeeded"}
            client.update_status(p)

    th = threading.Thread(target=finish)
    th.start()
    t0 = time.monotonic()
    objs, ok = wait_for(client, "v1", "Pod", lambda o: len(o) == 3 and all(
        (p.get("status") or {}).get("phase") == "Succeeded" for p in o.values()),
        namespace="ns", label_selector="run=x", timeout=10, poll_s=5.0)
    th.join()
    assert ok and sorted(objs) == ["p0", "p1", "p2"]
    assert time.monotonic() - t0 < 2.0  # event-driven, not one poll_s per check
    # a single object by name; a timeout returns the last state
    objs, ok = wait_for(client, "v1", "Pod", lambda o: False, namespace="ns", name="p1", timeout=0.3)
    assert not ok and list(objs) == ["p1"]


def test_wait_for_falls_back_to_listing():
    """No watch permission: wait_for lists every poll_s instead."""
    from amdgpu_operator.kube.client import wait_for
    from amdgpu_operator.kube.fakeapi import ApiError

    class NoWatch(LocalClient):
        def watch(self, *a, **kw):
            raise ApiError(403, "Forbidden", "watch not allowed")
            yield  # pragma: no cover

    c = NoWatch(FakeApiServer())
    c.create(R.new("v1", "Node", "a"))
    threading.Timer(0.2, lambda: c.patch("v1", "Node", "a", {"metadata": {"labels": {"x": "1"}}})).start()
    objs, ok = wait_for(c, "v1", "Node", lambda o: "x" in (o.get("a", {}).get("metadata", {}).get("labels") or {}),
                        name="a", timeout=5, poll_s=0.05)
    assert ok


def test_token_file_auth_follows_rotation(tmp_path):
    """In-cluster: the projected service-account token rotates; the client
    re-reads it (at most every reload period), as client-go does."""
    from amdgpu_operator.kube.client import TokenFileAuth

    now = [0.0]
    tok = tmp_path / "token"
    tok.write_text("first\n")
    auth = TokenFileAuth(str(tok), reload_s=60.0, clock=lambda: now[0])

    class Req:
        headers: dict = {}

    r = Req()
    r.headers = {}
    assert auth(r).headers["Authorization"] == "Bearer first"
    tok.write_text("second\n")
    now[0] = 30.0
    assert auth(r).headers["Authorization"] == "Bearer first"  # within the reload period
    now[0] = 61.0
    assert auth(r).headers["Authorization"] == "Bearer second"
    tok.unlink()
    now[0] = 200.0
    assert auth(r).headers["Authorization"] == "Bearer second"  # unreadable: keep the last one


def test_rest_client_sends_the_rotated_token(tmp_path):
    """End to end over HTTP: every request carries the current token."""
    import http.server
    import json as _json
    import threading as _th

    seen = []

    class H(http.server.BaseHTTPRequestHandler):
        def log_message(self, *a):
            pass

        def do_GET(self):
            seen.append(self.headers.get("Authorization"))
            body = _json.dumps({"apiVersion": "v1", "kind": "Node", "metadata": {"name": "a"}}).encode()
            self.send_response(200)
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), H)
    _th.Thread(target=srv.serve_forever, daemon=True).start()
    try:
        tok = tmp_path / "token"
        tok.write_text("t1")
        c = RestClient(f"http://127.0.0.1:{srv.server_address[1]}", token_file=str(tok))
        c.session.auth.reload_s = 0.0
        c.get("v1", "Node", "a")
        tok.write_text("t2")
        c.get("v1", "Node", "a")
        assert seen == ["Bearer t1", "Bearer t2"]
    finally:
        srv.shutdown()


def test_rest_client_retries_throttling_and_reads():
    """429 / 503 with Retry-After are retried for every verb (the server did
    not act); a refused connection only for reads."""
    import http.server
    import json as _json
    import threading as _th

    hits = {"GET": 0, "POST": 0}

    class H(http.server.BaseHTTPRequestHandler):
        def log_message(self, *a):
            pass

        def _reply(self, verb):
            hits[verb] += 1
            if hits[verb] <= 2:
                self.send_response(429 if verb == "GET" else 503)
                self.send_header("Retry-After", "0")
                self.send_header("Content-Length", "0")
                self.end_headers()
                return
            body = _json.dumps({"apiVersion": "v1", "kind": "Node", "metadata": {"name": "a"}}).encode()
            self.send_response(200 if verb == "GET" else 201)
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

        def do_GET(self):
            self._reply("GET")

        def do_POST(self):
            n = int(self.headers.get("Content-Length") or 0)
            self.rfile.read(n)
            self._reply("POST")

    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), H)
    _th.Thread(target=srv.serve_forever, daemon=True).start()
    port = srv.server_address[1]
    try:
        c = RestClient(f"http://127.0.0.1:{port}")
        assert c.get("v1", "Node", "a")["metadata"]["name"] == "a" and hits["GET"] == 3
        assert c.create(R.new("v1", "Node", "a"))["metadata"]["name"] == "a" and hits["POST"] == 3
    finally:
        srv.shutdown()
        srv.server_close()
    dead = RestClient(f"http://127.0.0.1:{port}")
    dead.RETRIES = 1
    with pytest.raises(ConnectionError):
        dead.create(R.new("v1", "Node", "b"))  # a write is not repeated blindly
    with pytest.raises(ConnectionError):
        dead.get("v1", "Node", "a")
