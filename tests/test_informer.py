"""kube/informer.py: watch-backed read caches for the operator loop."""

import threading
import time

import pytest

from amdgpu_operator.kube import resources as R
from amdgpu_operator.kube.client import LocalClient, NotFound, RestClient, apply_object
from amdgpu_operator.kube.fakeapi import FakeApiServer
from amdgpu_operator.kube.httpapi import HttpApiServer
from amdgpu_operator.kube.informer import CachedClient


@pytest.fixture(params=["local", "rest"])
def server(request):
    api = FakeApiServer()
    if request.param == "local":
        yield api, LocalClient(api)
        return
    srv = HttpApiServer(api).start()
    try:
        yield api, RestClient(srv.url)
    finally:
        srv.stop()


def until(cond, timeout=5.0):
    deadline = time.monotonic() + timeout
    while time.monotonic() < deadline:
        if cond():
            return True
        time.sleep(0.005)
    return False


def test_reads_come_from_the_cache_and_follow_the_watch(server):
    api, client = server
    other = LocalClient(api)  # someone else writing
    other.create(R.new("v1", "Namespace", "ns"))
    other.create(R.new("v1", "Node", "a", labels={"gpu": "yes"}))
    stop = threading.Event()
    seen = []
    c = CachedClient(client, [("v1", "Node", None, True), ("v1", "ServiceAccount", "ns")], stop, on_event=seen.append)
    try:
        assert c.wait_synced(5)
        before = api.request_count
        assert c.get("v1", "Node", "a")["metadata"]["labels"] == {"gpu": "yes"}
        assert [n["metadata"]["name"] for n in c.list("v1", "Node", label_selector="gpu=yes")] == ["a"]
        assert api.request_count == before  # no server round trip
        other.patch("v1", "Node", "a", {"metadata": {"labels": {"gpu": "no"}}})
        assert until(lambda: c.get("v1", "Node", "a")["metadata"]["labels"]["gpu"] == "no")
        assert "Node" in seen
        other.delete("v1", "Node", "a")
        assert until(lambda: not c.list("v1", "Node"))
        with pytest.raises(NotFound):
            c.get("v1", "Node", "a")
        # a namespaced kind outside the informer's namespace reads through
        other.create(R.new("v1", "Namespace", "elsewhere"))
        other.create(R.new("v1", "ServiceAccount", "sa", "elsewhere"))
        assert c.get("v1", "ServiceAccount", "sa", "elsewhere")["metadata"]["name"] == "sa"
    finally:
        stop.set()


def test_write_through_and_stale_events(server):
    api, client = server
    LocalClient(api).create(R.new("v1", "Namespace", "ns"))
    stop = threading.Event()
    c = CachedClient(client, [("v1", "ServiceAccount", "ns")], stop)
    try:
        assert c.wait_synced(5)
        sa = c.create(R.new("v1", "ServiceAccount", "sa", "ns"))
        assert c.get("v1", "ServiceAccount", "sa", "ns")["metadata"]["uid"] == sa["metadata"]["uid"]  # at once
        inf = c.informers[("v1", "ServiceAccount")]
        newer = c.patch("v1", "ServiceAccount", "sa", {"metadata": {"labels": {"v": "2"}}}, "ns")
        inf.put(sa)  # an older event arriving late must not win
        assert c.get("v1", "ServiceAccount", "sa", "ns")["metadata"]["resourceVersion"] == \
            newer["metadata"]["resourceVersion"]
        c.delete("v1", "ServiceAccount", "sa", "ns")
        with pytest.raises(NotFound):
            c.get("v1", "ServiceAccount", "sa", "ns")
    finally:
        stop.set()


def test_apply_recovers_from_a_stale_cache():
    api = FakeApiServer()
    client = LocalClient(api)
    client.create(R.new("v1", "Namespace", "ns"))
    stop = threading.Event()
    c = CachedClient(client, [("apps/v1", "DaemonSet", "ns")], stop)
    try:
        assert c.wait_synced(5)
        ds = R.new("apps/v1", "DaemonSet", "d", "ns", spec={"template": {"spec": {"containers": [{"name": "x"}]}}})
        assert apply_object(c, ds)[1] == "created"
        # someone else changes the object; the cache is made stale on purpose
        inf = c.informers[("apps/v1", "DaemonSet")]
        stale = c.get("apps/v1", "DaemonSet", "d", "ns")
        client.patch("apps/v1", "DaemonSet", "d", {"spec": {"template": {"spec": {"containers": [{"name": "y"}]}}}},
                     "ns")
        until(lambda: c.get("apps/v1", "DaemonSet", "d", "ns")["spec"]["template"]["spec"]["containers"][0]["name"]
              == "y")
        with inf._lock:  # roll the cache back to the stale copy
            import pickle

            inf._store[("ns", "d")] = pickle.dumps(stale)
            inf._rvs[("ns", "d")] = int(stale["metadata"]["resourceVersion"])
        want = R.deep(ds)
        want["spec"]["template"]["spec"]["containers"][0]["name"] = "z"
        # stale resourceVersion -> Conflict -> re-read from the server (not the cache) -> update
        assert apply_object(c, want)[1] == "updated"
        assert client.get("apps/v1", "DaemonSet", "d", "ns")["spec"]["template"]["spec"]["containers"][0]["name"] == "z"
    finally:
        stop.set()


def test_kind_the_server_does_not_serve_reads_through():
    """An informer whose list 404s (a CRD that is not installed) gives up and
    reads go to the server."""
    from amdgpu_operator.kube.fakeapi import ApiError

    class NoMonitors(LocalClient):
        def list_rv(self, api_version, kind, *a, **kw):
            if kind == "ServiceMonitor":
                raise ApiError(404, "NotFound", "the server could not find the requested resource")
            return super().list_rv(api_version, kind, *a, **kw)

    api = FakeApiServer()
    stop = threading.Event()
    c = CachedClient(NoMonitors(api), [("monitoring.coreos.com/v1", "ServiceMonitor", "ns")], stop)
    try:
        assert c.wait_synced(5)
        assert c.informers[("monitoring.coreos.com/v1", "ServiceMonitor")].failed.is_set()
        with pytest.raises(NotFound):
            c.get("monitoring.coreos.com/v1", "ServiceMonitor", "m", "ns")
    finally:
        stop.set()


def test_reconciler_loop_rebuilds_its_caches_per_run():
    """Leadership lost and regained: run() ends (its informers stop with it)
    and a later run() must not read from the stopped caches."""
    from amdgpu_operator.api.clusterpolicy import cluster_policy, spec_from_values
    from amdgpu_operator.controller.reconciler import ClusterPolicyReconciler
    from amdgpu_operator.helm.render import load_crd
    from amdgpu_operator.kube.informer import CachedClient

    api = FakeApiServer()
    client = LocalClient(api)
    client.create(load_crd())
    client.create(R.new("v1", "Namespace", "gpu-operator-resources"))  # helm --create-namespace
    client.create(cluster_policy("cluster-policy", spec_from_values({})))
    rec = ClusterPolicyReconciler(client, "gpu-operator-resources")
    for _ in range(2):
        stop = threading.Event()
        seen = []
        th = threading.Thread(target=rec.run, args=(stop,), kwargs={"resync_s": 0.2, "on_result": seen.append},
                              daemon=True)
        th.start()
        assert until(lambda: len(seen) >= 2)
        assert isinstance(rec.client, CachedClient)
        stop.set()
        th.join(5)
        assert rec.client is client
    assert client.list("apps/v1", "DaemonSet", "gpu-operator-resources")  # the operands were applied


def test_informer_survives_an_api_server_restart():
    """kube-apiserver restarts (upgrades, failover) end every watch: the
    informer relists and keeps following changes made meanwhile."""
    api = FakeApiServer()
    srv = HttpApiServer(api).start()
    port = srv.httpd.server_address[1]
    client = RestClient(srv.url, timeout=2.0)
    local = LocalClient(api)
    local.create(R.new("v1", "Node", "a"))
    stop = threading.Event()
    c = CachedClient(client, [("v1", "Node", None, True)], stop)
    try:
        assert c.wait_synced(5)
        srv.stop()
        local.create(R.new("v1", "Node", "b"))  # changes while the server is away
        local.delete("v1", "Node", "a")
        srv = HttpApiServer(api, port=port).start()
        assert until(lambda: [n["metadata"]["name"] for n in c.list("v1", "Node")] == ["b"], timeout=10)
        local.create(R.new("v1", "Node", "c"))
        assert until(lambda: len(c.list("v1", "Node")) == 2, timeout=5)
    finally:
        stop.set()
        srv.stop()


def test_timed_out_watch_resumes_without_a_relist():
    """A watch that ends at its timeout resumes from the last version seen
    (client-go's reflector); only an error costs a full list."""
    from amdgpu_operator.kube.informer import Informer

    c = LocalClient(FakeApiServer())
    c.create(R.new("v1", "Namespace", "ns"))
    lists = []
    orig = c.list_rv
    c.list_rv = lambda *a, **kw: (lists.append(1), orig(*a, **kw))[1]
    stop = threading.Event()
    inf = Informer(c, "v1", "ConfigMap", "ns", watch_timeout_s=0.2).start(stop)
    try:
        assert inf.synced.wait(5)
        for i in range(3):
            c.create(R.new("v1", "ConfigMap", f"cm{i}", "ns"))
            time.sleep(0.3)  # each watch times out between writes
        deadline = time.time() + 5
        while time.time() < deadline and len(inf.list("ns")) < 3:
            time.sleep(0.01)
        assert [R.name_of(o) for o in inf.list("ns")] == ["cm0", "cm1", "cm2"]
        assert len(lists) == 1
    finally:
        stop.set()


def test_echoes_of_own_writes_trigger_nothing():
    """A CachedClient's own writes come back on the watch: the cache takes
    them, but the change callback (the operator's reconcile trigger) is not
    called for them; another party's write to the same object is."""
    import threading
    import time

    from amdgpu_operator.kube import resources as R
    from amdgpu_operator.kube.client import LocalClient
    from amdgpu_operator.kube.fakeapi import FakeApiServer
    from amdgpu_operator.kube.informer import CachedClient

    server = LocalClient(FakeApiServer())
    seen, stop = [], threading.Event()
    cc = CachedClient(server, [("v1", "Node", None, True)], stop, on_event=seen.append)
    try:
        assert cc.wait_synced(5)
        time.sleep(0.05)
        seen.clear()
        cc.create(R.new("v1", "Node", "n1"))
        cc.patch("v1", "Node", "n1", {"metadata": {"labels": {"a": "1"}}})
        time.sleep(0.2)
        assert seen == [] and cc.get("v1", "Node", "n1")["metadata"]["labels"] == {"a": "1"}
        server.patch("v1", "Node", "n1", {"metadata": {"labels": {"b": "2"}}})  # someone else
        deadline = time.time() + 2
        while not seen and time.time() < deadline:
            time.sleep(0.01)
        assert seen == ["Node"]
    finally:
        stop.set()
