"""The device plugin's gRPC stack against a grpc-go-shaped kubelet.

The kubelet that registers and drives a device plugin on a real node is a
grpc-go program (/root/reference/README.md:205,211,220: the device plugin
advertises the GPUs through it).  grpc-go itself cannot run here (no Go
toolchain), so tests/helpers/h2go.py reproduces the parts of its wire
behaviour that the grpcio interop tests (tests/test_rpc.py) do not cover:
HPACK with incremental indexing and eviction (grpc-go's encoder indexes
every field; grpcio's does not the same way), the server's BDP and
graceful-stop pings, two-phase GOAWAY, ``grpc-message`` sent empty on
success, Trailers-Only errors, and multiplexed calls on one connection.
What a real grpc-go peer does beyond that stand-in stays parity unpinned.
"""

import time

import pytest

from amdgpu_operator.deviceplugin import api
from amdgpu_operator.deviceplugin.server import DevicePluginManager, PluginConfig
from amdgpu_operator.rpc import wire
from amdgpu_operator.testing import fakesys
from tests.helpers import h2go


def _path(name):
    return api.method_path(api.DEVICE_PLUGIN_SERVICE, name)


def _wait(pred, timeout: float = 5.0) -> bool:
    """Peers record frames on their reader threads: poll for the effect."""
    deadline = time.monotonic() + timeout
    while not pred():
        if time.monotonic() >= deadline:
            return False
        time.sleep(0.005)
    return True


def _dec(name, out, idx=0):
    return api.DEVICE_PLUGIN_METHODS[name][1].FromString(out["messages"][idx])


def _register_handler(seen: list):
    req_cls = api.REGISTRATION_METHODS["Register"][0]

    def handler(method, body):
        if method != api.method_path(api.REGISTRATION_SERVICE, "Register"):
            return 12, f"unknown method {method}", b""
        req = req_cls.FromString(body)
        seen.append(req)
        if req.version != api.VERSION:
            return 3, f"unsupported version {req.version}: 100% wrong", b""
        return 0, "", b""
    return handler


@pytest.fixture
def node(tmp_path):
    root = str(tmp_path / "host")
    fakesys.build_node(root, 8)
    sock_dir = tmp_path / "dp"
    sock_dir.mkdir()
    return root, str(sock_dir)


def test_go_kubelet_registers_and_drives_the_real_plugin(node):
    """The production plugin registers with a grpc-go-shaped Registration
    server, then that "kubelet" dials the plugin and makes the device
    manager's calls on one multiplexed connection: options, a ListAndWatch
    left open, GetPreferredAllocation and Allocate interleaved with it,
    a plugin-side health flip streamed, and a cancel by RST_STREAM."""
    root, sock_dir = node
    seen = []
    kubelet = h2go.GoServer(f"{sock_dir}/kubelet.sock", _register_handler(seen))
    m = DevicePluginManager(PluginConfig(socket_dir=sock_dir, sysfs_root=root, watch_interval_s=0.05))
    m.start()
    try:
        deadline = time.monotonic() + 10
        while not seen and time.monotonic() < deadline:
            time.sleep(0.01)
        assert seen and seen[0].resource_name == "amd.com/gpu" and seen[0].options.get_preferred_allocation_available
        assert kubelet.bdp_pings_sent == 1 and _wait(lambda: h2go.BDP_PING in kubelet.conns[0].pings_acked)  # acked
        # the kubelet dials the endpoint the plugin registered, authority = the socket path (older grpc-go)
        k = h2go.GoClient(f"{sock_dir}/{seen[0].endpoint}", authority=f"{sock_dir}/{seen[0].endpoint}")
        try:
            empty = api.pb["Empty"]().SerializeToString()
            opts = _dec("GetDevicePluginOptions", k.call(_path("GetDevicePluginOptions"), empty, timeout_s=5))
            assert opts.get_preferred_allocation_available
            law = k.start_call(_path("ListAndWatch"), empty)
            kind, hdrs, end = k.next_event(law)
            assert kind == "headers" and dict(hdrs)[":status"] == "200" and not end
            body = bytearray()
            while len(h2go.split_grpc(bytes(body))) < 1:
                kind, data, end = k.next_event(law)
                assert kind == "data" and not end
                body += data
            first = api.pb["ListAndWatchResponse"].FromString(h2go.split_grpc(bytes(body))[0])
            ids = [d.ID for d in first.devices]
            assert len(ids) == 8 and all(d.health == api.HEALTHY for d in first.devices)
            # preferred allocation and allocation on streams opened together, framed three ways
            pref = api.pb["PreferredAllocationRequest"]()
            pref.container_requests.add(available_deviceIDs=ids, allocation_size=4)
            alloc = api.pb["AllocateRequest"]()
            alloc.container_requests.add(devices_ids=ids[:2])
            s1 = k.start_call(_path("GetPreferredAllocation"), pref.SerializeToString(), timeout_s=5, framing="split")
            s2 = k.start_call(_path("Allocate"), alloc.SerializeToString(), timeout_s=5, framing="empty-end")
            k.ping()
            r2, r1 = k.finish(s2), k.finish(s1)
            for r in (r1, r2):
                assert r["headers"][":status"] == "200" and r["trailers"]["grpc-status"] == "0", r
            picked = list(_dec("GetPreferredAllocation", r1).container_responses[0].deviceIDs)
            assert len(picked) == 4 and set(picked) <= set(ids)
            resp = _dec("Allocate", r2).container_responses[0]
            assert resp.devices[0].host_path == "/dev/kfd" and len(resp.devices) == 3
            assert _wait(lambda: h2go.BDP_PING in k.conn.pings_acked)
            # an unknown device is refused with the plugin's status, on the same connection
            bad = api.pb["AllocateRequest"]()
            bad.container_requests.add(devices_ids=["no-such-gpu"])
            r = k.call(_path("Allocate"), bad.SerializeToString(), timeout_s=5)
            assert r["trailers"]["grpc-status"] == str(wire.StatusCode.INVALID_ARGUMENT.value)
            assert "no-such-gpu" in wire._pct_decode(r["trailers"]["grpc-message"])
            # a health flip on the plugin side reaches the open stream
            m.set_health(ids[3], False, "test")
            body = bytearray()
            while True:
                kind, data, end = k.next_event(law)
                assert kind == "data"
                body += data
                msgs = h2go.split_grpc(bytes(body))
                if msgs and any(d.ID == ids[3] and d.health == api.UNHEALTHY
                                for d in api.pb["ListAndWatchResponse"].FromString(msgs[-1]).devices):
                    break
            k.cancel(law)  # the kubelet stops the endpoint: the stream ends, the connection stays
            r = k.call(_path("GetDevicePluginOptions"), empty, timeout_s=5)
            assert r["trailers"]["grpc-status"] == "0"
            assert k.conn.enc.indexed_refs > 0  # later blocks referenced the dynamic table
        finally:
            k.close()
    finally:
        m.stop()
        kubelet.stop()


@pytest.fixture
def echo_server(tmp_path):
    class Svc:
        def Allocate(self, request, context):
            out = api.pb["AllocateResponse"]()
            r = out.container_responses.add()
            for i in (i for c in request.container_requests for i in c.devices_ids):
                r.envs[f"ID_{i}"] = i
            return out

    svc = Svc()
    name = "Allocate"
    req, resp, stream = api.DEVICE_PLUGIN_METHODS[name]
    srv = wire.Server({_path(name): wire.MethodHandler(svc.Allocate, req.FromString, resp.SerializeToString, stream)})
    path = str(tmp_path / "echo.sock")
    srv.add_unix(path)
    srv.start()
    yield path
    srv.stop(0.5)


def test_go_hpack_table_churn_on_one_connection(echo_server):
    """300 calls on one connection with per-call metadata and deadlines, as
    grpc-go indexes them: the dynamic table fills and evicts hundreds of
    times, and every header block still decodes on our side (a decoder out
    of step would route a call to the wrong method or drop the connection)."""
    k = h2go.GoClient(echo_server)
    try:
        for i in range(300):
            req = api.pb["AllocateRequest"]()
            req.container_requests.add(devices_ids=[f"d{i}"])
            framing = ("end-on-data", "empty-end", "split")[i % 3]
            md = [("x-pod-uid", f"{i:08x}-1f2e-4d3c-8b7a-{i * 7919:012x}"), ("x-attempt", str(i % 5))]
            out = k.call(_path("Allocate"), req.SerializeToString(), timeout_s=5 + i / 1000, framing=framing,
                         metadata=md)
            assert out["trailers"]["grpc-status"] == "0", (i, out)
            assert dict(_dec("Allocate", out).container_responses[0].envs) == {f"ID_d{i}": f"d{i}"}
            if i % 50 == 0:
                k.ping(bytes([i % 256]) * 8)
        assert k.conn.enc.evictions > 200 and k.conn.enc.indexed_refs > 300
        assert _wait(lambda: len(k.conn.pings_acked) == 6)
        # many calls in flight at once on the one connection
        sids = []
        for i in range(40):
            req = api.pb["AllocateRequest"]()
            req.container_requests.add(devices_ids=[f"m{i}"])
            sids.append(k.start_call(_path("Allocate"), req.SerializeToString(), timeout_s=5))
        for i, sid in reversed(list(enumerate(sids))):
            out = k.finish(sid)
            assert dict(_dec("Allocate", out).container_responses[0].envs) == {f"ID_m{i}": f"m{i}"}
    finally:
        k.close()


def test_our_client_against_go_shaped_registration_server(tmp_path):
    """Our client (the plugin's Register call) against grpc-go's server
    wire: responses indexed into the dynamic table, an empty grpc-message on
    success, a Trailers-Only error, the BDP ping answered, and a graceful
    stop (GOAWAY 2^31-1 + ping, then GOAWAY(last) and close) after which the
    next call opens a new connection."""
    seen = []
    path = str(tmp_path / "kubelet.sock")
    srv = h2go.GoServer(path, _register_handler(seen))
    req_cls, resp_cls, _ = api.REGISTRATION_METHODS["Register"]
    try:
        with wire.Channel(path) as ch:
            call = ch.unary_unary(api.method_path(api.REGISTRATION_SERVICE, "Register"),
                                  request_serializer=req_cls.SerializeToString, response_deserializer=resp_cls.FromString)
            ok = req_cls(version=api.VERSION, endpoint="amd.sock", resource_name="amd.com/gpu")
            for i in range(60):
                assert call(ok, timeout=5) == api.pb["Empty"]()
            assert srv.conns[0].enc.indexed_refs > 100  # :status/content-type/grpc-* by dynamic index
            with pytest.raises(wire.RpcError) as e:
                call(req_cls(version="v0"), timeout=5)
            assert e.value.code() is wire.StatusCode.INVALID_ARGUMENT
            assert e.value.details() == "unsupported version v0: 100% wrong"
            assert _wait(lambda: h2go.BDP_PING in srv.conns[0].pings_acked)
            srv.drain()
            assert call(ok, timeout=5) == api.pb["Empty"]()  # served under the first GOAWAY; ping acked
            assert _wait(lambda: h2go.GOAWAY_PING in srv.conns[0].pings_acked)
            assert srv.conns[0].closed.wait(5)
            for _ in range(3):
                assert call(ok, timeout=5) == api.pb["Empty"]()
            assert len(srv.conns) == 2 and {n for n, _, _ in srv.calls[-3:]} == {1}
            assert len(seen) == 65
            hdrs = srv.calls[0][2]
            assert hdrs[":authority"] == "localhost" and hdrs["te"] == "trailers" and "grpc-timeout" in hdrs
    finally:
        srv.stop()


def test_go_client_registration_concurrent_with_plugin_restart(node):
    """A plugin restarting (new socket, new server) while the grpc-go-shaped
    kubelet keeps its Registration server: both registrations arrive, each
    on its own connection, and the second plugin serves the kubelet."""
    root, sock_dir = node
    seen = []
    kubelet = h2go.GoServer(f"{sock_dir}/kubelet.sock", _register_handler(seen))
    try:
        for n in (1, 2):
            m = DevicePluginManager(PluginConfig(socket_dir=sock_dir, sysfs_root=root, watch_interval_s=0.05))
            m.start()
            try:
                deadline = time.monotonic() + 10
                while len(seen) < n and time.monotonic() < deadline:
                    time.sleep(0.01)
                assert len(seen) == n
                k = h2go.GoClient(f"{sock_dir}/{seen[-1].endpoint}")
                try:
                    out = k.call(_path("GetDevicePluginOptions"), api.pb["Empty"]().SerializeToString(), timeout_s=5)
                    assert out["trailers"]["grpc-status"] == "0"
                finally:
                    k.close()
            finally:
                m.stop()
        assert len({n for n, _, _ in kubelet.calls}) == 2
    finally:
        kubelet.stop()


def test_go_stand_in_encoder_matches_rfc7541_indexing():
    """The stand-in's encoder against our decoder on RFC 7541 C.3's request
    sequence (three blocks on one connection sharing the dynamic table)."""
    from amdgpu_operator.rpc import hpack

    enc, dec = h2go.GoEncoder(), hpack.Decoder()
    reqs = [[(":method", "GET"), (":scheme", "http"), (":path", "/"), (":authority", "www.example.com")],
            [(":method", "GET"), (":scheme", "http"), (":path", "/"), (":authority", "www.example.com"),
             ("cache-control", "no-cache")],
            [(":method", "GET"), (":scheme", "https"), (":path", "/index.html"), (":authority", "www.example.com"),
             ("custom-key", "custom-value")]]
    blocks = [enc.encode(r) for r in reqs]
    # C.4.1-C.4.3 (Huffman), which is what a Go encoder emits for these fields
    assert blocks[0].hex() == "828684418cf1e3c2e5f23a6ba0ab90f4ff"
    assert blocks[1].hex() == "828684be5886a8eb10649cbf"
    assert blocks[2].hex() == "828785bf408825a849e95ba97d7f8925a849e95bb8e8b4bf"
    assert [dec.decode(b) for b in blocks] == reqs
    assert enc.size == dec.size == 164
