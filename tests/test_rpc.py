"""The operator's own gRPC stack (rpc/proto.py, rpc/hpack.py, rpc/wire.py).

- protobuf codec: every kubelet message, random contents, both directions
  against google.protobuf's codec of the same schema (deviceplugin/protodef.py);
- HPACK: RFC 7541 Appendix C vectors (plain and Huffman-coded requests, a
  size-bounded dynamic table with evictions), malformed input rejected;
- HTTP/2 gRPC against grpcio in both directions: grpcio client -> our server
  (unary, server streaming, status codes, cancellation, messages larger than
  the flow-control windows and frames), our client -> grpcio server (status
  and message, deadlines, wait-for-ready, kept-alive connection across a
  server restart, large responses).
"""

import threading
import time
from concurrent import futures

import grpc
import pytest
from hypothesis import given, settings
from hypothesis import strategies as hs

from amdgpu_operator.deviceplugin import api
from amdgpu_operator.rpc import hpack, proto, wire

PB_DP, PB_PR = api.protobuf_classes()

_text = hs.text(max_size=12)
_i64 = hs.integers(-(1 << 63), (1 << 63) - 1)
_i32 = hs.integers(-(1 << 31), (1 << 31) - 1)


def _value(ftype, depth, schema):
    if ftype == "string":
        return _text
    if ftype == "bool":
        return hs.booleans()
    if ftype == "int64":
        return _i64
    if ftype == "int32":
        return _i32
    if ftype == "uint64":
        return hs.integers(0, (1 << 64) - 1)
    return _message_dict(ftype, schema, depth + 1)


def _message_dict(name, schema, depth=0):
    fields = {}
    for fname, _, ftype, label in schema[name]:
        if ftype.startswith("map<"):
            fields[fname] = hs.dictionaries(_text, _text, max_size=3)
        elif depth > 3 and ftype not in proto.SCALARS:
            continue
        elif label == "rep":
            fields[fname] = hs.lists(_value(ftype, depth, schema), max_size=3)
        else:
            fields[fname] = _value(ftype, depth, schema)
    return hs.fixed_dictionaries({}, optional=fields)


def _fill_pb(msg, d):
    """dict -> google.protobuf message (maps and nested messages included)."""
    for k, v in d.items():
        f = msg.DESCRIPTOR.fields_by_name[k]
        if f.message_type is not None and f.message_type.GetOptions().map_entry:
            getattr(msg, k).update(v)
        elif f.message_type is not None and f.is_repeated:
            for item in v:
                _fill_pb(getattr(msg, k).add(), item)
        elif f.message_type is not None:
            sub = getattr(msg, k)
            _fill_pb(sub, v)
            sub.SetInParent()
        elif f.is_repeated:
            getattr(msg, k).extend(v)
        else:
            setattr(msg, k, v)
    return msg


def _to_ours(cls, d):
    kw = {}
    for k, v in d.items():
        f = cls.BY_NAME[k]
        if f.is_message and f.repeated:
            kw[k] = [_to_ours(f.msg_cls, x) for x in v]
        elif f.is_message:
            kw[k] = _to_ours(f.msg_cls, v)
        else:
            kw[k] = v
    return cls(**kw)


def _as_dict(m):
    """Either codec's message -> plain data (proto3 defaults dropped)."""
    out = {}
    if isinstance(m, proto.Message):
        for f in type(m).FIELDS:
            v = getattr(m, f.name)
            if f.map_types is not None:
                v = dict(v)
            elif f.is_message and f.repeated:
                v = [_as_dict(x) for x in v]
            elif f.is_message:
                if not m.HasField(f.name):
                    continue
                v = _as_dict(v)
            elif f.repeated:
                v = list(v)
            if v or v == {} and f.is_message and not f.repeated:
                out[f.name] = v
        return out
    for f in m.DESCRIPTOR.fields:
        v = getattr(m, f.name)
        if f.message_type is not None and f.message_type.GetOptions().map_entry:
            v = dict(v)
        elif f.message_type is not None and f.is_repeated:
            v = [_as_dict(x) for x in v]
        elif f.message_type is not None:
            if not m.HasField(f.name):
                continue
            v = _as_dict(v)
        elif f.is_repeated:
            v = list(v)
        if v or v == {} and f.message_type is not None and not f.is_repeated:
            out[f.name] = v
    return out


def _has_map(name, schema):
    return any(ft.startswith("map<") or (ft in schema and _has_map(ft, schema)) for _, _, ft, _ in schema[name])


@pytest.mark.parametrize("family,name", [("dp", n) for n in api._MESSAGES] + [("pr", n) for n in api._PR_MESSAGES])
def test_codec_matches_google_protobuf(family, name):
    schema = api._MESSAGES if family == "dp" else api._PR_MESSAGES
    ours_cls = (api.pb if family == "dp" else api.podres)[name]
    ref_cls = (PB_DP if family == "dp" else PB_PR)[name]

    @settings(max_examples=60, deadline=None)
    @given(_message_dict(name, schema))
    def check(d):
        ours = _to_ours(ours_cls, d)
        ref = _fill_pb(ref_cls(), d)
        wire_ours, wire_ref = ours.SerializeToString(), ref.SerializeToString(deterministic=True)
        # both decoders read the other's bytes to the same content
        assert _as_dict(ref_cls.FromString(wire_ours)) == _as_dict(ref)
        assert _as_dict(ours_cls.FromString(wire_ref)) == _as_dict(ref)
        # byte-identical where no map ordering is involved
        if not _has_map(name, schema):
            assert wire_ours == wire_ref

    check()


def test_codec_details():
    req = api.pb["RegisterRequest"](version="v1beta1")
    assert not req.HasField("options")
    req.options.pre_start_required = False  # touching a sub-message leaves it absent while empty
    assert req.SerializeToString() == b"\n\x07v1beta1"
    req.options = api.pb["DevicePluginOptions"]()  # assigned: present even when empty
    assert req.SerializeToString() == b"\n\x07v1beta1\x22\x00"
    # negative int64, packed and unpacked repeated int64, unknown fields skipped
    m = api.podres["AllocatableResourcesResponse"](cpu_ids=[-1, 3])
    raw = m.SerializeToString()
    assert raw == bytes.fromhex("12" "0b" "ffffffffffffffffff01" "03")
    unpacked = bytes.fromhex("10" "05" "10" "07" "f80101" "2a0178")  # cpu_ids 5, 7; unknown varint 31 and len 5
    assert api.podres["AllocatableResourcesResponse"].FromString(unpacked).cpu_ids == [5, 7]
    assert api.podres["AllocatableResourcesResponse"].FromString(raw).cpu_ids == [-1, 3]
    with pytest.raises(proto.DecodeError):
        api.pb["Device"].FromString(b"\x0a\x05ab")  # truncated string
    with pytest.raises(AttributeError):
        api.pb["Device"](no_such_field=1)


# --------------------------------------------------------------------- HPACK

def _h(s):
    return bytes.fromhex(s.replace(" ", ""))


def test_hpack_rfc7541_requests_plain_and_huffman():
    for blocks in (("8286 8441 0f77 7777 2e65 7861 6d70 6c65 2e63 6f6d", "8286 84be 5808 6e6f 2d63 6163 6865",
                    "8287 85bf 400a 6375 7374 6f6d 2d6b 6579 0c63 7573 746f 6d2d 7661 6c75 65"),
                   ("8286 8441 8cf1 e3c2 e5f2 3a6b a0ab 90f4 ff", "8286 84be 5886 a8eb 1064 9cbf",
                    "8287 85bf 4088 25a8 49e9 5ba9 7d7f 8925 a849 e95b b8e8 b4bf")):
        d = hpack.Decoder()
        assert d.decode(_h(blocks[0])) == [(":method", "GET"), (":scheme", "http"), (":path", "/"),
                                           (":authority", "www.example.com")]
        assert d.size == 57
        assert d.decode(_h(blocks[1]))[-1] == ("cache-control", "no-cache")
        assert d.decode(_h(blocks[2])) == [(":method", "GET"), (":scheme", "https"), (":path", "/index.html"),
                                           (":authority", "www.example.com"), ("custom-key", "custom-value")]
        assert d.size == 164 and d.table[0] == ("custom-key", "custom-value")


def test_hpack_rfc7541_responses_with_eviction():
    d = hpack.Decoder(256)
    first = d.decode(_h("4882 6402 5885 aec3 771a 4b61 96d0 7abe 9410 54d4 44a8 2005 9504 0b81 66e0 82a6 2d1b ff6e"
                        "919d 29ad 1718 63c7 8f0b 97c8 e9ae 82ae 43d3"))
    assert first == [(":status", "302"), ("cache-control", "private"), ("date", "Mon, 21 Oct 2013 20:13:21 GMT"),
                     ("location", "https://www.example.com")]
    assert d.size == 222
    second = d.decode(_h("4883 640e ffc1 c0bf"))
    assert second[0] == (":status", "307") and second[1:] == first[1:]
    assert d.size == 222 and (":status", "302") not in d.table  # evicted


def test_hpack_encoder_roundtrip_and_errors():
    hdrs = [(":method", "POST"), (":scheme", "http"), (":path", "/v1beta1.DevicePlugin/Allocate"),
            (":authority", "localhost"), ("content-type", "application/grpc"), ("te", "trailers"),
            ("grpc-timeout", "5000m"), ("x-long", "v" * 300)]
    assert hpack.Decoder().decode(hpack.encode(hdrs)) == hdrs
    assert hpack.encode([(":status", "200")]) == b"\x88"
    with pytest.raises(hpack.HPACKError):
        hpack.huffman_decode(b"\xf1\xe3\xc2\x00")  # padding not all ones
    with pytest.raises(hpack.HPACKError):
        hpack.Decoder().decode(b"\xbe")  # dynamic index 62 on an empty table
    with pytest.raises(hpack.HPACKError):
        hpack.Decoder(4096).decode(b"\x3f\xe2\x1f")  # table size update to 4097, above the advertised 4096


# ---------------------------------------------------------- HTTP/2 gRPC, ours

DEV = api.pb["Device"]
LAW = api.pb["ListAndWatchResponse"]


class _Svc:
    def __init__(self):
        self.cancelled = threading.Event()
        self.updates = threading.Semaphore(0)

    def Allocate(self, request, context):  # echo the device ids, or fail as asked
        ids = [i for c in request.container_requests for i in c.devices_ids]
        if "bad" in ids:
            context.abort(wire.StatusCode.INVALID_ARGUMENT, "unknown device ids ['bad'] – ünïcode % sign")
        if "boom" in ids:
            raise RuntimeError("handler bug")
        out = api.pb["AllocateResponse"]()
        r = out.container_responses.add()
        for i in ids:
            r.envs[f"ID_{i[:8]}"] = i * (1000 if len(i) < 8 else 3)  # long ids make a large response
        return out

    def ListAndWatch(self, request, context):
        context.add_callback(self.cancelled.set)
        for n in range(3):
            yield LAW(devices=[DEV(ID=f"gpu{k}", health=api.HEALTHY) for k in range(n + 1)])
        while context.is_active():  # stays open until the client cancels
            if self.updates.acquire(timeout=0.05):
                yield LAW(devices=[DEV(ID="gpu0", health=api.UNHEALTHY)])


@pytest.fixture
def our_server(tmp_path):
    svc = _Svc()
    handlers = {api.method_path(api.DEVICE_PLUGIN_SERVICE, n): wire.MethodHandler(
        getattr(svc, n), api.DEVICE_PLUGIN_METHODS[n][0].FromString, api.DEVICE_PLUGIN_METHODS[n][1].SerializeToString,
        api.DEVICE_PLUGIN_METHODS[n][2]) for n in ("Allocate", "ListAndWatch")}
    path = str(tmp_path / "dp.sock")
    srv = wire.Server(handlers)
    srv.add_unix(path)
    srv.start()
    yield path, svc
    srv.stop(0.5)


def _grpcio_call(ch, name):
    req, resp, stream = api.DEVICE_PLUGIN_METHODS[name]
    mk = ch.unary_stream if stream else ch.unary_unary
    return mk(api.method_path(api.DEVICE_PLUGIN_SERVICE, name), request_serializer=req.SerializeToString,
              response_deserializer=resp.FromString)


def test_grpcio_client_against_our_server(our_server):
    path, svc = our_server
    with grpc.insecure_channel("unix:" + path) as ch:
        alloc = _grpcio_call(ch, "Allocate")
        req = api.pb["AllocateRequest"]()
        req.container_requests.add(devices_ids=["1", "2"])
        out = alloc(req, timeout=5)
        assert dict(out.container_responses[0].envs) == {"ID_1": "1" * 1000, "ID_2": "2" * 1000}
        # 300 KB response: beyond grpcio's 64 KiB initial windows and 16 KiB frames
        big = api.pb["AllocateRequest"]()
        big.container_requests.add(devices_ids=[str(k % 10) * 3 for k in range(100)] + ["x" * 100000])
        out = alloc(big, timeout=10)
        assert len(out.container_responses[0].envs) == 11
        for _ in range(20):  # many calls on one connection
            assert alloc(req, timeout=5) == alloc(req, timeout=5)
        with pytest.raises(grpc.RpcError) as e:
            bad = api.pb["AllocateRequest"]()
            bad.container_requests.add(devices_ids=["bad"])
            alloc(bad, timeout=5)
        assert e.value.code() == grpc.StatusCode.INVALID_ARGUMENT
        assert e.value.details() == "unknown device ids ['bad'] – ünïcode % sign"
        with pytest.raises(grpc.RpcError) as e:
            boom = api.pb["AllocateRequest"]()
            boom.container_requests.add(devices_ids=["boom"])
            alloc(boom, timeout=5)
        assert e.value.code() == grpc.StatusCode.UNKNOWN and "handler bug" in e.value.details()
        with pytest.raises(grpc.RpcError) as e:
            _grpcio_call(ch, "PreStartContainer")(api.pb["PreStartContainerRequest"](), timeout=5)
        assert e.value.code() == grpc.StatusCode.UNIMPLEMENTED
        # server streaming, then a client cancel reaches the handler
        it = _grpcio_call(ch, "ListAndWatch")(api.pb["Empty"]())
        assert [len(next(it).devices) for _ in range(3)] == [1, 2, 3]
        svc.updates.release()
        assert next(it).devices[0].health == api.UNHEALTHY
        it.cancel()
        assert svc.cancelled.wait(5)


def test_many_stream_updates_need_window_updates(our_server):
    """More streamed bytes than grpcio's initial stream window: our sender
    must wait for, and then use, the client's WINDOW_UPDATEs."""
    path, svc = our_server
    with grpc.insecure_channel("unix:" + path) as ch:
        it = _grpcio_call(ch, "ListAndWatch")(api.pb["Empty"]())
        for _ in range(3):
            next(it)
        n = 6000  # ~6000 x 20 B messages = 120 KB > 64 KiB
        for _ in range(n):
            svc.updates.release()
        for _ in range(n):
            assert next(it).devices[0].ID == "gpu0"
        it.cancel()


# ------------------------------------------------------- our client, grpcio

@pytest.fixture
def grpcio_server(tmp_path):
    path = str(tmp_path / "kubelet.sock")
    state = {"slow": 0.0}

    def register(request, context):
        if request.version != api.VERSION:
            context.abort(grpc.StatusCode.INVALID_ARGUMENT, f"unsupported version {request.version} – %")
        time.sleep(state["slow"])
        return api.pb["Empty"]()

    def allocatable(request, context):
        out = api.podres["AllocatableResourcesResponse"]()
        for k in range(state.get("n", 1)):
            out.devices.add(resource_name="amd.com/gpu", device_ids=[f"{k:04d}" + "z" * 200])
        return out

    def start():
        srv = grpc.server(futures.ThreadPoolExecutor(max_workers=4))
        req, resp, _ = api.REGISTRATION_METHODS["Register"]
        preq, presp, _ = api.POD_RESOURCES_METHODS["GetAllocatableResources"]
        srv.add_generic_rpc_handlers((
            grpc.method_handlers_generic_handler(api.REGISTRATION_SERVICE, {"Register": grpc.unary_unary_rpc_method_handler(
                register, request_deserializer=req.FromString, response_serializer=resp.SerializeToString)}),
            grpc.method_handlers_generic_handler(api.POD_RESOURCES_SERVICE, {
                "GetAllocatableResources": grpc.unary_unary_rpc_method_handler(
                    allocatable, request_deserializer=preq.FromString, response_serializer=presp.SerializeToString)}),
        ))
        srv.add_insecure_port("unix:" + path)
        srv.start()
        return srv

    box = {"srv": start()}
    yield path, state, box, start
    box["srv"].stop(0).wait()


def _register_call(ch):
    req, resp, _ = api.REGISTRATION_METHODS["Register"]
    return ch.unary_unary(api.method_path(api.REGISTRATION_SERVICE, "Register"),
                          request_serializer=req.SerializeToString, response_deserializer=resp.FromString)


def test_our_client_against_grpcio_server(grpcio_server):
    path, state, box, start = grpcio_server
    req_cls = api.REGISTRATION_METHODS["Register"][0]
    ok = req_cls(version=api.VERSION, endpoint="amd.sock", resource_name="amd.com/gpu")
    with wire.Channel(path) as ch:
        call = _register_call(ch)
        for _ in range(10):
            assert call(ok, timeout=5) == api.pb["Empty"]()
        with pytest.raises(wire.RpcError) as e:
            call(req_cls(version="v0"), timeout=5)
        assert e.value.code() is wire.StatusCode.INVALID_ARGUMENT
        assert e.value.details() == "unsupported version v0 – %"
        state["slow"] = 1.0
        t0 = time.monotonic()
        with pytest.raises(wire.RpcError) as e:
            call(ok, timeout=0.2)
        assert e.value.code() is wire.StatusCode.DEADLINE_EXCEEDED and time.monotonic() - t0 < 0.9
        state["slow"] = 0.0
        assert call(ok, timeout=5) == api.pb["Empty"]()  # the channel recovers after a deadline
        # large response through our receive windows
        state["n"] = 20000  # ~4.2 MB
        preq, presp, _ = api.POD_RESOURCES_METHODS["GetAllocatableResources"]
        pcall = ch.unary_unary(api.method_path(api.POD_RESOURCES_SERVICE, "GetAllocatableResources"),
                               request_serializer=preq.SerializeToString, response_deserializer=presp.FromString)
        out = pcall(preq(), timeout=10)
        assert len(out.devices) == 20000 and out.devices[-1].device_ids[0].startswith("19999")
        # a request larger than grpcio's 64 KiB windows: our sender reads the
        # server's WINDOW_UPDATEs itself (the calling thread is the only reader)
        assert call(req_cls(version=api.VERSION, endpoint="e" * (2 << 20)), timeout=10) == api.pb["Empty"]()
        with pytest.raises(wire.RpcError) as e:  # above grpcio's 4 MiB receive limit
            call(req_cls(version=api.VERSION, endpoint="e" * (5 << 20)), timeout=10)
        assert e.value.code() in (wire.StatusCode.RESOURCE_EXHAUSTED, wire.StatusCode.CANCELLED,
                                  wire.StatusCode.INTERNAL)
        assert call(ok, timeout=5) == api.pb["Empty"]()
        # the server restarts: the kept-alive connection is dead, the next call reconnects
        box["srv"].stop(0).wait()
        box["srv"] = start()
        assert call(ok, timeout=5) == api.pb["Empty"]()


def test_our_client_waits_for_ready(tmp_path):
    path = str(tmp_path / "late.sock")
    ch = wire.Channel(path)
    call = _register_call(ch)
    req = api.REGISTRATION_METHODS["Register"][0](version=api.VERSION)
    with pytest.raises(wire.RpcError) as e:
        call(req, timeout=1)  # no socket, no wait_for_ready: fails at once
    assert e.value.code() is wire.StatusCode.UNAVAILABLE
    srv = {}

    def late_start():
        time.sleep(0.3)
        s = grpc.server(futures.ThreadPoolExecutor(max_workers=1))
        r, resp, _ = api.REGISTRATION_METHODS["Register"]
        s.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(api.REGISTRATION_SERVICE, {
            "Register": grpc.unary_unary_rpc_method_handler(lambda q, c: api.pb["Empty"](), request_deserializer=r.FromString,
                                                            response_serializer=resp.SerializeToString)}),))
        s.add_insecure_port("unix:" + path)
        s.start()
        srv["s"] = s

    th = threading.Thread(target=late_start)
    th.start()
    try:
        assert call(req, timeout=5, wait_for_ready=True) == api.pb["Empty"]()
    finally:
        th.join()
        ch.close()
        srv["s"].stop(0).wait()


def test_our_client_and_server_together(our_server):
    path, _ = our_server
    with wire.Channel(path) as ch:
        req, resp, _ = api.DEVICE_PLUGIN_METHODS["Allocate"]
        call = ch.unary_unary(api.method_path(api.DEVICE_PLUGIN_SERVICE, "Allocate"),
                              request_serializer=req.SerializeToString, response_deserializer=resp.FromString)
        r = req()
        r.container_requests.add(devices_ids=["7"])
        assert call(r, timeout=5).container_responses[0].envs["ID_7"] == "7" * 1000
        r.container_requests[0].devices_ids.append("x" * 1_000_000)  # 1 MB request, 3 MB response
        assert len(call(r, timeout=10).container_responses[0].envs) == 2


def test_server_limits(our_server):
    """A request above 4 MiB is refused with RESOURCE_EXHAUSTED (gRPC's default
    receive limit); an oversized header block or an even client stream id
    ends the connection."""
    import socket
    import struct

    path, _ = our_server
    with grpc.insecure_channel("unix:" + path, options=[("grpc.max_send_message_length", 64 << 20)]) as ch:
        big = api.pb["AllocateRequest"]()
        big.container_requests.add(devices_ids=["y" * (5 << 20)])
        with pytest.raises(grpc.RpcError) as e:
            _grpcio_call(ch, "Allocate")(big, timeout=10)
        assert e.value.code() == grpc.StatusCode.RESOURCE_EXHAUSTED

    def raw(frames: bytes) -> bytes:
        s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        s.settimeout(5)
        s.connect(path)
        got = b""
        try:
            s.sendall(wire.PREFACE + wire.Connection.frame(wire.SETTINGS, 0, 0) + frames)
            while True:
                chunk = s.recv(65536)
                if not chunk:
                    break
                got += chunk
        except (ConnectionResetError, BrokenPipeError):  # closed with our frames still unread: also an end
            got += b"\x00\x00\x00\x07\x00\x00\x00\x00\x00"
        finally:
            s.close()
        return got

    def goaway(got: bytes) -> bool:
        pos = 0
        while pos + 9 <= len(got):
            n = int.from_bytes(got[pos:pos + 3], "big")
            if got[pos + 3] == wire.GOAWAY:
                return True
            pos += 9 + n
        return False

    hdr = hpack.encode([(":method", "POST"), (":path", "/x"), ("x-pad", "p" * 60000)])
    flood = wire.Connection.frame(wire.HEADERS, 0, 1, hdr) + b"".join(
        wire.Connection.frame(wire.CONTINUATION, 0, 1, hdr) for _ in range(5))
    assert goaway(raw(flood))  # closed once the block passed 256 KiB
    assert goaway(raw(wire.Connection.frame(wire.HEADERS, wire.END_HEADERS, 2, hpack.encode([(":path", "/x")]))))
    # a ping is answered with its payload
    got = raw(wire.Connection.frame(wire.PING, 0, 0, b"12345678") + wire.Connection.frame(wire.GOAWAY, 0, 0,
                                                                                          struct.pack(">II", 0, 0)))
    assert b"12345678" in got


def test_frames_after_end_stream_do_not_run_the_call_again(our_server):
    """a DATA or HEADERS frame with END_STREAM on a stream that
    already ended is dropped - one handler run, one reply, one trailer."""
    import socket

    path, _ = our_server
    req = api.pb["AllocateRequest"]()
    req.container_requests.add(devices_ids=["5"])
    msg = req.SerializeToString()
    body = b"\x00" + len(msg).to_bytes(4, "big") + msg
    head = [(":method", "POST"), (":scheme", "http"), (":authority", "x"),
            (":path", api.method_path(api.DEVICE_PLUGIN_SERVICE, "Allocate")),
            ("content-type", "application/grpc"), ("te", "trailers")]
    F = wire.Connection.frame
    frames = (F(wire.HEADERS, wire.END_HEADERS, 1, hpack.encode(head)) + F(wire.DATA, wire.END_STREAM, 1, body)
              + F(wire.DATA, wire.END_STREAM, 1, body)
              + F(wire.HEADERS, wire.END_HEADERS | wire.END_STREAM, 1, hpack.encode(head)))
    s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    s.connect(path)
    got = b""
    try:
        s.sendall(wire.PREFACE + F(wire.SETTINGS, 0, 0) + frames)
        s.settimeout(1.0)
        while True:
            try:
                chunk = s.recv(65536)
            except socket.timeout:
                break
            if not chunk:
                break
            got += chunk
    finally:
        s.close()
    seen = []
    pos = 0
    while pos + 9 <= len(got):
        n = int.from_bytes(got[pos:pos + 3], "big")
        ftype, flags, sid = got[pos + 3], got[pos + 4], int.from_bytes(got[pos + 5:pos + 9], "big") & 0x7FFFFFFF
        if sid == 1:
            seen.append((ftype, bool(flags & wire.END_STREAM)))
        pos += 9 + n
    assert seen.count((wire.DATA, False)) == 1  # the reply message
    assert sum(1 for t, end in seen if t == wire.HEADERS and end) == 1  # the trailers


def test_hpack_decoded_size_is_bounded():
    d = hpack.Decoder(4096, max_list_size=64 << 10)
    big = bytearray(b"\x40\x05x-big")  # literal with incremental indexing, new name
    hpack.encode_int(big, 4000, 7, 0)
    big += b"v" * 4000
    assert d.decode(bytes(big)) == [("x-big", "v" * 4000)]  # one 4 KB entry in the dynamic table
    with pytest.raises(hpack.HPACKError):
        d.decode(b"\xbe" * 100)  # 100 one-byte references to it: 400 KB decoded
