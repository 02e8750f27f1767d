"""gRPC over HTTP/2 on unix sockets, in plain Python: the kubelet's transport.

The reference's device plugin turns GPUs into an allocatable extended
resource through this kubelet API (/root/reference/README.md:122,205,211,220).

The device plugin serves ``v1beta1.DevicePlugin`` to the kubelet and calls
its ``Registration`` service; the validator and the metrics exporter call the
kubelet's ``v1.PodResourcesLister``.  All of that is unary calls plus one
server-streaming call (ListAndWatch) of small protobuf messages on a local
socket.  grpcio served it until round 3, but importing it cost the device
plugin ~0.1-0.13 s of its start-up on the MI355X box and the validator the
same again before its plugin check - both on the time-to-Ready critical path
(profiles/r3_grpc).  This module imports in a few milliseconds.

Protocol coverage (RFC 9113 + the gRPC HTTP/2 mapping):

- connection preface, SETTINGS exchange and ACKs, PING ACKs (gRPC's BDP and
  keepalive pings), GOAWAY, RST_STREAM (a cancelled ListAndWatch ends its
  handler), CONTINUATION, PADDED / PRIORITY flags, unknown frame types ignored;
- flow control both ways: DATA waits for the peer's connection and stream
  windows (WINDOW_UPDATE, SETTINGS_INITIAL_WINDOW_SIZE changes applied to open
  streams) and is split at the peer's SETTINGS_MAX_FRAME_SIZE; received DATA
  is returned to the peer with WINDOW_UPDATEs;
- HPACK with Huffman decoding and the dynamic table (rpc/hpack.py);
- gRPC: length-prefixed messages, ``grpc-timeout``, ``grpc-status`` /
  percent-encoded ``grpc-message`` trailers, Trailers-Only error responses,
  UNIMPLEMENTED for unknown methods or compressed messages.

The interface keeps the pieces of grpcio's the operator used: handlers take
``(request, context)`` with ``context.abort(code, details)``,
``add_callback`` and ``is_active``; clients get
``Channel(path).unary_unary(method, serializer, deserializer)(req, timeout=,
wait_for_ready=)`` and :class:`RpcError` with ``code()`` / ``details()``.
tests/test_rpc.py runs it against grpcio in both directions (grpcio client
-> this server, this client -> grpcio server), which is the peer a kubelet's
grpc-go stands in for; tests/test_rpc_grpcgo.py adds a frame-level stand-in
for grpc-go's own wire habits (HPACK incremental indexing and eviction, BDP
and graceful-stop pings, two-phase GOAWAY, Trailers-Only errors, multiplexed
calls) in both directions, the kubelet side driving the production plugin.
"""

from __future__ import annotations

import enum
import errno
import os
import socket
import struct
import threading
import time
from typing import Callable

from . import hpack

PREFACE = b"PRI * HTTP/2.0\r\n\r\nSM\r\n\r\n"

DATA, HEADERS, PRIORITY, RST_STREAM, SETTINGS, PUSH_PROMISE, PING, GOAWAY, WINDOW_UPDATE, CONTINUATION = range(10)
END_STREAM, ACK, END_HEADERS, PADDED, PRIORITY_FLAG = 0x1, 0x1, 0x4, 0x8, 0x20

S_HEADER_TABLE_SIZE, S_ENABLE_PUSH, S_MAX_CONCURRENT_STREAMS, S_INITIAL_WINDOW_SIZE, S_MAX_FRAME_SIZE, \
    S_MAX_HEADER_LIST_SIZE = range(1, 7)

DEFAULT_WINDOW = 65535
OUR_WINDOW = 1 << 24  # what we let a peer send before it hears from us
MAX_WINDOW = (1 << 31) - 1
CLIENT_MAX_MESSAGE = 64 << 20  # a response we accept (pod-resources List of a large node)
SERVER_MAX_MESSAGE = 4 << 20  # a request we accept (gRPC's default receive limit)
MAX_HEADER_BLOCK = 256 << 10
MAX_STREAMS = 128  # concurrent calls per connection (SETTINGS_MAX_CONCURRENT_STREAMS)

# HTTP/2 error codes
NO_ERROR, PROTOCOL_ERROR, INTERNAL_ERROR, FLOW_CONTROL_ERROR, _, STREAM_CLOSED, FRAME_SIZE_ERROR, REFUSED_STREAM, \
    CANCEL, COMPRESSION_ERROR = range(10)


class StatusCode(enum.Enum):
    OK = 0
    CANCELLED = 1
    UNKNOWN = 2
    INVALID_ARGUMENT = 3
    DEADLINE_EXCEEDED = 4
    NOT_FOUND = 5
    ALREADY_EXISTS = 6
    PERMISSION_DENIED = 7
    RESOURCE_EXHAUSTED = 8
    FAILED_PRECONDITION = 9
    ABORTED = 10
    OUT_OF_RANGE = 11
    UNIMPLEMENTED = 12
    INTERNAL = 13
    UNAVAILABLE = 14
    DATA_LOSS = 15
    UNAUTHENTICATED = 16


class RpcError(Exception):
    def __init__(self, code: StatusCode, details: str = ""):
        super().__init__(f"{code.name}: {details}")
        self._code, self._details = code, details

    def code(self) -> StatusCode:
        return self._code

    def details(self) -> str:
        return self._details


class ConnectionClosed(Exception):
    pass


def _pct_encode(s: str) -> str:
    out = []
    for b in s.encode():
        out.append(chr(b) if 0x20 <= b <= 0x7E and b != 0x25 else f"%{b:02X}")
    return "".join(out)


def _pct_decode(s: str) -> str:
    raw = s.encode("latin-1")
    out = bytearray()
    i = 0
    while i < len(raw):
        if raw[i] == 0x25 and i + 2 < len(raw):
            try:
                out.append(int(raw[i + 1:i + 3], 16))
                i += 3
                continue
            except ValueError:
                pass
        out.append(raw[i])
        i += 1
    return out.decode("utf-8", "replace")


def _timeout_header(seconds: float) -> str:
    ms = max(1, int(seconds * 1000))
    return f"{ms}m" if ms < 10 ** 8 else f"{max(1, int(seconds))}S"


def _parse_timeout(v: str) -> float | None:
    units = {"H": 3600.0, "M": 60.0, "S": 1.0, "m": 1e-3, "u": 1e-6, "n": 1e-9}
    try:
        return int(v[:-1]) * units[v[-1]]
    except (ValueError, KeyError, IndexError):
        return None


def grpc_frame(payload: bytes) -> bytes:
    return b"\x00" + struct.pack(">I", len(payload)) + payload


class _Stream:
    __slots__ = ("id", "headers", "trailers", "body", "ended", "reset", "send_window", "recv_consumed", "event",
                 "callbacks", "status_sent", "too_big")

    def __init__(self, sid: int, send_window: int):
        self.id = sid
        self.headers: list[tuple[str, str]] | None = None
        self.trailers: list[tuple[str, str]] | None = None
        self.body = bytearray()
        self.ended = False  # the peer's END_STREAM
        self.reset = None  # RST_STREAM error code from the peer, or a closed connection
        self.send_window = send_window
        self.recv_consumed = 0
        self.event = threading.Event()  # anything new for a waiting client call
        self.callbacks: list[Callable[[], None]] = []
        self.status_sent = False
        self.too_big = False  # the peer sent more than the message limit: the rest is dropped


class Connection:
    """One HTTP/2 connection; a reader thread (server) or the calling thread
    (client) reads frames, writers share one lock."""

    def __init__(self, sock: socket.socket, client: bool):
        self.sock = sock
        self.client = client
        self.max_message = CLIENT_MAX_MESSAGE if client else SERVER_MAX_MESSAGE
        self.wlock = threading.Lock()
        self.flow = threading.Condition()  # send windows
        self.decoder = hpack.Decoder()
        self.peer_initial_window = DEFAULT_WINDOW
        self.peer_max_frame = 16384
        self.conn_send_window = DEFAULT_WINDOW
        self.conn_recv_consumed = 0
        self.streams: dict[int, _Stream] = {}
        self.max_peer_sid = 0  # highest stream id the peer opened (ids only grow, RFC 9113 5.1.1)
        self.closed = False
        self.goaway = False
        self.next_id = 1
        self._buf = bytearray()
        self._hdr_block: tuple[int, int, bytearray] | None = None  # (stream, flags, fragments) awaiting CONTINUATION

    # ---------------------------------------------------------------- writing
    def _send(self, data: bytes) -> None:
        with self.wlock:
            if self.closed:
                raise ConnectionClosed("connection closed")
            try:
                self.sock.sendall(data)
            except OSError as e:
                self.closed = True
                raise ConnectionClosed(str(e)) from None

    @staticmethod
    def frame(ftype: int, flags: int, sid: int, payload: bytes = b"") -> bytes:
        n = len(payload)
        return struct.pack(">BHBBI", n >> 16, n & 0xFFFF, ftype, flags, sid & 0x7FFFFFFF) + payload

    def start(self) -> None:
        settings = struct.pack(">HI", S_ENABLE_PUSH, 0) + struct.pack(">HI", S_INITIAL_WINDOW_SIZE, OUR_WINDOW) + \
            struct.pack(">HI", S_MAX_FRAME_SIZE, 1 << 20) + struct.pack(">HI", S_MAX_CONCURRENT_STREAMS, MAX_STREAMS) + \
            struct.pack(">HI", S_MAX_HEADER_LIST_SIZE, MAX_HEADER_BLOCK)
        out = (PREFACE if self.client else b"") + self.frame(SETTINGS, 0, 0, settings) + \
            self.frame(WINDOW_UPDATE, 0, 0, struct.pack(">I", OUR_WINDOW - DEFAULT_WINDOW))
        self._send(out)

    def send_headers(self, sid: int, headers, end_stream: bool = False) -> None:
        block = hpack.encode(headers)
        first = True
        frames = bytearray()
        while True:
            chunk, block = block[:self.peer_max_frame], block[self.peer_max_frame:]
            last = not block
            if first:
                flags = (END_STREAM if end_stream else 0) | (END_HEADERS if last else 0)
                frames += self.frame(HEADERS, flags, sid, chunk)
                first = False
            else:
                frames += self.frame(CONTINUATION, END_HEADERS if last else 0, sid, chunk)
            if last:
                break
        self._send(bytes(frames))

    def send_data(self, st: _Stream, data: bytes, end_stream: bool = False, deadline: float | None = None,
                  pump: Callable[[float], None] | None = None) -> None:
        """DATA within the peer's windows.  A server's reader thread applies
        the peer's WINDOW_UPDATEs meanwhile; a client, whose calling thread is
        its only reader, passes ``pump(timeout)``, which reads and handles
        frames (a request larger than the server's window would otherwise wait
        for updates nobody reads)."""
        view = memoryview(data)
        while True:
            with self.flow:
                while True:
                    if self.closed or st.reset is not None:
                        raise ConnectionClosed("stream closed by the peer")
                    n = min(len(view), self.conn_send_window, st.send_window, self.peer_max_frame)
                    if n > 0 or not view:
                        break
                    left = None if deadline is None else deadline - time.monotonic()
                    if left is not None and left <= 0:
                        raise TimeoutError("flow-control window stayed closed")
                    if pump is not None:
                        break
                    self.flow.wait(0.5 if left is None else min(0.5, left))
                if n <= 0 and view:  # client: read the peer's frames, then look again
                    n = -1
                else:
                    self.conn_send_window -= n
                    st.send_window -= n
            if n < 0:
                left = None if deadline is None else deadline - time.monotonic()
                pump(0.5 if left is None else max(0.001, min(0.5, left)))
                continue
            chunk, view = view[:n], view[n:]
            last = not view
            self._send(self.frame(DATA, END_STREAM if (end_stream and last) else 0, st.id, bytes(chunk)))
            if last:
                return

    def send_rst(self, sid: int, code: int = CANCEL) -> None:
        try:
            self._send(self.frame(RST_STREAM, 0, sid, struct.pack(">I", code)))
        except ConnectionClosed:
            pass

    def close(self, code: int = NO_ERROR) -> None:
        if not self.closed:
            try:
                self._send(self.frame(GOAWAY, 0, 0, struct.pack(">II", 0, code)))
            except ConnectionClosed:
                pass
        with self.wlock:
            self.closed = True
        try:
            self.sock.shutdown(socket.SHUT_RDWR)
        except OSError:
            pass
        self.sock.close()
        self._fail_streams()

    def _fail_streams(self) -> None:
        with self.flow:
            self.closed = True
            self.flow.notify_all()
        for st in list(self.streams.values()):
            if st.reset is None:
                st.reset = CANCEL
            st.event.set()
            self._run_callbacks(st)

    @staticmethod
    def _run_callbacks(st: _Stream) -> None:
        cbs, st.callbacks = st.callbacks, []
        for cb in cbs:
            try:
                cb()
            except Exception:  # noqa: BLE001 - a callback must not break the transport
                pass

    # ---------------------------------------------------------------- reading
    def _read_exact(self, n: int) -> bytes:
        while len(self._buf) < n:
            chunk = self.sock.recv(max(65536, n - len(self._buf)))
            if not chunk:
                raise ConnectionClosed("peer closed the connection")
            self._buf += chunk
        out = bytes(self._buf[:n])
        del self._buf[:n]
        return out

    def read_preface(self) -> None:
        if self._read_exact(len(PREFACE)) != PREFACE:
            raise ConnectionClosed("not an HTTP/2 client preface")

    def read_frame(self) -> tuple[int, int, int, bytes]:
        h = self._read_exact(9)
        hi, lo, ftype, flags, sid = struct.unpack(">BHBBI", h)
        n = (hi << 16) | lo
        if n > (1 << 20):  # our SETTINGS_MAX_FRAME_SIZE
            raise ConnectionClosed(f"frame of {n} bytes above our max frame size")
        return ftype, flags, sid & 0x7FFFFFFF, self._read_exact(n)

    def handle_frame(self, ftype: int, flags: int, sid: int, payload: bytes,
                     on_headers: Callable[[_Stream, list, bool], None],
                     on_end: Callable[[_Stream], None]) -> None:
        """Connection-level frames are answered here; stream events go to
        ``on_headers(stream, headers, end_stream)`` / ``on_end(stream)``."""
        if self._hdr_block is not None and ftype != CONTINUATION:
            raise ConnectionClosed("expected CONTINUATION")
        if ftype == SETTINGS:
            if flags & ACK:
                return
            self._apply_settings(payload)
            self._send(self.frame(SETTINGS, ACK, 0))
        elif ftype == PING:
            if not flags & ACK:
                self._send(self.frame(PING, ACK, 0, payload[:8]))
        elif ftype == WINDOW_UPDATE:
            inc = struct.unpack(">I", payload[:4])[0] & 0x7FFFFFFF
            with self.flow:
                if sid == 0:
                    self.conn_send_window += inc
                elif sid in self.streams:
                    self.streams[sid].send_window += inc
                self.flow.notify_all()
        elif ftype == GOAWAY:
            self.goaway = True
            last = struct.unpack(">I", payload[:4])[0] & 0x7FFFFFFF
            for s, st in list(self.streams.items()):
                if s > last:  # never processed: the caller may retry elsewhere
                    st.reset = CANCEL
                    st.event.set()
        elif ftype == RST_STREAM:
            st = self.streams.get(sid)
            if st is not None:
                st.reset = struct.unpack(">I", payload[:4])[0]
                st.event.set()
                with self.flow:
                    self.flow.notify_all()
                self._run_callbacks(st)
        elif ftype in (HEADERS, CONTINUATION):
            if ftype == HEADERS:
                if self._hdr_block is not None:
                    raise ConnectionClosed("HEADERS inside a header block")
                payload = self._strip(flags, payload, headers=True)
                self._hdr_block = (sid, flags, bytearray(payload))
            else:
                if self._hdr_block is None or self._hdr_block[0] != sid:
                    raise ConnectionClosed("unexpected CONTINUATION")
                self._hdr_block[2].extend(payload)
            if len(self._hdr_block[2]) > MAX_HEADER_BLOCK:
                raise ConnectionClosed(f"header block above {MAX_HEADER_BLOCK} bytes")
            if flags & END_HEADERS:
                s, f0, block = self._hdr_block
                self._hdr_block = None
                try:
                    headers = self.decoder.decode(bytes(block))
                except hpack.HPACKError as e:
                    raise ConnectionClosed(f"HPACK: {e}") from None
                st = self.streams.get(s)
                if st is None:
                    if self.client:
                        return  # a stream we no longer track
                    if s % 2 == 0:
                        raise ConnectionClosed(f"client stream id {s} is even")
                    if s <= self.max_peer_sid:  # a frame for a stream that already closed: not a new call
                        return
                    self.max_peer_sid = s
                    if len(self.streams) >= MAX_STREAMS:
                        self.send_rst(s, REFUSED_STREAM)
                        return
                    st = self.streams[s] = _Stream(s, self.peer_initial_window)
                elif st.ended:  # the peer already closed its side: no second request or reply
                    return
                on_headers(st, headers, bool(f0 & END_STREAM))
                if f0 & END_STREAM:
                    st.ended = True
                    st.event.set()
                    on_end(st)
        elif ftype == DATA:
            data = self._strip(flags, payload)
            st = self.streams.get(sid)
            self._credit(st, len(payload))
            if st is None:
                return
            if st.ended:  # DATA after END_STREAM (half-closed remote): dropped, the call runs once
                return
            if not st.too_big:
                st.body += data
                if len(st.body) > self.max_message + 5:
                    st.too_big = True  # answered RESOURCE_EXHAUSTED once the stream ends
                    st.body = bytearray()
            if flags & END_STREAM:
                st.ended = True
                on_end(st)
            st.event.set()
        # PRIORITY, PUSH_PROMISE (disabled) and unknown types: ignored

    def _strip(self, flags: int, payload: bytes, headers: bool = False) -> bytes:
        pad = 0
        if flags & PADDED:
            pad = payload[0]
            payload = payload[1:]
        if headers and flags & PRIORITY_FLAG:
            payload = payload[5:]
        return payload[:len(payload) - pad] if pad else payload

    def _credit(self, st: _Stream | None, n: int) -> None:
        """Give received bytes back to the peer once half our window is used."""
        if n == 0:
            return
        out = b""
        self.conn_recv_consumed += n
        if self.conn_recv_consumed >= OUR_WINDOW // 2:
            out += self.frame(WINDOW_UPDATE, 0, 0, struct.pack(">I", self.conn_recv_consumed))
            self.conn_recv_consumed = 0
        if st is not None and not st.ended:
            st.recv_consumed += n
            if st.recv_consumed >= OUR_WINDOW // 2:
                out += self.frame(WINDOW_UPDATE, 0, st.id, struct.pack(">I", st.recv_consumed))
                st.recv_consumed = 0
        if out:
            self._send(out)

    def _apply_settings(self, payload: bytes) -> None:
        for i in range(0, len(payload) - len(payload) % 6, 6):
            key, val = struct.unpack(">HI", payload[i:i + 6])
            if key == S_INITIAL_WINDOW_SIZE:
                if val > MAX_WINDOW:
                    raise ConnectionClosed("initial window above 2^31-1")
                with self.flow:
                    delta = val - self.peer_initial_window
                    self.peer_initial_window = val
                    for st in self.streams.values():
                        st.send_window += delta
                    self.flow.notify_all()
            elif key == S_MAX_FRAME_SIZE:
                self.peer_max_frame = max(16384, min(val, (1 << 24) - 1))
            # header table size: our encoder never indexes, nothing to resize


def split_messages(body: bytes) -> list[bytes]:
    out = []
    pos = 0
    while pos < len(body):
        if pos + 5 > len(body):
            raise RpcError(StatusCode.INTERNAL, "truncated gRPC message prefix")
        compressed = body[pos]
        n = struct.unpack(">I", body[pos + 1:pos + 5])[0]
        if compressed:
            raise RpcError(StatusCode.UNIMPLEMENTED, "compressed gRPC messages are not supported")
        if pos + 5 + n > len(body):
            raise RpcError(StatusCode.INTERNAL, "truncated gRPC message")
        out.append(bytes(body[pos + 5:pos + 5 + n]))
        pos += 5 + n
    return out


# ===================================================================== server

class AbortError(Exception):
    def __init__(self, code: StatusCode, details: str):
        super().__init__(details)
        self.code, self.details = code, details


class ServicerContext:
    def __init__(self, conn: Connection, st: _Stream, deadline: float | None):
        self._conn, self._st, self._deadline = conn, st, deadline

    def add_callback(self, fn: Callable[[], None]) -> bool:
        if self._st.reset is not None:
            fn()
            return False
        self._st.callbacks.append(fn)
        return True

    def is_active(self) -> bool:
        return self._st.reset is None and not self._conn.closed

    def time_remaining(self) -> float | None:
        return None if self._deadline is None else max(0.0, self._deadline - time.monotonic())

    def abort(self, code: StatusCode, details: str = ""):
        raise AbortError(code, details)


class MethodHandler:
    """``fn(request, context)`` returning a response, or (``stream``) yielding them."""

    def __init__(self, fn: Callable, request_deserializer: Callable[[bytes], object],
                 response_serializer: Callable[[object], bytes], stream: bool = False):
        self.fn, self.deserialize, self.serialize, self.stream = fn, request_deserializer, response_serializer, stream


class Server:
    """Serves ``{"/pkg.Service/Method": MethodHandler}`` on unix sockets; a
    thread per connection reads frames, a thread per call runs its handler."""

    def __init__(self, handlers: dict[str, MethodHandler], name: str = "rpc"):
        self.handlers = dict(handlers)
        self.name = name
        self._listeners: list[socket.socket] = []
        self._paths: list[str] = []
        self._conns: set[Connection] = set()
        self._lock = threading.Lock()
        self._stopped = threading.Event()
        self._calls: set[threading.Thread] = set()

    def add_unix(self, path: str) -> None:
        s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        s.bind(path)
        s.listen(64)
        self._listeners.append(s)
        self._paths.append(path)

    def start(self) -> None:
        for s in self._listeners:
            threading.Thread(target=self._accept_loop, args=(s,), name=f"{self.name}-accept", daemon=True).start()

    def _accept_loop(self, ls: socket.socket) -> None:
        while not self._stopped.is_set():
            try:
                s, _ = ls.accept()
            except OSError:
                return
            conn = Connection(s, client=False)
            with self._lock:
                if self._stopped.is_set():
                    s.close()
                    return
                self._conns.add(conn)
            threading.Thread(target=self._serve_conn, args=(conn,), name=f"{self.name}-conn", daemon=True).start()

    def _serve_conn(self, conn: Connection) -> None:
        try:
            conn.start()
            conn.read_preface()
            while not self._stopped.is_set():
                ftype, flags, sid, payload = conn.read_frame()
                conn.handle_frame(ftype, flags, sid, payload, self._on_headers, lambda st: self._on_end(conn, st))
                if conn.goaway and not conn.streams:  # the client is done with this connection
                    break
        except (ConnectionClosed, OSError, struct.error):
            pass
        finally:
            with self._lock:
                self._conns.discard(conn)
            conn.close()

    def _on_headers(self, st: _Stream, headers: list, end_stream: bool) -> None:
        if st.headers is None:
            st.headers = headers

    def _on_end(self, conn: Connection, st: _Stream) -> None:
        th = threading.Thread(target=self._run_call, args=(conn, st), name=f"{self.name}-call", daemon=True)
        with self._lock:  # registered and started together: stop() never joins a thread not yet started
            self._calls.add(th)
            th.start()

    def _run_call(self, conn: Connection, st: _Stream) -> None:
        try:
            self._call(conn, st)
        except ConnectionClosed:
            pass
        finally:
            conn.streams.pop(st.id, None)
            Connection._run_callbacks(st)
            with self._lock:
                self._calls.discard(threading.current_thread())

    def _finish(self, conn: Connection, st: _Stream, code: StatusCode, details: str = "") -> None:
        trailers = [("grpc-status", str(code.value))]
        if details:
            trailers.append(("grpc-message", _pct_encode(details)))
        if st.status_sent:
            conn.send_headers(st.id, trailers, end_stream=True)
        else:  # Trailers-Only
            conn.send_headers(st.id, [(":status", "200"), ("content-type", "application/grpc")] + trailers,
                              end_stream=True)
            st.status_sent = True

    def _call(self, conn: Connection, st: _Stream) -> None:
        hdrs = dict(st.headers or [])
        path = hdrs.get(":path", "")
        if hdrs.get(":method") != "POST" or not hdrs.get("content-type", "").startswith("application/grpc"):
            self._finish(conn, st, StatusCode.UNIMPLEMENTED, "not a gRPC request")
            return
        h = self.handlers.get(path)
        if h is None:
            self._finish(conn, st, StatusCode.UNIMPLEMENTED, f"unknown method {path}")
            return
        tmo = _parse_timeout(hdrs["grpc-timeout"]) if "grpc-timeout" in hdrs else None
        deadline = None if tmo is None else time.monotonic() + tmo
        ctx = ServicerContext(conn, st, deadline)
        if st.too_big:
            self._finish(conn, st, StatusCode.RESOURCE_EXHAUSTED, f"request above {conn.max_message} bytes")
            return
        try:
            msgs = split_messages(bytes(st.body))
            if len(msgs) != 1:
                raise RpcError(StatusCode.INTERNAL, f"expected one request message, got {len(msgs)}")
            request = h.deserialize(msgs[0])
        except RpcError as e:
            self._finish(conn, st, e.code(), e.details())
            return
        except Exception as e:  # noqa: BLE001 - undecodable request
            self._finish(conn, st, StatusCode.INTERNAL, f"request: {e}")
            return
        try:
            if h.stream:
                for resp in h.fn(request, ctx):
                    if st.reset is not None or conn.closed:
                        return
                    self._send_message(conn, st, h.serialize(resp))
            else:
                resp = h.fn(request, ctx)
                self._send_message(conn, st, h.serialize(resp))
        except AbortError as e:
            self._finish(conn, st, e.code, e.details)
            return
        except ConnectionClosed:
            return
        except Exception as e:  # noqa: BLE001 - a handler bug is UNKNOWN to the caller, as in grpcio
            self._finish(conn, st, StatusCode.UNKNOWN, f"{type(e).__name__}: {e}")
            return
        if st.reset is None:
            self._finish(conn, st, StatusCode.OK)

    def _send_message(self, conn: Connection, st: _Stream, payload: bytes) -> None:
        if not st.status_sent:
            conn.send_headers(st.id, [(":status", "200"), ("content-type", "application/grpc")])
            st.status_sent = True
        conn.send_data(st, grpc_frame(payload))

    def stop(self, grace: float | None = None) -> threading.Event:
        """Stop accepting, end every connection (GOAWAY) and, within
        ``grace`` seconds, wait for running calls; returns a set event."""
        self._stopped.set()
        for s in self._listeners:
            try:
                s.shutdown(socket.SHUT_RDWR)  # wakes the accept() of the listener thread (close alone does not)
            except OSError:
                pass
            try:
                s.close()
            except OSError:
                pass
        with self._lock:
            conns, calls = list(self._conns), list(self._calls)
        for c in conns:
            c.close()
        if grace:
            end = time.monotonic() + grace
            for th in calls:
                th.join(max(0.0, end - time.monotonic()))
        done = threading.Event()
        done.set()
        return done


# ===================================================================== client

class Channel:
    """A client connection to one unix socket, opened at the first call and
    reused; calls on one channel are serialised (each reads its own stream
    to the end)."""

    def __init__(self, path: str, authority: str = "localhost"):
        self.path = path[5:] if path.startswith("unix:") else path
        self.authority = authority
        self._conn: Connection | None = None
        self._lock = threading.Lock()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def close(self) -> None:
        with self._lock:
            if self._conn is not None:
                self._conn.close()
                self._conn = None

    def _connect(self, deadline: float | None, wait_for_ready: bool) -> Connection:
        while True:
            s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
            try:
                s.settimeout(None if deadline is None else max(0.001, deadline - time.monotonic()))
                s.connect(self.path)
                s.settimeout(None)
                conn = Connection(s, client=True)
                conn.start()
                return conn
            except (FileNotFoundError, ConnectionRefusedError) as e:
                s.close()
                if not wait_for_ready or (deadline is not None and time.monotonic() >= deadline):
                    raise RpcError(StatusCode.UNAVAILABLE, f"connect {self.path}: {e}") from None
                time.sleep(0.005 if deadline is None else min(0.005, max(0.0, deadline - time.monotonic())))
            except socket.timeout:
                s.close()
                raise RpcError(StatusCode.DEADLINE_EXCEEDED, f"connect {self.path}: timed out") from None
            except ConnectionClosed as e:
                s.close()
                raise RpcError(StatusCode.UNAVAILABLE, f"connect {self.path}: {e}") from None
            except OSError as e:
                s.close()
                if e.errno in (errno.EAGAIN, errno.ECONNRESET) and wait_for_ready and (
                        deadline is None or time.monotonic() < deadline):
                    time.sleep(0.005)
                    continue
                raise RpcError(StatusCode.UNAVAILABLE, f"connect {self.path}: {e}") from None

    def unary_unary(self, method: str, request_serializer: Callable[[object], bytes],
                    response_deserializer: Callable[[bytes], object]):
        def call(request, timeout: float | None = None, wait_for_ready: bool = False, metadata=None):
            payload = request_serializer(request)
            deadline = None if timeout is None else time.monotonic() + timeout
            with self._lock:
                for attempt in range(2):
                    if self._conn is None or self._conn.closed or self._conn.goaway:
                        if self._conn is not None:
                            self._conn.close()
                        self._conn = self._connect(deadline, wait_for_ready)
                        fresh = True
                    else:
                        fresh = False
                    try:
                        resp = self._unary(self._conn, method, payload, deadline, metadata)
                    except _Retry:
                        self._conn.close()
                        self._conn = None
                        if fresh or attempt:
                            raise RpcError(StatusCode.UNAVAILABLE, "connection closed by the server") from None
                        continue  # a kept-alive connection the server had dropped: once more on a new one
                    return response_deserializer(resp)
        return call

    def _unary(self, conn: Connection, method: str, payload: bytes, deadline: float | None, metadata) -> bytes:
        sid = conn.next_id
        conn.next_id += 2
        st = conn.streams[sid] = _Stream(sid, conn.peer_initial_window)
        headers = [(":method", "POST"), (":scheme", "http"), (":path", method), (":authority", self.authority),
                   ("content-type", "application/grpc"), ("te", "trailers"), ("user-agent", "amdgpu-operator-rpc/1")]
        if deadline is not None:
            headers.append(("grpc-timeout", _timeout_header(max(0.001, deadline - time.monotonic()))))
        headers += list(metadata or [])
        def on_headers(s: _Stream, hdrs: list, end: bool) -> None:
            if s.headers is None:
                s.headers = hdrs
            else:
                s.trailers = hdrs
            if end and s.trailers is None:  # Trailers-Only
                s.trailers = hdrs

        def pump(timeout: float) -> None:  # the server's frames while our request waits for its window
            conn.sock.settimeout(timeout)
            try:
                ftype, flags, fsid, fp = conn.read_frame()
            except socket.timeout:
                return
            except OSError as e:
                raise ConnectionClosed(str(e)) from None
            finally:
                try:
                    conn.sock.settimeout(None)
                except OSError:
                    pass
            conn.handle_frame(ftype, flags, fsid, fp, on_headers, lambda s: None)

        try:
            try:
                conn.send_headers(sid, headers)
                conn.send_data(st, grpc_frame(payload), end_stream=True, deadline=deadline, pump=pump)
            except ConnectionClosed:
                if st.ended or st.reset is not None:  # the server answered (e.g. an error) before all of it
                    pass
                else:
                    raise _Retry() from None
            except TimeoutError:
                conn.send_rst(sid)
                raise RpcError(StatusCode.DEADLINE_EXCEEDED, "deadline exceeded (request not sent)") from None
            got_any = st.headers is not None

            while not st.ended and st.reset is None:
                if deadline is not None:
                    left = deadline - time.monotonic()
                    if left <= 0:
                        conn.send_rst(sid)
                        raise RpcError(StatusCode.DEADLINE_EXCEEDED, "deadline exceeded")
                    conn.sock.settimeout(left)
                try:
                    ftype, flags, fsid, fp = conn.read_frame()
                except socket.timeout:
                    conn.send_rst(sid)
                    conn.close()
                    raise RpcError(StatusCode.DEADLINE_EXCEEDED, "deadline exceeded") from None
                except (ConnectionClosed, OSError):
                    conn.closed = True
                    if not got_any:
                        raise _Retry() from None
                    raise RpcError(StatusCode.UNAVAILABLE, "connection lost during the call") from None
                finally:
                    try:
                        conn.sock.settimeout(None)
                    except OSError:
                        pass
                if fsid == sid:
                    got_any = True
                try:
                    conn.handle_frame(ftype, flags, fsid, fp, on_headers, lambda s: None)
                except ConnectionClosed as e:
                    conn.close(PROTOCOL_ERROR)
                    raise RpcError(StatusCode.INTERNAL, f"protocol error: {e}") from None
            if st.reset is not None and not st.ended:
                if not got_any and conn.goaway:
                    raise _Retry()
                raise RpcError(StatusCode.CANCELLED if st.reset == CANCEL else StatusCode.INTERNAL,
                               f"stream reset by the server (HTTP/2 error {st.reset})")
        finally:
            conn.streams.pop(sid, None)
        trailers = dict(st.trailers or st.headers or [])
        status = trailers.get("grpc-status")
        if status is None:
            http = dict(st.headers or []).get(":status", "?")
            raise RpcError(StatusCode.INTERNAL if http == "200" else StatusCode.UNAVAILABLE,
                           f"no grpc-status (HTTP {http})")
        try:
            code = StatusCode(int(status))
        except ValueError:
            code = StatusCode.UNKNOWN
        if code is not StatusCode.OK:
            raise RpcError(code, _pct_decode(trailers.get("grpc-message", "")))
        if st.too_big:
            raise RpcError(StatusCode.RESOURCE_EXHAUSTED, f"response above {conn.max_message} bytes")
        msgs = split_messages(bytes(st.body))
        if len(msgs) != 1:
            raise RpcError(StatusCode.INTERNAL, f"expected one response message, got {len(msgs)}")
        return msgs[0]


class _Retry(Exception):
    pass


def remove_socket(path: str) -> None:
    try:
        os.unlink(path)
    except FileNotFoundError:
        pass
