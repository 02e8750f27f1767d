"""A raw HTTP/2 gRPC peer that frames and HPACK-encodes the way grpc-go does.

The kubelet is a grpc-go program: it serves ``v1beta1.Registration`` and
dials every device plugin's socket.  No Go toolchain exists in this
environment, so the interop tests against grpcio (tests/test_rpc.py) are
joined by this stand-in, which reproduces the grpc-go wire behaviours that
grpcio (C-core) does not share [EXT, grpc-go internal/transport:
http2_client.go, http2_server.go, controlbuf.go, bdp_estimator.go;
golang.org/x/net/http2/hpack encode.go]:

* HPACK: every field not already in a table is sent as a literal WITH
  incremental indexing (name by index when static or dynamic table has it,
  the static table preferred), an exact table match as an indexed field,
  strings Huffman-coded only when that is shorter; so a connection's later
  header blocks are mostly references into the dynamic table, which
  evicts at 4096 bytes;
* client: SETTINGS with no parameters at start; header order ``:method``,
  ``:scheme``, ``:path``, ``:authority``, ``content-type``, ``user-agent``,
  ``te``, ``grpc-timeout``; a unary/server-streaming request's END_STREAM on
  its message DATA frame; a cancelled stream ends with RST_STREAM(CANCEL);
* server: SETTINGS{MAX_FRAME_SIZE=16384} at start; a BDP ping
  (``02 04 10 10 09 0e 07 07``) when DATA arrives; responses as HEADERS, DATA,
  trailers HEADERS carrying ``grpc-status`` AND an empty ``grpc-message``;
  errors as one Trailers-Only HEADERS frame; graceful stop as GOAWAY(2^31-1)
  plus a ping (``01 06 01 08 00 03 03 09``), then, once that ping is acked,
  GOAWAY(last stream id) and a close once its streams are done.

Flow control follows grpc-go's default (64 KiB windows, WINDOW_UPDATE once a
quarter of a window is consumed).  Only what the kubelet's calls need is
implemented (small messages, one connection per peer).
"""

from __future__ import annotations

import queue
import socket
import struct
import threading
import urllib.parse

from amdgpu_operator.rpc import hpack
from amdgpu_operator.rpc.hpack import STATIC_TABLE, encode_int, huffman_encode

PREFACE = b"PRI * HTTP/2.0\r\n\r\nSM\r\n\r\n"
DATA, HEADERS, PRIORITY, RST_STREAM, SETTINGS, PUSH_PROMISE, PING, GOAWAY, WINDOW_UPDATE, CONTINUATION = range(10)
END_STREAM, ACK, END_HEADERS = 0x1, 0x1, 0x4
CANCEL = 8
S_MAX_FRAME_SIZE = 5
BDP_PING = bytes([2, 4, 16, 16, 9, 14, 7, 7])
GOAWAY_PING = bytes([1, 6, 1, 8, 0, 3, 3, 9])
USER_AGENT = "grpc-go/1.65.0"
WINDOW = 65535


def frame(ftype: int, flags: int, sid: int, payload: bytes = b"") -> bytes:
    n = len(payload)
    return struct.pack(">BHBBI", n >> 16, n & 0xFFFF, ftype, flags, sid & 0x7FFFFFFF) + payload


def grpc_message(payload: bytes) -> bytes:
    return b"\x00" + struct.pack(">I", len(payload)) + payload


def split_grpc(body: bytes) -> list[bytes]:
    out, pos = [], 0
    while pos + 5 <= len(body):
        n = struct.unpack(">I", body[pos + 1:pos + 5])[0]
        out.append(body[pos + 5:pos + 5 + n])
        pos += 5 + n
    return out


class GoEncoder:
    """HPACK as golang.org/x/net/http2/hpack's Encoder writes it."""

    def __init__(self, max_size: int = 4096):
        self.table: list[tuple[str, str]] = []  # newest first: index 62 is table[0]
        self.size = 0
        self.max_size = max_size
        self.evictions = 0
        self.indexed_refs = 0  # exact matches sent as one index (dynamic-table ones counted)

    def _evict(self) -> None:
        while self.size > self.max_size and self.table:
            n, v = self.table.pop()
            self.size -= len(n) + len(v) + 32
            self.evictions += 1

    def _search(self, name: str, value: str) -> tuple[int, bool]:
        name_idx = 0
        for i, (n, v) in enumerate(STATIC_TABLE, 1):
            if n == name:
                if v == value:
                    return i, True
                name_idx = name_idx or i
        for j, (n, v) in enumerate(self.table, len(STATIC_TABLE) + 1):
            if n == name:
                if v == value:
                    return j, True
                name_idx = name_idx or j
        return name_idx, False

    @staticmethod
    def _str(out: bytearray, s: str) -> None:
        raw = s.encode()
        h = huffman_encode(raw)
        if len(h) < len(raw):
            encode_int(out, len(h), 7, 0x80)
            out += h
        else:
            encode_int(out, len(raw), 7, 0)
            out += raw

    def encode(self, fields) -> bytes:
        out = bytearray()
        for name, value in fields:
            idx, exact = self._search(name, value)
            if exact:
                encode_int(out, idx, 7, 0x80)
                self.indexed_refs += idx > len(STATIC_TABLE)
                continue
            entry = len(name) + len(value) + 32
            indexing = entry <= self.max_size
            encode_int(out, idx, 6, 0x40) if indexing else encode_int(out, idx, 4, 0x00)
            if idx == 0:
                self._str(out, name)
            self._str(out, value)
            if indexing:
                self.table.insert(0, (name, value))
                self.size += entry
                self._evict()
        return bytes(out)


class _Conn:
    """Frame I/O of one connection: a reader thread hands frames to
    ``on_frame``; connection-level frames are answered as grpc-go answers
    them (SETTINGS ACK, PING ACK, WINDOW_UPDATE credit)."""

    def __init__(self, sock: socket.socket):
        self.sock = sock
        self.enc = GoEncoder()
        self.dec = hpack.Decoder()
        self.wlock = threading.Lock()
        self.buf = bytearray()
        self.pings_acked: list[bytes] = []
        self.pings_received: list[bytes] = []
        self.consumed = 0
        self.closed = threading.Event()
        self._block: tuple[int, int, bytearray] | None = None

    def send(self, data: bytes) -> None:
        with self.wlock:
            self.sock.sendall(data)

    def send_headers(self, sid: int, fields, end_stream: bool = False) -> None:
        with self.wlock:  # encode and send in one order: the peer decodes in arrival order
            block = self.enc.encode(fields)
            self.sock.sendall(frame(HEADERS, END_HEADERS | (END_STREAM if end_stream else 0), sid, block))

    def _read(self, n: int) -> bytes:
        while len(self.buf) < n:
            chunk = self.sock.recv(65536)
            if not chunk:
                raise ConnectionError("peer closed")
            self.buf += chunk
        out = bytes(self.buf[:n])
        del self.buf[:n]
        return out

    def read_frame(self) -> tuple[int, int, int, bytes]:
        hi, lo, ftype, flags, sid = struct.unpack(">BHBBI", self._read(9))
        return ftype, flags, sid & 0x7FFFFFFF, self._read((hi << 16) | lo)

    def pump(self, on_headers, on_data, on_rst, on_goaway=None, on_ping_ack=None) -> None:
        try:
            while True:
                ftype, flags, sid, p = self.read_frame()
                if ftype == SETTINGS and not flags & ACK:
                    self.send(frame(SETTINGS, ACK, 0))
                elif ftype == PING:
                    if flags & ACK:
                        self.pings_acked.append(p)
                        if on_ping_ack:
                            on_ping_ack(p)
                    else:
                        self.pings_received.append(p)
                        self.send(frame(PING, ACK, 0, p))
                elif ftype in (HEADERS, CONTINUATION):
                    if ftype == HEADERS:
                        self._block = (sid, flags, bytearray(p))
                    else:
                        self._block[2].extend(p)
                    if flags & END_HEADERS:
                        s, f0, block = self._block
                        self._block = None
                        on_headers(s, self.dec.decode(bytes(block)), bool(f0 & END_STREAM))
                elif ftype == DATA:
                    if p:
                        self.consumed += len(p)
                        credit = b""
                        if self.consumed >= WINDOW // 4:
                            credit = frame(WINDOW_UPDATE, 0, 0, struct.pack(">I", self.consumed))
                            credit += frame(WINDOW_UPDATE, 0, sid, struct.pack(">I", self.consumed))
                            self.consumed = 0
                        if credit:
                            self.send(credit)
                    on_data(sid, p, bool(flags & END_STREAM))
                elif ftype == RST_STREAM:
                    on_rst(sid, struct.unpack(">I", p[:4])[0])
                elif ftype == GOAWAY and on_goaway:
                    on_goaway(struct.unpack(">I", p[:4])[0] & 0x7FFFFFFF, struct.unpack(">I", p[4:8])[0])
        except (ConnectionError, OSError):
            pass
        finally:
            self.closed.set()


class GoClient:
    """The kubelet's side of a plugin socket, grpc-go style: one connection,
    multiplexed calls; each call's events land in its own queue."""

    def __init__(self, path: str, authority: str = "localhost"):
        self.authority = authority
        self.sock = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        self.sock.connect(path)
        self.conn = _Conn(self.sock)
        self.next_id = 1
        self.streams: dict[int, queue.Queue] = {}
        self.goaways: list[tuple[int, int]] = []
        self.conn.send(PREFACE + frame(SETTINGS, 0, 0))
        self._reader = threading.Thread(target=self.conn.pump, args=(
            self._on_headers, self._on_data, self._on_rst, lambda last, code: self.goaways.append((last, code))),
            daemon=True)
        self._reader.start()

    def _q(self, sid: int) -> queue.Queue:
        return self.streams.setdefault(sid, queue.Queue())

    def _on_headers(self, sid, fields, end):
        self._q(sid).put(("headers", fields, end))

    def _on_data(self, sid, data, end):
        self._q(sid).put(("data", data, end))

    def _on_rst(self, sid, code):
        self._q(sid).put(("rst", code, True))

    def start_call(self, method: str, request: bytes, timeout_s: float | None = None, framing: str = "end-on-data",
                   metadata=()) -> int:
        """Send one request; ``framing``: ``end-on-data`` (grpc-go's unary and
        server-streaming calls), ``empty-end`` (message DATA, then an empty
        DATA with END_STREAM: a client-streaming CloseSend) or ``split`` (the
        5-byte prefix and the message in separate DATA frames)."""
        sid = self.next_id
        self.next_id += 2
        self._q(sid)
        fields = [(":method", "POST"), (":scheme", "http"), (":path", method), (":authority", self.authority),
                  ("content-type", "application/grpc"), ("user-agent", USER_AGENT), ("te", "trailers")]
        if timeout_s is not None:
            fields.append(("grpc-timeout", f"{max(1, int(timeout_s * 1e6))}u"))
        fields += list(metadata)
        body = grpc_message(request)
        self.conn.send_headers(sid, fields)
        if framing == "end-on-data":
            self.conn.send(frame(DATA, END_STREAM, sid, body))
        elif framing == "empty-end":
            self.conn.send(frame(DATA, 0, sid, body) + frame(DATA, END_STREAM, sid))
        elif framing == "split":
            self.conn.send(frame(DATA, 0, sid, body[:5]) + frame(DATA, END_STREAM, sid, body[5:]))
        else:
            raise ValueError(framing)
        return sid

    def next_event(self, sid: int, timeout: float = 10.0):
        return self.streams[sid].get(timeout=timeout)

    def finish(self, sid: int, timeout: float = 10.0) -> dict:
        """Events of a call up to its end: headers, messages, trailers."""
        out = {"headers": None, "messages": [], "trailers": None, "rst": None}
        body = bytearray()
        while True:
            kind, val, end = self.next_event(sid, timeout)
            if kind == "rst":
                out["rst"] = val
                break
            if kind == "headers":
                if out["headers"] is None and not end:
                    out["headers"] = dict(val)
                else:
                    out["trailers"] = dict(val)
            else:
                body += val
            if end:
                break
        out["messages"] = split_grpc(bytes(body))
        return out

    def call(self, method: str, request: bytes, **kw) -> dict:
        return self.finish(self.start_call(method, request, **kw))

    def ping(self, data: bytes = BDP_PING) -> None:
        self.conn.send(frame(PING, 0, 0, data))

    def cancel(self, sid: int) -> None:
        self.conn.send(frame(RST_STREAM, 0, sid, struct.pack(">I", CANCEL)))

    def close(self) -> None:
        try:
            self.sock.shutdown(socket.SHUT_RDWR)
        except OSError:
            pass
        self.sock.close()
        self._reader.join(5)


class GoServer:
    """A grpc-go-shaped unary server on a unix socket (the kubelet's
    Registration service).  ``handler(method, request_bytes)`` returns
    ``(code, message, response_bytes)``; a nonzero code is answered
    Trailers-Only.  :meth:`drain` performs grpc-go's graceful stop on the
    live connections."""

    def __init__(self, path: str, handler):
        self.path = path
        self.handler = handler
        self.ls = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        self.ls.bind(path)
        self.ls.listen(16)
        self.conns: list[_Conn] = []
        self.calls: list[tuple[int, str, dict]] = []  # (connection number, method, request headers)
        self.bdp_pings_sent = 0
        self._stop = threading.Event()
        self._draining: dict[int, dict] = {}
        self._lock = threading.Lock()
        threading.Thread(target=self._accept, daemon=True).start()

    def _accept(self) -> None:
        while not self._stop.is_set():
            try:
                s, _ = self.ls.accept()
            except OSError:
                return
            c = _Conn(s)
            with self._lock:
                self.conns.append(c)
                num = len(self.conns) - 1
            threading.Thread(target=self._serve, args=(c, num), daemon=True).start()

    def _serve(self, c: _Conn, num: int) -> None:
        try:
            if c._read(len(PREFACE)) != PREFACE:
                return
        except (ConnectionError, OSError):
            return
        c.send(frame(SETTINGS, 0, 0, struct.pack(">HI", S_MAX_FRAME_SIZE, 16384)))
        streams: dict[int, dict] = {}
        state = {"bdp_sent": False, "max_sid": 0, "final_goaway": False}

        def respond(sid):
            st = streams.pop(sid)
            method = st["headers"].get(":path", "")
            self.calls.append((num, method, st["headers"]))
            msgs = split_grpc(bytes(st["body"]))
            code, message, resp = self.handler(method, msgs[0] if msgs else b"")
            if code:
                c.send_headers(sid, [(":status", "200"), ("content-type", "application/grpc"),
                                     ("grpc-status", str(code)),
                                     ("grpc-message", urllib.parse.quote(message, safe=" "))], end_stream=True)
            else:
                c.send_headers(sid, [(":status", "200"), ("content-type", "application/grpc")])
                c.send(frame(DATA, 0, sid, grpc_message(resp)))
                c.send_headers(sid, [("grpc-status", "0"), ("grpc-message", "")], end_stream=True)
            if state["final_goaway"] and not streams:
                c.sock.shutdown(socket.SHUT_RDWR)

        def on_headers(sid, fields, end):
            state["max_sid"] = max(state["max_sid"], sid)
            streams[sid] = {"headers": dict(fields), "body": bytearray()}
            if end:
                respond(sid)

        def on_data(sid, data, end):
            if sid not in streams:
                return
            streams[sid]["body"] += data
            if data and not state["bdp_sent"]:  # grpc-go's BDP estimator: a ping when data arrives
                state["bdp_sent"] = True
                self.bdp_pings_sent += 1
                c.send(frame(PING, 0, 0, BDP_PING))
            if end:
                respond(sid)

        def on_rst(sid, code):
            streams.pop(sid, None)

        def on_ping_ack(p):
            if p == GOAWAY_PING:  # second phase of the graceful stop
                state["final_goaway"] = True
                c.send(frame(GOAWAY, 0, 0, struct.pack(">II", state["max_sid"], 0)))
                if not streams:
                    c.sock.shutdown(socket.SHUT_RDWR)

        c.pump(on_headers, on_data, on_rst, on_ping_ack=on_ping_ack)
        try:
            c.sock.close()
        except OSError:
            pass

    def drain(self) -> None:
        """grpc-go GracefulStop, first phase, on every live connection."""
        for c in list(self.conns):
            if not c.closed.is_set():
                c.send(frame(GOAWAY, 0, 0, struct.pack(">II", 0x7FFFFFFF, 0)) + frame(PING, 0, 0, GOAWAY_PING))

    def stop(self) -> None:
        self._stop.set()
        self.ls.close()
        for c in self.conns:
            try:
                c.sock.shutdown(socket.SHUT_RDWR)
            except OSError:
                pass
