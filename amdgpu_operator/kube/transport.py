"""HTTP(S) transport of :class:`~.client.RestClient`: HTTP/1.1 on sockets.

Every operand container talks to the API server, and every one of them pays
its client's import at start-up, inside the node's time-to-Ready.
``requests`` (urllib3, idna, charset detection, certifi) cost ~0.15 s of
import per process on this image; ``http.client`` still ~0.03 s, most of it
the ``email`` package it parses headers with (bench ``startup_s``: the
"client" phase).  This module speaks the small part of HTTP/1.1 the API
server needs on a socket of its own - request line and headers out;
status, headers and a body framed by Content-Length, chunked transfer
encoding or connection close back - and loads ``ssl`` only for https.  The
surface is the part of a ``requests.Session`` the client uses: ``verify`` /
``cert`` / ``auth`` / ``headers``, ``request()`` and a streaming ``get()``
with ``iter_lines()``.

Connections are kept alive per thread and per endpoint; a kept-alive
connection the server has since closed is detected before reuse, and a
request that finds it closed anyway is sent once more on a fresh connection
(nothing was processed on a dead socket).  Connection-level failures raise
:class:`ConnectionError` (an ``OSError``, as ``requests.ConnectionError``
is), which the callers' retry logic expects.
"""

from __future__ import annotations

import json
import select
import socket
import threading
from urllib.parse import urlsplit


class _Dead(Exception):
    """The peer closed the connection before a status line arrived."""


class _Conn:
    """One HTTP/1.1 connection (plain or TLS) with a buffered reader."""

    def __init__(self, host: str, port: int, timeout, ssl_context=None):
        self.host, self.port = host, port
        self.sock = None
        self._rfile = None
        self._timeout = timeout
        self._ctx = ssl_context

    def connect(self) -> None:
        sock = socket.create_connection((self.host, self.port), timeout=self._timeout)
        sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        if self._ctx is not None:
            sock = self._ctx.wrap_socket(sock, server_hostname=self.host)
        self.sock = sock
        self._rfile = sock.makefile("rb")

    def settimeout(self, timeout) -> None:
        self._timeout = timeout
        if self.sock is not None:
            self.sock.settimeout(timeout)

    def close(self) -> None:
        for x in (self._rfile, self.sock):
            if x is not None:
                try:
                    x.close()
                except OSError:
                    pass
        self.sock = self._rfile = None

    def send(self, method: str, path: str, headers: dict, body: bytes | None) -> None:
        if self.sock is None:
            self.connect()
        host = self.host if ":" not in self.host else f"[{self.host}]"
        lines = [f"{method} {path} HTTP/1.1", f"Host: {host}:{self.port}"]
        lines += [f"{k}: {v}" for k, v in headers.items() if k.lower() not in ("host", "content-length")]
        if body is not None or method in ("POST", "PUT", "PATCH"):
            lines.append(f"Content-Length: {len(body or b'')}")
        self.sock.sendall(("\r\n".join(lines) + "\r\n\r\n").encode("latin-1") + (body or b""))

    def read_head(self) -> tuple[int, list[tuple[str, str]], bool]:
        """Status, headers and whether the server closes after this response."""
        line = self._rfile.readline(65537)
        if not line:
            raise _Dead("connection closed")
        parts = line.decode("latin-1").split(None, 2)
        if len(parts) < 2 or not parts[0].startswith("HTTP/"):
            raise ConnectionError(f"bad status line {line[:80]!r}")
        status, version = int(parts[1]), parts[0]
        headers = []
        while True:
            h = self._rfile.readline(65537)
            if h in (b"\r\n", b"\n", b""):
                break
            k, _, v = h.decode("latin-1").partition(":")
            headers.append((k.strip(), v.strip()))
        conn_hdr = next((v.lower() for k, v in headers if k.lower() == "connection"), "")
        closes = conn_hdr == "close" or (version == "HTTP/1.0" and conn_hdr != "keep-alive")
        return status, headers, closes


class _Body:
    """A response body framed by Content-Length, chunked encoding or close."""

    def __init__(self, rfile, headers: dict, method: str, status: int):
        self._r = rfile
        te = headers.get("transfer-encoding", "").lower()
        self._chunked = "chunked" in te
        cl = headers.get("content-length")
        self._left = None if self._chunked or cl is None else int(cl)
        if method == "HEAD" or status in (204, 304) or 100 <= status < 200:
            self._left = 0
        self._chunk_left = 0
        self._done = self._left == 0

    def _next_chunk(self) -> bool:
        line = self._r.readline(65537)
        if not line:
            raise ConnectionError("connection closed inside a chunked body")
        size = int(line.split(b";", 1)[0].strip() or b"0", 16)
        if size == 0:  # trailer section up to the blank line
            while self._r.readline(65537) not in (b"\r\n", b"\n", b""):
                pass
            self._done = True
            return False
        self._chunk_left = size
        return True

    def read(self) -> bytes:
        if self._done:
            return b""
        if self._chunked:
            out = []
            while self._next_chunk():
                out.append(self._r.read(self._chunk_left))
                self._r.readline(3)  # CRLF after the chunk
            return b"".join(out)
        data = self._r.read() if self._left is None else self._r.read(self._left)
        if self._left is not None and len(data) < self._left:
            raise ConnectionError("connection closed inside the body")
        self._done = True
        return data

    def readline(self) -> bytes:
        """One line of the body (b"" at its end); lines may span chunks."""
        if self._done:
            return b""
        if not self._chunked:
            line = self._r.readline() if self._left is None else self._r.readline(self._left)
            if self._left is not None:
                self._left -= len(line)
                self._done = self._left <= 0
            elif not line:
                self._done = True
            return line
        buf = b""
        while True:
            if self._chunk_left == 0:
                if buf.endswith(b"\n") or not self._next_chunk():
                    return buf
            piece = self._r.readline(self._chunk_left)
            self._chunk_left -= len(piece)
            if self._chunk_left == 0:
                self._r.readline(3)  # CRLF after the chunk
            buf += piece
            if buf.endswith(b"\n"):
                return buf


class Headers(dict):
    """Case-insensitive response headers (``get`` only, as used)."""

    def __init__(self, items):
        super().__init__((k.lower(), v) for k, v in items)

    def get(self, key, default=None):
        return super().get(key.lower(), default)

    def __getitem__(self, key):
        return super().__getitem__(key.lower())

    def __contains__(self, key):
        return super().__contains__(key.lower())


class Response:
    def __init__(self, status: int, headers: Headers, reader: _Body | None = None, conn=None,
                 body: bytes | None = None):
        self.status_code = status
        self.headers = headers
        self._reader = reader
        self._conn = conn  # streaming: the connection this response owns
        self._body = body

    @property
    def content(self) -> bytes:
        if self._body is None:
            self._body = self._reader.read() if self._reader is not None else b""
        return self._body

    @property
    def text(self) -> str:
        return self.content.decode("utf-8", "replace")

    def json(self):
        return json.loads(self.content)

    def iter_lines(self, chunk_size=None):
        """Lines of a streamed body as they arrive (each watch event is one)."""
        while True:
            line = self._reader.readline()
            if not line:
                return
            yield line.rstrip(b"\r\n")

    def close(self) -> None:
        if self._conn is not None:
            self._conn.close()
            self._conn = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class PreparedRequest:
    """What an ``auth`` hook sees: mutable headers (TokenFileAuth sets one)."""

    def __init__(self, method: str, url: str, headers: dict):
        self.method, self.url, self.headers = method, url, headers


class Session:
    def __init__(self):
        self.verify = True       # True (system CAs), a CA bundle path, or False
        self.cert = None         # (certfile, keyfile)
        self.auth = None         # callable(PreparedRequest) -> PreparedRequest
        self.headers: dict[str, str] = {}
        self._local = threading.local()
        self._ssl = None
        self._ssl_key = None

    # ------------------------------------------------------------ internals
    def _context(self):
        import ssl  # https only: a plain-HTTP client never loads it

        key = (self.verify, self.cert)
        if self._ssl is None or self._ssl_key != key:
            if self.verify is False:
                ctx = ssl._create_unverified_context()  # noqa: SLF001 - insecure-skip-tls-verify
            else:
                ctx = ssl.create_default_context(cafile=self.verify if isinstance(self.verify, str) else None)
            if self.cert:
                ctx.load_cert_chain(*self.cert)
            self._ssl, self._ssl_key = ctx, key
        return self._ssl

    def _new_conn(self, scheme: str, netloc: str, timeout) -> _Conn:
        host, _, port = netloc.rpartition(":") if netloc.rsplit(":", 1)[-1].isdigit() else (netloc, "", "")
        host = host.strip("[]")
        if scheme == "https":
            return _Conn(host, int(port or 443), timeout, self._context())
        return _Conn(host, int(port or 80), timeout)

    @staticmethod
    def _dropped(conn) -> bool:
        """A kept-alive socket the server closed reads as ready (EOF)."""
        sock = conn.sock
        if sock is None:
            return True
        try:
            return bool(select.select([sock], [], [], 0)[0])
        except (OSError, ValueError):
            return True

    def _pooled(self, scheme: str, netloc: str, timeout):
        pool = getattr(self._local, "pool", None)
        if pool is None:
            pool = self._local.pool = {}
        conn = pool.get((scheme, netloc))
        if conn is not None and conn.sock is not None and self._dropped(conn):
            conn.close()
        if conn is None:
            conn = pool[(scheme, netloc)] = self._new_conn(scheme, netloc, timeout)
        conn.settimeout(timeout)
        return conn, conn.sock is not None

    def _prepare(self, method: str, url: str, data, headers):
        hdrs = dict(self.headers)
        hdrs.update(headers or {})
        req = PreparedRequest(method, url, hdrs)
        if self.auth is not None:
            req = self.auth(req)
        parts = urlsplit(url)
        path = (parts.path or "/") + (f"?{parts.query}" if parts.query else "")
        body = data.encode() if isinstance(data, str) else data
        return parts.scheme, parts.netloc, path, body, req.headers

    # --------------------------------------------------------------- public
    def request(self, method: str, url: str, timeout=None, data=None, headers=None, stream=False) -> Response:
        scheme, netloc, path, body, hdrs = self._prepare(method, url, data, headers)
        connect_t, read_t = timeout if isinstance(timeout, tuple) else (timeout, timeout)
        if stream:  # a connection of its own, closed with the response
            conn = self._new_conn(scheme, netloc, connect_t)
            try:
                conn.connect()
                conn.settimeout(read_t)
                conn.send(method, path, hdrs, body)
                status, headers, _ = conn.read_head()
                h = Headers(headers)
                return Response(status, h, _Body(conn._rfile, h, method, status), conn=conn)
            except (OSError, ValueError, _Dead) as e:
                conn.close()
                raise ConnectionError(f"{method} {url}: {e}") from e
        idempotent = method in ("GET", "HEAD", "OPTIONS")
        for attempt in (0, 1):
            conn, reused = self._pooled(scheme, netloc, connect_t)
            sent = False
            try:
                conn.send(method, path, hdrs, body)
                sent = True
                conn.settimeout(read_t)
                status, headers, closes = conn.read_head()
                h = Headers(headers)
                payload = _Body(conn._rfile, h, method, status).read()
                if closes or ("content-length" not in h and "chunked" not in h.get("transfer-encoding", "").lower()):
                    conn.close()
                return Response(status, h, body=payload)
            except (_Dead, ConnectionResetError, BrokenPipeError) as e:
                conn.close()
                # a kept-alive connection the server had closed: resend when the
                # request never left, or when running it twice is harmless; a
                # write that went out may have been applied, so it is not resent
                if reused and attempt == 0 and (not sent or idempotent):
                    continue
                raise ConnectionError(f"{method} {url}: {e}") from e
            except (OSError, ValueError) as e:
                conn.close()
                if isinstance(e, socket.timeout):
                    raise
                if isinstance(e, ConnectionError):
                    raise
                raise ConnectionError(f"{method} {url}: {e}") from e
        raise ConnectionError(f"{method} {url}: no connection")  # not reached

    def get(self, url: str, **kw) -> Response:
        return self.request("GET", url, **kw)
