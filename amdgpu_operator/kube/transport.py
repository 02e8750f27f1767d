"""HTTP(S) transport of :class:`~.client.RestClient` on the standard library.

Every operand container talks to the API server, and every one of them pays
its client's import at start-up, inside the node's time-to-Ready: ``requests``
(with urllib3, idna, charset detection, certifi) costs ~0.15 s of import per
process on this image, ``http.client`` + ``ssl`` a tenth of that, and the
operand images need one Python package less.  The surface is the small part
of a ``requests.Session`` the client uses: ``verify`` / ``cert`` / ``auth`` /
``headers``, ``request()`` and a streaming ``get()`` with ``iter_lines()``.

Connections are kept alive per thread and per endpoint (``http.client`` is not
thread-safe); a kept-alive connection the server has since closed is
detected before reuse, and a request that finds it closed anyway is sent
once more on a fresh connection (nothing was processed on a dead socket).
Connection-level failures raise :class:`ConnectionError` (an ``OSError``, as
``requests.ConnectionError`` is), which the callers' retry logic expects.
"""

from __future__ import annotations

import http.client
import json
import select
import socket
import ssl
import threading
from urllib.parse import urlsplit

_DEAD_CONN = (http.client.RemoteDisconnected, ConnectionResetError, BrokenPipeError, http.client.BadStatusLine,
              http.client.CannotSendRequest, http.client.ResponseNotReady)


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
    def __init__(self, resp: http.client.HTTPResponse, conn=None, body: bytes | None = None):
        self.status_code = resp.status
        self.headers = Headers(resp.getheaders())
        self._resp = resp
        self._conn = conn  # streaming: the connection this response owns
        self._body = body

    @property
    def content(self) -> bytes:
        if self._body is None:
            self._body = self._resp.read()
        return self._body

    @property
    def text(self) -> str:
        return self.content.decode("utf-8", "replace")

    def json(self):
        return json.loads(self.content)

    def iter_lines(self, chunk_size=None):
        """Lines of a streamed body as they arrive (each watch event is one)."""
        while True:
            line = self._resp.readline()
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
        self._ssl: ssl.SSLContext | None = None
        self._ssl_key = None

    # ------------------------------------------------------------ internals
    def _context(self) -> ssl.SSLContext:
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

    def _new_conn(self, scheme: str, netloc: str, timeout):
        host, _, port = netloc.rpartition(":") if netloc.rsplit(":", 1)[-1].isdigit() else (netloc, "", "")
        host = host.strip("[]")
        if scheme == "https":
            return http.client.HTTPSConnection(host, int(port or 443), timeout=timeout, context=self._context())
        return http.client.HTTPConnection(host, int(port or 80), timeout=timeout)

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
        conn.timeout = timeout
        if conn.sock is not None:
            conn.sock.settimeout(timeout)
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
                conn.sock.settimeout(read_t)
                conn.request(method, path, body=body, headers=hdrs)
                return Response(conn.getresponse(), conn=conn)
            except (OSError, http.client.HTTPException) as e:
                conn.close()
                raise ConnectionError(f"{method} {url}: {e}") from e
        for attempt in (0, 1):
            conn, reused = self._pooled(scheme, netloc, connect_t)
            try:
                conn.request(method, path, body=body, headers=hdrs)
                resp = conn.getresponse()
                payload = resp.read()
                if resp.will_close:
                    conn.close()
                return Response(resp, body=payload)
            except _DEAD_CONN as e:
                conn.close()
                if reused and attempt == 0:
                    continue  # the server had closed the kept-alive connection: nothing was processed
                raise ConnectionError(f"{method} {url}: {e}") from e
            except (OSError, http.client.HTTPException) as e:
                conn.close()
                if isinstance(e, socket.timeout):
                    raise
                raise ConnectionError(f"{method} {url}: {e}") from e
        raise ConnectionError(f"{method} {url}: no connection")  # not reached

    def get(self, url: str, **kw) -> Response:
        return self.request("GET", url, **kw)
