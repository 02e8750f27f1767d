"""The RestClient's socket-level HTTP/1.1 transport (kube/transport.py):
response framing (Content-Length, chunked - watch lines split across
chunks -, connection close), kept-alive connections and their silent loss,
and TLS with the server certificate checked against the configured CA."""

import socket
import ssl
import subprocess
import threading
import time

import pytest

from amdgpu_operator.kube import transport as T


class RawServer:
    """Accepts connections and answers each request with the next scripted
    response bytes (``None``: close the connection without answering; ``b""``:
    hold it unanswered for 2 s, then close)."""

    def __init__(self, responses, tls=None):
        self.responses = list(responses)
        self.requests: list[bytes] = []
        self.connections = 0
        self.sock = socket.socket()
        self.sock.bind(("127.0.0.1", 0))
        self.sock.listen(16)
        self.port = self.sock.getsockname()[1]
        self.tls = tls
        threading.Thread(target=self._serve, daemon=True).start()

    def _serve(self):
        while self.responses:
            try:
                c, _ = self.sock.accept()
            except OSError:
                return
            self.connections += 1
            if self.tls:
                try:
                    c = self.tls.wrap_socket(c, server_side=True)
                except (ssl.SSLError, OSError):
                    c.close()
                    continue
            f = c.makefile("rb")
            while self.responses:
                head = b""
                while not head.endswith(b"\r\n\r\n"):
                    line = f.readline()
                    if not line:
                        break
                    head += line
                if not head:
                    break
                n = next((int(h.split(b":")[1]) for h in head.split(b"\r\n") if h.lower().startswith(b"content-length")),
                         0)
                self.requests.append(head + f.read(n))
                out = self.responses.pop(0)
                if out is None:
                    break
                if out == b"":
                    time.sleep(2)
                    break
                c.sendall(out)
                if b"Connection: close" in out:
                    break
            f.close()  # the makefile holds the socket open too
            c.close()

    def url(self, scheme="http"):
        return f"{scheme}://127.0.0.1:{self.port}"


def ok(body: bytes, extra=b"") -> bytes:
    return b"HTTP/1.1 200 OK\r\nContent-Type: application/json\r\n" + extra + \
        b"Content-Length: " + str(len(body)).encode() + b"\r\n\r\n" + body


def test_content_length_and_keep_alive():
    srv = RawServer([ok(b'{"a": 1}'), ok(b'{"b": 2}')])
    s = T.Session()
    r1 = s.request("GET", srv.url() + "/x", timeout=5)
    r2 = s.request("POST", srv.url() + "/y", timeout=5, data='{"z": 3}', headers={"Content-Type": "application/json"})
    assert r1.status_code == 200 and r1.json() == {"a": 1} and r2.json() == {"b": 2}
    assert srv.connections == 1  # one kept-alive connection
    assert srv.requests[1].startswith(b"POST /y HTTP/1.1") and srv.requests[1].endswith(b'{"z": 3}')
    assert r1.headers.get("content-type") == "application/json"


def test_chunked_watch_lines_across_chunks():
    events = [b'{"type": "ADDED", "object": {"n": 1}}\n', b'{"type": "MODIFIED", "object": {"n": 2}}\n']
    blob = b"".join(events)
    chunks = [blob[:10], blob[10:45], blob[45:]]  # lines split anywhere
    body = b"".join(hex(len(c))[2:].encode() + b"\r\n" + c + b"\r\n" for c in chunks) + b"0\r\n\r\n"
    srv = RawServer([b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\n" + body])
    s = T.Session()
    with s.get(srv.url() + "/watch", stream=True, timeout=5) as r:
        lines = list(r.iter_lines())
    assert lines == [e.rstrip(b"\n") for e in events]


def test_chunked_full_body_and_close_delimited_body():
    body = b"5\r\nhello\r\n6\r\n world\r\n0\r\n\r\n"
    srv = RawServer([b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\n" + body,
                     b"HTTP/1.1 200 OK\r\nConnection: close\r\n\r\nuntil-close"])
    s = T.Session()
    assert s.request("GET", srv.url() + "/a", timeout=5).text == "hello world"
    assert s.request("GET", srv.url() + "/b", timeout=5).text == "until-close"


def test_a_kept_alive_connection_the_server_dropped_is_retried_once():
    srv = RawServer([ok(b"1"), None, ok(b"2")])  # the 2nd request meets a closed socket
    s = T.Session()
    assert s.request("GET", srv.url() + "/a", timeout=5).text == "1"
    assert s.request("GET", srv.url() + "/b", timeout=5).text == "2"
    assert srv.connections == 2


def test_a_write_the_dropped_connection_may_have_taken_is_not_resent():
    """the request went out whole before the server closed, so it
    may have been applied: a POST is not sent a second time."""
    srv = RawServer([ok(b"1"), None, ok(b"2")])
    s = T.Session()
    assert s.request("GET", srv.url() + "/a", timeout=5).text == "1"
    with pytest.raises(ConnectionError):
        s.request("POST", srv.url() + "/b", timeout=5, data="{}")
    assert [r.split(b" ")[0] for r in srv.requests] == [b"GET", b"POST"]
    assert s.request("GET", srv.url() + "/c", timeout=5).text == "2"  # a fresh connection


def test_the_read_timeout_holds_on_a_kept_alive_connection():
    srv = RawServer([ok(b"1"), b""])
    s = T.Session()
    assert s.request("GET", srv.url() + "/a", timeout=(5, 0.3)).text == "1"
    t0 = time.monotonic()
    with pytest.raises((socket.timeout, ConnectionError)):
        s.request("GET", srv.url() + "/b", timeout=(5, 0.3))
    assert time.monotonic() - t0 < 1.5


def test_connection_refused_is_a_connection_error():
    s = T.Session()
    with pytest.raises(ConnectionError):
        s.request("GET", "http://127.0.0.1:1/x", timeout=2)


def _ca_and_server_cert(tmp_path, name):
    d = tmp_path / name
    d.mkdir()

    def run(*args):
        subprocess.run(["openssl", *args], cwd=d, check=True, capture_output=True, timeout=60)

    run("req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", "ca.key", "-out", "ca.crt", "-days", "2",
        "-subj", f"/CN={name}")
    run("req", "-newkey", "rsa:2048", "-nodes", "-keyout", "s.key", "-out", "s.csr", "-subj", "/CN=127.0.0.1")
    (d / "ext").write_text("subjectAltName=IP:127.0.0.1\n")
    run("x509", "-req", "-in", "s.csr", "-CA", "ca.crt", "-CAkey", "ca.key", "-CAcreateserial", "-out", "s.crt",
        "-days", "2", "-extfile", "ext")
    return str(d / "ca.crt"), str(d / "s.crt"), str(d / "s.key")


def test_https_verifies_against_the_configured_ca(tmp_path):
    ca, crt, key = _ca_and_server_cert(tmp_path, "good")
    ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
    ctx.load_cert_chain(crt, key)
    srv = RawServer([ok(b'{"tls": true}')], tls=ctx)
    s = T.Session()
    s.verify = ca
    assert s.request("GET", srv.url("https") + "/x", timeout=5).json() == {"tls": True}
    other, _, _ = _ca_and_server_cert(tmp_path, "other")
    srv2 = RawServer([ok(b"{}")], tls=ctx)
    s2 = T.Session()
    s2.verify = other
    with pytest.raises(ConnectionError, match="CERTIFICATE_VERIFY_FAILED|certificate verify failed"):
        s2.request("GET", srv2.url("https") + "/x", timeout=5)
