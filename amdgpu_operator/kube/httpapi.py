"""HTTP front end for :class:`~.fakeapi.FakeApiServer` with real REST paths.

Serves ``/api/v1/...`` and ``/apis/<group>/<version>/...`` (namespaced and
cluster-scoped, ``/status`` subresource, ``?watch=1`` streaming JSON lines,
``labelSelector`` / ``fieldSelector``, merge-patch).  Lets the production
:class:`~.client.RestClient` be tested end-to-end over HTTP.
"""

from __future__ import annotations

import json
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from urllib.parse import parse_qs, unquote, urlparse

from . import resources as R
from .fakeapi import ApiError, FakeApiServer


def _parse_path(path: str):
    """-> (ResourceType, namespace, name, subresource)"""
    segs = [unquote(s) for s in path.strip("/").split("/") if s]
    if not segs:
        raise ApiError(404, "NotFound", path)
    if segs[0] == "api":
        group, version, rest = "", segs[1], segs[2:]
    elif segs[0] == "apis":
        group, version, rest = segs[1], segs[2], segs[3:]
    else:
        raise ApiError(404, "NotFound", path)
    ns = None
    if len(rest) >= 2 and rest[0] == "namespaces" and len(rest) > 2:
        ns, rest = rest[1], rest[2:]
    if not rest:
        raise ApiError(404, "NotFound", path)
    plural = rest[0]
    name = rest[1] if len(rest) > 1 else None
    sub = rest[2] if len(rest) > 2 else None
    t = R.BY_PLURAL.get((group, version, plural))
    if t is None:
        raise ApiError(404, "NotFound", f"no resource {group}/{version}/{plural}")
    return t, ns, name, sub


class _Handler(BaseHTTPRequestHandler):
    server_version = "fake-kube-apiserver/0.1"
    protocol_version = "HTTP/1.1"
    # headers and body go out in separate writes: with Nagle on, the body
    # waits for the client's delayed ACK of the headers (~40 ms per request)
    disable_nagle_algorithm = True
    api: FakeApiServer  # set on the subclass

    def log_message(self, fmt, *args):  # quiet
        pass

    def _send(self, code: int, body: dict) -> None:
        data = json.dumps(body).encode()
        self.send_response(code)
        self.send_header("Content-Type", "application/json")
        self.send_header("Content-Length", str(len(data)))
        self.end_headers()
        self.wfile.write(data)

    def _error(self, e: ApiError) -> None:
        self._send(e.code, {"kind": "Status", "apiVersion": "v1", "status": "Failure", "reason": e.reason,
                            "message": e.message, "code": e.code})

    def _body(self) -> dict:
        return json.loads(self._raw or b"{}")

    def _dispatch(self, method: str) -> None:
        # the body is read before anything can fail: an error answered with
        # the body still unread would leave it in the kept-alive connection,
        # where it becomes the next request's request line
        n = int(self.headers.get("Content-Length") or 0)
        self._raw = self.rfile.read(n) if n else b""
        u = urlparse(self.path)
        q = {k: v[-1] for k, v in parse_qs(u.query).items()}
        try:
            t, ns, name, sub = _parse_path(u.path)
            api = self.api
            authz = getattr(self.server, "authorizer", None)
            if authz is not None:  # kube/rbac.py: the caller's ServiceAccount must be granted the request
                from .rbac import verb_of

                auth = self.headers.get("Authorization", "")
                user = self.server.tokens.get(auth[7:] if auth.startswith("Bearer ") else "")
                if user is None:
                    raise ApiError(401, "Unauthorized", "no valid bearer token")
                verb = verb_of(method, name, method == "GET" and q.get("watch") in ("1", "true"))
                res = t.plural + (f"/{sub}" if sub else "")
                if not authz.allowed(user, verb, t.group, res, ns, name):
                    where = f' in the namespace "{ns}"' if ns else " at the cluster scope"
                    self.server.denied.append((user, verb, t.group, res, ns, name))
                    raise ApiError(403, "Forbidden", f'User "{user}" cannot {verb} resource "{res}" in API group '
                                                     f'"{t.group}"{where}')
            if method == "GET" and name is None:
                if q.get("watch") in ("1", "true"):
                    return self._watch(t, ns, q)
                items = api.list(t.api_version, t.kind, ns, q.get("labelSelector"), q.get("fieldSelector"))
                return self._send(200, {"apiVersion": t.api_version, "kind": t.kind + "List", "items": items,
                                        "metadata": {"resourceVersion": str(api.resource_version())}})
            if method == "GET":
                return self._send(200, api.get(t.api_version, t.kind, name, ns))
            if method == "POST":
                obj = self._body()
                if ns and t.namespaced:
                    obj.setdefault("metadata", {})["namespace"] = ns
                return self._send(201, api.create(obj))
            if method == "PUT":
                return self._send(200, api.update(self._body(), subresource=sub))
            if method == "PATCH":
                return self._send(200, api.patch(t.api_version, t.kind, name, self._body(), ns, subresource=sub))
            if method == "DELETE":
                grace = q.get("gracePeriodSeconds")
                api.delete(t.api_version, t.kind, name, ns, None if grace in (None, "") else int(grace))
                return self._send(200, {"kind": "Status", "apiVersion": "v1", "status": "Success"})
            raise ApiError(405, "MethodNotAllowed", method)
        except ApiError as e:
            self._error(e)
        except (ValueError, KeyError) as e:
            self._error(ApiError(400, "BadRequest", str(e)))

    def _watch(self, t, ns, q) -> None:
        timeout = float(q["timeoutSeconds"]) if q.get("timeoutSeconds") else None
        w = self.api.watch(t.api_version, t.kind, ns, q.get("labelSelector"), q.get("fieldSelector"),
                           q.get("resourceVersion"))
        self.send_response(200)
        self.send_header("Content-Type", "application/json")
        self.send_header("Transfer-Encoding", "chunked")
        self.end_headers()
        try:
            for etype, obj in w.stream(timeout=timeout, stop=self.server.stopping):
                line = (json.dumps({"type": etype, "object": obj}) + "\n").encode()
                self.wfile.write(b"%x\r\n%s\r\n" % (len(line), line))
                self.wfile.flush()
            self.wfile.write(b"0\r\n\r\n")
        except (BrokenPipeError, ConnectionResetError):
            pass
        finally:
            self.api.stop_watch(w)
            self.close_connection = True

    def do_GET(self):
        self._dispatch("GET")

    def do_POST(self):
        self._dispatch("POST")

    def do_PUT(self):
        self._dispatch("PUT")

    def do_PATCH(self):
        self._dispatch("PATCH")

    def do_DELETE(self):
        self._dispatch("DELETE")


class _Server(ThreadingHTTPServer):
    # the listen backlog: socketserver's default of 5 overflowed when the
    # operator's informers and a node's operand processes connected at once,
    # and a dropped SYN is retried by the client's kernel only after 1 s (a
    # watch that began a second late looked like a 1 s reconcile stall)
    request_queue_size = 512


class HttpApiServer:
    """Run the fake apiserver on ``127.0.0.1:<port>`` in a background thread."""

    def __init__(self, api: FakeApiServer, host: str = "127.0.0.1", port: int = 0):
        handler = type("Handler", (_Handler,), {"api": api})
        self.httpd = _Server((host, port), handler)
        self.httpd.daemon_threads = True
        self.httpd.stopping = threading.Event()
        self.httpd.authorizer = None  # enable_rbac()
        self.httpd.tokens = {}  # bearer token -> user
        self.httpd.denied = []  # (user, verb, group, resource, namespace, name) refused
        self.thread = threading.Thread(target=self.httpd.serve_forever, daemon=True, name="fake-apiserver-http")

    def enable_rbac(self) -> None:
        """Authorize every request against the RBAC objects in the API (kube/rbac.py)."""
        from .rbac import Authorizer

        self.httpd.authorizer = Authorizer(self.httpd.RequestHandlerClass.api)

    def token_for(self, namespace: str, service_account: str) -> str:
        """A bearer token that authenticates as ``namespace/service_account``."""
        token = f"sa-{namespace}-{service_account}"
        self.httpd.tokens[token] = f"system:serviceaccount:{namespace}:{service_account}"
        return token

    @property
    def denied(self) -> list:
        return self.httpd.denied

    @property
    def url(self) -> str:
        h, p = self.httpd.server_address[:2]
        return f"http://{h}:{p}"

    def start(self) -> "HttpApiServer":
        self.thread.start()
        return self

    def stop(self) -> None:
        self.httpd.stopping.set()
        self.httpd.shutdown()
        self.httpd.server_close()
