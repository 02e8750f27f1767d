"""N8, the native node-feature-discovery worker (``amdgpu-nfd``,
native/nfd/nfd_worker.cpp): the same labels as the Python worker
(discovery/labels.py nfd_labels), written to the Node over the API with a
merge patch - plain HTTP with a JSON kubeconfig, and HTTPS with the server
certificate verified against the configured CA."""

import json
import os
import signal
import ssl
import subprocess
import time

import pytest

from amdgpu_operator import native
from amdgpu_operator.discovery import labels as L
from amdgpu_operator.kube import resources as R
from amdgpu_operator.kube.fakeapi import FakeApiServer
from amdgpu_operator.kube.httpapi import HttpApiServer
from amdgpu_operator.testing import fakesys
from amdgpu_operator.wellknown import NFD_SCANNED_ANN

NFD = str(native.artefact("amdgpu-nfd"))
P = L.NFD_PREFIX


def _print(root):
    p = subprocess.run([NFD, "--print", "--host-root", root], capture_output=True, text=True, timeout=30)
    assert p.returncode == 0, p.stderr
    return json.loads(p.stdout)


@pytest.mark.parametrize("kind", ["synthetic", "mi355x-capture", "rdma"])
def test_labels_match_the_python_worker(tmp_path, kind):
    root = str(tmp_path / "host")
    if kind == "rdma":
        fakesys.add_rdma_nics(root, fakesys.build_node(root, 4, pcie_tree=True))
        assert L.nfd_labels(root)[P + "rdma.capable"] == L.nfd_labels(root)[P + "rdma.available"] == "true"
    if kind == "synthetic":
        fakesys.build_node(root, 4, kernel="6.8.0-45-generic")
    else:
        fakesys.build_from_real_fixture(root)
    assert _print(root) == L.nfd_labels(root)
    assert _print(root)[P + "pci-1002.present"] == "true"


def _cluster(tmp_path, labels=None, tls=None):
    api = FakeApiServer()
    api.create(R.new("v1", "Node", "n1", labels=labels or {}))
    http = HttpApiServer(api)
    server = "http://{}:{}".format(*http.httpd.server_address[:2])
    if tls:
        ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
        ctx.load_cert_chain(tls["cert"], tls["key"])
        http.httpd.socket = ctx.wrap_socket(http.httpd.socket, server_side=True)
        server = server.replace("http://", "https://")
    http.start()
    cluster = {"server": server}
    if tls:
        cluster["certificate-authority"] = tls["ca"]
    kc = tmp_path / "kubeconfig.json"
    kc.write_text(json.dumps({"apiVersion": "v1", "kind": "Config", "current-context": "t",
                              "clusters": [{"name": "t", "cluster": cluster}],
                              "users": [{"name": "u", "user": {"token": "abc"}}],
                              "contexts": [{"name": "t", "context": {"cluster": "t", "user": "u"}}]}))
    return api, http, str(kc)


def _run(kubeconfig, root, *args, timeout=30, **env):
    e = {k: v for k, v in os.environ.items() if k != "KUBERNETES_SERVICE_HOST"}
    e.update({"KUBECONFIG": kubeconfig, "NODE_NAME": "n1", "HOST_ROOT": root, **env})
    return subprocess.run([NFD, *args], env=e, capture_output=True, text=True, timeout=timeout)


def test_labels_the_node_and_removes_what_it_no_longer_sees(tmp_path):
    root = str(tmp_path / "host")
    fakesys.build_node(root, 2)
    api, http, kc = _cluster(tmp_path, labels={P + "pci-0300_10de.present": "true",  # a GPU that left the node
                                               "kubernetes.io/hostname": "n1"})
    try:
        ready = tmp_path / "ready"
        p = _run(kc, root, "--oneshot", AMDGPU_READY_FILE=str(ready))
        assert p.returncode == 0, p.stderr
        node = api.get("v1", "Node", "n1")
        labels = node["metadata"]["labels"]
        assert {k: v for k, v in labels.items() if k.startswith(P)} == L.nfd_labels(root)
        assert labels["kubernetes.io/hostname"] == "n1"  # not NFD's
        assert node["metadata"]["annotations"][NFD_SCANNED_ANN] == "true"
        assert float(ready.read_text()) >= float((tmp_path / "ready.started").read_text())
        rv = node["metadata"]["resourceVersion"]
        p = _run(kc, root, "--oneshot")  # nothing changed: no write
        assert p.returncode == 0 and api.get("v1", "Node", "n1")["metadata"]["resourceVersion"] == rv
        # the driver unloads: the module label goes
        os.unlink(os.path.join(root, "sys/module/amdgpu/initstate"))
        assert _run(kc, root, "--oneshot").returncode == 0
        assert P + "kernel-loadedmodule.amdgpu" not in api.get("v1", "Node", "n1")["metadata"]["labels"]
    finally:
        http.stop()


def test_stops_promptly_on_sigterm(tmp_path):
    root = str(tmp_path / "host")
    fakesys.build_node(root, 1)
    api, http, kc = _cluster(tmp_path)
    try:
        e = {k: v for k, v in os.environ.items() if k != "KUBERNETES_SERVICE_HOST"}
        e.update({"KUBECONFIG": kc, "NODE_NAME": "n1", "HOST_ROOT": root, "AMDGPU_READY_FILE": str(tmp_path / "r")})
        p = subprocess.Popen([NFD, "--interval", "600"], env=e, stderr=subprocess.PIPE, text=True)
        deadline = time.monotonic() + 20
        while not (tmp_path / "r").exists() and time.monotonic() < deadline:
            time.sleep(0.01)
        assert (tmp_path / "r").exists()
        t0 = time.monotonic()
        p.send_signal(signal.SIGTERM)
        assert p.wait(timeout=10) == 0 and time.monotonic() - t0 < 2.0
    finally:
        http.stop()


def _certs(tmp_path, name):
    """A CA and a server certificate for 127.0.0.1 signed by it (openssl CLI)."""
    d = tmp_path / name
    d.mkdir()

    def run(*args):
        subprocess.run(["openssl", *args], cwd=d, check=True, capture_output=True, timeout=60)

    run("req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", "ca.key", "-out", "ca.crt", "-days", "2",
        "-subj", f"/CN={name}-ca")
    run("req", "-newkey", "rsa:2048", "-nodes", "-keyout", "srv.key", "-out", "srv.csr", "-subj", "/CN=127.0.0.1")
    (d / "ext.cnf").write_text("subjectAltName=IP:127.0.0.1\n")
    run("x509", "-req", "-in", "srv.csr", "-CA", "ca.crt", "-CAkey", "ca.key", "-CAcreateserial", "-out", "srv.crt",
        "-days", "2", "-extfile", "ext.cnf")
    return {"ca": str(d / "ca.crt"), "cert": str(d / "srv.crt"), "key": str(d / "srv.key")}


def test_https_verifies_the_api_server_certificate(tmp_path):
    root = str(tmp_path / "host")
    fakesys.build_node(root, 1)
    good = _certs(tmp_path, "good")
    api, http, kc = _cluster(tmp_path, tls=good)
    try:
        p = _run(kc, root, "--oneshot")
        assert p.returncode == 0, p.stderr
        assert api.get("v1", "Node", "n1")["metadata"]["labels"][P + "pci-1002.present"] == "true"
        # a CA that did not sign the server's certificate: the handshake fails, nothing is written
        other = _certs(tmp_path, "other")
        cfg = json.loads(open(kc).read())
        cfg["clusters"][0]["cluster"]["certificate-authority"] = other["ca"]
        bad = tmp_path / "bad.json"
        bad.write_text(json.dumps(cfg))
        e = {k: v for k, v in os.environ.items() if k != "KUBERNETES_SERVICE_HOST"}
        e.update({"KUBECONFIG": str(bad), "NODE_NAME": "n1", "HOST_ROOT": root})
        proc = subprocess.Popen([NFD, "--oneshot"], env=e, stderr=subprocess.PIPE, text=True)
        time.sleep(1.0)
        proc.send_signal(signal.SIGTERM)
        _, err = proc.communicate(timeout=10)
        assert "TLS handshake" in err and "certificate verify failed" in err
    finally:
        http.stop()
