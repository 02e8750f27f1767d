"""Operand start-up stays light: an operand container is a fresh
``python -m amdgpu_operator <operand>`` process on the node's time-to-Ready
path, so the modules it runs must not pull in the operator's ClusterPolicy
model (pydantic), requests, YAML, grpcio or protobuf (bench --mode process breakdown,
tools/operand_start_probe.py)."""

import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OPERAND_MODULES = ["amdgpu_operator.cli.main", "amdgpu_operator.cli.operands", "amdgpu_operator.driver.manager",
                   "amdgpu_operator.validator.validate", "amdgpu_operator.toolkit.install",
                   "amdgpu_operator.deviceplugin.server", "amdgpu_operator.deviceplugin.config",
                   "amdgpu_operator.exporter.metrics", "amdgpu_operator.discovery.labels",
                   "amdgpu_operator.partition.manager", "amdgpu_operator.kube.client", "amdgpu_operator.kube.events",
                   "amdgpu_operator.testing.simnode", "amdgpu_operator.wellknown"]
HEAVY = ("pydantic", "requests", "yaml", "amdgpu_operator.api.clusterpolicy", "amdgpu_operator.controller.reconciler",
         # the kubelet gRPC runs on amdgpu_operator.rpc (grpcio + protobuf were ~0.1 s of the plugin's start)
         "grpc", "google.protobuf",
         # the simulated API server (the client imports kube.errors) and uuid's platform probe
         "amdgpu_operator.kube.fakeapi", "uuid")


def test_operand_modules_do_not_import_the_operator_model():
    code = ("import sys\n" + "".join(f"import {m}\n" for m in OPERAND_MODULES) +
            f"print(','.join(m for m in {HEAVY!r} if m in sys.modules))")
    p = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, p.stderr
    assert p.stdout.strip() == "", f"operand start-up imports {p.stdout.strip()}"


def test_the_api_client_stays_off_http_client():
    """The RestClient's transport speaks HTTP/1.1 on sockets: building a
    client and the critical-path operands' modules load neither
    ``http.client`` (its ``email`` header parsing was ~0.03 s per process)
    nor ``ssl`` for a plain-HTTP server."""
    code = ("import sys, json, os, tempfile\n"
            "import amdgpu_operator.cli.main, amdgpu_operator.cli.operands, amdgpu_operator.driver.manager\n"
            "import amdgpu_operator.toolkit.install, amdgpu_operator.validator.validate\n"
            "from amdgpu_operator.kube.client import RestClient\n"
            "RestClient('http://127.0.0.1:1')\n"
            "print(','.join(m for m in ('http.client', 'email.parser', 'ssl') if m in sys.modules))")
    p = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, p.stderr
    assert p.stdout.strip() == ""
