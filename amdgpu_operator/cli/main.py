"""``amdgpu-operator`` entry point (every operand image runs this).

Sub-commands:

* ``operator``              - the ClusterPolicy controller (Deployment in the chart)
* ``cleanup-crd``           - Helm pre-delete hook (``operator.cleanupCRD``, README.md:110)
* ``apply-crd``             - Helm pre-upgrade hook (CRD upgrade)
* ``verify``                - machine-checked version of README.md:113-215
* ``render``                - render the chart with ``--set`` flags (helm template)
* ``simulate``              - bring up a simulated cluster and report time-to-Ready
* ``driver|toolkit|validate|device-plugin|metrics-exporter|node-status-exporter|nfd|gfd|partition-manager``
                            - operand containers (see :mod:`.operands`)
"""

from __future__ import annotations

import argparse
import json
import sys
import threading

from .. import DEFAULT_NAMESPACE
from ..utils import logs

OPERAND_CMDS = {"driver", "toolkit", "validate", "device-plugin", "metrics-exporter", "node-status-exporter", "nfd",
                "gfd", "partition-manager"}


def _client(args):
    from ..kube.client import RestClient

    if getattr(args, "server", None):
        return RestClient(args.server, token=getattr(args, "token", None), verify=not getattr(args, "insecure", False))
    if getattr(args, "kubeconfig", None):
        return RestClient.from_kubeconfig(args.kubeconfig)
    try:
        return RestClient.from_incluster()
    except (KeyError, OSError):
        return RestClient.from_kubeconfig()


def _common(p):
    p.add_argument("--namespace", default=DEFAULT_NAMESPACE)
    p.add_argument("--kubeconfig", default=None)
    p.add_argument("--server", default=None, help="API server URL (tests / port-forward)")
    p.add_argument("--token", default=None)
    p.add_argument("--insecure", action="store_true")
    p.add_argument("--log-level", default="info")


def _health_server(port: int):
    from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

    class H(BaseHTTPRequestHandler):
        def log_message(self, *a):
            pass

        def do_GET(self):
            self.send_response(200 if self.path.startswith("/healthz") else 404)
            self.end_headers()
            self.wfile.write(b"ok\n")

    srv = ThreadingHTTPServer(("0.0.0.0", port), H)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    return srv


def main(argv: list[str] | None = None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    if argv and argv[0] in OPERAND_CMDS:
        from ..kube.client import RestClient
        from ..nodeenv import NodeEnv
        from .operands import run_operand

        logs.setup()
        try:
            client = RestClient.from_incluster()
        except (KeyError, OSError):
            client = None  # node-local operands (driver, toolkit) work without the API
        env = NodeEnv.from_environ(client)
        import os

        return run_operand(env, argv, threading.Event(), container_env=dict(os.environ))

    ap = argparse.ArgumentParser(prog="amdgpu-operator")
    sub = ap.add_subparsers(dest="cmd", required=True)
    op = sub.add_parser("operator", help="run the ClusterPolicy controller")
    _common(op)
    op.add_argument("--health-port", type=int, default=8081)
    op.add_argument("--resync", type=float, default=30.0)
    cl = sub.add_parser("cleanup-crd", help="delete ClusterPolicies and the CRD")
    _common(cl)
    ac = sub.add_parser("apply-crd", help="create/update the ClusterPolicy CRD")
    _common(ac)
    ve = sub.add_parser("verify", help="check the install like README.md:113-215")
    _common(ve)
    ve.add_argument("--json", action="store_true")
    ve.add_argument("--expect-gpus", type=int, default=None)
    rn = sub.add_parser("render", help="render the Helm chart (helm template)")
    rn.add_argument("--set", action="append", default=[])
    rn.add_argument("--namespace", default=DEFAULT_NAMESPACE)
    rn.add_argument("--release", default="gpu-operator")
    sm = sub.add_parser("simulate", help="simulated cluster bring-up (time-to-Ready)")
    sm.add_argument("--gpus", type=int, default=8)
    sm.add_argument("--partition", default="SPX")
    sm.add_argument("--set", action="append", default=[])
    sm.add_argument("--real-gpus", action="store_true", help="use this machine's GPUs and sysfs")
    sm.add_argument("--timeout", type=float, default=120)
    args = ap.parse_args(argv)
    logs.setup(getattr(args, "log_level", "info"))

    if args.cmd == "operator":
        from ..controller.reconciler import ClusterPolicyReconciler

        _health_server(args.health_port)
        rec = ClusterPolicyReconciler(_client(args), args.namespace)
        rec.run(threading.Event(), resync_s=args.resync)
        return 0
    if args.cmd == "cleanup-crd":
        from ..controller.reconciler import cleanup_crd

        print(json.dumps({"crd_deleted": cleanup_crd(_client(args))}))
        return 0
    if args.cmd == "apply-crd":
        from ..helm.crd import crd
        from ..kube.client import apply_object

        _, action = apply_object(_client(args), crd())
        print(json.dumps({"crd": action}))
        return 0
    if args.cmd == "verify":
        from .verify import main_verify

        return main_verify(_client(args), args.namespace, args.json, args.expect_gpus)
    if args.cmd == "render":
        import yaml

        from ..helm.render import render_chart

        docs = render_chart(set_flags=args.set, release_name=args.release, namespace=args.namespace)
        sys.stdout.write(yaml.safe_dump_all(docs, sort_keys=False))
        return 0
    if args.cmd == "simulate":
        import tempfile

        from ..api.clusterpolicy import parse_set_flags
        from ..testing.simcluster import NodeSpec, SimCluster
        from .verify import verify

        d = tempfile.mkdtemp(prefix="amdgpu-sim-")
        node = NodeSpec("node-0", args.gpus, args.partition, sysfs_root="/" if args.real_gpus else None)
        c = SimCluster(d, [node], fake_gpu=not args.real_gpus).start()
        try:
            c.install_operator(parse_set_flags(args.set))
            ttr = c.wait_ready(args.timeout)
            rep = verify(c.client, c.namespace)
            print(json.dumps({"time_to_ready_s": round(ttr, 4), "verify": rep.as_dict()}, indent=1))
            return 0 if rep.ok else 1
        finally:
            c.stop()
    return 2


if __name__ == "__main__":
    sys.exit(main())
