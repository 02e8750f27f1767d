"""``amdgpu-operator`` entry point (every operand image runs this).

Sub-commands:

* ``operator``              - the ClusterPolicy controller (Deployment in the chart)
* ``cleanup-crd``           - Helm pre-delete hook (``operator.cleanupCRD``, README.md:110)
* ``apply-crd``             - Helm pre-upgrade hook (CRD upgrade)
* ``verify``                - machine-checked version of README.md:113-215
* ``render``                - render the chart with ``--set`` flags (helm template)
* ``simulate``              - bring up a simulated cluster and report time-to-Ready
* ``preflight``             - node prerequisites of README.md:5-49 + the GPU/driver state, checked (``--fix``)
* ``collectives``           - RCCL sweep (all-reduce / all-gather / reduce-scatter, algBW + busBW);
                              one rank per GPU under ``torch.distributed.run``
* ``driver|toolkit|validate|device-plugin|metrics-exporter|node-status-exporter|nfd|gfd|partition-manager``
                            - operand containers (see :mod:`.operands`)
"""

from __future__ import annotations

import json
import sys
import threading

from .. import DEFAULT_NAMESPACE
from ..utils import logs

OPERAND_CMDS = {"driver", "toolkit", "validate", "device-plugin", "metrics-exporter", "node-status-exporter", "nfd",
                "gfd", "partition-manager", "vfio-manager", "sandbox-device-plugin", "dra-driver"}


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


def _ready_signal():
    """``AMDGPU_READY_FILE``: the operand's readiness as a file (written when
    the operand calls ``ready()``), for a supervisor without in-process
    callbacks - the simulated kubelet of a ``process_containers`` SimCluster,
    or a file-based readinessProbe.  ``<file>.started`` records when the
    operand's main began (interpreter + imports done)."""
    import os

    path = os.environ.get("AMDGPU_READY_FILE")
    if not path:
        return lambda: None

    def write(p, text):
        tmp = f"{p}.tmp.{os.getpid()}"
        with open(tmp, "w") as f:
            f.write(text)
        os.replace(tmp, p)

    import time

    write(path + ".started", repr(time.time()))
    return lambda: write(path, repr(time.time()))


def _stop_on_signals() -> threading.Event:
    """An event set by SIGTERM / SIGINT (how the kubelet stops a container)."""
    import signal

    stop = threading.Event()
    for sig in (signal.SIGTERM, signal.SIGINT):
        signal.signal(sig, lambda *_: stop.set())
    return stop


def _common(p):
    p.add_argument("--namespace", default=DEFAULT_NAMESPACE)
    p.add_argument("--kubeconfig", default=None)
    p.add_argument("--server", default=None, help="API server URL (tests / port-forward)")
    p.add_argument("--token", default=None)
    p.add_argument("--insecure", action="store_true")
    p.add_argument("--log-level", default="info")


def _health_server(port: int, metrics=None):
    """``/healthz`` (liveness/readiness probes) and ``/metrics`` (operator self-metrics)."""
    from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

    class H(BaseHTTPRequestHandler):
        def log_message(self, *a):
            pass

        def do_GET(self):
            if self.path.startswith("/metrics") and metrics is not None:
                body = metrics.render().encode()
                self.send_response(200)
                self.send_header("Content-Type", "text/plain; version=0.0.4")
                self.end_headers()
                self.wfile.write(body)
                return
            self.send_response(200 if self.path.startswith("/healthz") else 404)
            self.end_headers()
            self.wfile.write(b"ok\n")

    srv = ThreadingHTTPServer(("0.0.0.0", port), H)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    return srv


def main(argv: list[str] | None = None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    if argv and argv[0] in OPERAND_CMDS:
        import os
        import time

        trace = os.environ.get("AMDGPU_STARTUP_TRACE")  # "<file>": wall time of each start-up phase

        def mark(what):
            if trace:
                with open(trace, "a") as f:
                    f.write(f"{what} {time.time():.4f}\n")

        mark("main")
        from ..kube.client import RestClient
        from ..nodeenv import NodeEnv
        from .operands import run_operand

        mark("imports")
        logs.setup()
        try:
            client = RestClient.from_incluster()
        except (KeyError, OSError):
            # outside a pod: a kubeconfig if one is named (the simulated
            # cluster's operand processes), else node-local operands (driver,
            # toolkit) work without the API
            client = RestClient.from_kubeconfig() if os.environ.get("KUBECONFIG") else None
        mark("client")
        env = NodeEnv.from_environ(client)
        if os.environ.get("AMDGPU_SIM_NODE") == "1":
            from ..testing.simnode import adopt_sim_node_env

            adopt_sim_node_env(env)
        mark("env")
        import gc

        gc.freeze()  # the start-up heap (modules, config) is never garbage: later collections skip it
        # the kubelet stops a container with SIGTERM: operands then run their
        # shutdown (toolkit cleanup, vfio unbind, plugin socket removal)
        return run_operand(env, argv, _stop_on_signals(), ready=_ready_signal(), container_env=dict(os.environ))

    import argparse  # not on the operands' start-up path (cli/argspec.py)

    ap = argparse.ArgumentParser(prog="amdgpu-operator")
    sub = ap.add_subparsers(dest="cmd", required=True)
    op = sub.add_parser("operator", help="run the ClusterPolicy controller")
    _common(op)
    op.add_argument("--health-port", type=int, default=8081)
    op.add_argument("--resync", type=float, default=30.0)
    op.add_argument("--debounce", type=float, default=0.003,
                    help="an event within this long after a pass waits out the rest of it (bursts cost one pass; "
                         "the echoes of the operator's own writes trigger no pass at all, kube/informer.py)")
    op.add_argument("--leader-elect", action="store_true",
                    help="run the controller only while holding the Lease (replicas > 1: warm standbys)")
    op.add_argument("--leader-election-id", default="amd-gpu-operator-leader")
    op.add_argument("--lease-seconds", type=float, default=15.0)
    cl = sub.add_parser("cleanup-crd", help="delete ClusterPolicies and the CRD")
    _common(cl)
    ac = sub.add_parser("apply-crd", help="create/update the ClusterPolicy CRD")
    _common(ac)
    ve = sub.add_parser("verify", help="check the install like README.md:113-215")
    _common(ve)
    ve.add_argument("--json", action="store_true")
    ve.add_argument("--expect-gpus", type=int, default=None)
    ve.add_argument("--run-pod", action="store_true",
                    help="also run one 1-GPU pod per GPU node (device plugin or DRA claim) and require it to succeed")
    ve.add_argument("--pod-image", default=None,
                    help="image of the --run-pod pod (default: the ClusterPolicy's validator image)")
    ve.add_argument("--pod-timeout", type=float, default=120.0)
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
    sm.add_argument("--nodes", type=int, default=1, help="GPU nodes in the simulated cluster")
    sm.add_argument("--http-api", action="store_true",
                    help="operator and operands talk to the API server over HTTP (RestClient), as in a cluster")
    sm.add_argument("--run-pod", action="store_true", help="verify --run-pod after the bring-up (a 1-GPU pod per node)")
    pf = sub.add_parser("preflight", help="check (and --fix) a node's prerequisites before kubeadm join")
    pf.add_argument("--root", default="/")
    pf.add_argument("--fix", action="store_true")
    pf.add_argument("--json", action="store_true")
    pf.add_argument("--expect-gpus", type=int, default=None)
    pf.add_argument("--no-gpu", action="store_true", help="control-plane / CPU node: skip the GPU checks")
    mg = sub.add_parser("must-gather", help="archive cluster + node state for troubleshooting (README.md:172-187)")
    _common(mg)
    mg.add_argument("--output", default="amdgpu-must-gather.tar.gz")
    mg.add_argument("--node-root", default=None, help="also collect this host's GPU state (e.g. / on a GPU node)")
    mg.add_argument("--validations-dir", default="/run/amd/validations")
    mg.add_argument("--no-cluster", action="store_true", help="node state only (no API access)")
    co = sub.add_parser("collectives", help="RCCL collective sweep (run under torch.distributed.run)")
    co.add_argument("--min-bytes", type=int, default=8)
    co.add_argument("--max-bytes", type=int, default=1 << 30)
    co.add_argument("--factor", type=int, default=4)
    co.add_argument("--ops", default="allreduce,allgather,reducescatter")
    co.add_argument("--dtype", default="float32", choices=("float32", "bfloat16"))
    co.add_argument("--iters", type=int, default=10)
    co.add_argument("--backend", default=None, help="nccl (RCCL, default with a GPU) or gloo")
    co.add_argument("--json", action="store_true")
    args = ap.parse_args(argv)
    logs.setup(getattr(args, "log_level", "info"))

    if args.cmd == "operator":
        from ..controller.reconciler import ClusterPolicyReconciler

        client = _client(args)
        rec = ClusterPolicyReconciler(client, args.namespace)
        _health_server(args.health_port, rec.metrics)
        # a rollout or pod delete (SIGTERM) ends the reconcile loop and, with
        # leader election, releases the Lease so the standby takes over at once
        stop = _stop_on_signals()
        signal_ready = _ready_signal()  # AMDGPU_READY_FILE: after the first pass (informers live)
        import gc

        # a long-running controller: the import-time heap (pydantic models,
        # the CRD schema) stays out of every later collection
        gc.collect()
        gc.freeze()
        passes = [0]

        def on_result(_res):
            passes[0] += 1
            if passes[0] == 1:
                signal_ready()

        if not args.leader_elect:
            rec.run(stop, resync_s=args.resync, debounce_s=args.debounce, on_result=on_result)
            return 0
        import os
        import socket

        from ..kube.leader import LeaderElector

        identity = os.environ.get("POD_NAME") or f"{socket.gethostname()}_{os.getpid()}"
        elector = LeaderElector(client, args.leader_election_id, args.namespace, identity,
                                lease_s=args.lease_seconds, renew_deadline_s=args.lease_seconds * 2 / 3,
                                retry_period_s=args.lease_seconds / 7.5)
        lost = elector.run(stop, lambda ended: rec.run(ended, resync_s=args.resync, debounce_s=args.debounce,
                                                      on_result=on_result))
        # leadership lost: exit so the Deployment restarts this replica as a standby
        return 1 if lost else 0
    if args.cmd == "cleanup-crd":
        from ..controller.reconciler import cleanup_crd

        print(json.dumps({"crd_deleted": cleanup_crd(_client(args))}))
        return 0
    if args.cmd == "apply-crd":
        from ..helm.crd import crd, driver_crd
        from ..kube.client import apply_object

        client = _client(args)
        out = {c["metadata"]["name"]: apply_object(client, c)[1] for c in (crd(), driver_crd())}
        print(json.dumps({"crds": out}))
        return 0
    if args.cmd == "verify":
        from .verify import main_verify

        return main_verify(_client(args), args.namespace, args.json, args.expect_gpus, args.run_pod,
                           args.pod_image, args.pod_timeout)
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
        if args.real_gpus and args.nodes != 1:
            raise SystemExit("--real-gpus simulates one node (this machine)")
        nodes = [NodeSpec(f"node-{i}", args.gpus, args.partition, sysfs_root="/" if args.real_gpus else None)
                 for i in range(args.nodes)]
        c = SimCluster(d, nodes, fake_gpu=not args.real_gpus, http_api=args.http_api).start()
        try:
            c.install_operator(parse_set_flags(args.set))
            ttr = c.wait_ready(args.timeout)
            rep = verify(c.agent_client, c.namespace, run_pods=args.run_pod)
            print(json.dumps({"time_to_ready_s": round(ttr, 4), "nodes": args.nodes, "http_api": args.http_api,
                              "verify": rep.as_dict()}, indent=1))
            return 0 if rep.ok else 1
        finally:
            c.stop()
    if args.cmd == "collectives":
        return _collectives(args)
    if args.cmd == "must-gather":
        from .gather import must_gather

        summary = must_gather(None if args.no_cluster else _client(args), args.namespace, args.output,
                              args.node_root, args.validations_dir)
        print(json.dumps({"output": args.output, "summary": summary}, indent=1))
        return 0
    if args.cmd == "preflight":
        from .preflight import main_preflight

        return main_preflight(args.root, args.fix, args.json, args.expect_gpus, not args.no_gpu)
    return 2


def _collectives(args) -> int:
    import os

    import torch
    import torch.distributed as dist

    from ..parallel import collectives as C

    cuda = torch.cuda.is_available()
    backend = args.backend or ("nccl" if cuda else "gloo")
    if "RANK" not in os.environ:  # single process: world of one
        os.environ.update(RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=os.environ.get(
            "MASTER_PORT", "29531"))
    local = int(os.environ.get("LOCAL_RANK", os.environ["RANK"]))
    device = torch.device("cuda", local) if backend == "nccl" else torch.device("cpu")
    if backend == "nccl":
        torch.cuda.set_device(device)
    dist.init_process_group(backend, device_id=device if backend == "nccl" else None)
    try:
        rows = C.sweep(C.default_sizes(args.min_bytes, args.max_bytes, args.factor), tuple(args.ops.split(",")),
                       getattr(torch, args.dtype), device, iters=args.iters)
        if dist.get_rank() == 0:
            print(json.dumps(C.rows_as_dicts(rows)) if args.json else C.format_table(rows))
        return 0 if all(r.ok for r in rows) else 1
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
