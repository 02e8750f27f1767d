"""Per-node environment shared by the operands (host paths, API client).

In a real cluster every operand container builds this from its environment
(``NODE_NAME``, ``OPERATOR_NAMESPACE``) and the host paths mounted by its
DaemonSet (``controller/manifests.py``).  The simulated cluster
(``testing/simcluster.py``) builds one per simulated node pointing at
temporary directories, so the operand code paths are identical.
"""

from __future__ import annotations

import json
import os
import subprocess
import threading
import time
from .utils.record import field, record
from typing import Callable

from . import DEFAULT_NAMESPACE


@record
class ProcResult:
    rc: int
    stdout: str
    stderr: str
    seconds: float


# In a child's environment: its result is final once it has printed its JSON
# report and closed stdout/stderr (amdgpu-validator does), so the caller need
# not wait for the process exit - the kernel's teardown of a GPU process
# (KFD queues, VM, device memory) then runs off the time-to-Ready path.
REPORT_EARLY_ENV = "AMDGPU_REPORT_EARLY"


def report_rc(stdout: str) -> int:
    """Exit status implied by the last stdout line (a JSON report with ``ok``)."""
    lines = stdout.strip().splitlines()
    try:
        return 0 if lines and json.loads(lines[-1]).get("ok") is True else 1
    except ValueError:
        return 1


class PipeReader:
    """Drain a child's stdout and stderr on two threads (no pipe can fill up)."""

    def __init__(self, proc: subprocess.Popen):
        self.proc = proc
        self._out: list[str] = []
        self._err: list[str] = []
        self._threads = [threading.Thread(target=lambda: self._out.append(proc.stdout.read()), daemon=True),
                         threading.Thread(target=lambda: self._err.append(proc.stderr.read()), daemon=True)]
        for th in self._threads:
            th.start()

    def eof(self) -> bool:
        return not any(th.is_alive() for th in self._threads)

    def join(self, timeout: float | None) -> bool:
        deadline = None if timeout is None else time.monotonic() + timeout
        for th in self._threads:
            th.join(None if deadline is None else max(0.0, deadline - time.monotonic()))
        return self.eof()

    def text(self) -> tuple[str, str]:
        return "".join(self._out), "".join(self._err)

    def result(self, t0: float) -> ProcResult:
        """At EOF: the exit status if the child is gone, else the report's
        verdict (a reaper thread collects the exit later)."""
        out, err = self.text()
        rc = self.proc.poll()
        if rc is None:
            rc = report_rc(out)
            threading.Thread(target=self.proc.wait, daemon=True).start()
        return ProcResult(rc, out, err, time.perf_counter() - t0)


def run_local(argv: list[str], env: dict | None = None, timeout: float = 300.0) -> ProcResult:
    """Run a native tool as a child process (never exec in-process)."""
    t0 = time.perf_counter()
    full_env = dict(os.environ)
    full_env.update(env or {})
    if full_env.get(REPORT_EARLY_ENV) == "1":
        p = subprocess.Popen(argv, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=full_env)
        reader = PipeReader(p)
        if not reader.join(timeout):
            p.kill()
            reader.join(5)
            try:
                p.wait(5)
            except subprocess.TimeoutExpired:
                pass
            out, err = reader.text()
            return ProcResult(124, out, err + "\ntimeout", time.perf_counter() - t0)
        return reader.result(t0)
    try:
        p = subprocess.run(argv, capture_output=True, text=True, env=full_env, timeout=timeout)
        return ProcResult(p.returncode, p.stdout, p.stderr, time.perf_counter() - t0)
    except subprocess.TimeoutExpired as e:
        return ProcResult(124, e.stdout or "", (e.stderr or "") + "\ntimeout", time.perf_counter() - t0)


@record
class NodeEnv:
    node_name: str
    client: object
    host_root: str = "/"                      # sysfs/devfs root the topology library reads
    validations_dir: str = "/run/amd/validations"
    device_plugin_dir: str = "/var/lib/kubelet/device-plugins"
    pod_resources_socket: str = "/var/lib/kubelet/pod-resources/kubelet.sock"
    cdi_dir: str = "/var/run/cdi"
    containerd_config: str = "/etc/containerd/config.toml"
    crio_config_dir: str = "/etc/crio/crio.conf.d"
    docker_config: str = "/etc/docker/daemon.json"
    install_dir: str = "/usr/local/amd"
    namespace: str = DEFAULT_NAMESPACE
    poll_s: float = 1.0
    # how GPU processes are started: (argv, env, device_index or None) -> ProcResult.
    # The bench routes device d to the torch.distributed rank that owns GPU d.
    launcher: Callable[..., ProcResult] | None = None
    extra: dict = field(default_factory=dict)

    @classmethod
    def from_environ(cls, client) -> "NodeEnv":
        e = os.environ
        return cls(
            node_name=e.get("NODE_NAME", os.uname().nodename),
            client=client,
            host_root=e.get("HOST_ROOT", "/host" if os.path.isdir("/host/sys") else "/"),
            validations_dir=e.get("VALIDATIONS_DIR", "/run/amd/validations"),
            device_plugin_dir=e.get("DEVICE_PLUGIN_DIR", "/var/lib/kubelet/device-plugins"),
            pod_resources_socket=e.get("POD_RESOURCES_SOCKET", "/var/lib/kubelet/pod-resources/kubelet.sock"),
            cdi_dir=e.get("CDI_SPEC_DIR", "/var/run/cdi"),
            containerd_config=e.get("CONTAINERD_CONFIG", "/etc/containerd/config.toml"),
            crio_config_dir=e.get("CRIO_CONFIG_DIR", "/etc/crio/crio.conf.d"),
            docker_config=e.get("DOCKER_CONFIG", "/etc/docker/daemon.json"),
            install_dir=e.get("INSTALL_DIR", "/usr/local/amd"),
            namespace=e.get("OPERATOR_NAMESPACE", DEFAULT_NAMESPACE),
            poll_s=float(e.get("VALIDATION_POLL_S", "1.0")),
        )

    def waits(self, first_s: float = 0.002, factor: float = 1.5, cap_s: float = 0.02):
        """Sleep lengths for polling a cheap local condition that no event
        announces (the driver's sysfs, the kubelet's device list): start at
        ``first_s`` and grow to ``min(cap_s, poll_s)``.  One check costs ~0.1
        ms, so the 20 ms cap keeps a long wait at 0.5% of a core while a
        condition is seen within 20 ms of turning true.  (Ready files are
        waited for with inotify: utils/fswait.py.)"""
        cap = min(cap_s, self.poll_s)
        d = min(first_s, cap)
        while True:
            yield d
            d = min(cap, d * factor)

    def validation_file(self, name: str) -> str:
        return os.path.join(self.validations_dir, name)

    def sysfs_root(self) -> str:
        """Root for the topology library (host sysfs is mounted at /host/sys)."""
        return self.host_root

    def launch(self, argv: list[str], env: dict | None = None, device: int | None = None,
               timeout: float = 300.0) -> ProcResult:
        if self.launcher is not None:
            return self.launcher(argv, env or {}, device, timeout)
        return run_local(argv, env, timeout)
