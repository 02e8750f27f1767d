"""Driver DaemonSet logic (``amd-driver-daemonset``: ``amd-driver-ctr`` +
``amd-driver-health``, init ``amd-driver-manager``).

Reference parity: the driver DaemonSet "installs the NVIDIA driver on the
node" (/root/reference/README.md:212); its pods run ``2/2`` containers
(README.md:138-139) and the driver container ships the SMI tool
(README.md:152).  On MI355X:

* ``install``  - build/load the amdgpu DKMS module and ROCm userspace for
  gfx950 (``deploy/images/amd-driver/install.sh`` inside the image), then wait
  for the N1 probe (``/dev/kfd``, KFD GPU nodes, render nodes) and write
  ``driver-ready``.  Where the module is already live (preinstalled host
  driver, or the simulated node) the install step is a verification.
* ``monitor``  - the second container: re-probes periodically and removes
  ``driver-ready`` when the driver disappears (driver crash / unload), so the
  dependent operands re-gate.
* ``prepare-upgrade`` - init container: when the loaded driver differs from
  the requested version, evict GPU pods from the node (drain) and clear the
  validation files before the new driver is installed.
* ``smi``      - ``amd-smi``-style device table inside ``amd-driver-ctr``
  (the ``kubectl exec ... nvidia-smi`` check of README.md:152).
"""

from __future__ import annotations

import os
import subprocess
import threading
import time

from ..nodeenv import NodeEnv
from ..utils.logs import get_logger
from ..validator.validate import READY_FILES, clear_ready, write_ready

log = get_logger("amdgpu.driver")
INSTALL_SCRIPT = "/usr/local/bin/amd-driver-install.sh"


def loaded_version(env: NodeEnv) -> str:
    try:
        with open(os.path.join(env.sysfs_root(), "sys/module/amdgpu/version")) as f:
            return f.read().strip()
    except OSError:
        return ""


def install(env: NodeEnv, timeout: float = 600.0, stop: threading.Event | None = None) -> dict:
    from ..discovery import topology

    t0 = time.perf_counter()
    ran_script = False
    if os.path.exists(INSTALL_SCRIPT) and os.access(INSTALL_SCRIPT, os.X_OK):
        ok, _ = topology.probe(env.sysfs_root())
        if not ok:
            subprocess.run([INSTALL_SCRIPT], check=True, timeout=timeout)
            ran_script = True
    deadline = time.monotonic() + timeout
    while True:
        ok, msg = topology.probe(env.sysfs_root())
        if ok:
            break
        if time.monotonic() >= deadline:
            raise RuntimeError(f"driver did not come up: {msg}")
        if (stop.wait(env.poll_s) if stop is not None else (time.sleep(env.poll_s) or False)):
            raise RuntimeError("stopped")
    gpus = topology.enumerate_gpus(env.sysfs_root())
    out = {"ok": True, "message": msg, "gpus": len(gpus), "driver_version": loaded_version(env),
           "installed": ran_script, "seconds": time.perf_counter() - t0}
    write_ready(env, "driver", out)
    return out


def monitor_once(env: NodeEnv) -> bool:
    from ..discovery import topology

    ok, msg = topology.probe(env.sysfs_root())
    path = env.validation_file(READY_FILES["driver"])
    if not ok and os.path.exists(path):
        log.error("driver lost: %s", msg)
        clear_ready(env, ("driver", "toolkit", "workload", "plugin", "complete"))
    return ok


def monitor(env: NodeEnv, stop: threading.Event, interval: float = 10.0) -> None:
    while not stop.wait(interval):
        monitor_once(env)


def prepare_upgrade(env: NodeEnv, desired_version: str, drain: bool = True) -> dict:
    cur = loaded_version(env)
    if not cur or not desired_version or cur == desired_version:
        return {"upgrade": False, "loaded": cur}
    from ..partition.manager import evict_gpu_pods

    evicted = evict_gpu_pods(env) if drain else []
    clear_ready(env, ("driver", "toolkit", "workload", "plugin", "complete"))
    return {"upgrade": True, "loaded": cur, "desired": desired_version, "evicted": evicted}


def smi_table(env: NodeEnv) -> str:
    """Human table like ``amd-smi``/``nvidia-smi`` (README.md:157-167)."""
    from ..discovery import topology

    gpus = topology.enumerate_gpus(env.sysfs_root())
    metrics = {}
    try:
        with topology.Smi() as smi:
            metrics = {m.bdf: m.values for m in smi.collect()}
    except Exception:  # noqa: BLE001 - table without live metrics
        pass
    lines = [f"amd-gpu-operator driver {loaded_version(env) or 'unknown'}",
             "+-----+--------------+--------+-----+-----------+-----------------+---------+-------+",
             "| GPU | BDF          | Arch   | CUs | Partition | HBM used/total  | Power W | Temp C|",
             "+-----+--------------+--------+-----+-----------+-----------------+---------+-------+"]
    for g in gpus:
        m = metrics.get(g.bdf, {})
        used = m.get("vram_used_bytes", 0) / 2**20
        total = m.get("vram_total_bytes", g.vram_bytes) / 2**20
        lines.append(f"| {g.index:3d} | {g.bdf:12s} | {g.arch:6s} | {g.cu_count:3d} | "
                     f"{(g.compute_partition or 'SPX') + '/' + (g.memory_partition or 'NPS1'):9s} | "
                     f"{used:6.0f}/{total:6.0f}MiB | {m.get('socket_power_w', 0):7.0f} | {m.get('temp_hotspot_c', 0):5.0f} |")
    lines.append("+-----+--------------+--------+-----+-----------+-----------------+---------+-------+")
    return "\n".join(lines)
