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
  the requested version or driver spec, evict GPU pods from the node (drain),
  clear the validation files and unload the old module before the new driver
  is installed.
* ``smi``      - ``amd-smi``-style device table inside ``amd-driver-ctr``
  (the ``kubectl exec ... nvidia-smi`` check of README.md:152).
"""

from __future__ import annotations

import json
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
    """``/sys/module/amdgpu/version``; empty for an inbox / built-in module."""
    try:
        with open(os.path.join(env.sysfs_root(), "sys/module/amdgpu/version")) as f:
            return f.read().strip()
    except OSError:
        return ""


class HostModule:
    """The node's real amdgpu module: ``install.sh`` of the driver image and
    ``modprobe -r``.  The simulated cluster substitutes
    :class:`~amdgpu_operator.testing.fakesys.SimModule` (``env.extra["kmod"]``)."""

    def __init__(self, script: str | None = None):
        self.script = script or INSTALL_SCRIPT

    def can_install(self) -> bool:
        return os.path.exists(self.script) and os.access(self.script, os.X_OK)

    def install(self, env: NodeEnv, cenv: dict, timeout: float) -> None:
        subprocess.run([self.script], check=True, timeout=timeout, env={**os.environ, **cenv})

    def load(self, env: NodeEnv, timeout: float = 120.0) -> None:
        """Load the module the host provides (no installer in this image)."""
        subprocess.run(["modprobe", "amdgpu"], check=True, timeout=timeout, capture_output=True)

    def load_rdma(self, env: NodeEnv, timeout: float = 120.0) -> None:
        """The RDMA core for GPU peer memory (driver.rdma): ``ib_uverbs``
        brings ``ib_core``; the NIC's own driver comes with the host stack."""
        subprocess.run(["modprobe", "ib_uverbs"], check=True, timeout=timeout, capture_output=True)

    def unload(self, env: NodeEnv, timeout: float = 120.0, retry_s: float = 5.0) -> None:
        # a process that just exited may still be releasing its device files
        deadline = time.monotonic() + retry_s
        while True:
            p = subprocess.run(["modprobe", "-r", "amdgpu"], capture_output=True, text=True, timeout=timeout)
            if p.returncode == 0:
                return
            if time.monotonic() >= deadline:
                raise RuntimeError(f"modprobe -r amdgpu failed ({p.returncode}): {p.stderr.strip()}")
            time.sleep(0.5)


def _kmod(env: NodeEnv):
    return env.extra.get("kmod") or HostModule(INSTALL_SCRIPT)


def _state_path(env: NodeEnv) -> str:
    """What the operator last installed on this node (``/run/amd/driver-state.json``:
    survives driver pod restarts, not reboots - like the loaded module)."""
    return os.path.join(os.path.dirname(env.validations_dir.rstrip("/")), "driver-state.json")


def read_state(env: NodeEnv) -> dict:
    try:
        with open(_state_path(env)) as f:
            return json.load(f)
    except (OSError, ValueError):
        return {}


def _write_state(env: NodeEnv, state: dict | None) -> None:
    path = _state_path(env)
    if state is None:
        try:
            os.unlink(path)
        except FileNotFoundError:
            pass
        return
    os.makedirs(os.path.dirname(path), exist_ok=True)
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        json.dump(state, f)
    os.replace(tmp, path)


def outdated(env: NodeEnv, desired_version: str, spec_hash: str = "") -> str:
    """Why the live module does not satisfy the requested driver ("" = it does).

    A module that reports a version must report the requested one; one the
    operator installed must have been installed for the current driver spec
    (module parameters, image and ROCm release are in the hash, not in the
    module version).  An inbox / built-in module reports no version: it is
    replaced only when the image can install one (see :func:`install`)."""
    cur = loaded_version(env)
    if desired_version and cur and cur != desired_version:
        return f"loaded {cur}, requested {desired_version}"
    rec = read_state(env).get("specHash", "")
    if spec_hash and rec and rec != spec_hash:
        return f"loaded for driver spec {rec}, current spec {spec_hash}"
    return ""


def _release_gated_validators(env: NodeEnv, timeout: float = 5.0) -> list[str]:
    """Validator processes waiting at their start gate may hold /dev/kfd
    (validator/validate.py prespawn_safe; with an "init" verdict their HIP
    runtime is starting): abort them before the module goes, and wait until
    they are gone - each holds ``<gate>.held`` locked for its lifetime (the
    native validator, validator_main.cpp) - and until the kernel has torn
    down their GPU state (:func:`wait_kfd_settled`).  Returns the gates that
    were aborted."""
    from ..validator.validate import abort_start_gates

    aborted = abort_start_gates(env)
    if not aborted:
        return aborted
    t0 = time.monotonic()
    deadline = t0 + timeout
    left = [g for g in aborted if not _wait_unlocked(env.validation_file(g) + ".held", deadline)]
    settled = wait_kfd_settled(env, deadline)
    log.info("aborted %d validator start gate(s) before the driver change: gone after %.3f s%s%s", len(aborted),
             time.monotonic() - t0, f", {len(left)} still running" if left else "",
             "" if settled else ", KFD teardown still under way")
    return aborted


def _wait_unlocked(path: str, deadline: float) -> bool:
    """Until nobody holds ``path`` flock-ed (its holder exited) or ``deadline``
    (monotonic); a missing file has no holder."""
    import fcntl

    try:
        fd = os.open(path, os.O_RDONLY | os.O_CLOEXEC)
    except FileNotFoundError:
        return True
    try:
        while True:
            try:
                fcntl.flock(fd, fcntl.LOCK_EX | fcntl.LOCK_NB)
                fcntl.flock(fd, fcntl.LOCK_UN)
                return True
            except BlockingIOError:
                if time.monotonic() >= deadline:
                    return False
                time.sleep(0.001)
    finally:
        os.close(fd)


def wait_kfd_settled(env: NodeEnv, deadline: float) -> bool:
    """Until no exited process still has KFD state (a ``kfd/proc/<pid>`` entry
    whose PID is gone from /proc: the kernel's teardown of it is under way,
    and the module counts it as a user) or ``deadline``.  The driver
    container runs in the host PID namespace, where both lists name the same
    PIDs."""
    proc = os.path.join(env.sysfs_root(), "proc")
    while True:
        stale = [p for p in kfd_users(env) if not os.path.exists(os.path.join(proc, p))]
        if not stale:
            return True
        if time.monotonic() >= deadline:
            return False
        time.sleep(0.002)


def install(env: NodeEnv, timeout: float = 600.0, stop: threading.Event | None = None,
            cenv: dict | None = None) -> dict:
    """``amd-driver-ctr``: make the requested driver live, then publish it.

    ``cenv`` is the container environment of the driver spec
    (``AMDGPU_DRIVER_VERSION``, ``AMDGPU_DRIVER_SPEC_HASH``, module params ...).
    The install script runs when the module is not live, or when the live one
    is not the requested one (it unloads it first).  Without an installer
    (preinstalled host driver) a live module is accepted as host-managed, but
    a live module of another version fails loudly.  After the module is up
    the loaded version is checked against the request, recorded on the host
    and published as node annotations for the upgrade controller."""
    from ..wellknown import LOADED_HASH_ANN, LOADED_VERSION_ANN
    from ..discovery import topology

    cenv = dict(cenv or {})
    want = cenv.get("AMDGPU_DRIVER_VERSION", "")
    spec_hash = cenv.get("AMDGPU_DRIVER_SPEC_HASH", "")
    kmod = _kmod(env)
    t0 = time.perf_counter()
    ran_script = False
    live, _ = topology.probe(env.sysfs_root())
    why = "" if not live else outdated(env, want, spec_hash)
    if not live or why:
        if kmod.can_install():
            if why:
                log.info("replacing the live driver: %s", why)
                cenv["AMDGPU_FORCE_RELOAD"] = "true"
            if live:
                _release_gated_validators(env)
            kmod.install(env, cenv, timeout)
            ran_script = True
        elif why:
            raise RuntimeError(f"driver mismatch and no installer in this image: {why}")
    deadline = time.monotonic() + timeout
    for delay in env.waits():
        ok, msg = topology.probe(env.sysfs_root())
        if ok:
            break
        if time.monotonic() >= deadline:
            raise RuntimeError(f"driver did not come up: {msg}")
        if (stop.wait(delay) if stop is not None else (time.sleep(delay) or False)):
            raise RuntimeError("stopped")
    cur = loaded_version(env)
    if ran_script and want and cur != want:
        raise RuntimeError(f"installed driver reports version {cur or 'none'}, requested {want}")
    rdma = None
    if cenv.get("AMDGPU_RDMA_ENABLED") == "true":
        rdma = ensure_rdma(env, kmod, cenv.get("AMDGPU_RDMA_USE_HOST_MOFED") == "true", deadline, stop)
    # a restarted driver pod finds the module its predecessor installed: it stays ours
    prev = read_state(env)
    installed = ran_script or bool(prev.get("installed") and prev.get("version") == cur and live)
    host_managed = not installed and not cur
    # this pod now owns the module: a predecessor still shutting down (a
    # force-deleted pod whose container outlives its API object) must not
    # unload it from under us (cleanup_on_exit)
    _write_state(env, {"version": cur, "specHash": spec_hash, "installed": installed, "hostManaged": host_managed,
                       "owner": owner_id(cenv), "ts": round(time.time(), 3)})
    gpus = topology.enumerate_gpus(env.sysfs_root())
    out = {"ok": True, "message": msg, "gpus": len(gpus), "driver_version": cur, "installed": ran_script,
           "host_managed": host_managed, "seconds": time.perf_counter() - t0}
    if rdma is not None:
        out["rdma"] = rdma
    write_ready(env, "driver", out)  # the node's operands wait on this file, not on the annotation below
    try:  # for the upgrade controller (the loaded version / spec it compares with the policy)
        env.client.patch("v1", "Node", env.node_name, {"metadata": {"annotations": {
            LOADED_VERSION_ANN: cur or "host", LOADED_HASH_ANN: spec_hash or None}}})
    except Exception as e:  # noqa: BLE001 - the upgrade controller re-reads it on its next pass
        log.warning("could not annotate node %s: %s", env.node_name, e)
    # The module went away since the node was last validated (lost, or
    # unloaded by a driver container's exit): what the validator and the
    # device plugin hold belongs to the old driver instance - their pods
    # (waiting in stop, or serving stale device handles) are restarted, so the
    # node is validated and advertised afresh on this driver.
    if _claim_lost_marker(env):
        out["restarted"] = _restart_node_operands(env)
        log.info("driver back after a loss/unload; restarted %s", out["restarted"])
    return out


def ensure_rdma(env: NodeEnv, kmod, host_stack: bool, deadline: float, stop: threading.Event | None = None) -> dict:
    """driver.rdma: GPU memory reachable by the node's RDMA NICs before the
    driver is declared ready (upstream: nvidia-peermem after MOFED).  On
    MI355X the path is amdgpu's dma-buf export imported by the RDMA core, so
    this needs the core loaded - by the host's MOFED / inbox stack
    (``useHostMofed``: waited for) or here (``modprobe ib_uverbs``) - and a
    kernel whose RDMA core imports dma-bufs.  NICs without an ACTIVE port are
    reported, not waited for: a cable is not the driver's business.  The
    validator's ``dmabuf`` step then exports HBM on the device itself."""
    from ..discovery import rdma

    st = rdma.readiness(env.sysfs_root())
    if not st["dmabuf"]:
        raise RuntimeError(f"driver.rdma: kernel {st['kernel']} cannot hand GPU memory to an RDMA NIC (needs >= 5.12)")
    loaded = False
    for delay in env.waits():
        st = rdma.readiness(env.sysfs_root())
        if all(st["modules"].values()):
            break
        if not host_stack and not loaded:
            kmod.load_rdma(env)
            loaded = True
            continue
        if time.monotonic() >= deadline:
            raise RuntimeError("driver.rdma: RDMA core not loaded: " + "; ".join(st["problems"]))
        if (stop.wait(delay) if stop is not None else (time.sleep(delay) or False)):
            raise RuntimeError("stopped")
    st["loaded_here"] = loaded
    if st["problems"]:
        log.warning("driver.rdma: %s", "; ".join(st["problems"]))
    return st


def _claim_lost_marker(env: NodeEnv) -> bool:
    """Take the loss marker (True for exactly one of the driver container and
    its health monitor, whichever sees the driver back first)."""
    marker = env.validation_file(LOST_MARKER)
    claimed = f"{marker}.claimed.{os.getpid()}.{threading.get_ident()}"
    try:
        os.replace(marker, claimed)
    except FileNotFoundError:
        return False
    os.unlink(claimed)
    return True


def _withdraw_validation(env: NodeEnv, reason: str) -> None:
    """The node's validation no longer holds: remember why (the loss marker,
    :func:`_claim_lost_marker`), drop every ready file and the node's
    ``amd.com/gpu.validated`` labels."""
    from ..validator.validate import MFMA_LABEL, MFMA_RATE_LABEL, VALIDATED_LABEL

    os.makedirs(env.validations_dir, exist_ok=True)
    tmp = env.validation_file(f"{LOST_MARKER}.tmp.{os.getpid()}.{threading.get_ident()}")
    with open(tmp, "w") as f:
        f.write(reason)
    os.replace(tmp, env.validation_file(LOST_MARKER))
    clear_ready(env, ("driver", "toolkit", "workload", "plugin", "complete"))
    if env.client is not None:
        try:
            env.client.patch("v1", "Node", env.node_name, {"metadata": {"labels": {
                VALIDATED_LABEL: None, MFMA_LABEL: None, MFMA_RATE_LABEL: None}}})
        except Exception as e:  # noqa: BLE001
            log.warning("could not withdraw %s: %s", VALIDATED_LABEL, e)


RELOAD_REQUEST = ".driver-reload-request"  # partition/manager.py: a memory-partition change needs a reload


def reload_module(env: NodeEnv, cenv: dict, reason: str, timeout: float = 600.0, stop=None) -> dict:
    """Unload and load amdgpu again (a memory-partition change takes effect
    only at the module load).  The validations go first - the health monitor
    must not read the planned unload as a loss - and pending validator gates
    are aborted; then the module is loaded the way this container loads it:
    its install script (container-installed) or ``modprobe amdgpu`` (host
    module), and ``driver-ready`` is written again by :func:`install`."""
    kmod = _kmod(env)
    _release_gated_validators(env)
    # withdrawn like a loss, marker included: if the unload or the load fails
    # half-way, the health monitor (monitor_once) restores driver-ready as soon
    # as a module is live again - the old one that would not unload, or a later
    # load - and restarts the validator and device plugin on it; a successful
    # reload takes the marker in install()
    _withdraw_validation(env, f"planned reload: {reason}")
    log.info("reloading amdgpu: %s", reason)
    try:
        kmod.unload(env)
        if kmod.can_install():
            kmod.install(env, {**cenv, "AMDGPU_FORCE_RELOAD": "true"}, timeout)
        else:
            kmod.load(env, timeout)
    except Exception:
        monitor_once(env)  # the module still (or again) live: the node keeps its driver-ready
        raise
    return install(env, timeout, stop, cenv)


def serve_reload_requests(env: NodeEnv, stop: threading.Event, cenv: dict) -> None:
    """``amd-driver-ctr`` after its install: the node's module owner, it
    performs the reloads other node agents ask for (``.driver-reload-request``)
    until the container stops."""
    from ..utils.fswait import wait_for_file

    req = env.validation_file(RELOAD_REQUEST)
    while not stop.is_set():
        if not wait_for_file(req, 3600.0, stop, max(env.poll_s, 0.05)):
            continue
        try:
            with open(req) as f:
                reason = json.load(f).get("reason", "requested")
        except (OSError, ValueError):
            reason = "requested"
        try:
            reload_module(env, cenv, reason, stop=stop)
        except Exception as e:  # noqa: BLE001 - the requester times out and reports the failure
            log.error("driver reload failed: %s", e)
        finally:
            try:
                os.unlink(req)
            except FileNotFoundError:
                pass


def kfd_users(env: NodeEnv) -> list[str]:
    """PIDs with the GPU open (``/sys/class/kfd/kfd/proc/<pid>``)."""
    try:
        return sorted(p for p in os.listdir(os.path.join(env.sysfs_root(), "sys/class/kfd/kfd/proc")) if p.isdigit())
    except OSError:
        return []


def owner_id(cenv: dict) -> str:
    """The driver pod instance (downward API ``POD_UID``, else ``POD_NAME``)."""
    return cenv.get("POD_UID") or cenv.get("POD_NAME") or ""


def cleanup_on_exit(env: NodeEnv, owner: str = "") -> dict:
    """``amd-driver-ctr`` stopped (SIGTERM: helm uninstall, driver disabled, node
    left the GPU pool): unload the module this container installed, like the
    upstream driver container's shutdown.  A host-managed or inbox module is
    left alone, and so is one that still has GPU users (logged: the next driver
    pod's ``prepare-upgrade`` handles a version change after the drain)."""
    st = read_state(env)
    if not st.get("installed"):
        return {"unloaded": False, "reason": "module not installed by the driver container"}
    if owner and st.get("owner") and st["owner"] != owner:
        log.info("driver stays loaded: taken over by driver pod %s", st["owner"])
        return {"unloaded": False, "reason": f"taken over by {st['owner']}"}
    users = kfd_users(env)
    if users:
        log.warning("driver stays loaded: GPU in use by %d process(es) %s", len(users), users[:8])
        return {"unloaded": False, "reason": f"in use by {users[:8]}"}
    _release_gated_validators(env)
    # as for a lost driver: the node is unvalidated from here on, and the next
    # driver pod's install restarts the validator and device plugin
    _withdraw_validation(env, "amdgpu unloaded on driver container exit")
    try:
        _kmod(env).unload(env)
    except Exception as e:  # noqa: BLE001 - leave it loaded, say why
        log.warning("driver unload on exit failed: %s", e)
        return {"unloaded": False, "reason": str(e)}
    _write_state(env, None)
    log.info("amdgpu unloaded on driver container exit")
    return {"unloaded": True}


LOST_MARKER = ".driver-lost"
# operands that hold per-driver-instance state: restarted once the driver is back
RESTART_ON_RECOVERY = ("amd-operator-validator", "amd-device-plugin-daemonset")


def _restart_node_operands(env: NodeEnv, apps=RESTART_ON_RECOVERY) -> list[str]:
    out = []
    if env.client is None:
        return out
    for app in apps:
        try:
            pods = env.client.list("v1", "Pod", env.namespace, label_selector=f"app={app}",
                                   field_selector=f"spec.nodeName={env.node_name}")
            for pod in pods:
                env.client.delete("v1", "Pod", pod["metadata"]["name"], env.namespace)
                out.append(pod["metadata"]["name"])
        except Exception as e:  # noqa: BLE001 - next monitor pass retries nothing; log it
            log.warning("could not restart %s on %s: %s", app, env.node_name, e)
    return out


def monitor_once(env: NodeEnv) -> bool:
    """``amd-driver-health``: one pass of the driver watch.

    Driver lost (probe fails while ``driver-ready`` stands): every validation
    is withdrawn, the node's ``amd.com/gpu.validated`` label with it, and the
    loss is remembered.  Driver back after a loss: ``driver-ready`` is written
    again (the toolkit reinstalls on it) and the validator and device-plugin
    pods of this node are restarted, so the GPUs are validated and advertised
    afresh; until then the ClusterPolicy reports the node not validated."""
    from ..discovery import topology

    t_probe = time.time()
    ok, msg = topology.probe(env.sysfs_root())
    path = env.validation_file(READY_FILES["driver"])
    marker = env.validation_file(LOST_MARKER)
    try:
        fresh = os.stat(path).st_mtime >= t_probe
    except FileNotFoundError:
        fresh = False
    if not ok and os.path.exists(path) and not fresh:
        # (a driver-ready written since this probe began is a reload that
        # finished meanwhile, not the loss the probe saw: withdrawing it would
        # leave the node unvalidated on a live module)
        log.error("driver lost: %s", msg)
        _withdraw_validation(env, msg)
    elif ok and os.path.exists(marker) and not os.path.exists(path):
        gpus = topology.enumerate_gpus(env.sysfs_root())
        write_ready(env, "driver", {"ok": True, "message": msg, "gpus": len(gpus), "recovered": True,
                                    "driver_version": loaded_version(env), "seconds": 0.0})
        if _claim_lost_marker(env):
            restarted = _restart_node_operands(env)
            log.info("driver back (%s); restarted %s", msg, restarted)
    publish_smi(env, ok and os.path.exists(path))
    return ok


def monitor(env: NodeEnv, stop: threading.Event, interval: float = 10.0) -> None:
    """Watch the driver every ``interval``; while it is lost, every second
    (the node is unvalidated until the driver is seen again).  A change in
    the validations directory (a loss marker another agent wrote, a ready
    file withdrawn) triggers a pass at once."""
    from ..utils.fswait import DirWatch

    lost = env.validation_file(LOST_MARKER)
    os.makedirs(env.validations_dir, exist_ok=True)
    w = DirWatch(env.validations_dir)
    try:
        monitor_once(env)
        while not stop.is_set():
            period = min(interval, 1.0) if os.path.exists(lost) else interval
            deadline = time.monotonic() + period
            while not stop.is_set() and time.monotonic() < deadline:
                if w.active:
                    if w.wait(min(0.25, max(0.0, deadline - time.monotonic()))):
                        break  # something changed: look now
                elif stop.wait(min(0.25, max(0.0, deadline - time.monotonic()))):
                    break
            if stop.is_set():
                return
            monitor_once(env)
    finally:
        w.close()


def prepare_upgrade(env: NodeEnv, desired_version: str, drain: bool = True, spec_hash: str = "",
                    drain_timeout: float = 300.0) -> dict:
    """``amd-driver-manager`` init container of a (new) driver pod.

    When the live module is not the requested one (version, or the driver
    spec it was installed for), GPU pods are evicted, the validations are
    cleared and the old module is unloaded, so ``amd-driver-ctr`` installs
    the new one.  An unload failure raises: the init container fails and the
    kubelet retries it, instead of the node passing as upgraded with the old
    module still loaded."""
    from ..discovery import topology

    cur = loaded_version(env)
    live, _ = topology.probe(env.sysfs_root())
    why = outdated(env, desired_version, spec_hash) if live else ""
    if not why:
        return {"upgrade": False, "loaded": cur}
    kmod = _kmod(env)
    if not kmod.can_install():
        raise RuntimeError(f"driver upgrade needed ({why}) but this image has no installer")
    from ..partition.manager import evict_gpu_pods, wait_gpu_pods_gone

    log.info("driver upgrade: %s", why)
    evicted = evict_gpu_pods(env) if drain else []
    clear_ready(env, ("driver", "toolkit", "workload", "plugin", "complete"))
    if not wait_gpu_pods_gone(env, drain_timeout):
        log.warning("GPU pods still on the node after %.0f s; unloading anyway", drain_timeout)
    _release_gated_validators(env)
    kmod.unload(env)
    _write_state(env, None)
    still, _ = topology.probe(env.sysfs_root())
    if still:
        raise RuntimeError("amdgpu still live after unload")
    return {"upgrade": True, "loaded": cur, "desired": desired_version, "reason": why, "evicted": evicted,
            "unloaded": True}


def smi_snapshot(env: NodeEnv) -> dict:
    """What ``amd-smi`` shows from inside the driver image: per-GPU live
    metrics (power, temperature, HBM use) through the image's libamd_smi; on
    a simulated node without a GPU the captured MI355X metrics
    (``env.extra["metrics_fixture"]``).  ``ok`` only when every physical GPU
    reports live power and temperature; otherwise ``error`` says why."""
    from ..discovery import topology

    gpus = topology.enumerate_gpus(env.sysfs_root())
    snap = {"source": "amd-smi", "error": "", "version": "", "metrics": {}}
    try:
        with topology.Smi() as smi:
            snap["metrics"] = {m.bdf: m.values for m in smi.collect()}
            snap["version"] = smi.driver_version()
    except Exception as e:  # noqa: BLE001 - reported, never a zero reading
        snap["error"] = f"amd-smi unavailable: {e}"
        fx = env.extra.get("metrics_fixture")
        if fx:
            from ..exporter.metrics import FixtureSource

            samples = FixtureSource(fx).collect()  # captured on one MI355X: every simulated GPU reads it
            if samples:
                snap.update(source="fixture", error="",
                            metrics={g.bdf: samples[i % len(samples)].values for i, g in enumerate(gpus)})
    live = [b for b, v in snap["metrics"].items() if "socket_power_w" in v and "temp_hotspot_c" in v]
    physical = len({g.physical_index for g in gpus})
    snap.update(gpus=len(gpus), physical=physical, live=len(live))
    if not snap["error"] and (physical == 0 or len(live) < physical):
        snap["error"] = f"live power/temperature for {len(live)} of {physical} GPUs"
    snap["ok"] = not snap["error"]
    return snap


def smi_status(snap: dict) -> str:
    """One-line form for the node annotation ``verify`` reads."""
    if snap["ok"]:
        return f"ok: {snap['live']}/{snap['physical']} GPUs live ({snap['source']})"
    return f"error: {snap['error']}"[:250]


def publish_smi(env: NodeEnv, driver_ok: bool, refresh_s: float = 60.0) -> str:
    """``amd-driver-health``: keep ``amd.com/gpu.driver-smi`` on the Node
    current - the machine-checked form of ``kubectl exec ... -c
    amd-driver-ctr -- nvidia-smi`` (README.md:152).  amd-smi is asked again
    when the driver comes back and every ``refresh_s``; the Node is patched
    only when the status line changes."""
    from ..wellknown import DRIVER_SMI_ANN

    from ..utils import smihold

    last, at = env.extra.get("_smi_published", ("", 0.0))
    now = time.monotonic()
    if not driver_ok:
        status = "error: driver not live"
    elif last.startswith("ok") and now - at < refresh_s:
        return last
    else:
        # a partition change holds the node's amd-smi clients off (utils/smihold.py):
        # this poll is skipped, not raced against the apply
        with smihold.client(env.validations_dir) as allowed:
            if not allowed:
                return last
            status = smi_status(smi_snapshot(env))
    if status != last and env.client is not None:
        try:
            env.client.patch("v1", "Node", env.node_name, {"metadata": {"annotations": {DRIVER_SMI_ANN: status}}})
        except Exception as e:  # noqa: BLE001 - next pass retries
            log.warning("could not publish amd-smi status: %s", e)
            return last
    env.extra["_smi_published"] = (status, now)
    return status


def smi_table(env: NodeEnv, snap: dict | None = None) -> str:
    """Human table like ``amd-smi``/``nvidia-smi`` (README.md:157-167).  A
    GPU amd-smi gives no reading for shows ``n/a``, and the reason is the
    table's last line - never a zero that reads like a measurement."""
    from ..discovery import topology

    gpus = topology.enumerate_gpus(env.sysfs_root())
    snap = snap or smi_snapshot(env)
    metrics = snap["metrics"]
    version = loaded_version(env) or snap["version"]  # inbox/DKMS modules without a sysfs version
    from ..discovery.labels import rocm_version

    rocm = rocm_version(env.sysfs_root())

    def num(m, key, width):
        return f"{m[key]:{width}.0f}" if key in m else "n/a".rjust(width)

    lines = [f"amd-gpu-operator driver {version or 'unknown'}" + (f"   ROCm {rocm}" if rocm else ""),
             "+-----+--------------+--------+-----+-----------+-----------------+---------+-------+",
             "| GPU | BDF          | Arch   | CUs | Partition | HBM used/total  | Power W | Temp C|",
             "+-----+--------------+--------+-----+-----------+-----------------+---------+-------+"]
    for g in gpus:
        m = metrics.get(g.bdf, {})
        used = f"{m['vram_used_bytes'] / 2**20:6.0f}" if "vram_used_bytes" in m else "n/a".rjust(6)
        total = m.get("vram_total_bytes", g.vram_bytes) / 2**20
        lines.append(f"| {g.index:3d} | {g.bdf:12s} | {g.arch:6s} | {g.cu_count:3d} | "
                     f"{(g.compute_partition or 'SPX') + '/' + (g.memory_partition or 'NPS1'):9s} | "
                     f"{used}/{total:6.0f}MiB | {num(m, 'socket_power_w', 7)} | {num(m, 'temp_hotspot_c', 5)} |")
    lines.append("+-----+--------------+--------+-----+-----------+-----------------+---------+-------+")
    lines.append(f"amd-smi: {smi_status(snap)}")
    return "\n".join(lines)
