"""Driver DaemonSet (C3): the amdgpu/ROCm install script run
against a fake root with stub package/module commands (SURVEY.md §7.5 item 5:
no module loads on the box), and the Python driver manager (install gating,
driver-loss monitor, upgrade drain, SMI table)."""

import os
import stat
import subprocess

import pytest

from amdgpu_operator.driver import manager as DM
from amdgpu_operator.kube import resources as R
from amdgpu_operator.kube.client import LocalClient
from amdgpu_operator.kube.fakeapi import FakeApiServer
from amdgpu_operator.nodeenv import NodeEnv
from amdgpu_operator.testing import fakesys
from amdgpu_operator.validator import validate as V

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCRIPT = os.path.join(ROOT, "deploy/images/amd-driver/install.sh")

# stub commands: log argv; `modprobe amdgpu` brings the fake driver up unless
# FAKE_MODPROBE_NO_KFD is set (module loads but the KFD node never appears) and
# logs the kernel's firmware search path as it was at load time
STUB = r"""#!/bin/bash
echo "$(basename "$0") $*" >> "$FAKE_LOG"
case "$(basename "$0")" in
  modprobe)
    if [ "$1" = "-r" ]; then
      [ -z "${FAKE_MODPROBE_BUSY:-}" ] || { echo "modprobe: FATAL: Module amdgpu is in use." >&2; exit 1; }
      rm -f "$AMDGPU_SYS_ROOT/module/amdgpu/initstate" "$AMDGPU_SYS_ROOT/module/amdgpu/version" "$AMDGPU_DEV_ROOT/kfd"
      exit 0
    fi
    echo "fwpath=$(cat "$AMDGPU_SYS_ROOT/module/firmware_class/parameters/path")" >> "$FAKE_LOG"
    mkdir -p "$AMDGPU_SYS_ROOT/module/amdgpu"
    echo live > "$AMDGPU_SYS_ROOT/module/amdgpu/initstate"
    echo "${FAKE_MODULE_VERSION:-$AMDGPU_DRIVER_VERSION}" > "$AMDGPU_SYS_ROOT/module/amdgpu/version"
    [ -n "${FAKE_MODPROBE_NO_KFD:-}" ] || : > "$AMDGPU_DEV_ROOT/kfd" ;;
  modinfo) [ -n "${FAKE_MODINFO_VERSION:-}" ] || exit 1; echo "$FAKE_MODINFO_VERSION" ;;
  curl) echo "-----BEGIN PGP PUBLIC KEY BLOCK-----" ;;
  gpg) while [ $# -gt 0 ]; do [ "$1" = "-o" ] && { cat > "$2"; exit 0; }; shift; done; cat > /dev/null ;;
  apt-get) if [ -n "${FAKE_APT_FAIL_HEADERS:-}" ] && [[ "$*" == *linux-headers* ]]; then exit 100; fi ;;
esac
exit 0
"""
KVER = "6.8.0-45-generic"


@pytest.fixture
def fake_host(tmp_path):
    bindir = tmp_path / "bin"
    bindir.mkdir()
    for cmd in ("apt-get", "modprobe", "modinfo", "dpkg", "dkms", "curl", "gpg"):
        p = bindir / cmd
        p.write_text(STUB)
        p.chmod(p.stat().st_mode | stat.S_IXUSR)
    for d in ("sys/module/firmware_class/parameters", "dev", "etc", "usr/src", "host/usr/src", "debs"):
        (tmp_path / d).mkdir(parents=True)
    (tmp_path / "sys/module/firmware_class/parameters/path").write_text("\n")  # the kernel's default: unset
    (tmp_path / "etc/os-release").write_text('ID=ubuntu\nVERSION_CODENAME=noble\n')
    fw = tmp_path / "image-fw/amdgpu"  # amdgpu-dkms-firmware, baked at image build
    fw.mkdir(parents=True)
    for f in ("gc_9_5_0_mec.bin", "psp_13_0_14_sos.bin", "sdma_4_4_5.bin"):
        (fw / f).write_bytes(b"\0" * 16)
    env = {"PATH": f"{bindir}:{os.environ['PATH']}", "FAKE_LOG": str(tmp_path / "calls.log"),
           "AMDGPU_SYS_ROOT": str(tmp_path / "sys"), "AMDGPU_DEV_ROOT": str(tmp_path / "dev"),
           "AMDGPU_ETC_ROOT": str(tmp_path / "etc"), "AMDGPU_USR_SRC": str(tmp_path / "usr/src"),
           "AMDGPU_HOST_SRC": str(tmp_path / "host/usr/src"), "AMDGPU_DEB_DIR": str(tmp_path / "debs"),
           "AMDGPU_FIRMWARE_SRC": str(tmp_path / "image-fw"), "AMDGPU_HOST_FIRMWARE_DIR": str(tmp_path / "run/amd/firmware"),
           "AMDGPU_PRECOMPILED_ROOT": str(tmp_path / "opt/amdgpu"),
           "KVER": KVER, "AMDGPU_WAIT_SECONDS": "2", "AMDGPU_DRIVER_VERSION": "6.12.12", "ROCM_VERSION": "7.2.0"}
    return tmp_path, env


def run_script(env, **extra):
    return subprocess.run(["bash", SCRIPT], env={**env, **extra}, capture_output=True, text=True, timeout=60)


def calls(tmp):
    p = tmp / "calls.log"
    return p.read_text().splitlines() if p.exists() else []


def fetched(log):
    return [c for c in log if c.split()[0] in ("curl", "apt-get", "gpg")]


def _fw_path_at_load(tmp, log):
    """The firmware search path the kernel saw when `modprobe amdgpu` ran,
    and the value the script left behind."""
    i = next(i for i, c in enumerate(log) if c.startswith("modprobe") and "-r" not in c.split())
    return log[i + 1].split("=", 1)[1], (tmp / "sys/module/firmware_class/parameters/path").read_text()


def test_dkms_install_loads_module_and_waits_for_kfd(fake_host):
    tmp, env = fake_host
    r = run_script(env, AMDGPU_MODULE_PARAMS="noretry=1 ras_enable=1")
    assert r.returncode == 0, r.stdout + r.stderr
    log = calls(tmp)
    assert f"apt-get install -y linux-headers-{KVER} linux-modules-extra-{KVER}" in log
    assert "apt-get install -y amdgpu-dkms" in log
    assert log.index("apt-get install -y amdgpu-dkms") < log.index(f"dkms autoinstall -k {KVER}") \
        < log.index("modprobe amdgpu noretry=1 ras_enable=1")
    assert not any("amd-smi-lib" in c for c in log)  # amd-smi is baked in the image, never fetched at start
    assert (tmp / "dev/kfd").exists()
    src = (tmp / "etc/apt/sources.list.d/amdgpu.list").read_text()
    assert "repo.radeon.com/amdgpu/6.12.12/ubuntu noble main" in src
    assert (tmp / "etc/modprobe.d/amd-gpu-operator-blacklist.conf").read_text() == "blacklist amdgpu\n"
    assert "live" in r.stdout.splitlines()[-1]


def test_firmware_path_is_set_before_modprobe_and_restored(fake_host):
    tmp, env = fake_host
    host_fw = env["AMDGPU_HOST_FIRMWARE_DIR"]
    (tmp / "sys/module/firmware_class/parameters/path").write_text("/opt/site-firmware\n")  # an admin's own path
    r = run_script(env)
    assert r.returncode == 0, r.stdout + r.stderr
    at_load, after = _fw_path_at_load(tmp, calls(tmp))
    assert at_load == host_fw  # the kernel looked in the staged copy while amdgpu probed
    assert after.strip() == "/opt/site-firmware"  # and the admin's path is back afterwards
    assert sorted(os.listdir(os.path.join(host_fw, "amdgpu"))) == ["gc_9_5_0_mec.bin", "psp_13_0_14_sos.bin",
                                                                   "sdma_4_4_5.bin"]
    assert not os.path.exists(os.path.join(host_fw, ".amdgpu.new"))


def test_firmware_path_is_restored_when_the_load_fails(fake_host):
    tmp, env = fake_host
    r = run_script(env, FAKE_MODPROBE_NO_KFD="1", AMDGPU_WAIT_SECONDS="1")
    assert r.returncode == 1 and "kfd missing" in r.stdout
    at_load, after = _fw_path_at_load(tmp, calls(tmp))
    assert at_load == env["AMDGPU_HOST_FIRMWARE_DIR"] and after.strip() == ""


def test_offline_dkms_with_host_headers_and_baked_package(fake_host):
    """No network at pod start: the .deb baked in the image builds against the
    host's /usr/src (hostPath), and the firmware comes from the image."""
    tmp, env = fake_host
    (tmp / f"host/usr/src/linux-headers-{KVER}").mkdir()
    (tmp / "host/usr/src/linux-headers-6.8.0-45").mkdir()  # Ubuntu's common tree
    deb = tmp / "debs/amdgpu-dkms_6.12.12-2187269.24.04_all.deb"
    deb.write_bytes(b"!<arch>\n")
    r = run_script(env)
    assert r.returncode == 0, r.stdout + r.stderr
    log = calls(tmp)
    assert fetched(log) == []
    assert log.index(f"dpkg -i {deb}") < log.index(f"dkms autoinstall -k {KVER}") < log.index("modprobe amdgpu")
    for tree in (f"linux-headers-{KVER}", "linux-headers-6.8.0-45"):
        assert os.readlink(tmp / "usr/src" / tree) == str(tmp / "host/usr/src" / tree)
    assert "using the host's headers" in r.stdout


def test_module_already_built_for_this_kernel_is_not_rebuilt(fake_host):
    tmp, env = fake_host
    r = run_script(env, FAKE_MODINFO_VERSION="6.12.12")
    assert r.returncode == 0, r.stdout + r.stderr
    log = calls(tmp)
    assert fetched(log) == [] and not any(c.split()[0] in ("dpkg", "dkms") for c in log)
    assert f"modinfo -k {KVER} -F version amdgpu" in log and "modprobe amdgpu" in log
    # a module built for another version is rebuilt
    (tmp / "calls.log").unlink()
    (tmp / "dev/kfd").unlink()
    (tmp / "sys/module/amdgpu/initstate").unlink()
    r = run_script(env, FAKE_MODINFO_VERSION="6.10.5")
    assert r.returncode == 0 and f"dkms autoinstall -k {KVER}" in calls(tmp)


def _precompiled_image(tmp, kernels=(KVER,)):
    root = tmp / "opt/amdgpu"
    for k in kernels:
        (root / "lib/modules" / k / "updates").mkdir(parents=True)
        (root / "lib/modules" / k / "updates/amdgpu.ko").write_bytes(b"\x7fELF")
    (root / "firmware/amdgpu").mkdir(parents=True)
    (root / "firmware/amdgpu/gc_9_5_0_mec.bin").write_bytes(b"\0")
    return root


def test_precompiled_image_loads_without_network(fake_host):
    tmp, env = fake_host
    root = _precompiled_image(tmp)
    r = run_script(env, AMDGPU_USE_PRECOMPILED="true", AMDGPU_BLACKLIST_INBOX="false",
                   AMDGPU_MODULE_PARAMS="noretry=1")
    assert r.returncode == 0, r.stdout + r.stderr
    log = calls(tmp)
    assert fetched(log) == [] and not any(c.split()[0] in ("dpkg", "dkms", "modinfo") for c in log)
    assert f"modprobe -d {root} amdgpu noretry=1" in log
    at_load, _ = _fw_path_at_load(tmp, log)
    assert at_load == env["AMDGPU_HOST_FIRMWARE_DIR"]
    assert os.listdir(os.path.join(at_load, "amdgpu")) == ["gc_9_5_0_mec.bin"]
    assert not (tmp / "etc/modprobe.d/amd-gpu-operator-blacklist.conf").exists()


def test_precompiled_image_for_another_kernel_fails_and_names_it(fake_host):
    tmp, env = fake_host
    _precompiled_image(tmp, kernels=("6.5.0-1-generic",))
    r = run_script(env, AMDGPU_USE_PRECOMPILED="true")
    assert r.returncode == 1
    assert "built for: 6.5.0-1-generic" in r.stdout and f"6.12.12-{KVER}" in r.stdout
    assert not any(c.startswith("modprobe") for c in calls(tmp)) and fetched(calls(tmp)) == []


def test_package_mirror(fake_host):
    tmp, env = fake_host
    r = run_script(env, AMDGPU_REPO_BASE="http://mirror.local")
    assert r.returncode == 0, r.stderr
    assert "curl -fsSL http://mirror.local/rocm/rocm.gpg.key" in calls(tmp)
    assert "mirror.local/amdgpu/6.12.12/ubuntu noble" in (tmp / "etc/apt/sources.list.d/amdgpu.list").read_text()


def test_already_live_driver_is_left_alone(fake_host):
    tmp, env = fake_host
    (tmp / "sys/module/amdgpu").mkdir(parents=True)
    (tmp / "sys/module/amdgpu/initstate").write_text("live\n")
    (tmp / "dev/kfd").write_text("")
    r = run_script(env)
    assert r.returncode == 0 and "nothing to install" in r.stdout
    assert calls(tmp) == []
    assert (tmp / "sys/module/firmware_class/parameters/path").read_text() == "\n"  # untouched


def test_loaded_module_without_kfd_fails(fake_host):
    tmp, env = fake_host
    r = run_script(env, FAKE_MODPROBE_NO_KFD="1", AMDGPU_WAIT_SECONDS="1")
    assert r.returncode == 1 and "kfd missing" in r.stdout


def test_inbox_module_is_unloaded_before_the_new_one(fake_host):
    tmp, env = fake_host
    (tmp / "sys/module/amdgpu").mkdir(parents=True)
    (tmp / "sys/module/amdgpu/initstate").write_text("live\n")  # inbox module live, no KFD node
    r = run_script(env)
    assert r.returncode == 0, r.stderr
    log = calls(tmp)
    assert log.index("modprobe -r amdgpu") < log.index("modprobe amdgpu")


def _live_module(tmp, version="6.12.12"):
    (tmp / "sys/module/amdgpu").mkdir(parents=True, exist_ok=True)
    (tmp / "sys/module/amdgpu/initstate").write_text("live\n")
    (tmp / "sys/module/amdgpu/version").write_text(version + "\n")
    (tmp / "dev/kfd").write_text("")


def test_live_module_of_another_version_is_replaced(fake_host):
    tmp, env = fake_host
    _live_module(tmp, "6.10.5")
    r = run_script(env)  # requests 6.12.12
    assert r.returncode == 0, r.stdout + r.stderr
    log = calls(tmp)
    assert log.index("modprobe -r amdgpu") < log.index("modprobe amdgpu")
    assert (tmp / "sys/module/amdgpu/version").read_text().strip() == "6.12.12"
    assert "6.10.5 live, 6.12.12 requested: replacing" in r.stdout


def test_force_reload_replaces_a_matching_module(fake_host):
    tmp, env = fake_host
    _live_module(tmp, "6.12.12")
    r = run_script(env, AMDGPU_FORCE_RELOAD="true", AMDGPU_MODULE_PARAMS="noretry=0")
    assert r.returncode == 0, r.stderr
    log = calls(tmp)
    assert log.index("modprobe -r amdgpu") < log.index("modprobe amdgpu noretry=0")


def test_unload_failure_fails_the_install(fake_host):
    tmp, env = fake_host
    _live_module(tmp, "6.10.5")
    r = run_script(env, FAKE_MODPROBE_BUSY="1")
    assert r.returncode == 1 and "could not unload" in r.stdout
    assert "modprobe amdgpu" not in calls(tmp)  # never loads over the old module
    assert (tmp / "sys/module/amdgpu/version").read_text().strip() == "6.10.5"


def test_wrong_version_after_load_fails(fake_host):
    tmp, env = fake_host
    r = run_script(env, FAKE_MODULE_VERSION="6.8.0")
    assert r.returncode == 1 and "6.8.0 loaded, 6.12.12 requested" in r.stdout


def test_no_headers_anywhere_fails_clearly_and_version_is_required(fake_host):
    tmp, env = fake_host
    r = run_script(env, FAKE_APT_FAIL_HEADERS="1")
    assert r.returncode == 1 and f"no headers for {KVER}" in r.stdout and "usePrecompiled" in r.stdout
    assert not any(c.startswith("modprobe") for c in calls(tmp))
    env2 = dict(env)
    env2.pop("AMDGPU_DRIVER_VERSION")
    r = run_script(env2)
    assert r.returncode != 0 and "AMDGPU_DRIVER_VERSION" in r.stderr


# ------------------------------------------------------------ Python manager

@pytest.fixture
def node_env(tmp_path):
    root = str(tmp_path / "host")
    fakesys.build_node(root, 2)
    c = LocalClient(FakeApiServer())
    c.create(R.new("v1", "Node", "n1"))
    return NodeEnv("n1", c, host_root=root, validations_dir=str(tmp_path / "val"), poll_s=0.01)


def test_manager_install_runs_script_only_when_probe_fails(node_env, tmp_path, monkeypatch):
    marker = tmp_path / "ran"
    script = tmp_path / "install.sh"
    root = node_env.sysfs_root()
    # the "install" brings the driver back: restore initstate + /dev/kfd
    script.write_text(f"#!/bin/bash\ntouch {marker}\necho live > {root}/sys/module/amdgpu/initstate\n"
                      f": > {root}/dev/kfd\n")
    script.chmod(0o755)
    monkeypatch.setattr(DM, "INSTALL_SCRIPT", str(script))
    out = DM.install(node_env, timeout=5)
    assert out["ok"] and not out["installed"] and not marker.exists()  # driver already live
    os.unlink(f"{root}/sys/module/amdgpu/initstate")
    os.unlink(f"{root}/dev/kfd")
    out = DM.install(node_env, timeout=5)
    assert out["ok"] and out["installed"] and marker.exists() and out["gpus"] == 2
    assert V.read_ready(node_env, "driver")["ok"]


def test_monitor_clears_validations_when_driver_disappears(node_env):
    DM.install(node_env, timeout=5)
    V.write_ready(node_env, "workload", {"ok": True})
    assert DM.monitor_once(node_env)
    os.unlink(os.path.join(node_env.sysfs_root(), "dev/kfd"))
    assert not DM.monitor_once(node_env)
    assert V.read_ready(node_env, "driver") is None and V.read_ready(node_env, "workload") is None


def test_install_replaces_a_mismatched_module_through_the_backend(node_env):
    kmod = fakesys.SimModule(node_env.sysfs_root())
    node_env.extra["kmod"] = kmod
    out = DM.install(node_env, timeout=5, cenv={"AMDGPU_DRIVER_VERSION": "6.14.0", "AMDGPU_DRIVER_SPEC_HASH": "h2"})
    assert out["installed"] and out["driver_version"] == "6.14.0"
    assert kmod.log == ["unload", "install 6.14.0"]
    assert DM.read_state(node_env) | {"ts": 0} == {"version": "6.14.0", "specHash": "h2", "installed": True,
                                                   "hostManaged": False, "owner": "", "ts": 0}
    ann = node_env.client.get("v1", "Node", "n1")["metadata"]["annotations"]
    assert ann["amd.com/gpu-driver.version"] == "6.14.0" and ann["amd.com/gpu-driver.spec-hash"] == "h2"
    # same version, same spec: nothing to do
    out = DM.install(node_env, timeout=5, cenv={"AMDGPU_DRIVER_VERSION": "6.14.0", "AMDGPU_DRIVER_SPEC_HASH": "h2"})
    assert not out["installed"] and kmod.log == ["unload", "install 6.14.0"]
    # same version, new spec (e.g. module params): reloaded
    out = DM.install(node_env, timeout=5, cenv={"AMDGPU_DRIVER_VERSION": "6.14.0", "AMDGPU_DRIVER_SPEC_HASH": "h3",
                                                "AMDGPU_MODULE_PARAMS": "noretry=1"})
    assert out["installed"] and kmod.log[-1] == "install 6.14.0 noretry=1"


def test_install_without_installer(node_env, monkeypatch, tmp_path):
    monkeypatch.setattr(DM, "INSTALL_SCRIPT", str(tmp_path / "absent.sh"))
    with pytest.raises(RuntimeError, match="loaded 6.12.12, requested 6.14.0"):
        DM.install(node_env, timeout=5, cenv={"AMDGPU_DRIVER_VERSION": "6.14.0"})
    assert V.read_ready(node_env, "driver") is None
    # an inbox / built-in module reports no version: accepted as host-managed
    os.unlink(os.path.join(node_env.sysfs_root(), "sys/module/amdgpu/version"))
    out = DM.install(node_env, timeout=5, cenv={"AMDGPU_DRIVER_VERSION": "6.14.0"})
    assert out["host_managed"] and not out["installed"]
    assert node_env.client.get("v1", "Node", "n1")["metadata"]["annotations"]["amd.com/gpu-driver.version"] == "host"


def test_driver_container_exit_unloads_only_its_own_idle_module(node_env):
    kmod = fakesys.SimModule(node_env.sysfs_root())
    node_env.extra["kmod"] = kmod
    cenv = {"AMDGPU_DRIVER_VERSION": "6.14.0", "AMDGPU_DRIVER_SPEC_HASH": "h2"}
    DM.install(node_env, timeout=5, cenv=cenv)
    # a restarted driver pod keeps the module as container-installed
    assert not DM.install(node_env, timeout=5, cenv=cenv)["installed"] and DM.read_state(node_env)["installed"]
    kfd_proc = os.path.join(node_env.sysfs_root(), "sys/class/kfd/kfd/proc/4242")
    os.makedirs(kfd_proc)
    out = DM.cleanup_on_exit(node_env)  # a GPU process holds it: stays
    assert not out["unloaded"] and "4242" in out["reason"] and DM.loaded_version(node_env) == "6.14.0"
    os.rmdir(kfd_proc)
    V.write_ready(node_env, "workload", {"ok": True})
    assert DM.cleanup_on_exit(node_env)["unloaded"]
    assert kmod.log[-1] == "unload" and DM.loaded_version(node_env) == "" and DM.read_state(node_env) == {}
    assert V.read_ready(node_env, "driver") is None and V.read_ready(node_env, "workload") is None


def test_driver_container_exit_withdraws_validation_and_next_install_restarts_operands(node_env):
    """An unload on exit is a driver loss for the node: the validated labels
    go at once, and the next driver pod's install restarts the validator and
    device-plugin pods so the node is validated again on the new module."""
    kmod = fakesys.SimModule(node_env.sysfs_root())
    node_env.extra["kmod"] = kmod
    c = node_env.client
    cenv = {"AMDGPU_DRIVER_VERSION": "6.14.0", "AMDGPU_DRIVER_SPEC_HASH": "h2"}
    DM.install(node_env, timeout=5, cenv=cenv)
    c.create(R.new("v1", "Namespace", node_env.namespace))
    c.patch("v1", "Node", "n1", {"metadata": {"labels": {V.VALIDATED_LABEL: "true", V.MFMA_LABEL: "bf16"}}})
    for app in ("amd-operator-validator", "amd-device-plugin-daemonset", "amd-metrics-exporter"):
        c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": f"{app}-x", "namespace": node_env.namespace,
                                                                    "labels": {"app": app}},
                  "spec": {"nodeName": "n1"}})
    assert DM.cleanup_on_exit(node_env)["unloaded"]
    labels = c.get("v1", "Node", "n1")["metadata"].get("labels") or {}
    assert V.VALIDATED_LABEL not in labels and V.MFMA_LABEL not in labels
    assert os.path.exists(node_env.validation_file(DM.LOST_MARKER))
    out = DM.install(node_env, timeout=5, cenv=cenv)  # the replacement driver pod
    assert out["installed"] and sorted(out["restarted"]) == ["amd-device-plugin-daemonset-x", "amd-operator-validator-x"]
    assert not os.path.exists(node_env.validation_file(DM.LOST_MARKER))
    left = {p["metadata"]["name"] for p in c.list("v1", "Pod", node_env.namespace)}
    assert left == {"amd-metrics-exporter-x"}
    # and only once: the health monitor finds nothing left to recover
    assert DM.monitor_once(node_env) and "restarted" not in DM.install(node_env, timeout=5, cenv=cenv)


def test_driver_pod_that_was_taken_over_leaves_the_module(node_env):
    """A force-deleted driver pod can still be shutting down when its
    replacement has started: the replacement owns the module from its install
    on, and the old pod's exit must not unload it from under it."""
    kmod = fakesys.SimModule(node_env.sysfs_root())
    node_env.extra["kmod"] = kmod
    cenv = {"AMDGPU_DRIVER_VERSION": "6.14.0", "AMDGPU_DRIVER_SPEC_HASH": "h2"}
    DM.install(node_env, timeout=5, cenv={**cenv, "POD_UID": "old"})
    DM.install(node_env, timeout=5, cenv={**cenv, "POD_UID": "new"})  # replacement: takes over
    assert DM.read_state(node_env)["owner"] == "new"
    out = DM.cleanup_on_exit(node_env, owner="old")
    assert not out["unloaded"] and "taken over by new" in out["reason"]
    assert DM.loaded_version(node_env) == "6.14.0" and V.read_ready(node_env, "driver") is not None
    assert DM.cleanup_on_exit(node_env, owner="new")["unloaded"]


def test_driver_container_exit_leaves_a_host_module(node_env):
    kmod = fakesys.SimModule(node_env.sysfs_root())
    node_env.extra["kmod"] = kmod
    DM.install(node_env, timeout=5, cenv={"AMDGPU_DRIVER_VERSION": "6.12.12"})  # already live: not ours
    out = DM.cleanup_on_exit(node_env)
    assert not out["unloaded"] and kmod.log == [] and DM.loaded_version(node_env) == "6.12.12"


def test_prepare_upgrade_unloads_the_old_module(node_env):
    kmod = fakesys.SimModule(node_env.sysfs_root())
    node_env.extra["kmod"] = kmod
    DM.install(node_env, timeout=5, cenv={"AMDGPU_DRIVER_VERSION": "6.12.12", "AMDGPU_DRIVER_SPEC_HASH": "h1"})
    assert DM.prepare_upgrade(node_env, "6.12.12", spec_hash="h1")["upgrade"] is False
    out = DM.prepare_upgrade(node_env, "6.12.12", spec_hash="h2")  # same version, new driver spec
    assert out["upgrade"] and out["unloaded"] and "driver spec h1" in out["reason"]
    assert kmod.log == ["unload"] and DM.loaded_version(node_env) == ""
    assert DM.read_state(node_env) == {}
    # the driver container then installs the requested module
    out = DM.install(node_env, timeout=5, cenv={"AMDGPU_DRIVER_VERSION": "6.12.12", "AMDGPU_DRIVER_SPEC_HASH": "h2"})
    assert out["installed"] and DM.read_state(node_env)["specHash"] == "h2"


def test_prepare_upgrade_fails_when_the_module_cannot_be_unloaded(node_env):
    kmod = fakesys.SimModule(node_env.sysfs_root())
    kmod.busy = True
    node_env.extra["kmod"] = kmod
    with pytest.raises(RuntimeError, match="in use"):
        DM.prepare_upgrade(node_env, "6.14.0", drain_timeout=0.1)
    assert DM.loaded_version(node_env) == "6.12.12"


def test_prepare_upgrade_without_installer_refuses(node_env, monkeypatch, tmp_path):
    monkeypatch.setattr(DM, "INSTALL_SCRIPT", str(tmp_path / "absent.sh"))
    with pytest.raises(RuntimeError, match="no installer"):
        DM.prepare_upgrade(node_env, "6.14.0")


def test_prepare_upgrade_drains_only_on_version_change(node_env):
    node_env.extra["kmod"] = fakesys.SimModule(node_env.sysfs_root())
    DM.install(node_env, timeout=5)
    cur = DM.loaded_version(node_env)
    assert cur
    assert DM.prepare_upgrade(node_env, cur)["upgrade"] is False
    gpu_pod = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "train", "namespace": "default"},
               "spec": {"nodeName": "n1", "containers": [{"name": "c", "resources": {"limits": {"amd.com/gpu": "1"}}}]}}
    cpu_pod = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "web", "namespace": "default"},
               "spec": {"nodeName": "n1", "containers": [{"name": "c"}]}}
    node_env.client.create(gpu_pod)
    node_env.client.create(cpu_pod)
    out = DM.prepare_upgrade(node_env, "99.0", drain_timeout=1)
    assert out["upgrade"] and out["desired"] == "99.0" and out["unloaded"]
    names = {p["metadata"]["name"] for p in node_env.client.list("v1", "Pod", "default")}
    assert "web" in names and "train" not in names
    assert V.read_ready(node_env, "driver") is None


def test_smi_table_lists_every_gpu(node_env):
    table = DM.smi_table(node_env)
    rows = [ln for ln in table.splitlines() if ln.startswith("|") and "gfx950" in ln]
    assert len(rows) == 2 and "SPX/NPS1" in rows[0]


def test_smi_without_amd_smi_says_so_instead_of_printing_zeros(node_env):
    """No GPU here: amd-smi has no reading, and the table says n/a plus why
    (round 2 printed 0 W / 0 C, which reads like a measurement)."""
    snap = DM.smi_snapshot(node_env)
    assert not snap["ok"] and snap["error"]
    table = DM.smi_table(node_env, snap)
    rows = [ln for ln in table.splitlines() if "gfx950" in ln]
    assert all(ln.count("n/a") == 3 for ln in rows), table  # HBM used, power, temperature
    assert table.splitlines()[-1].startswith("amd-smi: error: ")


def test_smi_from_the_captured_mi355x_metrics(node_env):
    node_env.extra["metrics_fixture"] = os.path.join(fakesys.REAL_FIXTURE, "amd-smi-metric.json")
    snap = DM.smi_snapshot(node_env)
    assert snap["ok"] and snap["source"] == "fixture" and snap["live"] == snap["physical"] == 2
    rows = [ln for ln in DM.smi_table(node_env, snap).splitlines() if "gfx950" in ln]
    for r in rows:
        cells = [c.strip() for c in r.strip("|").split("|")]
        assert float(cells[6]) > 0 and float(cells[7]) > 0
    assert DM.smi_status(snap) == "ok: 2/2 GPUs live (fixture)"


def test_health_container_publishes_the_smi_status(node_env):
    from amdgpu_operator.cli.verify import verify
    from amdgpu_operator.wellknown import DRIVER_SMI_ANN

    def ann():
        return (node_env.client.get("v1", "Node", "n1")["metadata"].get("annotations") or {}).get(DRIVER_SMI_ANN)

    DM.install(node_env, timeout=5)
    DM.monitor_once(node_env)
    assert ann().startswith("error: amd-smi unavailable") or ann().startswith("error: live power")
    node_env.extra["metrics_fixture"] = os.path.join(fakesys.REAL_FIXTURE, "amd-smi-metric.json")
    node_env.extra.pop("_smi_published")
    DM.monitor_once(node_env)
    assert ann() == "ok: 2/2 GPUs live (fixture)"
    node_env.client.patch("v1", "Node", "n1", {"metadata": {"labels": {"amd.com/gpu.present": "true"}}})
    assert next(c for c in verify(node_env.client, "default").checks if c.name == "driver-smi[n1]").ok
    fakesys.SimModule(node_env.host_root).unload(node_env)  # driver lost
    DM.monitor_once(node_env)
    assert ann() == "error: driver not live"
    chk = next(c for c in verify(node_env.client, "default").checks if c.name == "driver-smi[n1]")
    assert not chk.ok and chk.detail == "error: driver not live"
