"""CDI specs the operator writes, checked against the CDI specification's
rules [EXT: cncf-tags/container-device-interface SPEC.md, v0.6.0] that
containerd/CRI-O enforce when they load a spec directory: a spec that breaks
them is skipped by the runtime and its devices cannot be injected.

Producers: the toolkit's node-wide spec (``amd.com/gpu``, the native OCI
hook's ``cdi`` mode, toolkit/install.py) and the DRA driver's per-claim specs
(``gpu.amd.com/claim``, dra/driver.py)."""

import json
import os
import re

import pytest

from amdgpu_operator.nodeenv import NodeEnv
from amdgpu_operator.testing import fakesys

_NAME = re.compile(r"[A-Za-z0-9][A-Za-z0-9_.-]*")
_DEVICE = re.compile(r"[A-Za-z0-9][A-Za-z0-9_.:-]*")
_SEMVER = re.compile(r"\d+\.\d+\.\d+")


def cdi_errors(spec: dict) -> list[str]:
    errs = []
    if not _SEMVER.fullmatch(str(spec.get("cdiVersion", ""))):
        errs.append(f"cdiVersion {spec.get('cdiVersion')!r}")
    vendor, _, cls = str(spec.get("kind", "")).partition("/")
    if not (vendor and cls and _NAME.fullmatch(vendor) and _NAME.fullmatch(cls)):
        errs.append(f"kind {spec.get('kind')!r} is not vendor/class")
    devices = spec.get("devices") or []
    if not devices:
        errs.append("no devices")
    names = [d.get("name", "") for d in devices]
    errs += [f"device name {n!r}" for n in names if not _DEVICE.fullmatch(n)]
    if len(set(names)) != len(names):
        errs.append("duplicate device names")

    def edits(e, where):
        for dn in e.get("deviceNodes") or []:
            if not str(dn.get("path", "")).startswith("/"):
                errs.append(f"{where}: device node path {dn.get('path')!r}")
            if dn.get("type") not in (None, "b", "c", "u", "p"):
                errs.append(f"{where}: device node type {dn.get('type')!r}")
            if dn.get("permissions") is not None and not re.fullmatch(r"[rwm]+", dn["permissions"]):
                errs.append(f"{where}: permissions {dn['permissions']!r}")
        for env in e.get("env") or []:
            if "=" not in env or env.startswith("="):
                errs.append(f"{where}: env {env!r} is not KEY=VALUE")
        for m in e.get("mounts") or []:
            if not str(m.get("containerPath", "")).startswith("/") or not m.get("hostPath"):
                errs.append(f"{where}: mount {m}")
        for h in e.get("hooks") or []:
            if h.get("hookName") not in ("prestart", "createRuntime", "createContainer", "startContainer",
                                         "poststart", "poststop") or not h.get("path"):
                errs.append(f"{where}: hook {h}")

    edits(spec.get("containerEdits") or {}, "containerEdits")
    for d in devices:
        if not d.get("containerEdits"):
            errs.append(f"device {d.get('name')!r}: containerEdits required")
        edits(d.get("containerEdits") or {}, f"device {d.get('name')!r}")
    return errs


@pytest.mark.parametrize("partition", ["SPX", "CPX"])
def test_toolkit_spec_is_valid_cdi(tmp_path, partition):
    from amdgpu_operator.toolkit.install import generate_cdi

    root = str(tmp_path / "h")
    fakesys.build_node(root, 8, compute_partition=partition)
    env = NodeEnv("n", None, host_root=root)
    path = generate_cdi(env, str(tmp_path / "cdi" / "amd.com-gpu.json"))
    with open(path) as f:
        spec = json.load(f)
    assert not cdi_errors(spec), cdi_errors(spec)
    assert spec["kind"] == "amd.com/gpu" and len(spec["devices"]) >= (8 if partition == "SPX" else 64)


def test_dra_claim_spec_is_valid_cdi(tmp_path):
    from amdgpu_operator.dra.driver import DraDriver

    root = str(tmp_path / "h")
    fakesys.build_node(root, 4)
    env = NodeEnv("n", None, host_root=root, cdi_dir=str(tmp_path / "cdi"),
                  device_plugin_dir=str(tmp_path / "k" / "device-plugins"))
    drv = DraDriver(env)
    ids = drv._write_cdi("0b4f6a3e-59d1-4c1d-b8f1-1e2a3b4c5d6e", ["gpu-0", "gpu-3"])
    with open(drv.cdi_path("0b4f6a3e-59d1-4c1d-b8f1-1e2a3b4c5d6e")) as f:
        spec = json.load(f)
    assert not cdi_errors(spec), cdi_errors(spec)
    # the fully-qualified names the kubelet hands the runtime resolve to devices of the spec
    assert all(i.split("=", 1)[0] == spec["kind"] and i.split("=", 1)[1] in {d["name"] for d in spec["devices"]}
               for i in ids)
    assert os.path.basename(drv.cdi_path("x")).endswith(".json")


def test_checker_rejects_broken_specs():
    bad = {"cdiVersion": "0.6", "kind": "amd.com", "devices": [{"name": "-x", "containerEdits": {
        "deviceNodes": [{"path": "dev/kfd", "permissions": "rwx"}], "env": ["=1"]}}]}
    errs = " | ".join(cdi_errors(bad))
    for want in ("cdiVersion", "not vendor/class", "device name '-x'", "device node path", "permissions", "env"):
        assert want in errs, (want, errs)


def test_runtime_dropins_are_valid_toml_with_the_keys_the_runtimes_read():
    """containerd (config version 2, the reference's `containerd config
    default`, README.md:15-17) and CRI-O read these files as TOML; a syntax
    error makes the runtime refuse to start."""
    import tomli

    from amdgpu_operator.toolkit import install as TK

    for default in (False, True):
        d = tomli.loads(TK.dropin_config("amd", "/usr/local/amd/amdgpu-oci-hook", "/var/run/cdi", ["--x"], default))
        cri = d["plugins"]["io.containerd.grpc.v1.cri"]
        assert d["version"] == 2 and cri["enable_cdi"] is True and "/var/run/cdi" in cri["cdi_spec_dirs"]
        rt = cri["containerd"]["runtimes"]["amd"]
        assert rt["runtime_type"] == "io.containerd.runc.v2" and rt["options"]["SystemdCgroup"] is True
        assert (cri["containerd"].get("default_runtime_name") == "amd") == default
    main = ('version = 2\n[plugins."io.containerd.grpc.v1.cri".containerd.runtimes.runc.options]\n'
            "  SystemdCgroup = true\n")
    patched = tomli.loads(TK.patch_containerd_config(main, "/etc/containerd/conf.d/99-amd.toml"))
    assert patched["imports"] == ["/etc/containerd/conf.d/99-amd.toml"]
    assert patched["plugins"]["io.containerd.grpc.v1.cri"]["containerd"]["runtimes"]["runc"]["options"]["SystemdCgroup"]
    for hooks in (None, "/usr/local/amd/oci-hooks-prestart.d"):
        c = tomli.loads(TK.crio_dropin("/var/run/cdi", hooks))["crio"]["runtime"]
        assert "/var/run/cdi" in c["cdi_spec_dirs"] and (("hooks_dir" in c) == bool(hooks))


# containerd 2.x's `containerd config default` (config version 3), trimmed to
# the parts the operator reads or must leave alone
CONTAINERD_V3_MAIN = """version = 3
root = '/var/lib/containerd'
state = '/run/containerd'

[plugins]
  [plugins.'io.containerd.cri.v1.images']
    snapshotter = 'overlayfs'

  [plugins.'io.containerd.cri.v1.runtime']
    enable_selinux = false

    [plugins.'io.containerd.cri.v1.runtime'.containerd]
      default_runtime_name = 'runc'

      [plugins.'io.containerd.cri.v1.runtime'.containerd.runtimes]
        [plugins.'io.containerd.cri.v1.runtime'.containerd.runtimes.runc]
          runtime_type = 'io.containerd.runc.v2'

          [plugins.'io.containerd.cri.v1.runtime'.containerd.runtimes.runc.options]
            SystemdCgroup = true
"""


def test_containerd_v2_and_v3_dropins_use_the_keys_each_version_reads():
    """containerd 2.x (config version 3) split the CRI plugin: runtime
    handlers, enable_cdi and cdi_spec_dirs moved to io.containerd.cri.v1.runtime.
    The drop-in follows the main config's version; a version-3 file keeps
    no key under the version-2 plugin name and the reverse."""
    import tomli

    from amdgpu_operator.toolkit import install as TK

    assert TK.containerd_config_version(CONTAINERD_V3_MAIN) == 3
    assert TK.containerd_config_version('version = 2\n[plugins]\n') == 2
    assert TK.containerd_config_version("[plugins]\nversion = 3\n") == 2  # a key of a table, not the file's version
    assert TK.containerd_config_version("") == TK.containerd_config_version(None) == 2
    for version, plugin, other in ((2, "io.containerd.grpc.v1.cri", "io.containerd.cri.v1.runtime"),
                                   (3, "io.containerd.cri.v1.runtime", "io.containerd.grpc.v1.cri")):
        d = tomli.loads(TK.dropin_config("amd", "/usr/local/amd/amdgpu-oci-hook", "/var/run/cdi", [], True, version))
        assert d["version"] == version and other not in d["plugins"]
        cri = d["plugins"][plugin]
        assert cri["enable_cdi"] is True and cri["cdi_spec_dirs"] == ["/var/run/cdi", "/etc/cdi"]
        assert cri["containerd"]["default_runtime_name"] == "amd"
        rt = cri["containerd"]["runtimes"]["amd"]
        assert rt["runtime_type"] == "io.containerd.runc.v2" and rt["pod_annotations"] == ["cdi.k8s.io/*"]
        assert rt["options"] == {"BinaryName": "runc", "SystemdCgroup": True}


def test_containerd_v3_install_is_idempotent_and_uninstall_restores(tmp_path):
    import tomli

    from amdgpu_operator.nodeenv import NodeEnv
    from amdgpu_operator.testing import fakesys
    from amdgpu_operator.toolkit import install as TK

    root = str(tmp_path / "host")
    fakesys.build_node(root, 2)
    cfg = tmp_path / "etc" / "containerd" / "config.toml"
    cfg.parent.mkdir(parents=True)
    cfg.write_text(CONTAINERD_V3_MAIN)
    env = NodeEnv("n1", None, host_root=root, validations_dir=str(tmp_path / "v"), cdi_dir=str(tmp_path / "cdi"),
                  containerd_config=str(cfg), install_dir=str(tmp_path / "amd"))
    out = TK.install(env)
    assert out["config_changed"]
    dropin = cfg.parent / "conf.d" / TK.DROPIN_NAME
    d = tomli.loads(dropin.read_text())
    assert d["version"] == 3 and "io.containerd.cri.v1.runtime" in d["plugins"]
    main = tomli.loads(cfg.read_text())
    assert main["version"] == 3 and main["imports"] == [str(dropin)]
    # the user's runc handler and images settings are untouched
    assert main["plugins"]["io.containerd.cri.v1.runtime"]["containerd"]["runtimes"]["runc"]["options"]["SystemdCgroup"]
    assert main["plugins"]["io.containerd.cri.v1.images"]["snapshotter"] == "overlayfs"
    assert not TK.install(env)["config_changed"]  # idempotent
    TK.uninstall(env)
    assert cfg.read_text() == CONTAINERD_V3_MAIN and not dropin.exists()
    # an upgrade from containerd 1.7 (v2 main config, v2 drop-in) to 2.x (v3 main): the drop-in follows
    cfg.write_text('version = 2\n[plugins."io.containerd.grpc.v1.cri".containerd.runtimes.runc.options]\n'
                   "  SystemdCgroup = true\n")
    TK.install(env)
    assert tomli.loads(dropin.read_text())["version"] == 2
    TK.uninstall(env)
    cfg.write_text(CONTAINERD_V3_MAIN)
    assert TK.install(env)["config_changed"] and tomli.loads(dropin.read_text())["version"] == 3
