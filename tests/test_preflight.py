"""``amdgpu-operator preflight``: the node-preparation steps of
/root/reference/README.md:5-49 as checks, on synthetic host trees."""

import json
import os

from amdgpu_operator.cli import preflight as PF
from amdgpu_operator.testing import fakesys

DEFAULT_CONTAINERD = """version = 2
[plugins."io.containerd.grpc.v1.cri".containerd.runtimes.runc.options]
            SystemdCgroup = false
"""


def _host(tmp_path, gpus=2, prepared=False):
    root = str(tmp_path / "host")
    fakesys.build_node(root, gpus)
    os.makedirs(f"{root}/etc/containerd", exist_ok=True)
    with open(f"{root}/etc/containerd/config.toml", "w") as f:
        f.write(DEFAULT_CONTAINERD.replace("false", "true") if prepared else DEFAULT_CONTAINERD)
    for m in ("overlay", "br_netfilter"):
        os.makedirs(f"{root}/sys/module/{m}", exist_ok=True)
    for k in PF.REQUIRED_SYSCTLS:
        path = f"{root}/proc/sys/" + k.replace(".", "/")
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "w") as f:
            f.write("1\n")
    os.makedirs(f"{root}/usr/bin", exist_ok=True)
    for t in ("kubelet", "kubeadm"):
        with open(f"{root}/usr/bin/{t}", "w") as f:
            f.write("#!/bin/sh\n")
        os.chmod(f"{root}/usr/bin/{t}", 0o755)
    if prepared:
        os.makedirs(f"{root}/etc/modules-load.d", exist_ok=True)
        with open(f"{root}/{PF.MODULES_FILE}", "w") as f:
            f.write("overlay\nbr_netfilter\n")
        os.makedirs(f"{root}/etc/sysctl.d", exist_ok=True)
        with open(f"{root}/{PF.SYSCTL_FILE}", "w") as f:
            f.write("".join(f"{k} = 1\n" for k in PF.REQUIRED_SYSCTLS))
    return root


def test_prepared_gpu_node_passes(tmp_path):
    rep = PF.preflight(_host(tmp_path, prepared=True), expect_gpus=2)
    assert rep.ok, rep.as_dict()
    names = [c.name for c in rep.checks]
    assert names[:4] == ["containerd", "kernel-modules", "sysctl", "kube-tools"]
    assert {c.name: c for c in rep.checks}["gpu-arch"].detail.startswith("2 GPU node(s)")


def test_fresh_node_fails_then_fix_writes_host_files(tmp_path):
    root = _host(tmp_path)
    rep = PF.preflight(root)
    bad = {c.name for c in rep.checks if not c.ok}
    assert bad == {"containerd", "kernel-modules", "sysctl"}
    fixed = PF.preflight(root, fix=True)
    assert fixed.ok, fixed.as_dict()
    assert "SystemdCgroup = true" in open(f"{root}/etc/containerd/config.toml").read()
    assert open(f"{root}/etc/containerd/config.toml.pre-preflight").read() == DEFAULT_CONTAINERD
    assert open(f"{root}/{PF.MODULES_FILE}").read() == "overlay\nbr_netfilter\n"
    assert "net.ipv4.ip_forward = 1" in open(f"{root}/{PF.SYSCTL_FILE}").read()
    assert any("systemctl restart containerd" in c.fix for c in fixed.checks)
    # idempotent: a second --fix changes nothing
    before = open(f"{root}/{PF.SYSCTL_FILE}").read()
    assert PF.preflight(root, fix=True).ok and open(f"{root}/{PF.SYSCTL_FILE}").read() == before


def test_node_without_gpu_driver(tmp_path):
    root = _host(tmp_path, gpus=0, prepared=True)
    rep = PF.preflight(root)
    by = {c.name: c for c in rep.checks}
    assert not rep.ok and not by["gpu-devices"].ok and not by["gpu-arch"].ok
    assert PF.preflight(root, gpu=False).ok  # control-plane node


def test_cli_json(tmp_path, capsys):
    from amdgpu_operator.cli.main import main

    root = _host(tmp_path, prepared=True)
    assert main(["preflight", "--root", root, "--json", "--expect-gpus", "2"]) == 0
    out = json.loads(capsys.readouterr().out)
    assert out["ok"] and all(c["ok"] for c in out["checks"])
    assert main(["preflight", "--root", root, "--expect-gpus", "3"]) == 1
