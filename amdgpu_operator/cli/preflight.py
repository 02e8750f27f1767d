"""``amdgpu-operator preflight``: node prerequisites, checked and optionally fixed.

The reference prepares every node by hand before ``kubeadm join``
(/root/reference/README.md:5-36: apt prerequisites, containerd with
``SystemdCgroup = true``, the ``overlay``/``br_netfilter`` modules and the
bridge/forwarding sysctls) and only discovers a missing GPU when a pod stays
Pending (README.md:186-187).  This command turns those steps into assertions
for an MI355X node, plus the GPU-side prerequisites the operator's driver
probe (N1) relies on:

  containerd     config present, SystemdCgroup = true (README.md:14-17)
  modules-load   overlay + br_netfilter persisted (README.md:23-27)
  sysctl         bridge-nf-call-ip(6)tables = 1, ip_forward = 1 (README.md:29-35)
  kube-tools     kubelet / kubeadm present (README.md:42-49)
  amdgpu         module loaded, /dev/kfd, KFD topology with gfx950 nodes,
                 a render node per GPU (amdgpu-probe semantics)
  hugepages/numa informational: NUMA nodes and the GPUs' NUMA affinity

``--fix`` writes the missing host files (modules-load.d, sysctl.d, the
containerd ``SystemdCgroup`` flip) under ``--root`` and prints the commands
that must run on the host (modprobe / sysctl --system / systemctl restart);
it never runs them itself.  Every path is taken relative to ``--root`` so
the whole check runs against a synthetic tree in tests.
"""

from __future__ import annotations

import json
import os
import re
import shutil
from dataclasses import asdict, dataclass, field

MODULES_FILE = "etc/modules-load.d/k8s.conf"
SYSCTL_FILE = "etc/sysctl.d/k8s.conf"
CONTAINERD_CONFIG = "etc/containerd/config.toml"
REQUIRED_MODULES = ("overlay", "br_netfilter")
REQUIRED_SYSCTLS = {
    "net.bridge.bridge-nf-call-iptables": "1",
    "net.bridge.bridge-nf-call-ip6tables": "1",
    "net.ipv4.ip_forward": "1",
}


@dataclass
class Check:
    name: str
    ok: bool
    detail: str
    reference: str = ""
    fix: list[str] = field(default_factory=list)  # host commands still to run


@dataclass
class Report:
    checks: list[Check]

    @property
    def ok(self) -> bool:
        return all(c.ok for c in self.checks)

    def as_dict(self) -> dict:
        return {"ok": self.ok, "checks": [asdict(c) for c in self.checks]}


def _p(root: str, rel: str) -> str:
    return os.path.join(root, rel)


def _read(path: str) -> str | None:
    try:
        with open(path) as f:
            return f.read()
    except OSError:
        return None


def _write(path: str, text: str) -> None:
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as f:
        f.write(text)


def _loaded_modules(root: str) -> set[str]:
    """Modules in /proc/modules plus everything under /sys/module (built-ins too)."""
    out = {ln.split()[0] for ln in (_read(_p(root, "proc/modules")) or "").splitlines() if ln.strip()}
    d = _p(root, "sys/module")
    if os.path.isdir(d):
        out |= set(os.listdir(d))
    return out


def _sysctl_value(root: str, key: str) -> str | None:
    v = _read(_p(root, "proc/sys/" + key.replace(".", "/")))
    return v.strip() if v is not None else None


def _persisted_sysctls(root: str) -> dict[str, str]:
    out: dict[str, str] = {}
    d = _p(root, "etc/sysctl.d")
    files = sorted(os.listdir(d)) if os.path.isdir(d) else []
    for name in files:
        for line in (_read(os.path.join(d, name)) or "").splitlines():
            m = re.match(r"\s*([\w.\-]+)\s*=\s*(\S+)", line)
            if m and not line.lstrip().startswith(("#", ";")):
                out[m.group(1)] = m.group(2)
    return out


def check_containerd(root: str, fix: bool) -> Check:
    path = _p(root, CONTAINERD_CONFIG)
    text = _read(path)
    ref = "README.md:11-19"
    if text is None:
        return Check("containerd", False, f"{CONTAINERD_CONFIG} missing", ref,
                     ["apt install -y containerd", "containerd config default > /etc/containerd/config.toml"])
    if re.search(r"^\s*SystemdCgroup\s*=\s*true", text, re.M):
        return Check("containerd", True, "SystemdCgroup = true", ref)
    if fix and re.search(r"^\s*SystemdCgroup\s*=\s*false", text, re.M):
        shutil.copyfile(path, path + ".pre-preflight")
        _write(path, re.sub(r"^(\s*SystemdCgroup\s*=\s*)false", r"\1true", text, flags=re.M))
        return Check("containerd", True, "SystemdCgroup flipped to true (backup .pre-preflight)", ref,
                     ["systemctl restart containerd"])
    return Check("containerd", False, "SystemdCgroup is not true (kubelet uses the systemd cgroup driver)", ref,
                 ["set SystemdCgroup = true under the runc options", "systemctl restart containerd"])


def check_modules(root: str, fix: bool) -> Check:
    ref = "README.md:21-27"
    persisted: set[str] = set()
    d = _p(root, "etc/modules-load.d")
    for name in sorted(os.listdir(d)) if os.path.isdir(d) else []:
        persisted |= {ln.strip() for ln in (_read(os.path.join(d, name)) or "").splitlines()
                      if ln.strip() and not ln.lstrip().startswith("#")}
    loaded = _loaded_modules(root)
    missing_p = [m for m in REQUIRED_MODULES if m not in persisted]
    missing_l = [m for m in REQUIRED_MODULES if m not in loaded]
    cmds = [f"modprobe {m}" for m in missing_l]
    if missing_p and fix:
        existing = _read(_p(root, MODULES_FILE)) or ""
        _write(_p(root, MODULES_FILE), existing + "".join(m + "\n" for m in missing_p))
        missing_p = []
    ok = not missing_p and not missing_l
    detail = "ok" if ok else f"not persisted: {missing_p or '-'}; not loaded: {missing_l or '-'}"
    return Check("kernel-modules", ok, detail, ref, cmds)


def check_sysctls(root: str, fix: bool) -> Check:
    ref = "README.md:29-35"
    persisted = _persisted_sysctls(root)
    missing_p = {k: v for k, v in REQUIRED_SYSCTLS.items() if persisted.get(k) != v}
    live_bad = [k for k, v in REQUIRED_SYSCTLS.items() if _sysctl_value(root, k) not in (None, v)]
    if missing_p and fix:
        existing = _read(_p(root, SYSCTL_FILE)) or ""
        _write(_p(root, SYSCTL_FILE), existing + "".join(f"{k} = {v}\n" for k, v in missing_p.items()))
        missing_p = {}
    ok = not missing_p and not live_bad
    cmds = ["sysctl --system"] if live_bad else []
    detail = "ok" if ok else f"not persisted: {sorted(missing_p) or '-'}; live value differs: {live_bad or '-'}"
    return Check("sysctl", ok, detail, ref, cmds)


def check_kube_tools(root: str) -> Check:
    ref = "README.md:42-49"
    found = {t: any(os.access(_p(root, d.lstrip("/") + "/" + t), os.X_OK)
                    for d in ("/usr/bin", "/usr/local/bin", "/bin")) for t in ("kubelet", "kubeadm")}
    missing = [t for t, ok in found.items() if not ok]
    return Check("kube-tools", not missing, "ok" if not missing else f"missing: {missing}", ref,
                 [f"install {' '.join(missing)} (pkgs.k8s.io, held)"] if missing else [])


def check_amdgpu(root: str, expect_gpus: int | None) -> list[Check]:
    from ..discovery import topology

    ref = "README.md:186-187"
    loaded = _loaded_modules(root)
    out = [Check("amdgpu-module", "amdgpu" in loaded, "loaded" if "amdgpu" in loaded else "amdgpu not loaded", ref,
                 [] if "amdgpu" in loaded else ["install amdgpu-dkms (ROCm) or enable the operator's driver"])]
    try:
        ok, msg = topology.probe(root or "/", expect_gpus or 0)
    except Exception as e:  # noqa: BLE001 - library missing is a failed check, not a crash
        ok, msg = False, f"probe unavailable: {e}"
    out.append(Check("gpu-devices", ok, msg, ref))
    try:
        gpus = topology.enumerate_gpus(root or "/")
    except Exception:  # noqa: BLE001
        gpus = []
    archs = sorted({g.arch for g in gpus})
    out.append(Check("gpu-arch", bool(gpus) and archs == ["gfx950"],
                     f"{len(gpus)} GPU node(s), arch {archs or '-'}", "SURVEY.md §2.B C6"))
    numa = sorted({g.numa_node for g in gpus})
    out.append(Check("numa-affinity", True, f"GPU NUMA nodes: {numa or '-'}", "informational"))
    return out


def preflight(root: str = "/", fix: bool = False, expect_gpus: int | None = None, gpu: bool = True) -> Report:
    root = root or "/"
    checks = [check_containerd(root, fix), check_modules(root, fix), check_sysctls(root, fix), check_kube_tools(root)]
    if gpu:
        checks += check_amdgpu(root, expect_gpus)
    return Report(checks)


def main_preflight(root: str, fix: bool, as_json: bool, expect_gpus: int | None, gpu: bool) -> int:
    rep = preflight(root, fix, expect_gpus, gpu)
    if as_json:
        print(json.dumps(rep.as_dict(), indent=1))
    else:
        for c in rep.checks:
            print(f"[{'ok' if c.ok else 'FAIL':>4}] {c.name:<15} {c.detail}" + (f"  ({c.reference})" if c.reference else ""))
            for cmd in c.fix:
                print(f"         run: {cmd}")
    return 0 if rep.ok else 1
