"""Host-code sanitizer builds (ASan + UBSan) of the native CPU tools, run on
synthetic inputs.  GPU sanitizers are not available on the
pool; the GPU kernels are covered by the numerics tests instead."""

import fcntl
import json
import os
import subprocess

import pytest

from amdgpu_operator import native
from amdgpu_operator.testing import fakesys

pytestmark = pytest.mark.slow


@pytest.fixture(scope="module")
def asan_bins():
    # xdist workers each build this fixture: serialise make so no worker runs
    # a binary another worker's make is relinking
    with open(os.path.join(str(native.NATIVE_SRC), ".sanitize.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        p = subprocess.run(["make", "-C", str(native.NATIVE_SRC), "sanitize"], capture_output=True, text=True,
                           timeout=600)
    if p.returncode != 0:
        pytest.skip(f"sanitizer toolchain unavailable: {p.stderr[-500:]}")
    return {n: str(native.artefact(n + ".asan")) for n in ("amdgpu-oci-hook", "amdgpu-probe", "amdgpu-nfd")}


def _run(argv, input_=None):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=99",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1:exitcode=98")
    return subprocess.run(argv, capture_output=True, text=True, input=input_, timeout=120, env=env)


def test_hook_under_asan(asan_bins, tmp_path):
    root = str(tmp_path / "host")
    fakesys.build_node(root, 8, "CPX")
    hook = asan_bins["amdgpu-oci-hook"]
    p = _run([hook, "cdi", "--root", root])
    assert p.returncode == 0, p.stderr[-3000:]
    assert len(json.loads(p.stdout)["devices"]) == 65
    b = tmp_path / "b"
    b.mkdir()
    (b / "config.json").write_text(json.dumps({"process": {"env": ["AMD_VISIBLE_DEVICES=all"]}, "linux": {}}))
    spec = (b / "config.json").read_text()
    for _ in range(2):
        p = _run([hook, "precreate", "--root", root], spec)
        assert p.returncode == 0, p.stderr[-3000:]
        assert len(json.loads(p.stdout)["linux"]["devices"]) == 65
    proc = tmp_path / "proc"
    (proc / "9/root").mkdir(parents=True)
    (proc / "9/cgroup").write_text("5:devices:/k/c\n")
    state = json.dumps({"bundle": str(b), "id": "x", "pid": 9})
    p = _run([hook, "prestart", "--root", root, "--proc-root", str(proc), "--dry-run"], state)
    assert p.returncode == 0, p.stderr[-3000:]
    assert len(json.loads(p.stdout)["mknod"]) == 65
    for bad in ("{", '{"bundle": []}', "\x00\x01", '{"a": "\\ud800"}', "[" * 1000 + "]" * 1000):
        p = _run([hook, "prestart", "--root", root], bad)
        assert p.returncode == 1, (bad[:20], p.returncode, p.stderr[-2000:])
    for bad in ("{", "\x00\x01", "[" * 1000 + "]" * 1000, '"spec"'):  # not a JSON object
        p = _run([hook, "precreate", "--root", root], bad)
        assert p.returncode == 1, (bad[:20], p.returncode, p.stderr[-2000:])


def test_probe_under_asan(asan_bins, tmp_path):
    root = fakesys.build_from_real_fixture(str(tmp_path / "real"))
    p = _run([asan_bins["amdgpu-probe"], "--root", root, "--json"])
    assert p.returncode == 0, p.stderr[-3000:]
    assert json.loads(p.stdout)["gpus"][0]["arch"] == "gfx950"
    p = _run([asan_bins["amdgpu-probe"], "--root", str(tmp_path / "none")])
    assert p.returncode == 1


@pytest.mark.parametrize("gpus,mode", [(1, "SPX"), (8, "SPX"), (8, "CPX"), (4, "DPX")])
def test_topology_library_under_asan(asan_bins, tmp_path, gpus, mode):
    """N3 (+ the N4/N6 unavailable paths) under ASan/UBSan, cross-checked with the ctypes view."""
    from amdgpu_operator.discovery import topology as T

    root = str(tmp_path / "host")
    fakesys.build_node(root, gpus, mode)
    p = _run([str(native.artefact("topo-selftest.asan")), root, "--smi"])
    assert p.returncode == 0, p.stderr[-3000:]
    rep = json.loads(p.stdout)
    py = T.enumerate_gpus(root)
    assert rep["enumerate_rc"] == 0 and rep["probe_rc"] == 0
    assert [g["bdf"] for g in rep["gpus"]] == [g.bdf for g in py]
    assert {g["partition"] for g in rep["gpus"]} == {mode}
    assert rep["links"] == len(T.links(root))
    if len(py) > 1:
        assert rep["nospc_rc"] == -28  # AT_ERR_NOSPC: short buffer reported, not overrun
    assert rep["smi_open_rc"] in (0, -95) and rep["health_poll_rc"] in (0, -95)


def test_topology_library_under_asan_real_fixture(asan_bins, tmp_path):
    root = fakesys.build_from_real_fixture(str(tmp_path / "real"))
    p = _run([str(native.artefact("topo-selftest.asan")), root])
    assert p.returncode == 0, p.stderr[-3000:]
    rep = json.loads(p.stdout)
    assert rep["gpus"][0]["arch"] == "gfx950" and rep["gpus"][0]["cu"] == 256


def test_nfd_worker_under_asan(asan_bins, tmp_path):
    """The native NFD worker's sysfs scan, kubeconfig parsing, HTTP exchange
    and merge patch under ASan/UBSan, against the fake API server over HTTP."""
    from amdgpu_operator.kube import resources as R
    from amdgpu_operator.kube.fakeapi import FakeApiServer
    from amdgpu_operator.kube.httpapi import HttpApiServer

    root = str(tmp_path / "host")
    fakesys.build_node(root, 8, "CPX")
    p = _run([asan_bins["amdgpu-nfd"], "--print", "--host-root", root])
    assert p.returncode == 0, p.stderr[-2000:]
    api = FakeApiServer()
    api.create(R.new("v1", "Node", "n1", labels={"feature.node.kubernetes.io/pci-0300_10de.present": "true"}))
    http = HttpApiServer(api).start()
    try:
        kc = tmp_path / "kc.json"
        kc.write_text(json.dumps({"current-context": "c", "clusters": [{"name": "c", "cluster": {"server": http.url}}],
                                  "users": [{"name": "u", "user": {"token": "t"}}],
                                  "contexts": [{"name": "c", "context": {"cluster": "c", "user": "u"}}]}))
        env = dict(os.environ, KUBECONFIG=str(kc), NODE_NAME="n1", HOST_ROOT=root,
                   ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=99",
                   UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1:exitcode=98")
        env.pop("KUBERNETES_SERVICE_HOST", None)
        for _ in range(2):  # a write, then a no-op pass
            p = subprocess.run([asan_bins["amdgpu-nfd"], "--oneshot"], capture_output=True, text=True, timeout=120,
                               env=env)
            assert p.returncode == 0, p.stderr[-2000:]
        labels = api.get("v1", "Node", "n1")["metadata"]["labels"]
        assert labels["feature.node.kubernetes.io/pci-1002.present"] == "true"
        assert "feature.node.kubernetes.io/pci-0300_10de.present" not in labels
    finally:
        http.stop()
