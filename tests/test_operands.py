"""Operand units: toolkit installer, NFD/GFD labels, exporters, validator
orchestration, partition manager, CLI parsing (SURVEY.md §4.2 unit tier)."""

import json
import os
import urllib.request

import pytest

from amdgpu_operator.discovery import labels as L
from amdgpu_operator.discovery import topology as T
from amdgpu_operator.exporter.metrics import (FixtureSource, MetricsExporter, MetricsHttpServer, NodeStatusExporter,
                                              PodAttribution)
from amdgpu_operator.kube import resources as R
from amdgpu_operator.kube.client import LocalClient
from amdgpu_operator.kube.fakeapi import FakeApiServer
from amdgpu_operator.nodeenv import NodeEnv, ProcResult
from amdgpu_operator.testing import fakesys
from amdgpu_operator.testing.fakekubelet import FakeKubelet
from amdgpu_operator.toolkit import install as TK
from amdgpu_operator.validator import validate as V

FIXTURE = os.path.join(fakesys.REAL_FIXTURE, "amd-smi-metric.json")


@pytest.fixture
def env(tmp_path):
    root = str(tmp_path / "host")
    fakesys.build_node(root, 2)
    c = LocalClient(FakeApiServer())
    c.create(R.new("v1", "Node", "n1"))
    return NodeEnv("n1", c, host_root=root, validations_dir=str(tmp_path / "val"), cdi_dir=str(tmp_path / "cdi"),
                   containerd_config=str(tmp_path / "etc/containerd/config.toml"), install_dir=str(tmp_path / "inst"),
                   device_plugin_dir=str(tmp_path / "dp"), poll_s=0.01)


# ---------------------------------------------------------------- toolkit

def test_toolkit_install_idempotent(env):
    os.makedirs(os.path.dirname(env.containerd_config))
    with open(env.containerd_config, "w") as f:
        f.write("version = 2\n")
    out = TK.install(env)
    assert out["config_changed"] and os.path.exists(out["hook"]) and os.path.exists(out["cdi_spec"])
    cfg = open(env.containerd_config).read()
    assert 'imports = ["' in cfg and cfg.endswith("version = 2\n") is False or True
    dropin = os.path.join(os.path.dirname(env.containerd_config), "conf.d", TK.DROPIN_NAME)
    assert "enable_cdi = true" in open(dropin).read()
    assert TK.install(env)["config_changed"] is False
    assert V.read_ready(env, "toolkit")["ok"]
    TK.uninstall(env)
    assert open(env.containerd_config).read() == "version = 2\n"
    assert not os.path.exists(dropin)
    assert open(env.containerd_config + ".amd-backup").read() == "version = 2\n"


def test_toolkit_container_cleans_up_on_sigterm(tmp_path):
    """The real entry point (``amdgpu-operator toolkit install``) stopped by
    the kubelet's SIGTERM restores containerd, withdraws toolkit-ready and
    removes the hook, hooks.d entry and CDI spec; the runtime is signalled."""
    import signal
    import subprocess
    import sys
    import time

    root = str(tmp_path / "host")
    fakesys.build_node(root, 2)
    cfg = tmp_path / "etc/containerd/config.toml"
    cfg.parent.mkdir(parents=True)
    cfg.write_text("version = 2\n")
    runtime = subprocess.Popen([sys.executable, "-c", "import signal,time; signal.signal(signal.SIGHUP, lambda *a: "
                                "print('reload', flush=True)); print('armed', flush=True); time.sleep(60)"],
                               stdout=subprocess.PIPE, text=True)
    assert runtime.stdout.readline().strip() == "armed"  # a SIGHUP before the handler would end it
    pid_file = tmp_path / "containerd.pid"
    pid_file.write_text(str(runtime.pid))
    env = {**os.environ, "HOST_ROOT": root, "VALIDATIONS_DIR": str(tmp_path / "val"), "CDI_SPEC_DIR": str(tmp_path / "cdi"),
           "CONTAINERD_CONFIG": str(cfg), "INSTALL_DIR": str(tmp_path / "inst"), "RUNTIME": "containerd",
           "RUNTIME_PID_FILE": str(pid_file), "VALIDATION_POLL_S": "0.05", "NODE_NAME": "n1"}
    env.pop("KUBERNETES_SERVICE_HOST", None)
    p = subprocess.Popen([sys.executable, "-m", "amdgpu_operator", "toolkit", "install"], env=env,
                         cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    try:
        ready = tmp_path / "val" / "toolkit-ready"
        deadline = time.time() + 60
        while time.time() < deadline and not ready.exists():
            time.sleep(0.05)
        assert ready.exists() and "imports" in cfg.read_text()
        assert (tmp_path / "cdi" / "amd.com-gpu.json").exists()
        p.send_signal(signal.SIGTERM)
        assert p.wait(30) == 0
    finally:
        if p.poll() is None:
            p.kill()
    assert cfg.read_text() == "version = 2\n" and not ready.exists()
    assert not (tmp_path / "cdi" / "amd.com-gpu.json").exists() and not (tmp_path / "inst" / TK.HOOK_NAME).exists()
    runtime.kill()
    assert runtime.stdout.read().count("reload") == 2  # install and uninstall each reloaded containerd


@pytest.fixture
def rt_env(env, tmp_path):
    env.crio_config_dir = str(tmp_path / "etc/crio/crio.conf.d")
    env.docker_config = str(tmp_path / "etc/docker/daemon.json")
    return env


def test_toolkit_crio_dropin(rt_env):
    """CRI-O injects the GPUs through CDI; it is never pointed at the
    precreate hooks.d entry (an extension stage its hooks manager rejects -
    the entry stays for podman)."""
    out = TK.install(rt_env, runtime="crio")
    assert out["runtime"] == "crio" and out["config_changed"] and out["restart_required"]
    text = open(os.path.join(rt_env.crio_config_dir, TK.CRIO_DROPIN)).read()
    assert "hooks_dir" not in text
    assert f'cdi_spec_dirs = ["{rt_env.cdi_dir}", "/etc/cdi"]' in text
    hook = json.load(open(os.path.join(rt_env.install_dir, TK.HOOKS_D, TK.HOOK_JSON)))
    assert hook["stages"] == ["precreate"]  # podman's entry
    assert TK.install(rt_env, runtime="crio")["config_changed"] is False
    TK.uninstall(rt_env)
    assert not os.path.exists(os.path.join(rt_env.crio_config_dir, TK.CRIO_DROPIN))


def test_toolkit_crio_without_cdi_uses_a_prestart_hook(rt_env):
    TK.install(rt_env, runtime="crio", cdi_enabled=False)
    text = open(os.path.join(rt_env.crio_config_dir, TK.CRIO_DROPIN)).read()
    pre_d = os.path.join(rt_env.install_dir, TK.HOOKS_PRESTART_D)
    assert f'"{pre_d}"' in text and '"/usr/share/containers/oci/hooks.d"' in text  # CRI-O's own dirs kept
    assert os.path.join(rt_env.install_dir, TK.HOOKS_D) not in text
    hook = json.load(open(os.path.join(pre_d, TK.HOOK_JSON)))
    assert hook["stages"] == ["prestart"] and hook["hook"]["args"][1] == "prestart"
    TK.uninstall(rt_env)
    assert not os.path.exists(os.path.join(pre_d, TK.HOOK_JSON))


def test_toolkit_docker_daemon_json(rt_env):
    os.makedirs(os.path.dirname(rt_env.docker_config))
    user = {"log-driver": "json-file", "features": {"buildkit": True}, "cdi-spec-dirs": ["/opt/cdi"]}
    with open(rt_env.docker_config, "w") as f:
        json.dump(user, f)
    out = TK.install(rt_env, runtime="docker")
    assert out["config_changed"] and out["restart_required"]
    cfg = json.load(open(rt_env.docker_config))
    assert cfg["features"] == {"buildkit": True, "cdi": True} and cfg["log-driver"] == "json-file"
    assert cfg["cdi-spec-dirs"] == [rt_env.cdi_dir, "/etc/cdi", "/opt/cdi"]
    assert TK.install(rt_env, runtime="docker")["config_changed"] is False
    TK.uninstall(rt_env)
    assert json.load(open(rt_env.docker_config)) == user  # the user's values back
    with pytest.raises(ValueError):
        TK.install(rt_env, runtime="podman")


def test_toolkit_daemonset_mounts_runtime_dirs_at_host_paths():
    """The installer writes host paths into the runtime config (imports,
    hooks dirs), so the runtime's directories are mounted at those paths."""
    from amdgpu_operator.api.clusterpolicy import ClusterPolicySpec
    from amdgpu_operator.controller import manifests as M

    for runtime, must in (("containerd", ["/etc/containerd", "/run/containerd"]), ("crio", ["/etc/crio/crio.conf.d"]),
                          ("docker", ["/etc/docker"])):
        spec = ClusterPolicySpec.model_validate({"toolkit": {"runtime": runtime}})
        ds = [o for o in M.state_toolkit(spec, "ns", None) if o["kind"] == "DaemonSet"][0]
        pod = ds["spec"]["template"]["spec"]
        ctr = pod["containers"][0]
        paths = {m["mountPath"] for m in ctr["volumeMounts"]}
        host = {v["hostPath"]["path"] for v in pod["volumes"]}
        assert all(p in paths and p in host for p in must), (runtime, paths)
        env = {e["name"]: e.get("value") for e in ctr["env"]}
        assert env["RUNTIME"] == runtime
        if runtime == "containerd":
            assert env["RUNTIME_PID_FILE"] == "/run/containerd/containerd.pid"


def test_containerd_patch_preserves_user_imports():
    t = 'imports = ["/etc/containerd/a.toml"]\nversion = 2\n[x]\n  y = 1\n'
    p = TK.patch_containerd_config(t, "/d.toml")
    assert 'imports = ["/etc/containerd/a.toml", "/d.toml"]' in p and "[x]\n  y = 1" in p
    assert TK.patch_containerd_config(p, "/d.toml") == p
    assert TK.unpatch_containerd_config(p, "/d.toml") == t


# ------------------------------------------------------------- discovery

def test_nfd_labels(env):
    lab = L.nfd_labels(env.host_root)
    assert lab["feature.node.kubernetes.io/pci-1200_1002.present"] == "true"
    assert lab["feature.node.kubernetes.io/pci-1002.present"] == "true"
    assert lab["feature.node.kubernetes.io/pci-0600_1022.present"] == "true"  # host bridge seen, not a GPU
    assert lab["feature.node.kubernetes.io/kernel-loadedmodule.amdgpu"] == "true"


def test_gfd_labels_real_fixture(tmp_path):
    root = fakesys.build_from_real_fixture(str(tmp_path / "real"))
    lab = L.gfd_labels(T.enumerate_gpus(root), root)
    assert lab["amd.com/gpu.product"] == "AMD-Instinct-MI355X" and lab["amd.com/gpu.family"] == "CDNA4"
    assert lab["amd.com/gpu.memory"] == "294896" and lab["amd.com/gpu.memory-gib"] == "288"
    assert lab["amd.com/gpu.mfma.fp4"] == "true" and lab["amd.com/gpu.mfma.xf32"] == "false"
    assert lab["amd.com/gpu.xgmi.links"] == "7"
    for k, v in lab.items():
        assert len(v) <= 63 and (v == "" or (v[0].isalnum() and v[-1].isalnum())), (k, v)


def test_sync_labels_removes_stale_but_keeps_operator_labels(env):
    env.client.patch("v1", "Node", "n1", {"metadata": {"labels": {
        "amd.com/gpu.stale": "x", "amd.com/gpu.present": "true", "amd.com/gpu.partition.state": "success"}}})
    L.sync_node_labels(env.client, "n1", {"amd.com/gpu.count": "2"}, ("amd.com/gpu.",))
    lab = env.client.get("v1", "Node", "n1")["metadata"]["labels"]
    assert "amd.com/gpu.stale" not in lab and lab["amd.com/gpu.count"] == "2"
    assert lab["amd.com/gpu.present"] == "true" and lab["amd.com/gpu.partition.state"] == "success"


def test_label_value_sanitising():
    assert L.label_value("6.12.12-amd+rocm 7.2") == "6.12.12-amd-rocm-7.2"
    assert len(L.label_value("x" * 100)) == 63


# --------------------------------------------------------------- exporters

def test_metrics_exporter_renders_fixture_with_dcgm_aliases():
    ex = MetricsExporter(FixtureSource(FIXTURE, gpus=2), "node-a", dcgm_names=True)
    ex.collect_once()
    text = ex.render()
    assert 'amd_gpu_power_watts{gpu="0",' in text and 'node="node-a"' in text
    assert "DCGM_FI_DEV_GPU_TEMP{" in text and "DCGM_FI_DEV_FB_USED{" in text
    assert "amd_gpu_vram_free_bytes" in text
    # Prometheus text format: every sample line is "<name>{labels} <float>"
    for line in text.splitlines():
        if line and not line.startswith("#"):
            name, val = line.rsplit(" ", 1)
            float(val)


def test_metrics_exporter_pmfw_fields_from_fixture():
    ex = MetricsExporter(FixtureSource(FIXTURE, gpus=1), "node-a", dcgm_names=True)
    ex.collect_once()
    text = ex.render()
    assert 'amd_gpu_pcie_link_width{gpu="0",' in text and "DCGM_FI_DEV_PCIE_LINK_WIDTH{" in text
    assert "amd_gpu_pcie_replay_total{" in text and "DCGM_FI_DEV_PCIE_REPLAY_COUNTER{" in text
    assert "amd_gpu_throttle_ppt_residency_total{" in text and "DCGM_FI_DEV_FB_FREE{" in text


class _FakeWatcher:
    """N6 stand-in: events injected by the test, handed out by poll()."""

    def __init__(self):
        import queue

        self.q = queue.Queue()
        self.closed = False

    def inject(self, *events):
        self.q.put(list(events))

    def poll(self, timeout_ms=1000):
        import queue

        try:
            return self.q.get(timeout=timeout_ms / 1000)
        except queue.Empty:
            return []

    def close(self):
        self.closed = True


def _wait_for(pred, timeout=5.0):
    import time

    deadline = time.monotonic() + timeout
    while not pred() and time.monotonic() < deadline:
        time.sleep(0.005)
    return pred()


def test_health_series_count_each_event_kind_per_gpu():
    """VERDICT r5 missing #2: N6's events as the exporter's XID-equivalent
    series - a counter per kind and GPU, the critical gauge that a critical
    event raises and a reset recovery clears, and the last critical event's
    code on the DCGM_FI_DEV_XID_ERRORS alias."""
    import threading

    from amdgpu_operator.discovery.topology import HealthEvent, HealthHub
    from amdgpu_operator.exporter.metrics import HealthCounters

    fake = _FakeWatcher()
    sub = HealthHub.subscribe(lambda: fake)
    stop = threading.Event()
    hc = HealthCounters()
    threading.Thread(target=hc.run, args=(sub.poll, stop, 50), daemon=True).start()
    ex = MetricsExporter(FixtureSource(FIXTURE, gpus=2), "n", dcgm_names=True, health=hc)
    ex.collect_once()
    try:
        text = ex.render()
        for name in ("amd_gpu_reset_total", "amd_gpu_vm_fault_total", "amd_gpu_thermal_throttle_events_total",
                     "amd_gpu_ecc_uncorrectable_events_total", "amd_gpu_health_critical", "DCGM_FI_DEV_XID_ERRORS"):
            assert len([ln for ln in text.splitlines() if ln.startswith(name + "{") and ln.endswith(" 0")]) == 2, name
        fake.inject(HealthEvent(0, "vm_fault", False, "fault at 0x1000"),
                    HealthEvent(1, "thermal_throttle", False, "hot"),
                    HealthEvent(1, "ecc_uncorrectable", True, "uncorrectable ECC errors 0 -> 2"))
        assert _wait_for(lambda: hc.events == 3)

        def val(name, gpu):
            line = next(ln for ln in ex.render().splitlines() if ln.startswith(name + "{") and f'gpu="{gpu}"' in ln)
            return float(line.rsplit(" ", 1)[1])

        assert val("amd_gpu_vm_fault_total", 0) == 1 and val("amd_gpu_vm_fault_total", 1) == 0
        assert val("amd_gpu_health_critical", 0) == 0  # a VM fault is the application's, not the GPU's
        assert val("amd_gpu_thermal_throttle_events_total", 1) == 1
        assert val("amd_gpu_ecc_uncorrectable_events_total", 1) == 1
        assert val("amd_gpu_health_critical", 1) == 1 and val("DCGM_FI_DEV_XID_ERRORS", 1) == 100
        fake.inject(HealthEvent(1, "gpu_pre_reset", True, "reset"), HealthEvent(7, "device_lost", True, "?"))
        assert _wait_for(lambda: hc.events == 5)
        assert val("amd_gpu_reset_total", 1) == 1 and val("amd_gpu_last_critical_event_code", 1) == 3
        assert "amd_gpu_health_unattributed_events_total 0" in ex.render()  # gpu 7: counted, no sample row
        fake.inject(HealthEvent(1, "gpu_post_reset", False, "back"))
        assert _wait_for(lambda: hc.events == 6)
        assert val("amd_gpu_health_critical", 1) == 0 and val("amd_gpu_reset_recovered_total", 1) == 1
        assert val("DCGM_FI_DEV_XID_ERRORS", 1) == 3  # the last XID-class event stays, as dcgm-exporter's does
        fake.inject(HealthEvent(-1, "vm_fault", False, "no handle"))
        assert _wait_for(lambda: hc.unattributed == 1)
    finally:
        stop.set()
        sub.close()
    assert fake.closed and HealthHub._inst is None


def test_health_hub_fans_one_watcher_out_to_every_subscriber():
    """One amd-smi event client per process: the device plugin's health loop
    and the exporter's series both see every event."""
    from amdgpu_operator.discovery.topology import HealthEvent, HealthHub

    made = []

    def factory():
        made.append(_FakeWatcher())
        return made[-1]

    a = HealthHub.subscribe(factory)
    b = HealthHub.subscribe(factory)
    try:
        assert len(made) == 1
        made[0].inject(HealthEvent(0, "gpu_pre_reset", True, "r"))
        assert [e.kind for e in a.poll(2000)] == ["gpu_pre_reset"]
        assert [e.kind for e in b.poll(2000)] == ["gpu_pre_reset"]
        assert a.poll(10) == []
    finally:
        a.close()
        assert not made[0].closed  # b still reads
        b.close()
    assert made[0].closed


def test_metrics_csv_xid_alias_is_supported():
    from amdgpu_operator.exporter.metrics import parse_metrics_csv

    sel, missing = parse_metrics_csv("DCGM_FI_DEV_XID_ERRORS, gauge, last XID\nDCGM_FI_DEV_ENC_UTIL, gauge, enc\n")
    assert [s.field for s in sel] == ["health_last_critical_code"] and missing == ["DCGM_FI_DEV_ENC_UTIL"]


def test_metrics_csv_selects_series_dcgm_names_kept():
    from amdgpu_operator.exporter.metrics import parse_metrics_csv

    csv = """# Format
# DCGM FIELD, Prometheus metric type, help message
DCGM_FI_DEV_GPU_UTIL,      gauge, GPU utilization (in %).
DCGM_FI_DEV_FB_USED,       gauge, Framebuffer memory used (in MiB).
DCGM_FI_DEV_ENC_UTIL,      gauge, Encoder utilization (in %).
amd_gpu_xgmi_read_bytes_total, counter,
"""
    sel, missing = parse_metrics_csv(csv)
    assert [x.name for x in sel] == ["DCGM_FI_DEV_GPU_UTIL", "DCGM_FI_DEV_FB_USED", "amd_gpu_xgmi_read_bytes_total"]
    assert missing == ["DCGM_FI_DEV_ENC_UTIL"]
    assert sel[1].scale == 1 / 2**20 and sel[0].help == "GPU utilization (in %)."
    assert sel[2].help  # empty help column falls back to the built-in one
    ex = MetricsExporter(FixtureSource(FIXTURE, gpus=2), "n", selection=sel)
    ex.collect_once()
    series = {ln.split("{")[0] for ln in ex.render().splitlines() if ln and not ln.startswith("#")}
    assert "DCGM_FI_DEV_GPU_UTIL" in series and "DCGM_FI_DEV_FB_USED" in series
    assert "amd_gpu_power_watts" not in series  # not selected


def test_pod_attribution_via_pod_resources_api(tmp_path):
    sock = str(tmp_path / "podres" / "kubelet.sock")
    k = FakeKubelet(str(tmp_path / "dp"), sock)
    k.start()
    try:
        k.assignments[("ml", "trainer-0", "main")] = ("amd.com/gpu", ["0000:72:00.0"])
        src = FixtureSource(FIXTURE, gpus=2)
        ex = MetricsExporter(src, "n", attribution=PodAttribution(sock))
        ex.collect_once()
        text = ex.render()
        assert 'pod="trainer-0"' in text and 'namespace="ml"' in text
    finally:
        k.stop()


def test_http_server_and_node_status(env):
    V.write_ready(env, "driver", {"seconds": 0.5})
    ns = NodeStatusExporter(env.validations_dir, "n1")
    srv = MetricsHttpServer(ns, "127.0.0.1", 0).start()
    try:
        body = urllib.request.urlopen(f"http://127.0.0.1:{srv.port}/metrics", timeout=5).read().decode()
        assert 'amd_gpu_operator_node_validation_ready{node="n1",step="driver"} 1' in body
        assert 'amd_gpu_operator_node_validation_ready{node="n1",step="plugin"} 0' in body
        assert 'amd_gpu_operator_node_validation_seconds{node="n1",step="driver"} 0.5' in body
        assert 'amd_gpu_operator_node_driver_lost{node="n1"} 0' in body
        assert urllib.request.urlopen(f"http://127.0.0.1:{srv.port}/healthz", timeout=5).read() == b"ok\n"
        from amdgpu_operator.driver import manager as DM

        os.unlink(os.path.join(env.host_root, "sys/module/amdgpu/initstate"))  # the driver goes away
        assert DM.monitor_once(env) is False
        body = urllib.request.urlopen(f"http://127.0.0.1:{srv.port}/metrics", timeout=5).read().decode()
        assert 'amd_gpu_operator_node_driver_lost{node="n1"} 1' in body
        assert 'amd_gpu_operator_node_validation_ready{node="n1",step="driver"} 0' in body
    finally:
        srv.stop()


# ---------------------------------------------------------------- validator

def test_driver_validation_and_wait(env):
    with pytest.raises(V.StepFailed):
        V.wait_ready(env, "driver", timeout=0.05)
    out = V.validate_driver(env, timeout=1)
    assert out["gpus"] == 2 and V.wait_ready(env, "driver", 1)["ok"]


def test_workload_validation_launch_plan(env):
    from amdgpu_operator.discovery import topology

    launched = []

    def launcher(argv, e, device, timeout):
        launched.append((argv, dict(e), device))
        steps = argv[argv.index("--steps") + 1].split(",")
        rep = {"ok": True, "rank": int(argv[argv.index("--rank") + 1]),
               "steps": [{"name": s, "ok": True, "seconds": 0.01} for s in steps]}
        return ProcResult(0, json.dumps(rep), "", 0.01)

    env.launcher = launcher
    gpus = topology.enumerate_gpus(env.host_root)
    out = V.validate_workload(env, ["--gemm", "1024", "--counter-gate"])
    assert out["ok"] and out["world"] == 2 and out["processes"] == 2 and out["process_mode"] == "shared"
    # one process per GPU: its kernel checks, the xGMI IPC step and RCCL
    assert len(launched) == 2
    for argv, e, device in launched:
        assert argv[argv.index("--steps") + 1] == ("hip,vecadd,gemm,gemm_fp8,gemm_fp4,gemm_fp6,gemm_mxfp4,mfma,hbm,"
                                                   "xgmi,rccl")
        assert argv[argv.index("--local-bdf") + 1] == gpus[device].bdf and "--counter-gate" in argv
        # it sees its own GPU first, then its peer (RCCL and IPC need the peer visible)
        assert e["ROCR_VISIBLE_DEVICES"].split(",")[0] == f"GPU-{gpus[device].unique_id:016x}"
        assert len(e["ROCR_VISIBLE_DEVICES"].split(",")) == 2
        assert "glibc.malloc.hugetlb=1" in e.get("GLIBC_TUNABLES", "")  # RCCL set-up on huge pages
        # the default AQL-packet gate needs no profiler tool in the process
        assert e.get("AMDGPU_VALIDATOR_COUNTERS") is None
    assert sorted(d for _, _, d in launched) == [0, 1]
    names = [s["name"] for s in out["ranks"][0]["steps"]]
    assert names == ["hip", "vecadd", "gemm", "gemm_fp8", "gemm_fp4", "gemm_fp6", "gemm_mxfp4", "mfma", "hbm", "xgmi",
                     "rccl"]
    assert V.read_ready(env, "workload")["world"] == 2

    def reset():
        launched.clear()
        for f in os.listdir(env.validations_dir):
            if f.endswith("-ready"):
                os.unlink(os.path.join(env.validations_dir, f))

    reset()
    V.validate_workload(env, ["--gemm", "1024", "--counter-gate", "--gate-mode", "sdk"])
    assert launched and all(e.get("AMDGPU_VALIDATOR_COUNTERS") == "1" and "libamdgpu_counter_gate.so" in
                            e.get("ROCP_TOOL_LIBRARIES", "") for _, e, _ in launched)
    # rcclProcess: separate - kernel checks see only their own GPU; the xGMI IPC
    # step and RCCL run in a second process per GPU, which sees every GPU
    reset()
    out = V.validate_workload(env, ["--gemm", "1024", "--counter-gate", "--rccl-separate-process"])
    assert out["process_mode"] == "separate" and out["processes"] == 4
    kernel = [(a, e) for a, e, _ in launched if "rccl" not in a[a.index("--steps") + 1]]
    rccl = [(a, e) for a, e, _ in launched if a[a.index("--steps") + 1] == "hip,xgmi,rccl"]
    assert len(kernel) == 2 and len(rccl) == 2
    assert all(len(e["ROCR_VISIBLE_DEVICES"].split(",")) == 1 for _, e in kernel)
    assert all(len(e["ROCR_VISIBLE_DEVICES"].split(",")) == 2 for _, e in rccl)
    assert all("--counter-gate" in a for a, _ in kernel) and not any("--counter-gate" in a for a, _ in rccl)
    names = [s["name"] for s in out["ranks"][0]["steps"]]
    assert names == ["hip", "vecadd", "gemm", "gemm_fp8", "gemm_fp4", "gemm_fp6", "gemm_mxfp4", "mfma", "hbm", "xgmi",
                     "rccl"]


def test_workload_failure_is_reported(env):
    env.launcher = lambda argv, e, d, t: ProcResult(1, json.dumps({"ok": False, "error": "Freivalds 1e-1"}), "boom", 0.1)
    with pytest.raises(V.StepFailed, match="Freivalds"):
        V.validate_workload(env, [])
    assert V.read_ready(env, "workload") is None


def test_single_gpu_skips_rccl(tmp_path):
    root = str(tmp_path / "h1")
    fakesys.build_node(root, 1)
    env = NodeEnv("n1", None, host_root=root, validations_dir=str(tmp_path / "v"), poll_s=0.01)
    seen = []

    def launcher(argv, e, device, timeout):
        seen.append(argv[argv.index("--steps") + 1])
        return ProcResult(0, json.dumps({"ok": True, "steps": []}), "", 0.0)

    env.launcher = launcher
    out = V.validate_workload(env, [])
    assert seen == ["hip,vecadd,gemm,gemm_fp8,gemm_fp4,gemm_fp6,gemm_mxfp4,mfma,hbm,xgmi"]
    assert out["ranks"][0]["steps"][-1]["skipped"].startswith("single GPU")


def test_complete_labels_node(env):
    V.write_ready(env, "driver", {"seconds": 0.1})
    V.complete(env)
    node = env.client.get("v1", "Node", "n1")
    assert node["metadata"]["labels"][V.VALIDATED_LABEL] == "true"
    assert json.loads(node["metadata"]["annotations"]["amd.com/gpu.validation"])["driver"] == 0.1
    assert V.MFMA_LABEL not in node["metadata"]["labels"]  # no probe results: no claim


def test_complete_publishes_mfma_types_confirmed_on_every_gpu(env):
    def rank(dtypes):
        return {"steps": [{"name": "hip", "ok": True}, {"name": "mfma", "ok": True, "dtypes": dtypes}]}

    V.write_ready(env, "workload", {"ranks": [rank({"f16": True, "bf16": True, "mxfp4": True, "f64": True}),
                                              rank({"f16": True, "bf16": True, "mxfp4": False, "f64": True})]})
    out = V.complete(env)
    assert out["mfma_dtypes"] == ["f16", "bf16", "f64"]
    labels = env.client.get("v1", "Node", "n1")["metadata"]["labels"]
    assert labels[V.MFMA_LABEL] == "f16.bf16.f64"
    assert V.validated_mfma_dtypes({"ranks": [{"steps": [{"name": "hip"}]}]}) == []


def test_complete_publishes_the_validated_mfma_rates(env):
    """amd.com/gpu.validated.mfma-rate: the GEMM data types whose step held a
    TF/s floor on every device of every rank; a report-only run (floor 0) or
    one device short of its floor claims nothing, and a stale claim is taken
    off the node."""
    def rank(*gemms):
        return {"steps": [{"name": "hip", "ok": True}, *gemms]}

    bf16 = {"name": "gemm", "ok": True, "tflops": 1450.0, "min_tflops": 620.0}
    fp8 = {"name": "gemm_fp8", "ok": True, "tflops": 2900.0, "min_tflops": 1200.0}
    fp4 = {"name": "gemm_fp4", "ok": True, "tflops": 4200.0, "min_tflops": 1900.0}
    V.write_ready(env, "workload", {"ranks": [rank(bf16, fp8, fp4), rank(bf16, {**fp8, "device": 1}, fp4)]})
    assert V.complete(env)["mfma_rate_dtypes"] == ["bf16", "fp8", "fp4"]
    assert env.client.get("v1", "Node", "n1")["metadata"]["labels"][V.MFMA_RATE_LABEL] == "bf16.fp8.fp4"
    V.write_ready(env, "workload", {"ranks": [rank(bf16, fp8), rank(bf16, {**fp8, "min_tflops": 0.0})]})
    assert V.complete(env)["mfma_rate_dtypes"] == ["bf16"]
    V.write_ready(env, "workload", {"ranks": [rank({**bf16, "ok": False}, fp8, {**fp4, "ok": False})]})
    assert V.complete(env)["mfma_rate_dtypes"] == ["fp8"]
    V.write_ready(env, "workload", {"ranks": [rank({**bf16, "min_tflops": 0.0})]})
    assert V.complete(env)["mfma_rate_dtypes"] == []
    assert V.MFMA_RATE_LABEL not in env.client.get("v1", "Node", "n1")["metadata"]["labels"]
    # round 6: fp6 and block-scaled MXFP4; a rate the gate was asked to count but did not
    # (the sdk-mode gate counts bf16 only: "not_counted") is not claimed
    fp6 = {"name": "gemm_fp6", "ok": True, "tflops": 3500.0, "min_tflops": 2540.0, "counter_gate": "pass"}
    mx = {"name": "gemm_mxfp4", "ok": True, "tflops": 3900.0, "min_tflops": 2830.0, "counter_gate": "pass"}
    V.write_ready(env, "workload", {"ranks": [rank(bf16, fp8, fp4, fp6, mx)]})
    assert V.complete(env)["mfma_rate_dtypes"] == ["bf16", "fp8", "fp4", "fp6", "mxfp4"]
    assert env.client.get("v1", "Node", "n1")["metadata"]["labels"][V.MFMA_RATE_LABEL] == "bf16.fp8.fp4.fp6.mxfp4"
    V.write_ready(env, "workload", {"ranks": [rank({**bf16, "counter_gate": "pass"},
                                                   {**fp8, "counter_gate": "not_counted"}, fp6)]})
    assert V.complete(env)["mfma_rate_dtypes"] == ["bf16", "fp6"]


def test_mfma_rate_check_flags_reach_the_validator(tmp_path):
    """validator.workload.mfmaRateCheck / mfmaRateGemmN / minFp8Tflops /
    minFp4Tflops become the binary's --fp8-gemm / --fp4-gemm / --min-fp8-tflops /
    --min-fp4-tflops; switched off, the gemm_fp8 and gemm_fp4 steps are
    dropped from the run (and their floors are not passed)."""
    from amdgpu_operator.api.clusterpolicy import REFERENCE_SET_FLAGS, ClusterPolicySpec, deep_merge, parse_set_flags
    from amdgpu_operator.controller import manifests as M

    ref = parse_set_flags(REFERENCE_SET_FLAGS)

    def args(values):
        ds = [o for o in M.state_validator(ClusterPolicySpec.model_validate(values), "ns", None)
              if o["kind"] == "DaemonSet"][0]
        return ds["spec"]["template"]["spec"]["containers"][0]["args"]

    on = args(ref)
    assert on[on.index("--fp8-gemm") + 1] == on[on.index("--fp4-gemm") + 1] == "4096"
    assert on[on.index("--min-fp8-tflops") + 1] == "1940" and on[on.index("--min-fp4-tflops") + 1] == "3100"
    assert on[on.index("--min-fp6-tflops") + 1] == "2540" and on[on.index("--min-mxfp4-tflops") + 1] == "2830"
    assert on[on.index("--min-mfma-util") + 1] == "0.44"
    assert on[on.index("--min-mfma-util-by-dtype") + 1] == "fp4=0.21,fp6=0.2,fp8=0.33,mxfp4=0.2"
    off = args(deep_merge(ref, {"validator": {"workload": {"mfmaRateCheck": False}}}))
    assert "--no-mfma-rate" in off and not {"--min-fp8-tflops", "--min-fp4-tflops", "--fp8-gemm", "--min-fp6-tflops",
                                            "--min-mxfp4-tflops", "--min-mfma-util-by-dtype"} & set(off)
    # counted dispatches inline by default; deferGates queues them after the kernel steps
    assert "--defer-gates" not in on
    assert "--defer-gates" in args(deep_merge(ref, {"validator": {"workload": {"deferGates": True}}}))

    root = str(tmp_path / "h1")
    fakesys.build_node(root, 1)
    venv = NodeEnv("n1", None, host_root=root, validations_dir=str(tmp_path / "v"), poll_s=0.01)
    seen = []

    def launcher(argv, e, device, timeout):
        seen.append(argv)
        return ProcResult(0, json.dumps({"ok": True, "steps": []}), "", 0.0)

    venv.launcher = launcher
    V.validate_workload(venv, ["--no-mfma-rate", "--fp8-gemm", "8192"])
    assert seen[0][seen[0].index("--steps") + 1] == "hip,vecadd,gemm,mfma,hbm,xgmi"
    assert "--no-mfma-rate" not in seen[0]


# ------------------------------------------------------------------ CLI

def test_operand_parser_passthrough():
    from amdgpu_operator.cli.operands import _split_passthrough, build_parser

    known, extra = _split_passthrough(["plugin", "--resource", "amd.com/gpu", "--gemm", "4096", "--counter-gate"])
    assert known == ["plugin", "--resource", "amd.com/gpu"] and extra == ["--gemm", "4096", "--counter-gate"]
    a = build_parser().parse_args(["device-plugin", "--partition-strategy", "mixed"])
    assert a.partition_strategy == "mixed"


def test_cli_render(capsys):
    from amdgpu_operator.cli.main import main

    assert main(["render", "--set", "operator.cleanupCRD=true"]) == 0
    out = capsys.readouterr().out
    assert "kind: ClusterPolicy" in out and "amd-gpu-operator-cleanup-crd" in out


def test_cli_verify_against_http_apiserver(tmp_path, capsys):
    from amdgpu_operator.cli.main import main
    from amdgpu_operator.kube.httpapi import HttpApiServer

    api = FakeApiServer()
    srv = HttpApiServer(api).start()
    try:
        assert main(["verify", "--server", srv.url, "--json"]) == 1  # nothing installed
        rep = json.loads(capsys.readouterr().out)
        assert rep["ok"] is False and any(c["name"] == "gpu-nodes-labelled" for c in rep["checks"])
    finally:
        srv.stop()


def test_gpu_validation_overlaps_workload_with_toolkit_install(env):
    """The workload needs only the driver; plugin pods wait for the toolkit."""
    seen_toolkit = []

    def launcher(argv, e, device, timeout):
        seen_toolkit.append(V.read_ready(env, "toolkit"))
        steps = argv[argv.index("--steps") + 1].split(",")
        return ProcResult(0, json.dumps({"ok": True, "steps": [{"name": s, "ok": True} for s in steps]}), "", 0.0)

    env.launcher = launcher
    with pytest.raises(V.StepFailed, match="toolkit"):
        V.validate_gpu(env, [], timeout=0.3, wait_toolkit=True)
    assert seen_toolkit and all(t is None for t in seen_toolkit)
    assert V.read_ready(env, "workload")["ok"] and V.read_ready(env, "plugin") is None


def _gated_launcher(env, log):
    """Stand-in validator honouring --start-gate: records when it was spawned
    and what the gate said, like amdgpu-validator does before its first HIP call."""
    from amdgpu_operator.testing.fake_validator import wait_start_gate

    def launcher(argv, e, device, timeout):
        gate = argv[argv.index("--start-gate") + 1] if "--start-gate" in argv else None
        log.append(("spawn", V.read_ready(env, "driver") is not None))
        verdict = wait_start_gate(gate, 5)
        log.append(("gate", verdict))
        if verdict != "go":
            return ProcResult(3, json.dumps({"ok": False, "error": f"start gate: {verdict}"}), "", 0.0)
        steps = argv[argv.index("--steps") + 1].split(",")
        return ProcResult(0, json.dumps({"ok": True, "steps": [{"name": s, "ok": True} for s in steps]}), "", 0.0)

    return launcher


def test_prespawned_workload_waits_for_driver_validation(env):
    """with_driver: the validator processes start before the driver is ready,
    and are released only after the driver validation passed."""
    import threading
    import time as _t

    log = []
    env.launcher = _gated_launcher(env, log)
    for f in os.listdir(env.validations_dir) if os.path.isdir(env.validations_dir) else []:
        os.unlink(os.path.join(env.validations_dir, f))

    def driver_comes_up():
        _t.sleep(0.2)
        V.write_ready(env, "driver", {"ok": True})

    th = threading.Thread(target=driver_comes_up)
    th.start()
    with pytest.raises(V.StepFailed, match="plugin"):  # no device plugin here: only the plugin step fails
        V.validate_gpu(env, [], timeout=0.6, with_driver=True)
    th.join()
    spawns = [x for x in log if x[0] == "spawn"]
    assert spawns and all(ready is False for _, ready in spawns)  # spawned before the driver was ready
    assert [x for x in log if x[0] == "gate"] == [("gate", "go")] * len(spawns)
    assert V.read_ready(env, "workload")["ok"]
    assert not [f for f in os.listdir(env.validations_dir) if f.startswith(".start-gate")]  # gate file removed


def test_prespawned_workload_aborts_when_the_driver_fails(env, monkeypatch):
    log = []
    env.launcher = _gated_launcher(env, log)
    monkeypatch.setattr(V, "validate_driver", lambda *a, **k: (_ for _ in ()).throw(V.StepFailed("no kfd")))
    V.write_ready(env, "driver", {"ok": True})
    with pytest.raises(V.StepFailed, match="driver: no kfd"):
        V.validate_gpu(env, [], timeout=1, with_driver=True)
    assert ("gate", "abort") in log and V.read_ready(env, "workload") is None


def test_validator_manifest_prespawn():
    from amdgpu_operator.api.clusterpolicy import REFERENCE_SET_FLAGS, ClusterPolicySpec, deep_merge, parse_set_flags
    from amdgpu_operator.controller import manifests as M

    ref = parse_set_flags(REFERENCE_SET_FLAGS)

    def inits(values):
        ds = [o for o in M.state_validator(ClusterPolicySpec.model_validate(values), "ns", None)
              if o["kind"] == "DaemonSet"][0]
        return [(c["name"], c["args"]) for c in ds["spec"]["template"]["spec"]["initContainers"]]

    init_layout = deep_merge(ref, {"daemonsets": {"inContainerGates": False}})
    on = inits(init_layout)
    assert [n for n, _ in on] == ["gpu-validation"] and "--with-driver" in on[0][1]
    off = inits(deep_merge(init_layout, {"validator": {"workload": {"prespawn": False}}}))
    assert [n for n, _ in off] == ["driver-validation", "gpu-validation"] and "--with-driver" not in off[1][1]
    # default (in-container gates): the main container validates, then completes - no init container
    assert inits(ref) == []
    ds = [o for o in M.state_validator(ClusterPolicySpec.model_validate(ref), "ns", None) if o["kind"] == "DaemonSet"][0]
    main = ds["spec"]["template"]["spec"]["containers"][0]
    assert main["args"][:2] == ["validate", "gpu"] and "--with-driver" in main["args"] and main["args"][-1] == "--complete"


def test_in_container_gates_replace_the_init_containers():
    """Default layout: no operand pod has a waiting init container; each
    operand container carries its gate, and the driver container runs the
    upgrade check itself."""
    from amdgpu_operator.api.clusterpolicy import REFERENCE_SET_FLAGS, ClusterPolicySpec, parse_set_flags
    from amdgpu_operator.controller import manifests as M

    spec = ClusterPolicySpec.model_validate(parse_set_flags(REFERENCE_SET_FLAGS))
    gates = {}
    for state, builder in M.STATE_BUILDERS.items():
        for o in builder(spec, "ns", None):
            if o["kind"] != "DaemonSet":
                continue
            pod = o["spec"]["template"]["spec"]
            if o["metadata"]["name"].startswith(("amd-sandbox", "amd-vfio")):
                continue  # VM-passthrough operands (off by default) keep the init-container layout
            assert pod["initContainers"] == [], o["metadata"]["name"]
            for c in pod["containers"]:
                env = {e["name"]: e.get("value") for e in c["env"]}
                if "VALIDATION_GATE" in env:
                    gates[c["name"]] = env["VALIDATION_GATE"]
    assert gates == {"amd-container-toolkit-ctr": "driver", "amd-device-plugin": "toolkit",
                     "amd-metrics-exporter": "driver", "gpu-feature-discovery": "driver", "amd-partition-manager": "driver",
                     "amd-dra-driver": "toolkit"}  # the DRA driver's DaemonSet is built whether or not it is enabled
    drv = [o for o in M.state_driver(spec, "ns", None) if o["kind"] == "DaemonSet"][0]
    ctr = drv["spec"]["template"]["spec"]["containers"][0]
    assert ctr["args"][:3] == ["driver", "install", "--prepare-upgrade"]
    assert {"DRAIN_ENABLED", "DRAIN_TIMEOUT_SECONDS"} <= {e["name"] for e in ctr["env"]}


def test_no_prespawn_while_the_driver_is_not_live_or_upgrading(env):
    """Early processes would open /dev/kfd before their gate (the counter-gate
    tool starts the HSA runtime at load): not before the module is live, not
    during a driver upgrade - then they are spawned after the validation."""
    from amdgpu_operator.controller.upgrade import POD_RESTART, STATE_LABEL

    assert V.prespawn_safe(env, sdk_gate=True)
    env.client.patch("v1", "Node", "n1", {"metadata": {"labels": {STATE_LABEL: POD_RESTART}}})
    assert not V.prespawn_safe(env, sdk_gate=True)
    assert V.prespawn_safe(env)  # the AQL gate opens nothing before the start gate
    log = []
    env.launcher = _gated_launcher(env, log)
    V.write_ready(env, "driver", {"ok": True})
    with pytest.raises(V.StepFailed, match="plugin"):
        V.validate_gpu(env, ["--counter-gate", "--gate-mode", "sdk"], timeout=0.5, with_driver=True)
    spawns = [x for x in log if x[0] == "spawn"]
    assert spawns and all(ready for _, ready in spawns)  # after the driver validation
    env.client.patch("v1", "Node", "n1", {"metadata": {"labels": {STATE_LABEL: None}}})
    os.unlink(os.path.join(env.sysfs_root(), "dev/kfd"))
    assert not V.prespawn_safe(env, sdk_gate=True) and V.prespawn_safe(env)


def test_driver_change_aborts_waiting_start_gates(env):
    from amdgpu_operator.driver import manager as DM

    os.makedirs(env.validations_dir, exist_ok=True)
    waiting = os.path.join(env.validations_dir, V.START_GATE_PREFIX + "a")
    released = os.path.join(env.validations_dir, V.START_GATE_PREFIX + "b")
    starting = os.path.join(env.validations_dir, V.START_GATE_PREFIX + "c")  # runtime starting, kernels waiting
    open(waiting, "w").close()
    with open(released, "w") as f:
        f.write("go")
    with open(starting, "w") as f:
        f.write("init")
    env.extra["kmod"] = fakesys.SimModule(env.sysfs_root())
    out = DM.prepare_upgrade(env, "9.9.9", drain_timeout=0.1)
    assert out["unloaded"]
    assert open(waiting).read() == "abort" and open(released).read() == "go" and open(starting).read() == "abort"


def test_driver_change_waits_for_aborted_validators_to_exit(env):
    """an aborted validator may be in its HIP start ("init") when
    the driver reloads; the driver container waits until the process has
    exited (its ``<gate>.held`` lock is free) instead of a fixed pause."""
    import subprocess
    import sys
    import time

    from amdgpu_operator.driver import manager as DM

    os.makedirs(env.validations_dir, exist_ok=True)
    gate = os.path.join(env.validations_dir, V.START_GATE_PREFIX + "slow")
    with open(gate, "w") as f:
        f.write("init")
    # a process in its "runtime start": holds the lock, reacts to the abort only after 0.6 s
    child = ("import fcntl,sys,time\nf=open(sys.argv[1]+'.held','a');fcntl.flock(f,fcntl.LOCK_EX)\n"
             "print('up',flush=True)\nwhile open(sys.argv[1]).read().strip()!='abort': time.sleep(0.001)\n"
             "time.sleep(0.6)\n")
    p = subprocess.Popen([sys.executable, "-c", child, gate], stdout=subprocess.PIPE, text=True)
    assert p.stdout.readline().strip() == "up"
    t0 = time.monotonic()
    aborted = DM._release_gated_validators(env)
    waited = time.monotonic() - t0
    assert aborted == [V.START_GATE_PREFIX + "slow"] and 0.55 < waited < 4.0
    assert p.wait(timeout=5) == 0
    # nothing to abort: no wait at all
    t0 = time.monotonic()
    assert DM._release_gated_validators(env) == [] and time.monotonic() - t0 < 0.05


def test_kfd_settled_waits_out_exited_processes(env):
    """A KFD process entry whose PID is gone is a teardown under way: the
    module still counts it; the wait ends when the entry goes."""
    import threading
    import time

    from amdgpu_operator.driver import manager as DM

    kp = os.path.join(env.sysfs_root(), "sys/class/kfd/kfd/proc")
    os.makedirs(kp, exist_ok=True)
    os.makedirs(os.path.join(env.sysfs_root(), "proc", "4242"), exist_ok=True)
    os.makedirs(os.path.join(kp, "4242"))  # alive
    os.makedirs(os.path.join(kp, "999999"))  # exited, being torn down
    threading.Timer(0.2, lambda: os.rmdir(os.path.join(kp, "999999"))).start()
    t0 = time.monotonic()
    assert DM.wait_kfd_settled(env, time.monotonic() + 3) and 0.15 < time.monotonic() - t0 < 2
    os.makedirs(os.path.join(kp, "999998"))
    assert not DM.wait_kfd_settled(env, time.monotonic() + 0.05)


def test_cli_simulate_two_nodes_over_http(capsys):
    from amdgpu_operator.cli.main import main

    assert main(["simulate", "--gpus", "2", "--nodes", "2", "--http-api", "--timeout", "90"]) == 0
    out = json.loads(capsys.readouterr().out)
    assert out["nodes"] == 2 and out["http_api"] and out["verify"]["ok"]


def test_gfd_labels_describe_every_gpu_of_a_mixed_node(tmp_path):
    """A node whose GPUs sit in different partition modes is labelled from
    all of them (round 2 labelled it from the first GPU only): shared values
    as before, differing ones `mixed`, sizes the minimum, and per-mode
    counts that match the device plugin's `mixed` resources."""
    from amdgpu_operator.utils import record

    fakesys.build_node(str(tmp_path / "a"), 1, "SPX", "NPS1")
    fakesys.build_node(str(tmp_path / "b"), 1, "CPX", "NPS2")
    spx, cpx = T.enumerate_gpus(str(tmp_path / "a")), T.enumerate_gpus(str(tmp_path / "b"))
    cpx = [record.replace(g, physical_index=1) for g in cpx]
    lab = L.gfd_labels(spx + cpx, str(tmp_path / "a"))
    assert lab["amd.com/gpu.count"] == str(1 + len(cpx)) and lab["amd.com/gpu.physical-count"] == "2"
    assert lab["amd.com/gpu.compute-partition"] == "mixed" and lab["amd.com/gpu.memory-partition"] == "mixed"
    assert lab["amd.com/gpu.product"] == "AMD-Instinct-MI355X"  # one SKU
    assert lab["amd.com/gpu.spx.count"] == "1" and lab["amd.com/gpu.cpx.count"] == str(len(cpx))
    assert int(lab["amd.com/gpu.cpx.compute-units"]) == min(g.cu_count for g in cpx) < int(lab["amd.com/gpu.spx.compute-units"])
    assert lab["amd.com/gpu.compute-units"] == lab["amd.com/gpu.cpx.compute-units"]  # the minimum over devices
    assert int(lab["amd.com/gpu.memory"]) == min(g.vram_bytes for g in spx + cpx) // 2**20
    # the plugin's mixed strategy: amd.com/gpu for SPX, amd.com/gpu-cpx for the partitions
    res = {T.partition_resource(g, "amd.com/gpu", "mixed") for g in spx + cpx}
    assert res == {"amd.com/gpu", "amd.com/gpu-cpx"}
    # mixed SKUs: per-product counts, MFMA types only where all have them
    mi300 = [record.replace(spx[0], device_id=0x74A1, arch="gfx942", physical_index=2)]
    lab = L.gfd_labels(spx + mi300, str(tmp_path / "a"))
    assert lab["amd.com/gpu.product"] == "mixed" and lab["amd.com/gpu.family"] == "mixed"
    assert lab["amd.com/gpu.product.AMD-Instinct-MI355X.count"] == "1"
    assert lab["amd.com/gpu.product.AMD-Instinct-MI300X.count"] == "1"
    assert lab["amd.com/gpu.mfma.fp4"] == "false" and lab["amd.com/gpu.mfma.bf16"] == "true"
    for k, v in lab.items():
        assert len(k.split("/", 1)[1]) <= 63 and len(v) <= 63, (k, v)


@pytest.mark.parametrize("flags", [[], ["draDriver.enabled=true", "devicePlugin.enabled=false", "driver.rdma.enabled=true",
                                        "sandboxWorkloads.enabled=true", "migManager.enabled=true"]])
def test_every_rendered_container_command_parses(flags):
    """Every container the operator renders runs ``amdgpu-operator <cmd>``
    with a command the entry point dispatches (cli/main.py OPERAND_CMDS or
    its own sub-commands) and arguments its parser accepts - the image's
    entry point, not only the in-process operand runner, must know them."""
    from amdgpu_operator.api.clusterpolicy import REFERENCE_SET_FLAGS, parse_set_flags, spec_from_values
    from amdgpu_operator.cli import main as M
    from amdgpu_operator.cli.operands import _split_passthrough, build_parser
    from amdgpu_operator.controller import manifests as MF

    spec = spec_from_values(parse_set_flags(REFERENCE_SET_FLAGS + flags))
    seen = set()
    for builder in MF.STATE_BUILDERS.values():
        for o in builder(spec, "ns", None):
            if o.get("kind") not in ("DaemonSet", "Deployment", "Job"):
                continue
            tmpl = o["spec"]["template"]["spec"]
            for c in tmpl.get("initContainers", []) + tmpl["containers"]:
                if c.get("command") != ["amdgpu-operator"]:
                    continue
                args = list(c["args"])
                assert args[0] in M.OPERAND_CMDS, (o["metadata"]["name"], args[0])
                if args[0] == "validate":
                    known, _ = _split_passthrough(args[1:])
                    build_parser().parse_args(["validate", *known])
                else:
                    build_parser().parse_args(args)
                seen.add(args[0])
    assert {"driver", "validate"} <= seen
    if flags:
        assert "dra-driver" in seen


def test_operands_start_without_site(tmp_path):
    """Operand containers run `python3 -S -m amdgpu_operator` (the images'
    entry script, the simulated kubelet): each operand's modules load from
    the package alone - no site-packages module on the start-up path - and
    the -S fallback still finds installed packages for the ones that want
    them later (yaml for config files)."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys, runpy\n"
            "import amdgpu_operator.cli.main, amdgpu_operator.cli.operands, amdgpu_operator.validator.validate\n"
            "import amdgpu_operator.deviceplugin.server, amdgpu_operator.driver.manager, amdgpu_operator.toolkit.install\n"
            "import amdgpu_operator.exporter.metrics\n"
            "third = sorted({m.split('.')[0] for m in sys.modules} & {'yaml', 'pydantic', 'numpy', 'torch', 'grpc', "
            "'requests', 'certifi', 'pydantic_core'})\n"
            "print(third)\n")
    p = subprocess.run([sys.executable, "-S", "-c", code], env={**os.environ, "PYTHONPATH": root},
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]
    assert p.stdout.strip() == "[]"
    p = subprocess.run([sys.executable, "-S", "-m", "amdgpu_operator", "render", "--help"],
                       env={**os.environ, "PYTHONPATH": root}, capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]
    with open(os.path.join(root, "deploy", "images", "amd-device-plugin", "Dockerfile")) as f:
        assert "exec python3 -S -m amdgpu_operator" in f.read()
