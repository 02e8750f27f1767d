"""N7 gate lock (native/include/gate_lock.h) on the CPU: the per-GPU lock the
counter gate holds exclusively around its counted dispatch and the operator's
other GPU work (plugin-validation pod, RCCL processes) holds shared.  Driven
through ``amdgpu-validator --gate-lock-probe`` (no GPU involved) against
Python's flock on the same file: the two are one lock."""

import fcntl
import json
import os
import subprocess
import time

import pytest

from amdgpu_operator import native

BIN = os.path.join(os.path.dirname(native.__file__), "_native", "amdgpu-validator")


def probe(lock_dir, mode, timeout=0.3, hold=0.0, bdf="0000:75:00.0", background=False):
    argv = [BIN, "--gate-lock-probe", f"{bdf},{mode},{timeout},{hold}"]
    env = dict(os.environ, AMDGPU_GATE_LOCK_DIR=str(lock_dir))
    if background:
        return subprocess.Popen(argv, env=env, stdout=subprocess.PIPE, text=True)
    p = subprocess.run(argv, env=env, capture_output=True, text=True, timeout=30)
    return p.returncode, json.loads(p.stdout)


@pytest.fixture()
def lock_dir(tmp_path):
    if not os.path.exists(BIN):
        pytest.fail(f"{BIN} not built (make -C native)")
    return tmp_path


def hold(lock_dir, how, bdf="0000:75:00.0"):
    f = open(os.path.join(lock_dir, "gate-" + bdf.lower().replace(":", "-").replace(".", "-") + ".lock"), "a+")
    fcntl.flock(f, how)
    return f


def test_lock_file_is_named_by_the_gpu(lock_dir):
    rc, out = probe(lock_dir, "ex", bdf="0000:F5:00.0")
    assert rc == 0 and out["state"] == "held" and out["file"] == "gate-0000-f5-00-0.lock"
    assert os.path.exists(lock_dir / "gate-0000-f5-00-0.lock")


def test_exclusive_waits_for_a_shared_holder_and_gives_up_at_its_bound(lock_dir):
    f = hold(lock_dir, fcntl.LOCK_SH)
    try:
        t0 = time.monotonic()
        rc, out = probe(lock_dir, "ex", timeout=0.3)
        assert rc == 1 and out["state"] == "timeout" and 0.3 <= out["wait_s"] < 2.0
        assert time.monotonic() - t0 < 5
        rc, out = probe(lock_dir, "sh")  # co-workers share it
        assert rc == 0 and out["state"] == "held" and out["wait_s"] < 0.1
    finally:
        f.close()
    rc, out = probe(lock_dir, "ex")
    assert rc == 0 and out["state"] == "held"


def test_exclusive_gets_the_lock_once_the_shared_holder_lets_go(lock_dir):
    f = hold(lock_dir, fcntl.LOCK_SH)
    p = probe(lock_dir, "ex", timeout=5.0, background=True)
    time.sleep(0.3)
    f.close()
    out = json.loads(p.communicate(timeout=30)[0])
    assert p.returncode == 0 and out["state"] == "held" and 0.25 <= out["wait_s"] < 2.0


def test_shared_waits_while_a_gate_counts(lock_dir):
    gate = probe(lock_dir, "ex", hold=0.4, background=True)
    time.sleep(0.15)
    rc, out = probe(lock_dir, "sh", timeout=3.0)
    assert rc == 0 and out["state"] == "held" and out["wait_s"] >= 0.1
    gate.communicate(timeout=30)


def test_other_gpus_do_not_contend(lock_dir):
    f = hold(lock_dir, fcntl.LOCK_EX, bdf="0000:75:00.0")
    try:
        rc, out = probe(lock_dir, "ex", bdf="0000:05:00.0")
        assert rc == 0 and out["state"] == "held" and out["wait_s"] < 0.1
    finally:
        f.close()


def test_no_lock_dir_means_no_locking(tmp_path):
    p = subprocess.run([BIN, "--gate-lock-probe", "0000:75:00.0,ex,0.1,0"], capture_output=True, text=True,
                       env={k: v for k, v in os.environ.items() if k != "AMDGPU_GATE_LOCK_DIR"}, timeout=30)
    assert p.returncode == 0 and json.loads(p.stdout)["state"] == "off"


def test_validator_processes_and_plugin_pods_get_the_lock_dir(tmp_path):
    """validate.py hands every validator process and the plugin-validation
    pod the same lock directory (the pod-results hostPath the pod mounts)."""
    from amdgpu_operator.nodeenv import NodeEnv
    from amdgpu_operator.validator import validate as V

    env = NodeEnv("n", None, host_root=str(tmp_path), validations_dir=str(tmp_path / "v"))
    d = V.gate_lock_env(env)[V.GATE_LOCK_ENV]
    assert d == os.path.join(str(tmp_path / "v"), V.POD_RESULTS) and os.path.isdir(d)
    pod = {"metadata": {"name": "p"}, "spec": {"containers": [{"name": "c", "args": []}]}}
    pod = V._with_result_file(env, pod, "--result-file")
    ctr = pod["spec"]["containers"][0]
    assert {"name": V.GATE_LOCK_ENV, "value": d} in ctr["env"]
    assert any(m["mountPath"] == d for m in ctr["volumeMounts"])
