"""Bounded failure of multi-rank validator runs (N >= 2), on the CPU.

The native ``amdgpu-validator`` keeps a liveness record per rank in the
run's rendezvous directory and watches its peers' while it waits on them
(validator_main.cpp Rendezvous); its ``peers`` step waits for every rank
before any GPU call, so the protocol runs here without a GPU.  The RCCL
set-up path that uses the same watch (ncclCommInitRank on its own thread,
abandoned when a peer cannot arrive) is covered on the MI355X in
tests/test_validator_multirank_gpu.py.

validate_workload's sibling cancellation (the abort file) runs with the
stand-in validator (testing/fake_validator.py, same protocol) and injected
faults."""

import json
import os
import signal
import subprocess
import sys
import time

import pytest

from amdgpu_operator import native
from amdgpu_operator.nodeenv import NodeEnv, ProcResult, run_local
from amdgpu_operator.testing import fakesys
from amdgpu_operator.validator import validate as V

VALIDATOR = str(native.binary("amdgpu-validator"))


def _rank(rdv, rank, world=2, extra=(), **kw):
    return subprocess.Popen([VALIDATOR, "--rank", str(rank), "--world", str(world), "--rendezvous", str(rdv),
                             "--run-id", "t", "--steps", "peers", *extra],
                            stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, **kw)


def _report(p, timeout=20):
    out, err = p.communicate(timeout=timeout)
    return p.returncode, json.loads(out.strip().splitlines()[-1])


def test_rank_never_started_is_named_within_the_peer_timeout(tmp_path):
    t0 = time.monotonic()
    rc, rep = _report(_rank(tmp_path, 0, extra=["--peer-timeout", "1"]))
    took = time.monotonic() - t0
    assert rc == 1 and not rep["ok"]
    assert rep["failed_peer"] == 1 and rep["peer_state"] == "missing"
    assert "rank 1 never started" in rep["error"]
    assert 0.9 < took < 5
    # its own failure is published for its siblings
    assert (tmp_path / "t-failed-0").read_text().startswith("rank 1 never started")


def test_rank_killed_after_publishing_is_named_at_once(tmp_path):
    gate = tmp_path / "gate"
    gate.write_text("")  # rank 1 waits at its start gate: alive, published
    r1 = _rank(tmp_path, 1, extra=["--start-gate", str(gate)])
    deadline = time.monotonic() + 10
    while not (tmp_path / "t-alive-1").exists():
        assert time.monotonic() < deadline
        time.sleep(0.01)
    r1.kill()
    r1.wait()
    t0 = time.monotonic()
    rc, rep = _report(_rank(tmp_path, 0, extra=["--peer-timeout", "60"]))
    assert time.monotonic() - t0 < 3  # not the 60 s peer timeout
    assert rc == 1 and rep["failed_peer"] == 1 and rep["peer_state"] == "dead"
    assert f"pid {r1.pid}" in rep["error"]


def test_zombie_peer_counts_as_dead(tmp_path):
    gate = tmp_path / "gate"
    gate.write_text("")
    r1 = _rank(tmp_path, 1, extra=["--start-gate", str(gate)])
    while not (tmp_path / "t-alive-1").exists():
        time.sleep(0.01)
    os.kill(r1.pid, signal.SIGKILL)
    time.sleep(0.2)  # not reaped yet: a zombie still has a /proc entry
    rc, rep = _report(_rank(tmp_path, 0, extra=["--peer-timeout", "60"]))
    r1.wait()
    assert rc == 1 and rep["peer_state"] == "dead"


def test_failed_peer_and_orchestrator_abort(tmp_path):
    (tmp_path / "t-failed-1").write_text("gemm: Freivalds 1e-1")
    rc, rep = _report(_rank(tmp_path, 0, extra=["--peer-timeout", "60"]))
    assert rc == 1 and rep["peer_state"] == "failed" and "Freivalds" in rep["error"]
    # abort file: a rank waiting on a peer that never comes stops at once
    d = tmp_path / "b"
    d.mkdir()
    p = _rank(d, 0, extra=["--peer-timeout", "60"])
    time.sleep(0.3)
    (d / "abort.tmp").write_text("t rank 1 failed (rc 1)")
    os.replace(d / "abort.tmp", d / "abort")  # as validate.py writes it: never seen half-written
    rc, rep = _report(p, timeout=5)
    assert rc == 1 and rep["peer_state"] == "aborted" and "rank 1 failed" in rep["error"]


def test_abort_file_releases_a_rank_waiting_at_its_start_gate(tmp_path):
    gate = tmp_path / "gate"
    gate.write_text("")
    p = _rank(tmp_path, 1, extra=["--start-gate", str(gate)])
    time.sleep(0.3)
    (tmp_path / "abort").write_text("sibling failed")
    rc, rep = _report(p, timeout=5)
    assert rc == 3 and "aborted" in rep["error"]
    assert (tmp_path / "t-failed-1").exists()


def test_all_peers_present_pass(tmp_path):
    gate = tmp_path / "gate"
    gate.write_text("")  # ranks 1 and 2 stay alive at their start gate
    others = [_rank(tmp_path, r, world=3, extra=["--start-gate", str(gate)]) for r in (1, 2)]
    rc, rep = _report(_rank(tmp_path, 0, world=3))
    # no GPU here: the peers step passes, the hip step after it cannot
    assert rep["steps"][0]["name"] == "peers" and rep["steps"][0]["ok"], rep
    gate.write_text("abort")
    for p in others:
        assert _report(p)[0] == 3


# ---------------------------------------------------- validate_workload ----

@pytest.fixture
def env8(tmp_path):
    root = str(tmp_path / "h")
    fakesys.build_node(root, 2)
    env = NodeEnv("n1", None, host_root=root, validations_dir=str(tmp_path / "v"), poll_s=0.01)

    def launcher(argv, e, device, timeout):
        return run_local([sys.executable, "-m", "amdgpu_operator.testing.fake_validator", *argv[1:]], e, timeout)

    env.launcher = launcher
    return env


def test_sibling_failure_cancels_a_hanging_rank(env8, monkeypatch):
    # rank 1 hangs (alive, not waiting on anyone); rank 0 fails: the
    # orchestrator's abort file ends the hang
    monkeypatch.setenv("AMDGPU_FAKE_VALIDATOR_FAULT", "*:1:hang,*:0:fail")
    t0 = time.monotonic()
    with pytest.raises(V.StepFailed) as ei:
        V.validate_workload(env8, ["--peer-timeout", "60"], timeout=120)
    assert time.monotonic() - t0 < 10
    msg = str(ei.value)
    assert msg.index("injected failure") < msg.index("then")  # cause first, consequences after
    assert "aborted" in msg
    assert not os.listdir(os.path.join(env8.validations_dir, "rendezvous"))  # run dir removed


def test_separate_rccl_process_hang_is_cancelled(env8, monkeypatch):
    # the second-process layout (rcclProcess: separate): its RCCL process hangs
    monkeypatch.setenv("AMDGPU_FAKE_VALIDATOR_FAULT", "-rccl:1:hang,*:0:fail")
    with pytest.raises(V.StepFailed, match="injected failure"):
        V.validate_workload(env8, ["--peer-timeout", "60", "--rccl-separate-process"], timeout=120)


def test_rank_exiting_without_report_is_named(env8, monkeypatch):
    monkeypatch.setenv("AMDGPU_FAKE_VALIDATOR_FAULT", "*:1:exit")
    t0 = time.monotonic()
    with pytest.raises(V.StepFailed) as ei:
        V.validate_workload(env8, ["--peer-timeout", "60"], timeout=120)
    assert time.monotonic() - t0 < 10
    assert "rank 1" in str(ei.value)


def test_rank_never_started_fails_within_peer_timeout(env8, monkeypatch):
    real = env8.launcher

    def launcher(argv, e, device, timeout):
        if argv[argv.index("--rank") + 1] == "1":
            time.sleep(0.1)
            return ProcResult(127, "", "exec failed: no such file", 0.1)  # never ran
        return real(argv, e, device, timeout)

    env8.launcher = launcher
    t0 = time.monotonic()
    with pytest.raises(V.StepFailed, match="rank 1"):
        V.validate_workload(env8, ["--peer-timeout", "2"], timeout=120)
    assert time.monotonic() - t0 < 10


def test_validate_flags_translate_to_the_binary(env8, monkeypatch):
    seen = []
    real = env8.launcher

    def launcher(argv, e, device, timeout):
        seen.append(argv)
        return real(argv, e, device, timeout)

    env8.launcher = launcher
    out = V.validate_workload(env8, ["--rccl-busbw-link-fraction", "0.2", "--xgmi-read-link-fraction", "0.25",
                                     "--require-xgmi-links", "--min-mfma-util", "0.2"])
    assert out["ok"] and out["fabric"]["ok"] and out["fabric"]["physical_gpus"] == 2
    # one 76 GB/s link per rank (KFD io_links): busBW 0.2 x 76 x 64/(64+16) MiB, reads 0.25 x 76
    assert out["floors"] == {"link_gbps_per_rank": [76.0, 76.0], "min_rccl_busbw_gbps": 12.2,
                             "min_xgmi_peer_read_gbps": 19.0}
    assert len(seen) == 2 and out["processes"] == 2 and out["process_mode"] == "shared"
    for a in seen:
        for own in ("--rccl-busbw-link-fraction", "--xgmi-read-link-fraction", "--require-xgmi-links",
                    "--max-gpu-processes"):
            assert own not in a
        assert a[a.index("--min-rccl-busbw-gbps") + 1] == "12.2"
        assert a[a.index("--min-xgmi-read-gbps") + 1] == "19"
        assert a[a.index("--min-mfma-util") + 1] == "0.2"
        # one process per GPU
        assert a[a.index("--steps") + 1] == "hip,vecadd,gemm,gemm_fp8,gemm_fp4,gemm_fp6,gemm_mxfp4,mfma,hbm,xgmi,rccl"


# ------------------------------------------- process layout and budget ----

def _fake_env(tmp_path, gpus, partition="SPX"):
    root = str(tmp_path / "h")
    fakesys.build_node(root, gpus, compute_partition=partition)
    env = NodeEnv("n1", None, host_root=root, validations_dir=str(tmp_path / "v"), poll_s=0.01)
    calls = []

    def launcher(argv, e, device, timeout):
        calls.append((argv, e, device))
        return run_local([sys.executable, "-m", "amdgpu_operator.testing.fake_validator", *argv[1:]], e, timeout)

    env.launcher = launcher
    return env, calls


def _by_rank(calls):
    return sorted(calls, key=lambda c: int(c[0][c[0].index("--rank") + 1]))


def test_eight_gpus_start_eight_processes_each_seeing_its_peers(tmp_path):
    from amdgpu_operator.discovery import topology

    env, calls = _fake_env(tmp_path, 8)
    gpus = topology.enumerate_gpus(env.host_root)
    out = V.validate_workload(env, ["--peer-timeout", "60"])
    assert out["processes"] == 8 and out["world"] == 8 and len(calls) == 8
    for rank, (argv, e, device) in enumerate(_by_rank(calls)):
        assert device == rank and argv[argv.index("--local-bdf") + 1] == gpus[rank].bdf
        ids = e["ROCR_VISIBLE_DEVICES"].split(",")
        assert len(ids) == 8 and ids[0] == f"GPU-{gpus[rank].unique_id:016x}"  # own GPU first, then its 7 peers


def test_separate_rccl_processes_only_within_the_budget(tmp_path):
    env, calls = _fake_env(tmp_path, 8)
    out = V.validate_workload(env, ["--peer-timeout", "60", "--rccl-separate-process"], budget=15)
    assert out["process_mode"] == "shared" and out["processes"] == 8  # 16 would not fit
    env2, calls2 = _fake_env(tmp_path / "b", 2)
    out = V.validate_workload(env2, ["--peer-timeout", "60", "--rccl-separate-process"], budget=15)
    assert out["process_mode"] == "separate" and out["processes"] == 4
    assert V.planned_workload_processes(env, ["--rccl-separate-process"], 15) == 8
    assert V.planned_workload_processes(env2, ["--rccl-separate-process"], 15) == 4


def test_cpx_node_validates_every_partition_from_one_process_per_gpu(tmp_path):
    """8 x CPX = 64 partitions: 8 processes (not 64 + 64), a communicator of 8
    physical ranks, and every partition's kernel steps reported."""
    env, calls = _fake_env(tmp_path, 8, "CPX")
    out = V.validate_workload(env, ["--peer-timeout", "60"])
    assert out["devices"] == 64 and out["world"] == 8 and out["processes"] == 8 and len(calls) == 8
    for rank, rep in enumerate(out["ranks"]):
        for step in ("vecadd", "gemm", "mfma", "hbm"):
            assert sorted(s["device"] for s in rep["steps"] if s["name"] == step) == list(range(8)), (rank, step)
        names = [s["name"] for s in rep["steps"]]
        assert names.count("xgmi") == 1 and names.count("rccl") == 1  # xGMI + RCCL across the physical GPUs
    for rank, (argv, e, _) in enumerate(_by_rank(calls)):
        assert argv[argv.index("--world") + 1] == "8" and argv[argv.index("--expect-devices") + 1] == "8"
        assert len(e["ROCR_VISIBLE_DEVICES"].split(",")) == 8 + 7  # its 8 partitions + one device of each peer


def test_a_partition_missing_from_a_rank_fails_the_run(tmp_path, monkeypatch):
    env, calls = _fake_env(tmp_path, 2, "CPX")
    real = env.launcher

    def launcher(argv, e, device, timeout):  # rank 1's process sees only 7 of its 8 partitions
        if argv[argv.index("--rank") + 1] == "1":
            argv = list(argv)
            argv[argv.index("--expect-devices") + 1] = "7"
        return real(argv, e, device, timeout)

    env.launcher = launcher
    with pytest.raises(V.StepFailed, match="rank 1: 7 of 8 devices validated"):
        V.validate_workload(env, ["--peer-timeout", "60"])


# ------------------------------------------------------------ fabric ----

class _M:
    def __init__(self, bdf, up, total=7, err=0):
        self.bdf, self.values = bdf, {"xgmi_links_up": up, "xgmi_links_total": total, "xgmi_links_error": err}


def test_fabric_check_on_an_8_gpu_hive(tmp_path):
    from amdgpu_operator.discovery import topology

    root = str(tmp_path / "h")
    fakesys.build_node(root, 8)
    env = NodeEnv("n1", None, host_root=root, validations_dir=str(tmp_path / "v"))
    gpus = topology.enumerate_gpus(root)
    ok = V.check_fabric(env, gpus, [_M(g.bdf, 7) for g in gpus])
    assert ok["ok"] and ok["physical_gpus"] == 8 and ok["kfd_xgmi_pairs"] == 28
    bad = V.check_fabric(env, gpus, [_M(g.bdf, 6 if g.index == 3 else 7, err=1 if g.index == 5 else 0) for g in gpus])
    assert not bad["ok"]
    assert any(gpus[3].bdf in p and "6 xGMI links up" in p for p in bad["problems"])
    assert any(gpus[5].bdf in p and "in error" in p for p in bad["problems"])


def test_fabric_check_finds_a_missing_kfd_link_and_a_split_hive(tmp_path):
    from amdgpu_operator.discovery import topology

    root = str(tmp_path / "h")
    fakesys.build_node(root, 2, xgmi=False)  # two GPUs, no hive, PCIe only
    env = NodeEnv("n1", None, host_root=root, validations_dir=str(tmp_path / "v"))
    out = V.check_fabric(env, topology.enumerate_gpus(root), [])
    assert not out["ok"]
    assert any("hive" in p for p in out["problems"]) and any("no XGMI link" in p for p in out["problems"])


def test_fabric_check_skips_partitions_of_one_gpu(tmp_path):
    from amdgpu_operator.discovery import topology

    root = str(tmp_path / "h")
    fakesys.build_node(root, 1, compute_partition="CPX", memory_partition="NPS2")
    env = NodeEnv("n1", None, host_root=root, validations_dir=str(tmp_path / "v"))
    gpus = topology.enumerate_gpus(root)
    assert len(gpus) == 8
    out = V.check_fabric(env, gpus, [])
    assert out["ok"] and out["physical_gpus"] == 1 and "skipped" in out


def test_half_rate_links_fail_closed(tmp_path):
    """Every link "up", but trained to half its rate: amd-smi's rate x width
    against the KFD nominal (76 GB/s per direction on MI355X) names it."""
    from amdgpu_operator.discovery import topology

    root = str(tmp_path / "h")
    fakesys.build_node(root, 8)
    env = NodeEnv("n1", None, host_root=root, validations_dir=str(tmp_path / "v"))
    gpus = topology.enumerate_gpus(root)

    def m(g, speed, width=16):
        x = _M(g.bdf, 7)
        x.values.update(xgmi_link_speed_gbps=speed, xgmi_link_width=width)
        return x

    ok = V.check_fabric(env, gpus, [m(g, 38) for g in gpus])
    assert ok["ok"] and ok["links"][gpus[0].bdf]["link_gbps"] == 76.0
    half = V.check_fabric(env, gpus, [m(g, 19) for g in gpus])
    assert not half["ok"] and all(any(g.bdf in p and "nominal 76 GB/s" in p for p in half["problems"]) for g in gpus)
    narrow = V.check_fabric(env, gpus, [m(g, 38, 8 if g.index == 2 else 16) for g in gpus])
    assert not narrow["ok"] and len(narrow["problems"]) == 1 and gpus[2].bdf in narrow["problems"][0]


def test_throughput_floors_scale_with_the_links(tmp_path):
    from amdgpu_operator.discovery import topology

    root = str(tmp_path / "h")
    fakesys.build_node(root, 8)
    env = NodeEnv("n1", None, host_root=root, validations_dir=str(tmp_path / "v"))
    gpus = topology.enumerate_gpus(root)
    plan = V.rank_plan(gpus)
    f = V.fabric_floors(env, plan, gpus, 0.2, 0.25, 64 << 20)
    assert f["link_gbps_per_rank"] == [532.0] * 8  # 7 links x 76 GB/s
    assert f["min_rccl_busbw_gbps"] == 85.1 and f["min_xgmi_peer_read_gbps"] == 133.0
    small = V.fabric_floors(env, plan, gpus, 0.2, 0.25, 1 << 20)  # latency-bound size: a lower busBW floor
    assert small["min_rccl_busbw_gbps"] < 10
    four = V.fabric_floors(env, plan[:4], gpus, 0.2, 0.25, 64 << 20)
    assert four["link_gbps_per_rank"] == [228.0] * 4
