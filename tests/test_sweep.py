"""The collective sweep (validator/sweep.py) and the fabric floors' fallback.

The merge is the part that decides what the driver's multi-GPU record says:
one row per (op, size) at the slowest rank, busBW from that time with the
rccl-tests factors, a row with any rank's mismatch (or a missing rank) not
ok.  The 8-rank end-to-end run is in test_launcher.py; the MI355X run in
test_bench.py (gpu) and test_native_gpu.py."""

import sys

import pytest

from amdgpu_operator.nodeenv import NodeEnv, run_local
from amdgpu_operator.testing import fakesys
from amdgpu_operator.validator import sweep as S
from amdgpu_operator.validator import validate as V


def _rep(rank, rows, links=None):
    steps = [{"name": "hip", "ok": True}, {"name": "sweep", "ok": True, "rows": rows}]
    if links is not None:
        steps.insert(1, {"name": "xgmi_links", "ok": True, "links": links})
    return {"ok": True, "rc": 0, "rank": rank, "steps": steps}


def test_sizes_match_the_native_schedule():
    s = S.sizes()
    assert s[0] == 8 and s[-1] == 1 << 30 and len(s) == 15 and all(b * 4 == c for b, c in zip(s, s[1:-1]))
    assert S.sizes(8, 100, 4) == [8, 32, 100]


def test_merge_takes_the_slowest_rank_and_rccl_tests_factors():
    row = lambda op, b, us, bad=0: {"op": op, "bytes": b, "us": us, "mismatches": bad}  # noqa: E731
    reps = [_rep(0, [row("allreduce", 1 << 20, 10.0), row("allgather", 1 << 20, 8.0)]),
            _rep(1, [row("allreduce", 1 << 20, 20.0), row("allgather", 1 << 20, 4.0, bad=1)])]
    out = S.merge_rows(2, reps)
    ar = out["allreduce"][0]
    assert ar["latency_us"] == 20.0 and ar["ok"]
    assert ar["algbw_gbps"] == round((1 << 20) / 20e-6 / 1e9, 2)
    assert ar["busbw_gbps"] == pytest.approx(ar["algbw_gbps"] * 2 * 1 / 2, abs=0.01)  # 2(n-1)/n at n = 2
    ag = out["allgather"][0]
    assert ag["latency_us"] == 8.0 and not ag["ok"]  # one rank's mismatch fails the row
    assert ag["busbw_gbps"] == pytest.approx(ag["algbw_gbps"] * 0.5, abs=0.01)
    # a rank that did not report a size: the row is not ok
    out = S.merge_rows(2, [reps[0], _rep(1, [row("allreduce", 1 << 20, 11.0)])])
    assert out["allreduce"][0]["ok"] and not out["allgather"][0]["ok"]
    # world 1: no bus factor
    assert S.merge_rows(1, [reps[0]])["allreduce"][0]["busbw_gbps"] == 0.0


def test_link_matrix_names_each_link():
    reps = [_rep(0, [], [{"peer": 1, "read_gbps": 50.0, "intact": True}, {"peer": 2, "read_gbps": 20.0, "intact": True}]),
            _rep(1, [], [{"peer": 2, "read_gbps": 51.0, "intact": True}, {"peer": 0, "read_gbps": 49.0, "intact": True}]),
            _rep(2, [], [{"peer": 0, "read_gbps": 48.0, "intact": False}, {"peer": 1, "read_gbps": 47.0, "intact": True}])]
    m = S.link_matrix(reps, 3)
    assert m["read_gbps"][0] == [None, 50.0, 20.0] and m["read_gbps"][2][2] is None
    assert m["min_read_gbps"] == 20.0 and m["max_read_gbps"] == 51.0 and m["intact"] is False


def _env(tmp_path, gpus, **kw):
    root = str(tmp_path / "h")
    fakesys.build_node(root, gpus, **kw)
    env = NodeEnv("n1", None, host_root=root, validations_dir=str(tmp_path / "v"), poll_s=0.01)
    env.launcher = lambda argv, e, device, timeout: run_local(
        [sys.executable, "-m", "amdgpu_operator.testing.fake_validator", *argv[1:]], e, timeout)
    return env


def test_sweep_on_four_stand_in_ranks(tmp_path):
    env = _env(tmp_path, 4)
    out = S.collective_sweep(env, max_bytes=1 << 24, timeout=60)
    assert out["ok"] and out["world"] == 4 and out["simulated"]
    assert set(out["ops"]) == set(S.OPS) and out["ops"]["allreduce"][-1]["bytes"] == 1 << 24
    ff = out["fabric_floors"]
    assert ff["link_gbps_per_rank"] == [228.0] * 4  # 3 x 76 GB/s
    assert all(v["ratio"] is None for v in ff["allreduce_vs_floor"] if v["bytes"] < S.RATIO_FROM_BYTES)
    assert ff["min_allreduce_ratio"] > 1 and ff["min_link_read_floor_gbps"] == 19.0 and ff["links_below_floor"] == []
    assert out["xgmi_links"]["min_read_gbps"] > 0


def test_sweep_reports_a_failed_rank(tmp_path, monkeypatch):
    env = _env(tmp_path, 2)
    monkeypatch.setenv("AMDGPU_FAKE_VALIDATOR_FAULT", "*:1:fail")
    out = S.collective_sweep(env, max_bytes=1 << 20, timeout=60)
    assert not out["ok"] and "rank 1" in out["error"] and out["ops"] == {}
    assert out["ranks"][1]["ok"] is False and out["ranks"][1]["error"] == "injected failure"


def test_floors_hold_a_node_without_kfd_xgmi_bandwidth_to_the_nominal(tmp_path):
    """a multi-GPU node whose KFD reports no XGMI io_link (PCIe
    routed) summed to 0 - "no floor".  The pairs now count at the xGMI
    nominal, so such a node keeps (and, PCIe-routed, fails) its floors."""
    from amdgpu_operator.discovery import topology

    root = str(tmp_path / "h")
    fakesys.build_node(root, 2, xgmi=False)
    env = NodeEnv("n1", None, host_root=root, validations_dir=str(tmp_path / "v"))
    gpus = topology.enumerate_gpus(root)
    f = V.fabric_floors(env, V.rank_plan(gpus), gpus, 0.2, 0.25, 64 << 20)
    assert f["link_gbps_per_rank"] == [76.0, 76.0] and f["nominal_pairs"] == 2
    assert f["min_rccl_busbw_gbps"] == 12.2 and f["min_xgmi_peer_read_gbps"] == 19.0


def test_workload_failure_leaves_a_record_with_floors(tmp_path):
    env = _env(tmp_path, 2)
    with pytest.raises(V.StepFailed):
        V.validate_workload(env, ["--peer-timeout", "60", "--rccl-busbw-link-fraction", "50"])
    rec = V.read_failure(env, "workload")
    assert rec["world"] == 2 and rec["failed_ranks"] == [0, 1] and rec["floors"]["min_rccl_busbw_gbps"] == 3040.0
    rccl = next(s for s in rec["ranks"][0]["steps"] if s["name"] == "rccl")
    assert rccl["perf_ok"] is False and rccl["busbw_gbps"] < rccl["min_busbw_gbps"]
    # the next pass clears it
    V.validate_workload(env, ["--peer-timeout", "60"])
    assert V.read_failure(env, "workload") is None and V.read_ready(env, "workload")["ok"]
