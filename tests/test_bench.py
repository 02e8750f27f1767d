"""bench.py contract (driver runs it with --gpus/--steps/--warmup)."""

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}
HEAD = ["metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step"]
LINE_BUDGET = 3000


def _bench():
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    return b


def _line(stdout: str) -> str:
    lines = [x for x in stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, stdout[-2000:]
    return lines[0]


def test_bench_json_line_contract(tmp_path):
    detail = str(tmp_path / "detail.json")
    p = subprocess.run([sys.executable, "bench.py", "--steps", "2", "--warmup", "1", "--fake-gpu", "--detail", detail],
                       cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [x for x in p.stdout.splitlines() if x.strip()]
    assert len(lines) == 1
    assert len(lines[0]) <= LINE_BUDGET  # the driver keeps a ~9 KB tail of stdout + stderr (BENCH_r05)
    assert len(p.stderr) < 1500, p.stderr  # a few progress lines, no log records
    out = json.loads(lines[0])
    assert KEYS <= set(out)
    assert list(out)[:len(HEAD)] == HEAD  # headline fields first
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        assert out["metric"] == json.load(f)["metric"]
    assert out["unit"] == "s" and out["higher_is_better"] is False and out["steps"] == 2 and out["warmup"] == 1
    assert out["n_gpus"] == 1 and out["config"]["allocatable_amd_com_gpu"] == 1
    assert 0 < out["value"] < 60 and abs(out["vs_baseline"] - out["value"] / 600.0) < 1e-4
    assert out["config"]["parallelism"] == "dp1"
    cfg = out["config"]
    assert cfg["operand_mode"] == "process" and cfg["other_mode_time_to_ready_s"]["mode"] == "thread"
    assert len(cfg["other_mode_time_to_ready_s"]["s"]) == 2
    # both halves of the metric (README.md:122), summarised
    assert cfg["ttr_s"]["mean"] == pytest.approx(out["value"], abs=1e-3) and len(cfg["time_to_ready_s"]) == 2
    assert 0 < cfg["allocatable_visible_s"]["mean"] <= cfg["allocatable_visible_s"]["p95"]
    assert cfg["slow_steps"]["count"] == 0  # fewer than 3 steps: nothing is judged slow
    assert cfg["rates"]["counter_gate"]["bf16"] == "pass" and cfg["kfd_holders"]["ready_max"] == 0
    gr = cfg["gate_retries"]  # every timed bring-up's counted dispatches
    assert gr["gates"] >= 2 and 0 <= gr["retried"] <= gr["gates"] and gr["max_attempts"] >= 1
    col = cfg["collectives"]
    assert col["ok"] and col["world"] == 1 and col["sizes"] == 15
    assert cfg["pod_workload"]["ok"] and cfg["detail"] == detail
    # everything else is in the detail file the line names
    with open(detail) as f:
        d = json.load(f)
    assert d["summary"] == out
    cps = d["critical_path"]
    assert len(cps) == 2 and all(c["ttr"] > 0 and "complete" in c["at"] and "ready_gap" in c for c in cps)
    # the detail keeps 4 decimals, the line 3: compare at the line's precision (no double rounding)
    assert [c["ttr"] for c in cps] == pytest.approx(cfg["time_to_ready_s"], abs=6e-4)
    ops = d["operands"]
    assert ops["amd-device-plugin-daemonset/amd-device-plugin"]["ready_s"] > 0
    assert ops["amd-operator-validator/amd-operator-validator"]["ready_s"] > 0
    assert set(d["collectives"]["ops"]) == {"allreduce", "allgather", "reducescatter"}
    assert [r["bytes"] for r in d["collectives"]["ops"]["allreduce"]][-1] == 1 << 30
    assert all(set(h) == {"start", "ready"} for h in d["kfd_holders"])


def test_bench_floor_failure_prints_a_structured_line(tmp_path):
    """A bring-up that fails its floors (here the RCCL busBW fraction set 250x
    above the link model) ends at once with the JSON line: value null, the
    failing step, ranks and floor vs measured, and the collective curve
    measured after it; rc non-zero.  At N = 8 the line and everything printed
    after it stay inside the driver's tail."""
    detail = str(tmp_path / "detail.json")
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=8",
                        "--master-addr", "127.0.0.1", "--master-port=29617", "bench.py", "--gpus", "8", "--steps", "20",
                        "--warmup", "0", "--fake-gpu-procs", "--compare", "0", "--detail", detail,
                        "--set", "validator.workload.rcclBusbwLinkFraction=50"],
                       cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert p.returncode != 0
    line = _line(p.stdout)
    assert len(line) <= LINE_BUDGET
    assert len(p.stdout) + len(p.stderr) < 8000, p.stderr[-3000:]  # the driver's tail holds ~8.9 KB
    out = json.loads(line)
    assert KEYS <= set(out) and out["value"] is None and out["vs_baseline"] is None
    e = out["error"]
    assert e["phase"] == "timed" and e["bring_up"] == 1 and e["failed_steps"][0] in ("gpu", "workload")
    assert e["world"] == 8 and e["failed_ranks"] == list(range(8))
    assert e["floors"]["min_rccl_busbw_gbps"] == 21280.0  # 50 x 532 GB/s x 64/(64+16) MiB
    ff = e["first_failed"]
    assert ff["name"] == "rccl" and ff["busbw_gbps"] < ff["min_busbw_gbps"]
    col = out["config"]["collectives"]
    assert col["ok"] and col["world"] == 8 and col["min_read_gbps"] > 0 and col["links_below_floor"] == 0
    with open(out["config"]["detail"]) as f:
        d = json.load(f)
    rec = d["errors"][0]["records"]["workload"]
    for r in rec["ranks"]:
        rccl = next(s for s in r["steps"] if s["name"] == "rccl")
        assert rccl["ok"] is False and rccl["perf_ok"] is False and rccl["busbw_gbps"] < rccl["min_busbw_gbps"]
    assert d["errors"][0]["collectives"]["fabric_floors"]["rccl_busbw_link_fraction"] == 0.2
    assert "Traceback" in d["errors"][0]["traceback"]


def test_bench_setup_failure_prints_a_structured_line(tmp_path):
    """A run that fails before its first bring-up (here: two GPUs asked of a
    node whose KFD topology has one) still ends with one parseable line,
    value null and phase "setup", and a non-zero exit."""
    from amdgpu_operator.testing import fakesys

    root = str(tmp_path / "host")
    fakesys.build_node(root, 1)
    os.makedirs(os.path.join(root, "dev"), exist_ok=True)
    open(os.path.join(root, "dev", "kfd"), "w").close()
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "1", "--warmup", "0",
                        "--sysfs-root", root, "--detail", str(tmp_path / "d.json")],
                       cwd=ROOT, capture_output=True, text=True, timeout=120)
    assert p.returncode == 1, p.stderr[-2000:]
    line = _line(p.stdout)
    assert len(line) <= LINE_BUDGET
    out = json.loads(line)
    assert out["value"] is None and out["n_gpus"] == 2 and out["steps"] == 1
    assert out["error"]["phase"] == "setup"
    assert "node exposes 1" in out["error"]["message"]
    assert list(out)[:len(HEAD)] == HEAD


def test_fit_line_sheds_optional_fields_to_the_budget():
    b = _bench()
    out = {"metric": "m", "value": 1.0, "config": {"model": "x", "time_to_ready_s": [0.25] * 400,
                                                    "collectives": {"ok": True, "pad": "y" * 900}}}
    line = b.fit_line(out, budget=1200)
    assert len(line) <= 1200
    got = json.loads(line)
    assert got["value"] == 1.0 and set(got["config"]["shed"]) == {"collectives", "time_to_ready_s"}


@pytest.mark.gpu
def test_bench_harness_never_opens_the_gpu():
    """N = 1 on the MI355X: the bench process itself never becomes a KFD
    process during a bring-up (only its children - validator, plugin pod -
    do), so the headline measures the operator's GPU processes, not a HIP
    context of the harness."""
    import time

    procs = "/sys/class/kfd/kfd/proc"
    if not os.path.isdir(procs):
        pytest.skip("no KFD process list in this container")
    p = subprocess.Popen([sys.executable, "bench.py", "--steps", "1", "--warmup", "0", "--compare", "0",
                          "--detail", "gpurun_out/test_bench_detail.json"],
                         cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    seen: set[str] = set()
    deadline = time.monotonic() + 240
    while p.poll() is None and time.monotonic() < deadline:
        try:
            seen.update(os.listdir(procs))
        except OSError:
            pass
        time.sleep(0.002)
    if p.poll() is None:
        p.kill()
    out, err = p.communicate()
    assert p.returncode == 0, err[-3000:]
    line = json.loads([x for x in out.splitlines() if x.startswith("{")][0])
    assert line["config"]["harness_holds_kfd"] is False
    assert str(p.pid) not in seen
    assert seen - {str(os.getpid())}, "no GPU process seen at all: the KFD process list is not being read"
    assert len(out.splitlines()[-1]) <= LINE_BUDGET
    # the collective block on the device (world 1: RCCL's single-rank path, the curve's shape)
    assert line["config"]["collectives"]["ok"] and not line["config"]["collectives"]["simulated"]
    with open(os.path.join(ROOT, line["config"]["detail"])) as f:
        col = json.load(f)["collectives"]
    assert col["ok"] and col["world"] == 1 and not col["simulated"], col
    assert len(col["ops"]["allreduce"]) >= 14 and all(r["ok"] and r["latency_us"] > 0 for r in col["ops"]["allreduce"])
    assert col["ops"]["allreduce"][-1]["algbw_gbps"] > 100  # a 1 GiB single-rank all-reduce is an HBM copy


def test_slow_steps_name_the_part_that_grew():
    """the record names the cause of any bring-up above 1.3 x the
    median - the critical-path part that grew most against its own median."""
    b = _bench()

    def cp(ttr, hsa_init=0.06, proc=0.12):
        return {"ttr": ttr, "at": {"driver": 0.09, "registered": 0.08, "pods_created": 0.11},
                "wl": {"proc": proc}, "pod": {"hsa_init": hsa_init, "hsa": 0.011, "main_at": 0.14},
                "ready_gap": 0.008, "stall_ms": 3.0}

    cps = [cp(0.24), cp(0.23), cp(0.25), cp(0.42, hsa_init=0.25), cp(0.33, proc=0.22), cp(0.24)]
    slow = b.slow_steps(cps)
    assert [s["step"] for s in slow] == [3, 4]
    assert slow[0]["cause"] == "plugin pod HSA start-up (hsa_init)" and slow[0]["cause_s"] == 0.25
    assert slow[0]["cause_median_s"] == 0.06 and slow[0]["median_ttr"] == 0.245
    assert slow[1]["cause"] == "workload validator process" and slow[1]["cause_s"] == 0.22
    assert b.slow_steps(cps[:2]) == []
