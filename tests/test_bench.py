"""bench.py contract (driver runs it with --gpus/--steps/--warmup)."""

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def test_bench_json_line_contract():
    p = subprocess.run([sys.executable, "bench.py", "--steps", "2", "--warmup", "1", "--fake-gpu"], cwd=ROOT,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [x for x in p.stdout.splitlines() if x.strip()]
    assert len(lines) == 1
    out = json.loads(lines[0])
    assert KEYS <= set(out)
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        assert out["metric"] == json.load(f)["metric"]
    assert out["unit"] == "s" and out["higher_is_better"] is False and out["steps"] == 2 and out["warmup"] == 1
    assert out["n_gpus"] == 1 and out["config"]["allocatable_amd_com_gpu"] == 1
    assert 0 < out["value"] < 60 and abs(out["vs_baseline"] - out["value"] / 600.0) < 1e-4
    assert out["config"]["parallelism"] == "dp1"
    # headline: operands as processes, with their start-up breakdown; in-process figure next to it
    cfg = out["config"]
    assert cfg["operand_mode"] == "process" and len(cfg["thread_mode_time_to_ready_s"]) == 2
    ops = cfg["operands"]
    assert ops["amd-device-plugin-daemonset/amd-device-plugin"]["ready_s"] > 0
    assert ops["amd-operator-validator/amd-operator-validator"]["ready_s"] > 0
    # both halves of the metric (README.md:122), and every timed step's critical path
    vis = cfg["allocatable_visible_s"]
    assert cfg["allocatable_visible_mean_s"] == pytest.approx(sum(vis) / 2, abs=1e-3) and cfg["allocatable_visible_p95_s"] == max(vis)
    cps = cfg["critical_path"]
    assert len(cps) == 2 and all(c["ttr"] > 0 and "complete" in c["at"] and "ready_gap" in c for c in cps)
    assert [c["ttr"] for c in cps] == cfg["time_to_ready_s"]
    assert isinstance(cfg["slow_steps"], list)  # fewer than 3 steps: nothing is judged slow
    # the collective block after the last timed bring-up (world 1 here; the 8-rank run: test_launcher.py)
    col = cfg["collectives"]
    assert col["ok"] and col["world"] == 1 and set(col["ops"]) == {"allreduce", "allgather", "reducescatter"}
    assert [r["bytes"] for r in col["ops"]["allreduce"]][-1] == 1 << 30


def test_bench_floor_failure_prints_a_structured_line():
    """A bring-up that fails its floors (here the RCCL busBW fraction set 250x
    above the link model) ends at once with the JSON line: value null, the
    failing step, ranks and floor vs measured, and the collective curve
    measured after it; rc non-zero."""
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr", "127.0.0.1", "--master-port=29617", "bench.py", "--gpus", "2", "--steps", "3",
                        "--warmup", "0", "--fake-gpu-procs", "--compare", "0",
                        "--set", "validator.workload.rcclBusbwLinkFraction=50"],
                       cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert p.returncode != 0
    lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:] + p.stderr[-2000:]
    out = json.loads(lines[0])
    assert KEYS <= set(out) and out["value"] is None and out["vs_baseline"] is None
    e = out["error"]
    assert e["phase"] == "timed" and e["bring_up"] == 1 and e["failed_steps"][0] in ("gpu", "workload")
    assert e["world"] == 2 and e["failed_ranks"] == [0, 1]
    assert e["floors"]["min_rccl_busbw_gbps"] == 3040.0  # 50 x 76 GB/s x 64/(64+16) MiB
    for r in e["ranks"]:
        rccl = next(s for s in r["steps"] if s["name"] == "rccl")
        assert rccl["ok"] is False and rccl["perf_ok"] is False and rccl["busbw_gbps"] < rccl["min_busbw_gbps"]
    col = out["config"]["collectives"]
    assert col["ok"] and col["world"] == 2 and col["xgmi_links"]["min_read_gbps"] > 0
    assert col["fabric_floors"]["rccl_busbw_link_fraction"] == 0.2  # the sweep reports against the default model


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
    p = subprocess.Popen([sys.executable, "bench.py", "--steps", "1", "--warmup", "0", "--compare", "0"],
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
    # the collective block on the device (world 1: RCCL's single-rank path, the curve's shape)
    col = line["config"]["collectives"]
    assert col["ok"] and col["world"] == 1 and not col["simulated"], col
    assert len(col["ops"]["allreduce"]) >= 14 and all(r["ok"] and r["latency_us"] > 0 for r in col["ops"]["allreduce"])
    assert col["ops"]["allreduce"][-1]["algbw_gbps"] > 100  # a 1 GiB single-rank all-reduce is an HBM copy


def test_slow_steps_name_the_part_that_grew():
    """the record names the cause of any bring-up above 1.3 x the
    median - the critical-path part that grew most against its own median."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)

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
