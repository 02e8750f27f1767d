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
