"""Rank launcher: GPU processes run on the rank that owns the GPU (gloo, CPU)."""

import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _torchrun(nproc: int, script: str, *args, port: int) -> subprocess.CompletedProcess:
    return subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
                           "--master-addr", "127.0.0.1", f"--master-port={port}", script, *args],
                          capture_output=True, text=True, timeout=240, cwd=os.path.dirname(HERE))


@pytest.mark.parametrize("nproc,port", [(2, 29611), (4, 29612)])
def test_processes_run_on_owner_rank(nproc, port):
    p = _torchrun(nproc, os.path.join(HERE, "helpers", "launcher_worker.py"), port=port)
    assert "LAUNCHER_OK" in p.stdout, p.stdout[-2000:] + p.stderr[-3000:]


@pytest.mark.parametrize("nproc,warmup,port,mode", [(2, 0, 29613, "thread"), (8, 1, 29614, "process")])
def test_bench_ranks_with_stand_in_validators(nproc, warmup, port, mode, tmp_path):
    """The driver's scaling launch (torchrun, one rank per GPU) on CPU: 8 ranks,
    a warm-up phase and the other-mode comparison exercise the launcher
    hand-over between phases; thread mode routes every GPU process through
    the rank that owns the GPU, process mode runs the operands as processes."""
    p = _torchrun(nproc, "bench.py", "--gpus", str(nproc), "--steps", "1", "--warmup", str(warmup),
                  "--fake-gpu-procs", "--mode", mode, "--compare", "1", "--detail", str(tmp_path / "detail.json"), port=port)
    assert p.returncode == 0, p.stderr[-3000:]
    import json

    lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1  # rank 0 prints the one JSON line
    out = json.loads(lines[0])
    assert out["n_gpus"] == nproc and out["config"]["allocatable_amd_com_gpu"] == nproc
    assert out["config"]["parallelism"] == f"dp{nproc}" and out["steps"] == 1 and out["warmup"] == warmup
    other = "thread" if mode == "process" else "process"
    assert out["config"]["operand_mode"] == mode
    assert out["config"]["other_mode_time_to_ready_s"]["mode"] == other
    assert len(out["config"]["other_mode_time_to_ready_s"]["s"]) == 1


def test_run_local_takes_the_report_before_the_exit():
    """AMDGPU_REPORT_EARLY: the result is the child's report once it closed its
    pipes; its (slow) exit is reaped in the background."""
    import time

    from amdgpu_operator.nodeenv import run_local

    child = ("import json,os,sys,time;print(json.dumps({'ok': %s}));sys.stdout.flush();"
             "n=os.open(os.devnull,os.O_WRONLY);os.dup2(n,1);os.dup2(n,2);time.sleep(3)")
    t0 = time.perf_counter()
    r = run_local([sys.executable, "-c", child % "True"], {"AMDGPU_REPORT_EARLY": "1"}, timeout=30)
    assert r.rc == 0 and time.perf_counter() - t0 < 2.0 and '"ok": true' in r.stdout
    r = run_local([sys.executable, "-c", child % "False"], {"AMDGPU_REPORT_EARLY": "1"}, timeout=30)
    assert r.rc == 1  # the report's verdict
    r = run_local([sys.executable, "-c", "import sys; sys.exit(7)"], {"AMDGPU_REPORT_EARLY": "1"}, timeout=30)
    assert r.rc == 7  # already exited: its real status
    r = run_local([sys.executable, "-c", "import time; time.sleep(5)"], {"AMDGPU_REPORT_EARLY": "1"}, timeout=0.5)
    assert r.rc == 124


def test_bench_n8_stays_within_the_gpu_process_budget(tmp_path):
    """The driver's N = 8 launch (torchrun, 8 ranks) on CPU with stand-in GPU
    processes: no harness rank opens a GPU (harness_holds_kfd false; the
    stand-ins are the only "GPU processes"), one validator process per GPU
    plus the plugin pod, and never more than 16 of them alive at once (the
    box's per-user GPU-process limit, tools/storm_probe.py)."""
    import json

    from test_simcluster import _peak_concurrency

    log_dir = str(tmp_path / "procs")
    env = dict(os.environ, AMDGPU_FAKE_GPU_PROC_LOG=log_dir)
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=8",
                        "--master-addr", "127.0.0.1", "--master-port=29615", "bench.py", "--gpus", "8", "--steps", "1",
                        "--warmup", "0", "--fake-gpu-procs", "--mode", "process", "--compare", "0",
                        "--detail", str(tmp_path / "detail.json")],
                       capture_output=True, text=True, timeout=240, cwd=os.path.dirname(HERE), env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [x for x in p.stdout.splitlines() if x.startswith("{")][0]
    # the driver's tail (~8.9 KB of stdout + stderr) holds the line at N = 8, with
    # room for 40 steps' time-to-Ready list (7 bytes each) on top of this 1-step run
    assert len(line) + 40 * 7 <= 3000, len(line)
    assert len(p.stdout) + len(p.stderr) < 8000
    out = json.loads(line)
    assert out["config"]["allocatable_amd_com_gpu"] == 8 and out["config"]["harness_holds_kfd"] is False
    with open(out["config"]["detail"]) as f:
        detail = json.load(f)
    assert out["config"]["pod_workload"]["ok"] and out["config"]["pod_workload"]["pods"] == 11
    pw = detail["pod_workload"]  # config 5 after Ready: 8 x 1 GPU, 1 x 8, 2 x 4
    assert pw["pods"] == 11 and pw["all_succeeded"] and pw["single_gpu_pods_distinct_devices"]
    assert pw["two_halves_numa_local"] and pw["two_halves_disjoint"]
    peak, roles = _peak_concurrency(log_dir)
    # 8 validator processes per pass: the bring-up's, then the collective sweep's
    assert roles == {"validator": 16, "pod": 1 + 11}, roles  # the plugin-validation pod + the workload's pods
    assert peak <= 16, peak
    # the collective curve at world 8 after the timed bring-up
    cs = out["config"]["collectives"]
    assert cs["ok"] and cs["world"] == 8 and cs["links_below_floor"] == 0 and cs["min_allreduce_ratio"] > 1
    assert cs["peak_busbw_gbps"] >= cs["busbw_256MiB_gbps"] > cs["busbw_1MiB_gbps"] > 0
    col = detail["collectives"]
    assert col["ok"] and col["world"] == 8
    for op in ("allreduce", "allgather", "reducescatter"):
        rows = col["ops"][op]
        assert len(rows) == 14 and rows[0]["bytes"] == 32 and rows[-1]["bytes"] == 1 << 30  # 8 B rounds up to 8 floats
        assert all(r["ok"] and r["latency_us"] > 0 and r["busbw_gbps"] >= 0 for r in rows)
        assert rows[-1]["busbw_gbps"] > rows[0]["busbw_gbps"]
    links = col["xgmi_links"]["read_gbps"]
    assert len(links) == 8 and all(links[r][r] is None and all(links[r][p] for p in range(8) if p != r) for r in range(8))
    ff = col["fabric_floors"]
    assert ff["link_gbps_per_rank"] == [532.0] * 8 and ff["min_allreduce_ratio"] > 1 and ff["links_below_floor"] == []
    assert len(detail["critical_path"]) == 1
