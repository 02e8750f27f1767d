"""Native components on a real MI355X: validator binary (incl. counter gate and
the IPC peer path), N3/N4/N6 over libamd_smi, probe on the real sysfs, and the
metrics exporter with live data."""

import json
import os
import pathlib
import re
import subprocess
import tempfile

import pytest

from amdgpu_operator import native

pytestmark = pytest.mark.gpu
VALIDATOR = str(native.binary("amdgpu-validator"))
_WPT = int(re.search(r"kGemmWavesPerTile = (\d+);", (pathlib.Path(__file__).resolve().parents[1] / "native" / "include"
                                                     / "gemm_default.h").read_text()).group(1))


def _run(args, env=None, timeout=120):
    p = subprocess.run([VALIDATOR, *args], capture_output=True, text=True, timeout=timeout,
                       env={**os.environ, **(env or {})})
    rep = json.loads(p.stdout.strip().splitlines()[-1])
    return p.returncode, rep


def test_validator_all_local_steps_with_counter_gate(tmp_path):
    # default gate: AQL profiling packets on the validator's own queue
    rc, rep = _run(["--rendezvous", str(tmp_path), "--steps", "hip,vecadd,gemm,mfma,hbm,xgmi", "--counter-gate"])
    assert rc == 0 and rep["ok"], rep
    steps = {s["name"]: s for s in rep["steps"]}
    assert steps["mfma"]["dtypes"] == {d: True for d in ("f16", "bf16", "fp8", "bf8", "i8", "mxfp8", "mxfp6", "mxfp4",
                                                         "f32", "f64")}
    assert steps["hip"]["arch"].startswith("gfx950") and steps["hip"]["cus"] == 256
    assert steps["vecadd"]["mismatches"] == 0
    g = steps["gemm"]
    assert g["freivalds_rel_err"] < 1e-4 and g["counter_gate"] == "pass"
    assert g["flop_per_mop"] == 512  # one MFMA "MOP" = 512 FLOP on gfx950 (16x16x32 bf16 = 32 MOPs)
    assert g["gate_mode"] == "aql" and g["gated_output_matches"]
    assert g["SQ_WAVES"] == (4096 // 256) ** 2 * _WPT  # 256x256 tiles, the default kernel's waves each
    assert g["samples"] == [32, 32, 32, 8]  # per-SE/XCC instances of the SQ counters, 8 GRBM
    assert g["tflops"] > 300
    assert steps["hbm"]["checksum_match"] and steps["hbm"]["gbps"] > 2000
    assert steps["xgmi"]["emulated"] and steps["xgmi"]["max_abs_err"] <= 8e-5


def test_validator_fp8_rate_step_with_counter_gate(tmp_path):
    """mfma-rate: the e4m3 GEMM on the f8f6f4 MFMA, Freivalds-checked, over
    its floor, and counted: SQ_INSTS_VALU_MFMA_MOPS_F8 == 2N^3/512 with the
    default kernel's waves.  Its gate reuses the HSA session the validator set
    up on a thread at its start (setup ~0 at the gate)."""
    rc, rep = _run(["--rendezvous", str(tmp_path), "--steps", "hip,gemm,gemm_fp8,gemm_fp4", "--counter-gate",
                    "--min-fp8-tflops", "1200", "--min-gemm-tflops", "620", "--min-fp4-tflops", "1900"])
    assert rc == 0 and rep["ok"], rep
    steps = {s["name"]: s for s in rep["steps"]}
    f = steps["gemm_fp8"]
    assert f["dtype"] == "e4m3" and f["n"] == 4096 and f["freivalds_rel_err"] < 1e-3
    assert f["counter_gate"] == "pass" and f["gated_output_matches"], f
    assert f["SQ_INSTS_VALU_MFMA_MOPS_F8"] * 512 == 2 * 4096 ** 3 and f["flop_per_mop"] == 512
    assert f["SQ_WAVES"] == (4096 // 256) ** 2 * _WPT
    assert f["perf_ok"] and f["tflops"] >= 1200 and f["min_tflops"] == 1200
    assert f["tflops"] > 1.3 * steps["gemm"]["tflops"]  # 2x the FLOP per clock of the bf16 MFMA
    # the gates' HSA set-up ran on a thread beside the first steps (avk_aql_gate_prepare)
    assert rep["gate_prepare"]["seconds"] > 0 and "error" not in rep["gate_prepare"], rep["gate_prepare"]
    assert f["gate_setup_seconds"] < 0.002
    # FP4 (e2m1) on the same instruction, cbsz = blgp = 4: SQ_INSTS_VALU_MFMA_MOPS_F6F4
    q = steps["gemm_fp4"]
    assert q["dtype"] == "e2m1" and q["freivalds_rel_err"] < 1e-3 and q["counter_gate"] == "pass", q
    assert q["SQ_INSTS_VALU_MFMA_MOPS_F6F4"] * 512 == 2 * 4096 ** 3 and q["SQ_WAVES"] == (4096 // 256) ** 2 * _WPT
    assert q["perf_ok"] and q["tflops"] > 1.3 * f["tflops"] and q["gate_setup_seconds"] < 0.002


def test_validator_fp6_and_mxfp4_rate_steps_with_counter_gate(tmp_path):
    """VERDICT r5 task 6: the fp6 (e2m3) and block-scaled MXFP4 GEMMs at
    4096^3 - Freivalds-checked against the decoded (and, for MX, scaled)
    operands, over a floor, and counted: SQ_INSTS_VALU_MFMA_MOPS_F6F4 ==
    2N^3/512 with the default kernel's waves."""
    rc, rep = _run(["--rendezvous", str(tmp_path), "--steps", "hip,gemm_fp4,gemm_fp6,gemm_mxfp4", "--counter-gate",
                    "--min-fp6-tflops", "1000", "--min-mxfp4-tflops", "1000", "--min-fp4-tflops", "1000"])
    assert rc == 0 and rep["ok"], rep
    steps = {s["name"]: s for s in rep["steps"]}
    for name, dtype in (("gemm_fp6", "e2m3"), ("gemm_mxfp4", "mxfp4")):
        g = steps[name]
        assert g["dtype"] == dtype and g["n"] == 4096 and g["freivalds_rel_err"] < 1e-3, g
        assert g["counter_gate"] == "pass" and g["gate_attempts"] == 1 and g["gated_output_matches"], g
        assert g["SQ_INSTS_VALU_MFMA_MOPS_F6F4"] * 512 == 2 * 4096 ** 3 and g["SQ_WAVES"] == (4096 // 256) ** 2 * _WPT
        assert g["perf_ok"] and g["tflops"] >= 1000 and g["min_tflops"] == 1000
    # fp6 moves fp8's bytes at the fp4 MFMA rate: well above the fp8 step's rate class
    assert steps["gemm_fp6"]["tflops"] > 0.6 * steps["gemm_fp4"]["tflops"]
    assert steps["gemm_mxfp4"]["tflops"] > 0.8 * steps["gemm_fp4"]["tflops"]  # the scales cost little


def test_shipped_floors_pass_and_a_floor_above_the_measured_rate_fails(tmp_path):
    """VERDICT r5 task 5: the Ready gate's shipped floors (WorkloadSpec) pass
    on a healthy MI355X; the same floors at 1.05 x what this GPU just
    measured fail the step - so the floors sit near the rate, not at 40 %."""
    from amdgpu_operator.api.clusterpolicy import WorkloadSpec

    w = WorkloadSpec()
    floors = ["--min-gemm-tflops", str(w.minGemmTflops), "--min-fp8-tflops", str(w.minFp8Tflops),
              "--min-fp4-tflops", str(w.minFp4Tflops), "--min-fp6-tflops", str(w.minFp6Tflops),
              "--min-mxfp4-tflops", str(w.minMxfp4Tflops), "--min-hbm-gbps", str(w.minHbmGbps),
              "--min-mfma-util", str(w.minMfmaUtil),
              "--min-mfma-util-by-dtype", ",".join(f"{k}={v}" for k, v in w.minMfmaUtilByDtype.items())]
    steps = "hip,gemm,gemm_fp8,gemm_fp4,gemm_fp6,gemm_mxfp4,hbm"
    rc, rep = _run(["--rendezvous", str(tmp_path / "a"), "--steps", steps, "--counter-gate", *floors])
    assert rc == 0 and rep["ok"], rep
    got = {s["name"]: s for s in rep["steps"]}
    for name, floor in (("gemm", w.minGemmTflops), ("gemm_fp8", w.minFp8Tflops), ("gemm_fp4", w.minFp4Tflops),
                        ("gemm_fp6", w.minFp6Tflops), ("gemm_mxfp4", w.minMxfp4Tflops)):
        assert got[name]["min_tflops"] == floor and got[name]["tflops"] < floor / 0.60, (name, got[name]["tflops"])
    assert got["hbm"]["gbps"] < w.minHbmGbps / 0.60
    # 1.05 x the rate: this run's, or the calibration median where this run
    # read lower (one best-of-3 reading spreads ~+-8 % for fp8 between
    # processes, profiles/r6_defer; the 60-run medians of profiles/r6_floors)
    medians = {"gemm": 1505.5, "gemm_fp8": 2706.2, "gemm_fp4": 4313.0, "gemm_fp6": 3533.7, "gemm_mxfp4": 3938.8}
    over = {"gemm": "--min-gemm-tflops", "gemm_fp8": "--min-fp8-tflops", "gemm_fp4": "--min-fp4-tflops",
            "gemm_fp6": "--min-fp6-tflops", "gemm_mxfp4": "--min-mxfp4-tflops"}
    for name, flag in over.items():
        rate = max(got[name]["tflops"], medians[name])
        rc, rep = _run(["--rendezvous", str(tmp_path / name), "--steps", f"hip,{name}", flag, f"{1.05 * rate:.1f}"])
        st = next(s for s in rep["steps"] if s["name"] == name)
        assert rc != 0 and st["perf_ok"] is False and st["tflops"] < st["min_tflops"], st


def test_counter_gates_pass_first_time_beside_a_process_dispatching_continuously(tmp_path):
    """VERDICT r5 task 3: a second process (the plugin-validation pod's check,
    here looping its kernel for seconds) dispatches on the GPU the whole time
    the validator's three counter gates run.  It holds the GPU's gate lock
    shared per dispatch and the gates hold it exclusively around their counted
    dispatch (gate_lock.h), so every gate passes on its first attempt."""
    import time

    locks = tmp_path / "locks"
    locks.mkdir()
    env = {"AMDGPU_GATE_LOCK_DIR": str(locks)}
    bg = subprocess.Popen([str(native.binary("amdgpu-gpu-check")), "--loop-seconds", "6", "--elems", str(1 << 22),
                           "--timeout", "30"], env={**os.environ, **env}, stdout=subprocess.PIPE, text=True)
    try:
        deadline = time.monotonic() + 20
        while not list(locks.glob("gate-*.lock")) and time.monotonic() < deadline:
            time.sleep(0.01)  # the loop's first lock: it is dispatching
        assert list(locks.glob("gate-*.lock")), "the background check never took its lock"
        rc, rep = _run(["--rendezvous", str(tmp_path), "--steps", "hip,gemm,gemm_fp8,gemm_fp4", "--counter-gate"],
                       env=env)
        assert bg.poll() is None, "the background dispatcher ended before the gates"
    finally:
        out = bg.communicate(timeout=60)[0]
    assert rc == 0 and rep["ok"], rep
    for name in ("gemm", "gemm_fp8", "gemm_fp4"):
        st = next(x for x in rep["steps"] if x["name"] == name)
        assert st["counter_gate"] == "pass" and st["gate_attempts"] == 1, st
        assert st["gate_lock"] == "held" and st["gate_lock_wait_s"] < 0.5, st
    bgrep = json.loads(out.strip().splitlines()[-1])
    vec = next(x for x in bgrep["steps"] if x["name"] == "vecadd")
    assert bgrep["ok"] and vec["dispatches"] > 10, bgrep  # it kept the GPU busy throughout
    hsa = next(x for x in bgrep["steps"] if x["name"] == "hsa")
    assert hsa["gate_lock"] == "held"
    # the pod (HSA agent BDF) and the gates (hipDeviceGetPCIBusId) named the same lock file
    assert [p.name for p in locks.glob("gate-*.lock")] == ["gate-" + hsa["bdf"].replace(":", "-").replace(".", "-")
                                                           + ".lock"]


def test_counter_gate_beside_another_partys_mfma_kernels(tmp_path):
    """A co-tenant that takes no gate lock (a PyTorch process running bf16
    GEMMs back to back) shares the device-wide counters with the counted
    window.  The gate never accepts such a window: it passes only with every
    equality exact on one attempt, and a window the other party's work
    explains (its waves, and for the bf16 gate its MFMA ops too) is counted
    again - up to 4 attempts - never failed outright on the first."""
    import sys
    import time

    code = ("import sys, time, torch\n"
            "a = torch.randn(4096, 4096, device='cuda', dtype=torch.bfloat16)\n"
            "b = torch.randn(4096, 4096, device='cuda', dtype=torch.bfloat16)\n"
            "(a @ b).sum().item()\n"
            "print('ready', flush=True)\n"
            "t = time.monotonic()\n"
            "while time.monotonic() - t < float(sys.argv[1]):\n"
            "    for _ in range(8):\n"
            "        c = a @ b\n"
            "    torch.cuda.synchronize()\n")
    bg = subprocess.Popen([sys.executable, "-c", code, "8"], stdout=subprocess.PIPE, text=True)
    try:
        assert bg.stdout.readline().strip() == "ready"
        t0 = time.monotonic()
        rc, rep = _run(["--rendezvous", str(tmp_path), "--steps", "hip,gemm,gemm_fp8", "--counter-gate"],
                       timeout=60)
        busy_throughout = bg.poll() is None
        took = time.monotonic() - t0
    finally:
        bg.communicate(timeout=60)
    assert busy_throughout, "the co-tenant ended before the gates"
    got = {x["name"]: x for x in rep["steps"]}
    assert got["gemm"]["counter_gate"] in ("pass", "fail"), rep
    for name, mops in (("gemm", "SQ_INSTS_VALU_MFMA_MOPS_BF16"), ("gemm_fp8", "SQ_INSTS_VALU_MFMA_MOPS_F8")):
        st = got.get(name)
        if st is None or st["counter_gate"] == "not_run":  # counted only while the earlier gates pass
            continue
        assert st["freivalds_rel_err"] < 1e-3, st  # the computation itself was right
        if st["counter_gate"] == "pass":
            assert st[mops] * 512 == 2 * 4096 ** 3 and st["SQ_WAVES"] == (4096 // 256) ** 2 * _WPT, st
        else:
            assert st["counter_gate"] == "fail" and st["gate_attempts"] == 4, st
        tries = [r for r in st.get("gate_retried_after", "").split("; ") if r]
        assert len(tries) == st["gate_attempts"] - (st["counter_gate"] == "pass"), st
        assert all(r.endswith(", preempted)") or r.endswith(", foreign_mfma)") for r in tries), st
    assert took < 30


def test_counter_gate_fails_closed_on_a_truncated_gemm(tmp_path):
    """The counted dispatch runs half the K loop (AMDGPU_GATE_TEST_TRUNCATE_K):
    its MFMA op count misses 2MNK/512 and its output differs, so the gate
    fails on its first attempt and is not retried."""
    for mode in ([], ["--defer-gates"]):
        rc, rep = _run(["--rendezvous", str(tmp_path / str(len(mode))), "--steps", "hip,gemm,gemm_fp8",
                        "--counter-gate", *mode], env={"AMDGPU_GATE_TEST_TRUNCATE_K": "1"})
        assert rc != 0 and not rep["ok"]
        g = next(x for x in rep["steps"] if x["name"] == "gemm")
        assert g["counter_gate"] == "fail" and g["gate_attempts"] == 1 and not g["ok"], g
        assert g["SQ_INSTS_VALU_MFMA_MOPS_BF16"] * 512 == 4096 ** 3  # half of 2 * 4096^3
        assert g["gated_output_matches"] is False and g["freivalds_rel_err"] < 1e-4  # the HIP GEMM itself was right
        f = next((x for x in rep["steps"] if x["name"] == "gemm_fp8"), None)
        if mode:  # deferred: the fp8 step ran, and after the failed gate its own is not counted
            assert g["gate_deferred"] and f["counter_gate"] == "not_run" and not f["ok"], f
        else:  # inline: the run stops at the failed step
            assert f is None


def test_counter_gates_run_after_the_kernel_steps(tmp_path):
    """PendingGate (--defer-gates, validator.workload.deferGates): each GEMM
    step is measured and checked in place, its counted dispatch runs once the
    kernel steps are done - after the HBM step here - and lands in the step's
    own record; by default the gate runs inside the step."""
    steps = "hip,gemm,gemm_fp8,hbm"
    rc, rep = _run(["--rendezvous", str(tmp_path / "d"), "--steps", steps, "--counter-gate", "--defer-gates"])
    assert rc == 0 and rep["ok"], rep
    got = {x["name"]: x for x in rep["steps"]}
    for name in ("gemm", "gemm_fp8"):
        assert got[name]["counter_gate"] == "pass" and got[name]["gate_deferred"] is True, got[name]
        assert got[name]["seconds"] >= got[name]["gate_seconds"]
    rc, rep = _run(["--rendezvous", str(tmp_path / "n"), "--steps", steps, "--counter-gate"])
    assert rc == 0 and rep["ok"], rep
    got = {x["name"]: x for x in rep["steps"]}
    assert got["gemm"]["counter_gate"] == "pass" and "gate_deferred" not in got["gemm"]


def test_validator_fp8_floor_fails_the_step(tmp_path):
    rc, rep = _run(["--rendezvous", str(tmp_path), "--steps", "hip,gemm_fp8", "--min-fp8-tflops", "100000"])
    assert rc != 0 and not rep["ok"]
    f = {s["name"]: s for s in rep["steps"]}["gemm_fp8"]
    assert f["perf_ok"] is False and f["min_tflops"] == 100000 and f["freivalds_rel_err"] < 1e-3


def test_start_gate_init_starts_the_runtime_and_go_the_kernels(tmp_path):
    """Two-phase start gate: "init" (the driver container has the module
    loaded) lets the HIP runtime start; the kernel steps wait for "go" (the
    validator's own driver check).  The second wait is reported."""
    import threading
    import time

    gate = tmp_path / "gate"
    gate.write_text("init")

    def release():
        time.sleep(1.5)
        (tmp_path / "gate.tmp").write_text("go")
        (tmp_path / "gate.tmp").replace(gate)

    th = threading.Thread(target=release)
    th.start()
    rc, rep = _run(["--rendezvous", str(tmp_path / "rv"), "--steps", "hip,vecadd", "--start-gate", str(gate)])
    th.join()
    assert rc == 0 and rep["ok"], rep
    sg = rep["start_gate"]
    # the runtime started during the 1.5 s (its start-up is ~0.1 s, up to
    # ~0.35 s right after another GPU process's exit): the kernels then waited
    assert sg["wait_s"] < 0.1 and 0.5 < sg["go_wait_s"] < 2.0, sg


def test_start_gate_abort_after_init_exits_before_the_kernels(tmp_path):
    import threading
    import time

    gate = tmp_path / "gate"
    gate.write_text("init")

    def release():
        time.sleep(0.3)
        gate.write_text("abort")

    th = threading.Thread(target=release)
    th.start()
    rc, rep = _run(["--rendezvous", str(tmp_path / "rv"), "--steps", "hip,vecadd", "--start-gate", str(gate)])
    th.join()
    assert rc == 3 and rep["error"] == "start gate: aborted" and rep["steps"] == []


def test_start_gate_abort_during_the_runtime_start_ends_the_process_at_once(tmp_path):
    """"abort" while the HIP runtime is still starting after "init"
    - the gate watcher thread ends the process within milliseconds, not after
    the runtime's start-up, and its ``.held`` lock is free once it is gone
    (what the driver container waits on before a reload)."""
    import fcntl
    import time

    gate = tmp_path / "gate"
    gate.write_text("init")
    p = subprocess.Popen([VALIDATOR, "--rendezvous", str(tmp_path / "rv"), "--steps", "hip,vecadd", "--start-gate",
                          str(gate)], stdout=subprocess.PIPE, text=True)
    held = tmp_path / "gate.held"
    deadline = time.monotonic() + 10
    while not held.exists() and time.monotonic() < deadline:
        time.sleep(0.0005)
    time.sleep(0.01)  # inside the runtime's start (~0.1 s)
    t0 = time.monotonic()
    gate.write_text("abort")
    line = p.stdout.readline()  # printed right before _exit
    answered = time.monotonic() - t0
    p.wait(timeout=30)
    rep = json.loads(line)
    assert p.returncode == 3 and rep["error"] == "start gate: aborted", rep
    assert answered < 0.05, answered
    with open(held) as f:
        fcntl.flock(f, fcntl.LOCK_EX | fcntl.LOCK_NB)  # released with the process


def test_validator_counter_gate_tool_library_from_env(tmp_path):
    # the operator's path: the tool library is named explicitly (validate.py)
    from amdgpu_operator.validator.validate import gate_env

    rc, rep = _run(["--rendezvous", str(tmp_path), "--steps", "hip,gemm", "--gemm", "1024", "--counter-gate",
                    "--gate-mode", "sdk"], gate_env())
    assert rc == 0 and rep["ok"], rep
    g = {s["name"]: s for s in rep["steps"]}["gemm"]
    assert g["counter_gate"] == "pass" and g["dispatches"] == 1 and g["flop_per_mop"] == 512


def test_validator_counter_gate_sdk_definitions(tmp_path):
    # the tool named by the caller with the SDK's own full counter set: the
    # gate must work with either definition file, as long as it is one set
    env = {**gate_env_full(), "AMDGPU_GATE_KERNEL_NAMES": "1"}
    rc, rep = _run(["--rendezvous", str(tmp_path), "--steps", "hip,gemm", "--gemm", "1024", "--counter-gate",
                    "--gate-mode", "sdk"], env)
    assert rc == 0 and rep["ok"], rep
    assert {s["name"]: s for s in rep["steps"]}["gemm"]["counter_gate"] == "pass"


def gate_env_full():
    from amdgpu_operator.validator.validate import gate_env

    env = gate_env()
    env.pop("ROCPROFILER_METRICS_PATH")
    return env


def test_validator_counter_gate_unavailable_fails_closed(tmp_path):
    # sdk gate requested but the tool was not activated: must not silently pass
    rc, rep = _run(["--rendezvous", str(tmp_path), "--steps", "hip,gemm", "--counter-gate", "--gate-mode", "sdk"])
    assert rc == 1 and not rep["ok"]
    assert {s["name"]: s for s in rep["steps"]}["gemm"]["counter_gate"] == "unavailable"


def test_validator_aql_gate_fails_closed_without_its_code_object(tmp_path):
    # the AQL gate dispatches the GEMM from validator_kernels.co next to the
    # binary: a copy of the binary without it cannot pass the gate
    import shutil

    exe = tmp_path / "amdgpu-validator"
    shutil.copy2(VALIDATOR, exe)
    p = subprocess.run([str(exe), "--rendezvous", str(tmp_path / "rv"), "--steps", "hip,gemm", "--gemm", "1024",
                        "--counter-gate"], capture_output=True, text=True, timeout=120)
    rep = json.loads(p.stdout.strip().splitlines()[-1])
    g = {s["name"]: s for s in rep["steps"]}["gemm"]
    assert p.returncode == 1 and g["counter_gate"] == "unavailable" and "validator_kernels.co" in g["gate_error"]


def test_validator_aql_gate_small_and_rectangular_work(tmp_path):
    # 1024^3: 16 workgroups; the gate must still count every wave and MOP
    rc, rep = _run(["--rendezvous", str(tmp_path), "--steps", "hip,gemm", "--gemm", "1024", "--counter-gate"])
    assert rc == 0 and rep["ok"], rep
    g = {s["name"]: s for s in rep["steps"]}["gemm"]
    assert g["SQ_WAVES"] == 16 * _WPT and g["SQ_INSTS_VALU_MFMA_MOPS_BF16"] * 512 == 2 * 1024 ** 3


def test_validator_ipc_peer_path_two_processes_one_gpu(tmp_path):
    # two ranks on the same GPU exercise the hipIpc handle exchange + peer-pointer
    # one-shot kernel (on a node the peers are other GPUs over xGMI)
    procs = [subprocess.Popen([VALIDATOR, "--rank", str(r), "--world", "2", "--device", "0", "--rendezvous",
                               str(tmp_path), "--run-id", "ipc", "--steps", "hip,xgmi", "--xgmi-elems", "1048576"],
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(2)]
    outs = [p.communicate(timeout=120) for p in procs]
    for p, (out, err) in zip(procs, outs):
        rep = json.loads(out.strip().splitlines()[-1])
        assert p.returncode == 0 and rep["ok"], (rep, err[-2000:])
        x = {s["name"]: s for s in rep["steps"]}["xgmi"]
        assert not x["emulated"] and x["peers"] == 2


def test_validator_single_rank_rccl(tmp_path):
    rc, rep = _run(["--rendezvous", str(tmp_path), "--steps", "hip,rccl", "--rccl-elems", "1048576"])
    assert rc == 0 and rep["ok"], rep
    r = {s["name"]: s for s in rep["steps"]}["rccl"]
    assert r["mismatches"] == 0
    assert set(r["collectives"]) == {"allreduce_f32", "allreduce_bf16", "allgather_f32", "reducescatter_f32"}
    assert all(c["mismatches"] == 0 and c["ms"] > 0 for c in r["collectives"].values())


def test_validator_sweep_step_one_rank(tmp_path):
    # the native sweep (validator_main.cpp step_sweep): every size checked on the
    # device, then timed; 8 B ... 16 MiB here
    rc, rep = _run(["--rendezvous", str(tmp_path), "--steps", "hip,sweep", "--sweep-max-bytes", str(16 << 20)])
    assert rc == 0 and rep["ok"], rep
    s = {x["name"]: x for x in rep["steps"]}["sweep"]
    assert s["world"] == 1 and s["mismatches"] == 0 and s["comm_init_s"] > 0
    rows = s["rows"]
    for op in ("allreduce", "allgather", "reducescatter"):
        mine = [r for r in rows if r["op"] == op]
        assert [r["bytes"] for r in mine] == [8 * 4 ** k for k in range(11)] + [16 << 20]
        assert all(r["mismatches"] == 0 and r["us"] > 0 and r["busbw_gbps"] == 0 for r in mine)  # world 1: no bus
    assert max(r["algbw_gbps"] for r in rows) > 50


def test_validator_xgmi_links_two_processes_one_gpu(tmp_path):
    # two ranks on one GPU take the per-link path (IPC, lockstep rounds, data
    # checked); on a node each round crosses a different xGMI link
    procs = [subprocess.Popen([VALIDATOR, "--rank", str(r), "--world", "2", "--device", "0", "--rendezvous",
                               str(tmp_path), "--run-id", "links", "--steps", "hip,xgmi_links",
                               "--link-bytes", str(16 << 20)],
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(2)]
    outs = [p.communicate(timeout=120) for p in procs]
    for r, (p, (out, err)) in enumerate(zip(procs, outs)):
        rep = json.loads(out.strip().splitlines()[-1])
        assert p.returncode == 0 and rep["ok"], (rep, err[-2000:])
        x = {s["name"]: s for s in rep["steps"]}["xgmi_links"]
        assert x["links"] == [dict(x["links"][0], peer=1 - r)] and x["links"][0]["intact"]
        assert x["min_read_gbps"] > 10


def test_collectives_sweep_rccl_one_gpu():
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, "-m", "amdgpu_operator", "collectives", "--max-bytes", str(64 << 20),
                        "--iters", "3", "--json"], capture_output=True, text=True, timeout=300, cwd=repo,
                       env={**os.environ, "PYTHONPATH": repo, "MASTER_PORT": "29611"})
    assert p.returncode == 0, p.stderr[-3000:]
    rows = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("[")][-1])
    assert rows and all(r["ok"] and r["world"] == 1 for r in rows)
    assert {r["op"] for r in rows} == {"allreduce", "allgather", "reducescatter"}


def test_validator_rejects_bad_arguments():
    p = subprocess.run([VALIDATOR, "--gemm", "1000"], capture_output=True, text=True, timeout=30)
    assert p.returncode == 2


def test_probe_and_topology_on_real_sysfs():
    from amdgpu_operator.discovery import topology as T

    ok, msg = T.probe("/")
    assert ok, msg
    gpus = T.enumerate_gpus("/")
    assert gpus and all(g.arch == "gfx950" and g.cu_count == 256 for g in gpus)
    assert all(g.vram_bytes > 280 * 2**30 for g in gpus)


def test_smi_collector_and_health_watcher():
    from amdgpu_operator.discovery import topology as T

    with T.Smi() as smi:
        assert smi.count() >= 1
        m = smi.collect()[0]
        assert m.values["vram_total_bytes"] > 280 * 2**30
        assert "socket_power_w" in m.values and "temp_hotspot_c" in m.values
        # PMFW metrics table (amdsmi_get_gpu_metrics_info): PCIe link, xGMI counters, HBM peak bandwidth
        assert m.values["pcie_link_width"] > 0 and m.values["vram_max_bandwidth_gbps"] > 1000
        assert "xgmi_read_bytes" in m.values and "ppt_residency" in m.values
        assert smi.partitions(0)[0] in ("SPX", "DPX", "QPX", "CPX", "")
    hw = T.HealthWatcher()
    try:
        events = hw.poll(100)
        assert all(not e.critical for e in events), events
    finally:
        hw.close()


def test_driver_smi_table_on_mi355x(tmp_path):
    """``kubectl exec ... -c amd-driver-ctr -- amdgpu-operator driver smi``:
    the table the reference reads off nvidia-smi (README.md:152-167), from the
    real sysfs and libamd_smi."""
    from amdgpu_operator.driver import manager as DM
    from amdgpu_operator.nodeenv import NodeEnv

    table = DM.smi_table(NodeEnv(node_name="box", client=None, host_root="/", validations_dir=str(tmp_path)))
    rows = [r for r in table.splitlines() if "gfx950" in r]
    assert rows, table
    for r in rows:
        cells = [c.strip() for c in r.strip("|").split("|")]
        assert cells[3] == "256"
        used, total = cells[5].removesuffix("MiB").split("/")
        assert int(total) > 280 * 1024 and 0 <= int(used) <= int(total)  # 288 GB HBM3E per GPU
        assert int(cells[6]) > 0 and int(cells[7]) > 0  # live power and temperature from amd-smi
    assert table.splitlines()[-1].startswith("amd-smi: ok: "), table


def test_pci_binding_view_on_mi355x():
    """vfio-manager's PCI sysfs reader on the real host: the MI355X is an AMD
    processing accelerator bound to amdgpu, so passthrough validation fails
    closed and the sandbox plugin has nothing to advertise."""
    from amdgpu_operator.discovery import topology as T
    from amdgpu_operator.sandbox import plugin as SP
    from amdgpu_operator.sandbox import vfio as VF

    pci = VF.PciSysfs("/")
    gpus = {g.bdf: g for g in pci.gpus()}
    kfd = [g.bdf for g in T.enumerate_gpus("/")]
    assert kfd and all(b in gpus for b in kfd), (kfd, sorted(gpus))
    for b in kfd:
        g = gpus[b]
        assert g.device == 0x75A3 and g.cls.startswith("12") and g.driver == "amdgpu", g
    ok, msg, _ = VF.check_bound(pci)
    assert not ok and "amdgpu" in msg
    assert SP.vfio_devices(pci) == [] and SP.resource_name(gpus[kfd[0]].device) == "amd.com/MI355X"


def test_metrics_exporter_live():
    from amdgpu_operator.exporter.metrics import MetricsExporter, SmiSource

    src = SmiSource()
    try:
        ex = MetricsExporter(src, "box")
        ex.collect_once()
        text = ex.render()
        assert "amd_gpu_vram_total_bytes{" in text and "amd_gpu_power_watts{" in text
        assert ex.errors == 0
        assert 'product="AMD-Instinct-MI355X"' in text  # not libdrm's generic name
    finally:
        src.close()


def test_metrics_exporter_health_series_live():
    """The XID-equivalent series on the MI355X: the exporter's amd-smi event
    client (the process's one HealthHub watcher) initialises, every series
    exists at 0 per GPU, and the stream reads as live."""
    import threading
    import time

    from amdgpu_operator.discovery.topology import HealthHub
    from amdgpu_operator.exporter.metrics import HealthCounters, MetricsExporter, SmiSource

    src = SmiSource()
    stop = threading.Event()
    sub = HealthHub.subscribe()
    sub2 = HealthHub.subscribe()  # a second consumer in the process shares the watcher
    try:
        assert sub._hub is sub2._hub
        hc = HealthCounters()
        th = threading.Thread(target=hc.run, args=(sub.poll, stop, 100), daemon=True)
        th.start()
        ex = MetricsExporter(src, "box", health=hc, dcgm_names=True)
        ex.collect_once()
        deadline = time.monotonic() + 5
        while not hc.live and time.monotonic() < deadline:
            time.sleep(0.01)
        text = ex.render()
        assert "amd_gpu_exporter_health_events_live 1" in text
        for name in ("amd_gpu_reset_total", "amd_gpu_vm_fault_total", "amd_gpu_thermal_throttle_events_total",
                     "amd_gpu_ecc_uncorrectable_events_total", "amd_gpu_health_critical", "DCGM_FI_DEV_XID_ERRORS"):
            rows = [ln for ln in text.splitlines() if ln.startswith(name + "{")]
            assert rows and all(ln.endswith(" 0") for ln in rows), (name, rows)
    finally:
        stop.set()
        sub.close()
        sub2.close()
        src.close()
    assert HealthHub._inst is None  # the last subscription closed the watcher


@pytest.mark.parametrize("mode", ["local", "http", "process"])
def test_sim_cluster_on_real_gpu(mode):
    """Bring-up on the MI355X; with ``http`` the operator and the operands
    use the production RestClient against the API server's HTTP front end;
    with ``process`` every operand container is its own process (the device
    plugin's amd-smi health watcher on)."""
    from amdgpu_operator.testing.simcluster import NodeSpec, SimCluster
    from amdgpu_operator.discovery import topology as T

    n = len(T.enumerate_gpus("/"))
    d = tempfile.mkdtemp()
    c = SimCluster(d, [NodeSpec("node-0", n, sysfs_root="/")], fake_gpu=False, poll_s=0.005, http_api=mode == "http",
                   process_containers=mode == "process", termination_s=0.0 if mode == "process" else None).start()
    try:
        c.install_operator({"validator": {"workload": {"gemmN": 1024, "hbmBytes": 1 << 26}}})
        ttr = c.wait_ready(120, {"node-0": n})
        assert ttr < 60
        from amdgpu_operator.validator.validate import read_ready

        wl = read_ready(c.nodes["node-0"].env, "workload")
        gemm = [s for s in wl["ranks"][0]["steps"] if s["name"] == "gemm"][0]
        assert gemm["counter_gate"] == "pass"
        if mode == "process":  # verify --run-pod: a user's 1-GPU pod runs its kernel on the MI355X
            from amdgpu_operator.cli.verify import verify

            rep = verify(c.client, c.namespace, run_pods=True, pod_timeout=60)
            pod = next(x for x in rep.checks if x.name == "gpu-pod[node-0]")
            assert pod.ok, rep.table()
    finally:
        c.stop()


def test_must_gather_node_state_on_mi355x(tmp_path):
    from amdgpu_operator.cli.gather import gather_node

    node = gather_node("/", str(tmp_path))
    assert node["probe"]["ok"] and node["gpus"] and all(g["arch"] == "gfx950" for g in node["gpus"])
    assert node["metrics"] and node["metrics"][0]["vram_total_bytes"] > 280 * 2**30
