"""amdgpu-validator --start-gate on the CPU: the process loads, waits at its
gate without any HIP call and leaves with status 3 when the gate says abort
(validator_main.cpp; validate.py validate_gpu prespawn)."""

import json
import subprocess
import threading
import time

from amdgpu_operator import native

VALIDATOR = str(native.binary("amdgpu-validator"))


def test_gate_abort_exits_before_any_hip_call(tmp_path):
    gate = tmp_path / "gate"
    gate.write_text("")  # no verdict yet

    def release():
        time.sleep(0.3)
        gate.write_text("abort")

    th = threading.Thread(target=release)
    t0 = time.perf_counter()  # before the releaser starts its 0.3 s sleep
    th.start()
    p = subprocess.run([VALIDATOR, "--rendezvous", str(tmp_path / "rv"), "--steps", "hip,vecadd", "--start-gate",
                        str(gate)], capture_output=True, text=True, timeout=30)
    th.join()
    assert p.returncode == 3 and time.perf_counter() - t0 >= 0.3
    rep = json.loads(p.stdout.strip().splitlines()[-1])
    assert rep["ok"] is False and rep["error"] == "start gate: aborted" and rep["steps"] == []


def test_gate_times_out(tmp_path):
    p = subprocess.run([VALIDATOR, "--rendezvous", str(tmp_path / "rv"), "--steps", "hip", "--start-gate",
                        str(tmp_path / "never"), "--timeout", "0.2"], capture_output=True, text=True, timeout=30)
    assert p.returncode == 3 and "start gate: timeout" in p.stdout
