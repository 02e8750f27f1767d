"""Stand-in for the native ``amdgpu-validator`` on machines without a GPU.

Accepts the same arguments, rendezvous with its peer ranks through the same
directory protocol as ``native/validator/validator_main.cpp`` (liveness
records ``<run>-alive-<r>`` / ``-failed-`` / ``-done-``, the orchestrator's
``abort`` file, ``--peer-timeout``), so multi-rank orchestration and its
bounded failure are exercised for real, and prints the same JSON report shape
with ``"simulated": true``.

``--expect-devices N`` (a rank validating a GPU's N partitions) reports the
kernel steps once per device, with ``"device"`` and ``local_devices``, as the
native binary does.

``AMDGPU_FAKE_GPU_PROC_LOG=<dir>``: every stand-in writes ``<dir>/<pid>.json``
with its start and end (``time.monotonic``, comparable across processes) and
its role, so a test can count how many "GPU processes" were alive at once.

Fault injection for the CPU tests: ``AMDGPU_FAKE_VALIDATOR_FAULT`` =
``<run-id suffix or *>:<rank>:<kind>`` with kind ``fail`` (report a failure at
once), ``exit`` (die without a report, after the liveness record) or ``hang``
(never reach the rendezvous; stops only when aborted).
"""

from __future__ import annotations

import json
import os
import sys
import time


def visible_count(env: dict) -> int | None:
    """GPUs a (stand-in) GPU process would see: the length of its
    ``ROCR_VISIBLE_DEVICES`` / ``HIP_VISIBLE_DEVICES`` (None: unrestricted)."""
    for k in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES"):
        if env.get(k) is not None:
            return len([x for x in env[k].split(",") if x])
    return None


_HELD: list = []


def _hold_for_life(path: str) -> None:
    """``<gate>.held`` locked until the process exits, as the native validator
    does (driver/manager.py _release_gated_validators waits on it)."""
    import fcntl

    try:
        f = open(path, "a")
        fcntl.flock(f, fcntl.LOCK_EX | fcntl.LOCK_NB)
        _HELD.append(f)
    except OSError:
        pass


def wait_start_gate(path: str | None, timeout: float = 120.0, abort_path: str | None = None) -> str:
    """The native validator's ``--start-gate``: block until the file has a
    verdict; "go" releases the process (same protocol as validator_main.cpp,
    where "init" already lets the runtime start: a stand-in has none, so it
    waits on for the final verdict).  An abort file in the run's rendezvous
    directory aborts the wait too."""
    if not path:
        return "go"
    _hold_for_life(path + ".held")
    deadline = time.time() + timeout
    while time.time() < deadline:
        try:
            with open(path) as f:
                text = f.read().strip()
            if text and text != "init":
                return text
        except FileNotFoundError:
            pass
        if abort_path and os.path.exists(abort_path):
            return "abort"
        time.sleep(0.001)
    return "timeout"


class PeerError(RuntimeError):
    def __init__(self, peer: int, state: str, msg: str):
        super().__init__(msg)
        self.peer = peer
        self.state = state


class Rendezvous:
    """Python twin of validator_main.cpp's Rendezvous liveness protocol."""

    def __init__(self, rdv: str, run_id: str, rank: int, world: int, peer_timeout: float):
        self.rdv, self.run_id, self.rank, self.world = rdv, run_id, rank, world
        self.peer_timeout = peer_timeout
        self.t0 = time.monotonic()

    def _p(self, name: str) -> str:
        return os.path.join(self.rdv, name)

    def marker(self, kind: str, r: int) -> str:
        return self._p(f"{self.run_id}-{kind}-{r}")

    def publish(self, path: str, text: str) -> None:
        tmp = f"{path}.tmp.{os.getpid()}"
        with open(tmp, "w") as f:
            f.write(text)
        os.replace(tmp, path)

    def announce(self) -> None:
        self.publish(self.marker("alive", self.rank), f"{os.getpid()} 0\n")

    def finish(self, ok: bool, error: str = "") -> None:
        self.publish(self.marker("done" if ok else "failed", self.rank), "ok" if ok else error)

    def _read(self, path: str) -> str | None:
        try:
            with open(path) as f:
                return f.read().strip()
        except FileNotFoundError:
            return None

    def peer(self, r: int) -> tuple[str, str]:
        if (t := self._read(self.marker("failed", r))) is not None:
            return "failed", t
        if self._read(self.marker("done", r)) is not None:
            return "done", ""
        t = self._read(self.marker("alive", r))
        if not t:
            return "missing", ""
        pid = int(t.split()[0])
        try:
            with open(f"/proc/{pid}/stat") as f:
                state = f.read().rsplit(")", 1)[1].split()[0]
            if state in ("Z", "X"):
                raise FileNotFoundError
        except (FileNotFoundError, IndexError):
            if self._read(self.marker("done", r)) is not None:
                return "done", ""
            return "dead", f"pid {pid}"
        return "alive", ""

    def watch(self, only: int = -1) -> None:
        if (why := self._read(self._p("abort"))) is not None:
            raise PeerError(-1, "aborted", f"run aborted by the orchestrator: {why}")
        age = time.monotonic() - self.t0
        for r in range(self.world):
            if r == self.rank or (only >= 0 and r != only):
                continue
            st, d = self.peer(r)
            if st == "failed":
                raise PeerError(r, "failed", f"rank {r} failed: {d}")
            if st == "dead":
                raise PeerError(r, "dead", f"rank {r} ({d}) exited before the rendezvous completed")
            if st == "missing" and age > self.peer_timeout:
                raise PeerError(r, "missing", f"rank {r} never started (no liveness record after {age:.1f} s)")

    def barrier(self, tag: str, timeout: float = 60.0) -> None:
        self.publish(self._p(f"{self.run_id}-barrier-{tag}-{self.rank}"), "1")
        deadline = time.monotonic() + timeout
        for r in range(self.world):
            while not os.path.exists(self._p(f"{self.run_id}-barrier-{tag}-{r}")):
                self.watch(r)
                if time.monotonic() > deadline:
                    raise RuntimeError(f"rendezvous: timeout waiting for rank {r}")
                time.sleep(0.002)


# The stand-in's fabric: every peer link at ~60 % of the MI355X xGMI nominal
# (76 GB/s per direction), collectives on the alpha-beta shape the floors use
# (validate.py RCCL_HALF_BW_BYTES).  Only the shape matters to the CPU tests:
# numbers that pass the default floors, and fail floors set far above them.
SIM_LINK_GBPS = 45.0
SIM_LATENCY_US = 12.0
# GEMM rates of the simulated GPU (TF/s at 4096^3): above the default floors
# (api/clusterpolicy.py WorkloadSpec), below floors set far above them
SIM_GEMM_TFLOPS = {"gemm": 1300.0, "gemm_fp8": 2600.0, "gemm_fp4": 4100.0, "gemm_fp6": 3600.0, "gemm_mxfp4": 4000.0}


def sim_busbw(world: int, nbytes: int) -> float:
    return SIM_LINK_GBPS * max(1, world - 1) * nbytes / (nbytes + (16 << 20))


def simulated_detail(step: str, argv: list[str], rank: int, world: int) -> dict:
    """Extra report fields of a simulated step: the measured-rate fields the
    native binary reports, from the model above, and the floor verdicts the
    binary applies to them (``--min-rccl-busbw-gbps``, ``--min-xgmi-read-gbps``)."""
    def arg(name, default):
        return argv[argv.index(name) + 1] if name in argv else default

    if step in SIM_GEMM_TFLOPS:  # the binary's floors apply from 4096^3 (validator_main.cpp gemm_floor)
        size_flag, floor_flag = {"gemm": ("--gemm", "--min-gemm-tflops"), "gemm_fp8": ("--fp8-gemm", "--min-fp8-tflops"),
                                 "gemm_fp4": ("--fp4-gemm", "--min-fp4-tflops"),
                                 "gemm_fp6": ("--fp8-gemm", "--min-fp6-tflops"),
                                 "gemm_mxfp4": ("--fp4-gemm", "--min-mxfp4-tflops")}[step]
        n = int(arg(size_flag, "4096"))
        tf = SIM_GEMM_TFLOPS[step]
        floor = float(arg(floor_flag, "0")) if n >= 4096 else 0.0
        ok = floor <= 0 or tf >= floor
        gated = "--counter-gate" in argv
        return {"ok": ok, "n": n, "tflops": tf, "min_tflops": floor, "perf_ok": ok,
                "counter_gate": "pass" if gated else "off", **({"gate_attempts": 1} if gated else {})}
    if step == "rccl" and world > 1:
        nbytes = 4 * int(arg("--rccl-elems", str(1 << 24)))
        bus = sim_busbw(world, nbytes)
        floor = float(arg("--min-rccl-busbw-gbps", "0"))
        ok = floor <= 0 or bus >= floor
        return {"ok": ok, "world": world, "bytes": nbytes, "busbw_gbps": round(bus, 1), "min_busbw_gbps": floor,
                "perf_ok": ok, "comm_init_s": 0.0}
    if step == "xgmi" and world > 1:
        read = SIM_LINK_GBPS * (world - 1)
        floor = float(arg("--min-xgmi-read-gbps", "0"))
        ok = floor <= 0 or read >= floor
        return {"ok": ok, "peers": world, "peer_read_gbps": round(read, 1), "min_peer_read_gbps": floor,
                "perf_ok": ok}
    if step == "xgmi_links" and world > 1:
        return {"world": world, "links": [{"peer": (rank + k) % world, "read_gbps": SIM_LINK_GBPS, "intact": True}
                                          for k in range(1, world)], "min_read_gbps": SIM_LINK_GBPS}
    if step == "sweep":
        lo, hi, f = int(arg("--sweep-min-bytes", "8")), int(arg("--sweep-max-bytes", str(1 << 30))), \
            int(arg("--sweep-factor", "4"))
        ops = arg("--sweep-ops", "allreduce,allgather,reducescatter").split(",")
        rows = []
        for op in ("allreduce", "allgather", "reducescatter"):
            if op not in ops:
                continue
            b = lo
            sizes = []
            while b <= hi:
                sizes.append(b)
                b *= f
            if not sizes or sizes[-1] != hi:
                sizes.append(hi)
            last = None
            for nbytes in sizes:
                n = max(world, (nbytes // 4) // world * world) * 4
                if n == last:  # as the native step: sizes below `world` floats round up to one tensor
                    continue
                last = n
                factor = (2.0 if op == "allreduce" else 1.0) * (world - 1) / world if world > 1 else 0.0
                peak = SIM_LINK_GBPS * max(1, world - 1)  # alpha-beta: latency + bytes on the wire / link rate
                us = SIM_LATENCY_US + (n * factor if world > 1 else n) / (peak * 1e3)
                algbw = n / (us * 1e-6) / 1e9
                rows.append({"op": op, "bytes": n, "iters": 1, "us": round(us, 2), "algbw_gbps": round(algbw, 2),
                             "busbw_gbps": round(algbw * factor, 2), "mismatches": 0})
        return {"world": world, "comm_init_s": 0.0, "mismatches": 0, "rows": rows}
    return {}


def _fault(run_id: str, rank: int) -> str | None:
    spec = os.environ.get("AMDGPU_FAKE_VALIDATOR_FAULT", "")
    for item in filter(None, spec.split(",")):
        where, r, kind = item.split(":")
        if (where == "*" or run_id.endswith(where)) and int(r) == rank:
            return kind
    return None


def _log_lifetime(t_start: float, argv: list[str]) -> None:
    d = os.environ.get("AMDGPU_FAKE_GPU_PROC_LOG")
    if not d:
        return
    os.makedirs(d, exist_ok=True)
    role = "validator" if "--rank" in argv or "--local-bdf" in argv else "pod"
    with open(os.path.join(d, f"{os.getpid()}.json"), "w") as f:
        json.dump({"start": t_start, "end": time.monotonic(), "role": role, "argv": argv}, f)


def main(argv: list[str]) -> int:
    t_start = time.monotonic()
    try:
        return _main(argv)
    finally:
        _log_lifetime(t_start, argv)


def _main(argv: list[str]) -> int:
    def arg(name, default):
        return argv[argv.index(name) + 1] if name in argv else default

    rank, world = int(arg("--rank", "0")), int(arg("--world", "1"))
    rdv, run_id = arg("--rendezvous", "/tmp/amdgpu-validator"), arg("--run-id", "run")
    os.makedirs(rdv, exist_ok=True)
    rv = Rendezvous(rdv, run_id, rank, world, float(arg("--peer-timeout", "30")))
    if world > 1:
        rv.announce()
    fault = _fault(run_id, rank)
    if fault == "exit":
        os._exit(9)
    verdict = wait_start_gate(arg("--start-gate", None), abort_path=os.path.join(rdv, "abort") if world > 1 else None)
    if verdict != "go":
        if world > 1:
            rv.finish(False, f"start gate: {verdict}")
        print(json.dumps({"ok": False, "error": f"start gate: {verdict}", "steps": []}))
        return 3

    steps = arg("--steps", "hip,vecadd,gemm,mfma,hbm,xgmi,rccl").split(",")
    t0 = time.perf_counter()
    if "--pod-check" in argv:  # a plugin-validation pod: every allocated GPU must be in the container
        expect, seen = int(arg("--expect-devices", "-1")), visible_count(dict(os.environ))
        if expect >= 0 and seen is not None and seen != expect:
            print(json.dumps({"ok": False, "simulated": True, "steps": [],
                              "error": f"{expect} GPU(s) allocated to the pod, {seen} visible"}))
            return 1
    ndev = max(1, int(arg("--expect-devices", "1")))
    per_device = ("vecadd", "gemm", "gemm_fp8", "gemm_fp4", "gemm_fp6", "gemm_mxfp4", "mfma", "hbm", "dmabuf")
    recs = []
    for s in steps:
        for d in (range(ndev) if s in per_device and ndev > 1 else [None]):
            recs.append({"name": s, "ok": True, "seconds": 0.0, "simulated": True, **({"device": d} if d is not None else {}),
                         **simulated_detail(s, argv, rank, world)})
    below = [r["name"] for r in recs if r.get("ok") is False]
    rep = {"ok": True, "simulated": True, "rank": rank, "world": world, "device": int(arg("--device", "0")),
           "owner_rank_env": os.environ.get("RANK"), "hip_visible_devices": os.environ.get("HIP_VISIBLE_DEVICES"),
           "rocr_visible_devices": os.environ.get("ROCR_VISIBLE_DEVICES"), "local_bdf": arg("--local-bdf", None),
           "local_devices": list(range(ndev)), "steps": recs}
    try:
        if fault == "fail":
            raise RuntimeError("injected failure")
        if fault == "hang":
            while True:  # ends only through the abort file (or a kill)
                rv.watch(rank)
                time.sleep(0.005)
        if world > 1 and any(s in steps for s in ("rccl", "xgmi", "peers", "sweep", "xgmi_links")):
            rv.barrier("rccl" if "rccl" in steps else "xgmi")  # like the RCCL unique-id exchange
        if below:  # a measured rate under its floor (the native binary's perf_ok)
            raise RuntimeError(f"step {below[0]} failed")
    except PeerError as e:
        rep.update(ok=False, error=str(e), failed_peer=e.peer, peer_state=e.state)
    except RuntimeError as e:
        rep.update(ok=False, error=str(e))
    rep["seconds"] = time.perf_counter() - t0
    if world > 1:
        rv.finish(rep["ok"], rep.get("error", ""))
    print(json.dumps(rep))
    sys.stdout.flush()
    # the report in a file as well, like the native checks: --result-file
    # (amdgpu-gpu-check) always, --ready-file (amdgpu-validator) when ok
    for flag, always in (("--result-file", True), ("--ready-file", False)):
        path = arg(flag, None)
        if path and (always or rep["ok"]):
            with open(path + ".tmp", "w") as f:
                f.write(json.dumps(rep))
            os.replace(path + ".tmp", path)
    if os.environ.get("AMDGPU_FAKE_POD_EXIT_S") and "--pod-check" in argv:
        # the kernel's release of a GPU process after its exit: a signal does
        # not cut it short, so the kubelet's stop waits it out
        import signal

        signal.signal(signal.SIGTERM, signal.SIG_IGN)
        time.sleep(float(os.environ["AMDGPU_FAKE_POD_EXIT_S"]))
    return 0 if rep["ok"] else 1


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
