"""N >= 2 validator runs that cannot complete end within their deadline, on
the one MI355X of the box (tests/test_validator_rendezvous.py has the CPU
side of the protocol).

Rank 0 runs the RCCL step (ncclCommInitRank on its set-up thread, awaited
against the rendezvous): its peer is either never launched, or launched and
killed after publishing its liveness record.  Either way rank 0 must report
the failed rank by number within the deadline, abandon the set-up thread
blocked in RCCL's bootstrap and exit - no process of the run may be left
holding the GPU.

Also here: the Ready-gate floors with teeth - the same binary with a floor
above what the GPU delivers fails the node."""

import json
import os
import subprocess
import time

import pytest

from amdgpu_operator import native

pytestmark = pytest.mark.gpu
VALIDATOR = str(native.binary("amdgpu-validator"))


def _spawn(rdv, rank, steps, extra=()):
    return subprocess.Popen([VALIDATOR, "--rank", str(rank), "--world", "2", "--device", "0", "--rendezvous", str(rdv),
                             "--run-id", "mr", "--steps", steps, "--rccl-elems", "1048576", *extra],
                            stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                            env={**os.environ, "AMDGPU_VALIDATOR_TEARDOWN": "0"})


def _gone(pid: int, timeout: float = 15.0) -> bool:
    deadline = time.monotonic() + timeout
    while time.monotonic() < deadline:
        if not os.path.exists(f"/proc/{pid}"):
            return True
        time.sleep(0.05)
    return False


def _kfd_holders(pids) -> list[int]:
    out = []
    for pid in pids:
        try:
            for fd in os.listdir(f"/proc/{pid}/fd"):
                if os.readlink(f"/proc/{pid}/fd/{fd}") == "/dev/kfd":
                    out.append(pid)
                    break
        except OSError:
            pass
    return out


def test_rccl_rank_never_launched_fails_within_deadline(tmp_path):
    t0 = time.monotonic()
    p0 = _spawn(tmp_path, 0, "hip,rccl", ["--peer-timeout", "4"])
    out, err = p0.communicate(timeout=60)
    took = time.monotonic() - t0
    rep = json.loads(out.strip().splitlines()[-1])
    print(json.dumps({"took_s": round(took, 3), "report": rep}))
    assert p0.returncode == 1 and not rep["ok"]
    assert rep["failed_peer"] == 1 and rep["peer_state"] == "missing", rep
    assert "rank 1 never started" in rep["error"] and "rccl init" in rep["error"]
    assert took < 4 + 10  # deadline + the hip step + a bounded abort
    p0.wait()
    assert _gone(p0.pid) and not _kfd_holders([p0.pid])


def test_rccl_rank_killed_after_publishing_fails_at_once(tmp_path):
    gate = tmp_path / "gate"
    gate.write_text("")
    p1 = _spawn(tmp_path, 1, "hip,rccl", ["--start-gate", str(gate)])
    deadline = time.monotonic() + 30
    while not (tmp_path / "mr-alive-1").exists():
        assert time.monotonic() < deadline and p1.poll() is None
        time.sleep(0.01)
    t0 = time.monotonic()
    p0 = _spawn(tmp_path, 0, "hip,rccl", ["--peer-timeout", "60"])
    time.sleep(0.5)  # rank 0 is in its RCCL set-up, rank 1 published and waits at its gate
    p1.kill()
    p1.wait()
    out, err = p0.communicate(timeout=60)
    took = time.monotonic() - t0
    rep = json.loads(out.strip().splitlines()[-1])
    print(json.dumps({"took_s": round(took, 3), "report": rep}))
    assert p0.returncode == 1 and rep["failed_peer"] == 1 and rep["peer_state"] == "dead", rep
    assert f"pid {p1.pid}" in rep["error"]
    assert took < 15  # not the 60 s peer timeout
    p0.wait()
    assert _gone(p0.pid) and _gone(p1.pid) and not _kfd_holders([p0.pid, p1.pid])


def _local(tmp_path, steps, extra):
    p = subprocess.run([VALIDATOR, "--rendezvous", str(tmp_path), "--steps", steps, *extra],
                       capture_output=True, text=True, timeout=120)
    rep = json.loads(p.stdout.strip().splitlines()[-1])
    return p.returncode, rep, {s["name"]: s for s in rep["steps"]}


def test_default_floors_pass_on_a_healthy_mi355x(tmp_path):
    rc, rep, st = _local(tmp_path, "hip,gemm,hbm", ["--counter-gate", "--min-gemm-tflops", "620",
                                                    "--min-hbm-gbps", "3700", "--min-mfma-util", "0.2"])
    print(json.dumps({k: {f: st[k].get(f) for f in ("tflops", "gbps", "mfma_util", "mfma_util_floor")} for k in st}))
    assert rc == 0 and rep["ok"], rep
    assert st["gemm"]["perf_ok"] and st["hbm"]["perf_ok"] and st["gemm"]["counter_gate"] == "pass"
    assert st["gemm"]["mfma_util"] >= 0.2


def test_floor_above_the_gpu_fails_the_node(tmp_path):
    rc, rep, st = _local(tmp_path, "hip,gemm", ["--min-gemm-tflops", "100000"])
    assert rc == 1 and not rep["ok"] and st["gemm"]["perf_ok"] is False
    rc, rep, st = _local(tmp_path, "hip,hbm", ["--min-hbm-gbps", "100000"])
    assert rc == 1 and st["hbm"]["perf_ok"] is False
    rc, rep, st = _local(tmp_path, "hip,gemm", ["--counter-gate", "--min-mfma-util", "0.99"])
    assert rc == 1 and st["gemm"]["counter_gate"] == "fail" and "below floor" in st["gemm"]["gate_reason"]


def test_small_gemm_gate_util_recorded(tmp_path):
    # the plugin-pod size: occupancy-scaled floor still passes
    rc, rep, st = _local(tmp_path, "hip,gemm", ["--gemm", "1024", "--counter-gate", "--min-mfma-util", "0.2"])
    print(json.dumps({f: st["gemm"].get(f) for f in ("mfma_util", "mfma_util_floor", "tflops")}))
    assert rc == 0 and st["gemm"]["counter_gate"] == "pass", rep


def test_kernel_check_process_restricted_to_its_gpu(tmp_path):
    """At N > 1 a kernel-check process sees only its own GPU
    (topology.visible_devices_env: ROCR_VISIBLE_DEVICES by KFD unique id) and
    addresses it as HIP device 0."""
    from amdgpu_operator.discovery import topology

    gpus = topology.enumerate_gpus("/")
    env = topology.visible_devices_env([gpus[-1]], gpus)
    assert "ROCR_VISIBLE_DEVICES" in env, env
    p = subprocess.run([VALIDATOR, "--rendezvous", str(tmp_path), "--device", "0", "--steps", "hip,vecadd,gemm",
                        "--gemm", "1024"], capture_output=True, text=True, timeout=120, env={**os.environ, **env})
    rep = json.loads(p.stdout.strip().splitlines()[-1])
    assert p.returncode == 0 and rep["ok"], (rep, p.stderr[-1000:])
    assert {s["name"]: s for s in rep["steps"]}["hip"]["arch"].startswith("gfx950")


def test_all_devices_validates_every_gpu_the_pod_holds(tmp_path):
    """The plugin-validation pod holds all of a resource's GPUs and checks
    each one from a single process (--all-devices): every visible device
    runs hip + vecadd, and each step record names its device."""
    rc, rep, _ = _local(tmp_path, "hip,vecadd", ["--all-devices"])
    assert rc == 0 and rep["ok"] and rep["device"] == -1, rep
    n = sum(1 for s in rep["steps"] if s["name"] == "hip")
    assert n >= 1 and [(s["device"], s["name"]) for s in rep["steps"]] == \
        [(d, step) for d in range(n) for step in ("hip", "vecadd")], rep["steps"]
    # peers-only steps are refused with it
    p = subprocess.run([VALIDATOR, "--all-devices", "--steps", "hip,rccl"], capture_output=True, text=True, timeout=30)
    assert p.returncode == 2 and "--all-devices" in p.stderr


def test_gpu_check_runs_a_kernel_per_visible_gpu():
    """The plugin pod's check (amdgpu-gpu-check): HSA runtime only, one
    host-verified kernel per visible GPU, report in the validator's shape."""
    check = str(native.binary("amdgpu-gpu-check"))
    p = subprocess.run([check, "--timeout", "20"], capture_output=True, text=True, timeout=60)
    rep = json.loads(p.stdout.strip().splitlines()[-1])
    assert p.returncode == 0 and rep["ok"] and rep["devices"] >= 1, rep
    adds = [s for s in rep["steps"] if s["name"] == "vecadd"]
    assert len(adds) == rep["devices"] and all(s["mismatches"] == 0 and s["elems"] == 65536 for s in adds)
    assert all(s["agent"].startswith("gfx950") for s in rep["steps"] if s["name"] == "hsa")


def test_local_bdf_selects_the_gpu_and_checks_the_device_count(tmp_path):
    """One process per physical GPU (validate.py rank_plan): --local-bdf picks
    every visible device at the GPU's PCI address (the GPU in SPX, its
    partitions otherwise); --expect-devices fails a process that sees fewer."""
    from amdgpu_operator.discovery import topology

    gpu = topology.enumerate_gpus("/")[0]
    rc, rep, st = _local(tmp_path, "hip,vecadd,gemm", ["--local-bdf", gpu.bdf.upper(), "--expect-devices", "1",
                                                        "--gemm", "1024", "--counter-gate"])
    assert rc == 0 and rep["ok"] and rep["local_devices"] == [0], rep
    assert st["gemm"]["counter_gate"] == "pass"
    rc, rep, _ = _local(tmp_path, "hip,vecadd", ["--local-bdf", gpu.bdf, "--expect-devices", "2"])
    assert rc == 1 and "2 device(s) expected, 1 visible" in rep["error"], rep
    rc, rep, _ = _local(tmp_path, "hip,vecadd", ["--local-bdf", "0000:ff:1f.7"])
    assert rc == 1 and "no visible device at 0000:ff:1f.7" in rep["error"], rep


def test_all_devices_threaded_path_with_counter_gate(tmp_path):
    """--all-devices runs each device's steps on a thread of its own (with
    several devices the gated GEMM goes last, GateTurns); on this box that
    is one device, in the single-device step order."""
    rc, rep, _ = _local(tmp_path, "hip,vecadd,gemm,hbm", ["--all-devices", "--gemm", "1024", "--counter-gate",
                                                          "--hbm-bytes", str(1 << 26)])
    assert rc == 0 and rep["ok"], rep
    names = [(s["device"], s["name"]) for s in rep["steps"]]
    assert names == [(0, "hip"), (0, "vecadd"), (0, "gemm"), (0, "hbm")], names
    g = [s for s in rep["steps"] if s["name"] == "gemm"][0]
    assert g["counter_gate"] == "pass" and g["gated_output_matches"]


def test_gpu_check_fails_when_an_allocated_gpu_is_missing():
    check = str(native.binary("amdgpu-gpu-check"))
    p = subprocess.run([check, "--timeout", "20", "--expect-devices", "2"], capture_output=True, text=True, timeout=60)
    rep = json.loads(p.stdout.strip().splitlines()[-1])
    assert p.returncode == 1 and "2 GPU(s) allocated to the pod, 1 visible" in rep["error"], rep
    p = subprocess.run([check, "--timeout", "20", "--expect-devices", "1"], capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, p.stdout


def test_ipc_one_shot_eight_processes_one_gpu(tmp_path):
    """K4's multi-process path at its full width: 8 ranks (8 processes) on one
    GPU exchange IPC handles and each reads all 8 buffers; a peer-read floor
    above what the device delivers fails every rank (the N >= 2 gate)."""
    def run(extra, tag):
        procs = [subprocess.Popen([VALIDATOR, "--rank", str(r), "--world", "8", "--device", "0", "--rendezvous",
                                   str(tmp_path / tag), "--run-id", tag, "--steps", "hip,xgmi", "--xgmi-elems",
                                   str(1 << 20), "--peer-timeout", "60", *extra],
                                  stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(8)]
        outs = [p.communicate(timeout=120) for p in procs]
        return [(p.returncode, json.loads(o.strip().splitlines()[-1]), e) for p, (o, e) in zip(procs, outs)]

    reps = run([], "ok")
    for rc, rep, err in reps:
        assert rc == 0 and rep["ok"], (rep, err[-2000:])
        x = {s["name"]: s for s in rep["steps"]}["xgmi"]
        assert not x["emulated"] and x["peers"] == 8 and x["max_abs_err"] <= 8e-5 and x["peer_read_gbps"] > 0
    print(json.dumps([{s["name"]: s for s in r["steps"]}["xgmi"]["peer_read_gbps"] for _, r, _ in reps]))
    for rc, rep, _ in run(["--min-xgmi-read-gbps", "1e9"], "floor"):
        x = {s["name"]: s for s in rep["steps"]}["xgmi"]
        assert rc == 1 and x["perf_ok"] is False and x["max_abs_err"] <= 8e-5


def test_xgmi_link_rate_matches_the_kfd_nominal_on_mi355x():
    """The link-rate check of validate.check_fabric on real data: amd-smi's
    xGMI rate x width of this GPU against the KFD nominal of its XGMI
    io_links (76 GB/s per direction) - a healthy GPU must pass."""
    from amdgpu_operator.discovery import topology

    with topology.Smi() as smi:
        ms = smi.collect()
    vals = ms[0].values
    nominal = [lk.max_bandwidth_mbps / 1000 for lk in topology.links("/") if lk.is_xgmi and lk.max_bandwidth_mbps]
    if not nominal:  # a one-GPU slice of a hive: the peers' KFD nodes are listed, not enumerated as GPUs
        import glob

        for p in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/io_links/*/properties"):
            try:
                with open(p) as f:
                    kv = dict(ln.split() for ln in f if len(ln.split()) == 2)
            except OSError:  # other GPUs' nodes may be unreadable here
                continue
            if kv.get("type") == "11" and int(kv.get("max_bandwidth", 0)):  # CRAT_IOLINK_TYPE_XGMI
                nominal.append(int(kv["max_bandwidth"]) / 1000)
    print(json.dumps({"speed": vals.get("xgmi_link_speed_gbps"), "width": vals.get("xgmi_link_width"),
                      "up": vals.get("xgmi_links_up"), "nominal": sorted(set(nominal))}))
    if not vals.get("xgmi_link_speed_gbps") or not vals.get("xgmi_link_width") or not nominal:
        pytest.skip("amd-smi reports no xGMI rate/width here")
    assert vals["xgmi_link_speed_gbps"] * vals["xgmi_link_width"] / 8 >= 0.9 * min(nominal)


def test_dmabuf_export_of_hbm_round_trips():
    """driver.rdma's device step: HBM exported as a dma-buf (what an RDMA NIC
    imports), the fd an amdgpu dma-buf of the buffer's size, and the buffer
    imported back aliasing the original both ways (validator_main.cpp
    step_dmabuf)."""
    p = subprocess.run([VALIDATOR, "--steps", "hip,dmabuf"], capture_output=True, text=True, timeout=90)
    rep = json.loads(p.stdout.strip().splitlines()[-1])
    s = {x["name"]: x for x in rep["steps"]}["dmabuf"]
    print(json.dumps(s))
    assert p.returncode == 0 and rep["ok"] and s["ok"], (s, p.stderr[-2000:])
    assert s["exporter"] in ("amdgpu", "drm") and s["dmabuf_bytes"] >= s["bytes"] == 64 << 20  # drm: PRIME
    assert s["read_match"] and s["write_through"] and not s["error"]


def test_rdma_discovery_on_the_real_host():
    """discovery/rdma.py on the box's own sysfs: its RDMA NICs (if any) with
    their PCIe paths, each GPU's nearest ones and the GFD labels."""
    from amdgpu_operator.discovery import labels, rdma, topology

    gpus = topology.enumerate_gpus("/")
    nics = rdma.enumerate_nics("/")
    out = {"readiness": rdma.readiness("/"),
           "nics": [{"name": n.name, "bdf": n.bdf, "numa": n.numa_node, "path": list(n.pci_path),
                     "ports": [list(p) for p in n.ports]} for n in nics],
           "gpus": [{"bdf": g.bdf, "numa": g.numa_node, "path": list(rdma.pci_path("/", g.bdf))} for g in gpus],
           "nearest": rdma.nearest_nics(gpus, nics), "labels": rdma.rdma_labels(gpus)}
    print(json.dumps(out))
    if not nics:
        pytest.skip("no RDMA device on this host")
    assert all(n.pci_path[0].startswith("pci") for n in nics)
    assert all(rdma.pci_path("/", g.bdf)[0].startswith("pci") for g in gpus)
    assert set(out["nearest"]) == {g.bdf for g in gpus} and all(out["nearest"].values())
    assert labels.gfd_labels(gpus)["amd.com/gpu.rdma.nics"] == str(sum(1 for n in nics if n.active))
