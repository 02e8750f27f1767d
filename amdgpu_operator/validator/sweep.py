"""The node's collective curve over RCCL and its xGMI links, one by one.

SURVEY.md §5.8 asks for algBW, busBW and latency per message size at
n = 2/4/8, and §2.E lists the sweep (8 B ... 1 GiB; all-reduce, all-gather,
reduce-scatter) next to the validator's fixed-size check.  The reference has
no collective at all (/root/reference/README.md:1-220 runs only
``nvidia-smi``); its GPU nodes are plural (README.md:138-139) and the scaling
configuration is BASELINE.json ``configs[4]`` (8 pods x 1 GPU + an RCCL
all-reduce validator).

:func:`collective_sweep` runs one ``amdgpu-validator`` process per physical
GPU, through the node's launcher (``NodeEnv.launch``: under
``torch.distributed.run`` the rank that owns the GPU starts it), with the
steps ``hip,xgmi_links,sweep``:

* ``sweep`` - every size of ``8 x 4^k`` up to ``max_bytes`` for each op,
  checked exactly on the device, then timed (``validator_main.cpp``
  ``step_sweep``);
* ``xgmi_links`` (N >= 2) - each xGMI link read on its own, in lockstep
  rounds, with the data checked (``step_xgmi_links``): the per-peer GB/s that
  names a slow link which the all-peers K4 read only shows as a lower sum.

The rows of all ranks merge into one row per (op, size) at the slowest rank
(a collective is as slow as its slowest member), and next to each all-reduce
row stands the floor the validator's Ready gate applies at that size
(validate.py ``rccl_busbw_floor``, from the KFD link model), so the first
multi-GPU run shows how far above (or below) the model-derived floors the
fabric really is.  It runs after the node is Ready (bench.py), not inside a
bring-up: it holds 2 x ``max_bytes`` of HBM per GPU and takes seconds.
"""

from __future__ import annotations

import json
import os
import shutil
import time
from concurrent.futures import ThreadPoolExecutor

from ..nodeenv import REPORT_EARLY_ENV, NodeEnv
from . import validate as V

OPS = ("allreduce", "allgather", "reducescatter")
RATIO_FROM_BYTES = 1 << 20
BUS_FACTOR = {"allreduce": lambda n: 2.0 * (n - 1) / n, "allgather": lambda n: (n - 1) / n,
              "reducescatter": lambda n: (n - 1) / n}


def sizes(min_bytes: int = 8, max_bytes: int = 1 << 30, factor: int = 4) -> list[int]:
    """The message sizes (validator_main.cpp ``sweep_sizes``, which accepts
    factors 2 ... 1024)."""
    if not 2 <= factor <= 1024 or min_bytes < 1:
        raise ValueError(f"sweep factor must be in [2, 1024] (got {factor}) and min_bytes >= 1")
    out, b = [], min_bytes
    while b <= max_bytes:
        out.append(b)
        b *= factor
    if not out or out[-1] != max_bytes:
        out.append(max_bytes)
    return out


def merge_rows(world: int, reports: list[dict]) -> dict[str, list[dict]]:
    """Per op, one row per size from every rank's ``sweep`` rows: the slowest
    rank's time, algBW / busBW recomputed from it, ``ok`` only if no rank saw
    a mismatch."""
    merged: dict[tuple[str, int], dict] = {}
    for rep in reports:
        step = next((s for s in rep.get("steps", []) if s.get("name") == "sweep"), None) or {}
        for row in step.get("rows", []):
            key = (row["op"], int(row["bytes"]))
            m = merged.setdefault(key, {"op": row["op"], "bytes": int(row["bytes"]), "us": 0.0, "mismatches": 0,
                                        "ranks": 0})
            m["us"] = max(m["us"], float(row["us"]))
            m["mismatches"] += int(row.get("mismatches", 0))
            m["ranks"] += 1
    out: dict[str, list[dict]] = {}
    for (op, nbytes), m in sorted(merged.items(), key=lambda kv: (OPS.index(kv[0][0]) if kv[0][0] in OPS else 9,
                                                                    kv[0][1])):
        algbw = nbytes / (m["us"] * 1e-6) / 1e9 if m["us"] > 0 else 0.0
        busbw = algbw * BUS_FACTOR[op](world) if world > 1 and op in BUS_FACTOR else 0.0
        out.setdefault(op, []).append({"bytes": nbytes, "latency_us": round(m["us"], 2),
                                       "algbw_gbps": round(algbw, 2), "busbw_gbps": round(busbw, 2),
                                       "ok": m["mismatches"] == 0 and m["ranks"] == len(reports)})
    return out


def link_matrix(reports: list[dict], world: int) -> dict:
    """Per-peer xGMI read GB/s: ``reads[r][p]`` = rank r reading rank p's
    buffer over their link (None on the diagonal)."""
    reads = [[None] * world for _ in range(world)]
    intact = True
    for r, rep in enumerate(reports):
        step = next((s for s in rep.get("steps", []) if s.get("name") == "xgmi_links"), None) or {}
        for ln in step.get("links", []):
            p = int(ln["peer"])
            if 0 <= p < world:
                reads[r][p] = ln.get("read_gbps")
            intact = intact and ln.get("intact", False) is True
    vals = [v for row in reads for v in row if v is not None]
    return {"read_gbps": reads, "min_read_gbps": min(vals) if vals else None,
            "max_read_gbps": max(vals) if vals else None, "intact": intact and bool(vals)}


def collective_sweep(env: NodeEnv, max_bytes: int = 1 << 30, min_bytes: int = 8, factor: int = 4,
                     link_bytes: int = 64 << 20, rccl_fraction: float = 0.2, xgmi_fraction: float = 0.25,
                     timeout: float = 120.0, ops: tuple[str, ...] = OPS) -> dict:
    """Run the sweep on every physical GPU of the node (module docstring)."""
    from ..discovery import topology

    t0 = time.perf_counter()
    gpus = topology.enumerate_gpus(env.sysfs_root())
    if not gpus:
        raise V.StepFailed("no GPUs to sweep")
    plan = V.rank_plan(gpus)
    world = len(plan)
    run_id = "sweep-" + os.urandom(5).hex()
    rdv = os.path.join(env.validations_dir, "rendezvous", run_id)
    os.makedirs(rdv, exist_ok=True)
    steps = "hip,xgmi_links,sweep" if world > 1 else "hip,sweep"
    args = ["--steps", steps, "--sweep-min-bytes", str(min_bytes), "--sweep-max-bytes", str(max_bytes),
            "--sweep-factor", str(factor), "--sweep-ops", ",".join(ops), "--link-bytes", str(link_bytes),
            "--peer-timeout", "60", "--collective-timeout", "60", "--expect-devices", "1"]
    jobs = []
    for r, devs in enumerate(plan):
        others = [plan[q][0] for q in range(world) if q != r]
        jenv = {**V.thp_malloc_env(), **topology.visible_devices_env([devs[0], *others], gpus), REPORT_EARLY_ENV: "1"}
        jobs.append((r, V.workload_argv(args + ["--local-bdf", devs[0].bdf], r, world, rdv, run_id, 0), jenv))

    def one(job):
        r, argv, jenv = job
        res = env.launch(argv, jenv, device=r, timeout=timeout)
        if world > 1 and (res.rc != 0 or V.report_rc(res.stdout) != 0):
            V.abort_run(rdv, f"{run_id} rank {r} failed (rc {res.rc})")
        return res

    try:
        with ThreadPoolExecutor(max_workers=len(jobs)) as ex:
            results = list(ex.map(one, jobs))
    finally:
        shutil.rmtree(rdv, ignore_errors=True)
    reports = []
    for res in results:
        try:
            rep = json.loads(res.stdout.strip().splitlines()[-1]) if res.stdout.strip() else {}
        except ValueError:
            rep = {"raw": res.stdout[-2000:]}
        rep["rc"] = res.rc
        if res.rc != 0:
            rep["stderr"] = res.stderr[-1500:]
        reports.append(rep)
    ok = all(r.get("rc") == 0 and r.get("ok") for r in reports)
    rows = merge_rows(world, reports) if ok else {}
    out: dict = {"ok": ok and all(row["ok"] for op_rows in rows.values() for row in op_rows), "world": world,
                 "sizes": max((len(v) for v in rows.values()), default=0), "ops": rows,
                 "comm_init_s": max((s.get("comm_init_s") or 0.0 for r in reports for s in r.get("steps", [])
                                     if s.get("name") == "sweep"), default=None),
                 "simulated": any(r.get("simulated") for r in reports)}
    if not ok:
        out["error"] = V.failure_summary(reports)
    if world > 1:
        out["xgmi_links"] = link_matrix(reports, world) if ok else None
        floors = V.fabric_floors(env, plan, gpus, rccl_fraction, xgmi_fraction, 0)
        link_sum = min(floors["link_gbps_per_rank"]) if floors["link_gbps_per_rank"] else 0.0
        # the Ready gate's floors at every all-reduce size, next to the measured busBW
        # (the ratio from 1 MiB up: below it the alpha-beta model's floor is a
        # few GB/s or less and the ratio says nothing about the links)
        vs = []
        for row in rows.get("allreduce", []):
            f = V.rccl_busbw_floor(link_sum, rccl_fraction, row["bytes"])
            vs.append({"bytes": row["bytes"], "busbw_gbps": row["busbw_gbps"], "floor_gbps": round(f, 2),
                       "ratio": round(row["busbw_gbps"] / f, 2) if f > 0 and row["bytes"] >= RATIO_FROM_BYTES
                       else None})
        per_link = {}
        links = V._xgmi_link_gbps(env, gpus)
        for r, devs in enumerate(plan):
            for q, peer in enumerate(plan):
                if q != r:
                    nominal = links.get((devs[0].index, peer[0].index)) or V.NOMINAL_XGMI_LINK_GBPS
                    per_link[f"{r}-{q}"] = round(xgmi_fraction * nominal, 1)
        lm = out.get("xgmi_links") or {}
        out["fabric_floors"] = {
            "link_gbps_per_rank": floors["link_gbps_per_rank"],
            "rccl_busbw_link_fraction": rccl_fraction, "xgmi_read_link_fraction": xgmi_fraction,
            "allreduce_vs_floor": vs,
            "min_allreduce_ratio": min((v["ratio"] for v in vs if v["ratio"] is not None), default=None),
            # one link alone: the K4 fraction of that link's nominal rate
            "min_link_read_floor_gbps": min(per_link.values()) if per_link else None,
            "links_below_floor": [k for k, f in per_link.items()
                                  if lm.get("read_gbps") and lm["read_gbps"][int(k.split("-")[0])][int(k.split("-")[1])]
                                  is not None and lm["read_gbps"][int(k.split("-")[0])][int(k.split("-")[1])] < f],
        }
        if floors.get("nominal_pairs"):
            out["fabric_floors"]["nominal_pairs"] = floors["nominal_pairs"]
    out["seconds"] = round(time.perf_counter() - t0, 3)
    if not ok:
        out["ranks"] = [{k: r.get(k) for k in ("rank", "rc", "ok", "error", "failed_peer", "peer_state")}
                        for r in reports]
    return out
