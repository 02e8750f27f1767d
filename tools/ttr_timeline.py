"""Compact per-step critical-path timeline from a ``bench.py --detail`` file.

Every time is seconds after ClusterPolicy creation:

  nfd / dp / val   spawn of the NFD worker, device-plugin and validator processes
  drv              the validator's driver validation (driver-ready seen, N1 probe)
  reg / k_list     plugin Register reaching the kubelet / the kubelet's first device list
  seen             validator sees the devices (pod-resources API)
  wl / plug        workload (kernel checks) and plugin-validation pod done
  done             node labelled validated
  val_written / val_ready   validator's ready file written / seen by the kubelet
  ttr              ClusterPolicy ready and node validated

usage: python tools/ttr_timeline.py DETAIL.json [OUT.json]
"""

from __future__ import annotations

import json
import statistics
import sys


def step_row(s: dict) -> dict:
    ops = s.get("operands") or {}
    tl = s.get("timeline_s") or {}

    def op(key):
        return next((v for k, v in ops.items() if k.endswith(key)), {})

    nfd, dp, val = op("/nfd-worker"), op("/amd-device-plugin"), op("/amd-operator-validator")
    row = {"ttr": round(s["time_to_ready_s"], 4), "nfd": nfd.get("spawn_at_s"), "dp": dp.get("spawn_at_s"),
           "val": val.get("spawn_at_s"), "drv": tl.get("driver"),
           "reg": (s.get("kubelet_register_at_s") or [None])[0],
           "k_list": next(iter((s.get("kubelet_first_list_at_s") or {}).values()), None),
           "seen": tl.get("plugin.devices_seen"), "wl": tl.get("workload"), "plug": tl.get("plugin"),
           "done": tl.get("complete")}
    if val.get("ready_written_s") is not None:
        row["val_written"] = round(val["spawn_at_s"] + val["ready_written_s"], 4)
    if val.get("ready_s") is not None:
        row["val_ready"] = round(val["spawn_at_s"] + val["ready_s"], 4)
    return row


def main() -> int:
    d = json.load(open(sys.argv[1]))
    rows = [step_row(s) for s in d["steps"]]
    keys = [k for k in rows[0] if all(isinstance(r.get(k), (int, float)) for r in rows)]
    out = {"summary": {k: d["summary"].get(k) for k in ("value", "n_gpus", "steps", "warmup", "ms_per_step")},
           "thread_mode_time_to_ready_s": d["summary"]["config"].get("thread_mode_time_to_ready_s"),
           "median": {k: round(statistics.median(r[k] for r in rows), 4) for k in keys}, "steps": rows}
    text = json.dumps(out, indent=1)
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            f.write(text + "\n")
    else:
        print(text)
    return 0


if __name__ == "__main__":
    sys.exit(main())
