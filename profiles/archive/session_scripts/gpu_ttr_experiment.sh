#!/bin/bash
# time-to-Ready start-up variance: default vs no counter gate vs plugin pods after the workload
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-ttr_exp}
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u bench.py --steps 8 --warmup 1 --detail $O/default.json > $O/default.out 2> $O/default.err || exit $?
timeout -k 10 300 python3 -u bench.py --steps 8 --warmup 1 --no-counter-gate --detail $O/nogate.json > $O/nogate.out 2> $O/nogate.err || exit $?
AMDGPU_EXPERIMENT_PLUGIN_AFTER_WORKLOAD=1 timeout -k 10 300 python3 -u bench.py --steps 8 --warmup 1 --detail $O/serial.json > $O/serial.out 2> $O/serial.err || exit $?
python3 - $O <<'PY'
import json, sys
for name in ("default", "nogate", "serial"):
    d = json.load(open(f"{sys.argv[1]}/{name}.json"))
    ttr = [round(s["time_to_ready_s"], 3) for s in d["steps"]]
    hip = [round(s["rank0_step_seconds"].get("hip") or 0, 3) for s in d["steps"]]
    proc = [s["workload_process_seconds"][0] for s in d["steps"]]
    print(name, "mean", round(sum(ttr) / len(ttr), 3), "ttr", ttr, "hip", hip, "proc", proc)
PY
