#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s15
mkdir -p $O
timeout -k 10 300 python3 $R/tools/startup_timing.py > $O/startup.json 2>&1
rc=$?; echo "rc=$rc"; cat $O/startup.json | grep -v '"out"' | head -80
