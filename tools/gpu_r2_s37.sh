#!/bin/bash
# Round 2: fault-injection soak on the real MI355X (operand pod deletions, kubelet restarts, policy
# edits; every revalidation runs the HIP/MFMA validator on the device)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2s37
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u tools/chaos_sim.py --real-gpu --seeds 1-3 --steps 8 --timeout 60 > $O/chaos_real_gpu.log 2>&1
rc=$?; echo "chaos rc=$rc"; grep -E "^seed|NOT" $O/chaos_real_gpu.log | tail -30
exit $rc
