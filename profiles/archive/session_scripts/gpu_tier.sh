#!/bin/bash
# GPU test tier + one live metrics-exporter scrape (profiles evidence)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-tier}
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -15 $O/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 60 python3 -c "
from amdgpu_operator.exporter.metrics import MetricsExporter, SmiSource
src = SmiSource(); ex = MetricsExporter(src, 'mi355x', dcgm_names=True); ex.collect_once(); print(ex.render())
" > $O/metrics_live.txt 2>&1
rc=$?; echo "scrape rc=$rc"; grep -E "^amd_gpu_(xgmi|pcie|throttle|vram_max)" $O/metrics_live.txt | head -20
exit $rc
