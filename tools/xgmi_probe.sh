set -u
mkdir -p gpurun_out/xgmi_probe
timeout -k 10 200 python -u -m pytest tests/test_validator_multirank_gpu.py -k "link_rate or eight_processes" -s -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/xgmi_probe/pytest.log 2>&1
rc=$?
tail -5 gpurun_out/xgmi_probe/pytest.log
timeout -k 10 60 python -u - > gpurun_out/xgmi_probe/smi.json 2>&1 <<'PY'
import json
from amdgpu_operator.discovery import topology
with topology.Smi() as smi:
    ms = smi.collect()
print(json.dumps({m.bdf: {k: v for k, v in m.values.items() if "xgmi" in k or "pcie" in k} for m in ms}, indent=1))
print(json.dumps([(l.src, l.dst, l.is_xgmi, l.max_bandwidth_mbps, l.weight) for l in topology.links("/")]))
PY
cat gpurun_out/xgmi_probe/smi.json | head -60
(ls /sys/class/kfd/kfd/topology/nodes/*/io_links/*/properties && head -20 /sys/class/kfd/kfd/topology/nodes/*/io_links/*/properties) > gpurun_out/xgmi_probe/io_links.txt 2>&1
timeout -k 5 30 amd-smi xgmi > gpurun_out/xgmi_probe/amd_smi_xgmi.txt 2>&1
timeout -k 5 30 amd-smi metric -x > gpurun_out/xgmi_probe/amd_smi_metric_x.txt 2>&1
exit $rc
