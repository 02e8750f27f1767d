cd /tmp
N=/root/repo/amdgpu_operator/_native
rm -f /tmp/g1; (sleep 1; echo go > /tmp/g1) &
AMDGPU_VALIDATOR_COUNTERS=1 ROCP_TOOL_LIBRARIES=$N/libamdgpu_counter_gate.so ROCPROFILER_METRICS_PATH=$N/gate-metrics timeout -k 5 60 $N/amdgpu-validator --rendezvous /tmp/rvk --steps hip,gemm --counter-gate --start-gate /tmp/g1 | cut -c1-400
wait
rm -f /tmp/g2; (sleep 1; echo go > /tmp/g2) &
timeout -k 5 60 $N/amdgpu-validator --rendezvous /tmp/rvk2 --steps hip,gemm --start-gate /tmp/g2 | cut -c1-300
wait
