#!/bin/bash
# validator step times after the SDMA-free read-backs and the gate set-up thread
set -o pipefail
export PYTHONPATH="$GRAFT_REPO_ROOT"
O=gpurun_out/r5_valfast
mkdir -p $O
N=amdgpu_operator/_native
A="--steps hip,vecadd,gemm,gemm_fp8,gemm_fp4,mfma,hbm --counter-gate --min-gemm-tflops 620 --min-fp8-tflops 1200 --min-fp4-tflops 1900 --min-hbm-gbps 3700"
for i in 1 2 3; do
  timeout -k 5 60 $N/amdgpu-validator --rendezvous /tmp/rv-vf $A > $O/val.$i.json || exit 1
  sleep 1
done
echo validator done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_native_gpu.py > $O/pytest_native_gpu.log 2>&1 || exit 1
echo pytest done
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-pod-workload --no-sweep > $O/bench.json 2> $O/bench.err || exit 1
echo bench done
