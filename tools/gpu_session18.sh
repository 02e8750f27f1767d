#!/bin/bash
# 8-phase GEMM variants: numerics, A/B kernel bench, then the full GPU tier + N=1 bench
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s18
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm" > $O/gemm_tests.log 2>&1
rc=$?; echo "gemm tests rc=$rc"; tail -3 $O/gemm_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u tools/kernel_bench.py > $O/kernel_bench.json 2> $O/kernel_bench.err
rc=$?; echo "kernel_bench rc=$rc"; grep -E "tflops|gbps" $O/kernel_bench.json | head -40
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 $O/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --detail $O/bench_detail.json > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; cat $O/bench.json; tail -3 $O/bench.err
exit $rc
