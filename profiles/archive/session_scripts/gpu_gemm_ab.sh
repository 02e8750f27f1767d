#!/bin/bash
# GEMM variant A/B: numerics of every variant, then the interleaved kernel bench
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-gemm_ab}
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm" > $O/gemm_tests.log 2>&1
rc=$?; echo "gemm tests rc=$rc"; tail -3 $O/gemm_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u tools/kernel_bench.py > $O/kernel_bench.json 2> $O/kernel_bench.err
rc=$?; echo "kernel_bench rc=$rc"; grep -E "tflops\"|gbps|\"n\"" $O/kernel_bench.json
exit $rc
