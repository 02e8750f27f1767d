#!/bin/bash
# repeated interleaved GEMM A/B of a few variants (DVFS noise: many rounds)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-gemm_rounds}
shift
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u tools/kernel_bench.py --rounds 15 --gemm-variants "$@" > $O/kernel_bench.json 2> $O/kernel_bench.err
rc=$?; echo "kernel_bench rc=$rc"; grep -E "tflops\"|\"n\"" $O/kernel_bench.json; tail -3 $O/kernel_bench.err
exit $rc
