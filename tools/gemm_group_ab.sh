#!/bin/bash
# 8-phase GEMM: tile rows per L2 band (GROUP_M 4 = shipped, lab variants 10/11/12/13 = 8/16/2/4).
# Outputs must equal the shipped kernel's bit for bit (same tiles, another order), then the interleaved timing.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${1:-gemm_group}; mkdir -p $O; cd $R
timeout -k 10 120 python3 - > $O/check.txt 2>&1 <<'PY'
import torch
from amdgpu_operator.ops import kernels as K
for n in (4096, 8192):
    a = torch.empty(n, n, device="cuda", dtype=torch.bfloat16); bt = torch.empty_like(a)
    K.fill_uniform_(a, 1); K.fill_uniform_(bt, 2)
    ref = K.gemm_bf16_nt(a, bt, out_dtype=torch.float32, variant=6)
    for v in (10, 11, 12):
        out = K.gemm_bf16_nt(a, bt, out_dtype=torch.float32, variant=v)
        print(n, v, "identical" if torch.equal(out, ref) else f"DIFFERENT max {float((out - ref).abs().max())}")
PY
rc=$?; cat $O/check.txt; [ $rc -ne 0 ] && exit $rc
grep -q DIFFERENT $O/check.txt && exit 1
timeout -k 10 300 python3 -u tools/kernel_bench.py --gemm-variants 6 10 11 12 --rounds 8 > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; python3 -c "
import json; d=json.load(open('$O/bench.json'))
for g in d['gemm']: print({k: v for k, v in g.items() if 'tflops' in k or k == 'n'})"
exit $rc
