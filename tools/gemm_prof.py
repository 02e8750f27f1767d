"""Drive the K2 GEMM variants for a rocprofv3 counter run (one process, fixed
random operands; see tools/pmc_summary.py for the aggregation)."""

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from amdgpu_operator.ops import kernels as K  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="+", default=[4096, 8192])
    ap.add_argument("--variants", type=int, nargs="+", default=[0, 1, 2])
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    for n in a.n:
        x = torch.empty(n, n, device="cuda", dtype=torch.bfloat16)
        w = torch.empty(n, n, device="cuda", dtype=torch.bfloat16)
        K.fill_uniform_(x, 1)
        K.fill_uniform_(w, 2)
        c = torch.empty(n, n, device="cuda", dtype=torch.bfloat16)
        for v in a.variants:
            for _ in range(a.iters):
                K.gemm_bf16_nt(x, w, out=c, variant=v)
            torch.cuda.synchronize()
        for _ in range(a.iters):
            torch.matmul(x, w.t(), out=c)
        torch.cuda.synchronize()
    return 0


if __name__ == "__main__":
    sys.exit(main())
