"""Drive the low-precision K2 GEMMs (fp8 e4m3, fp4 e2m1, fp6 e2m3, MXFP4 with
E8M0 block scales) for timing and rocprofv3 counter runs: fixed random
operands per size, ``--iters`` back-to-back dispatches per kernel, then one
JSON line per (kernel, size) with the fastest of ``--trials`` event-timed
trials.  Under ``rocprofv3 --pmc`` the counters of every dispatch are summed
per kernel by tools/pmc_summary.py.

  python tools/lowp_prof.py --n 4096 8192
"""

from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from amdgpu_operator.ops import kernels as K  # noqa: E402


def timed(fn, iters: int, trials: int) -> float:
    best = None
    for _ in range(trials):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        e1.synchronize()
        ms = e0.elapsed_time(e1) / iters
        best = ms if best is None else min(best, ms)
    return best


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="+", default=[4096, 8192])
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--trials", type=int, default=3)
    a = ap.parse_args()
    dev = "cuda"
    for n in a.n:
        out = torch.empty(n, n, device=dev, dtype=torch.bfloat16)
        a8, b8 = (torch.empty(n, n, device=dev, dtype=torch.uint8) for _ in range(2))
        K.fill_fp8_(a8, 1)
        K.fill_fp8_(b8, 2)
        a4, b4 = (torch.empty(n, n // 2, device=dev, dtype=torch.uint8) for _ in range(2))
        K.fill_fp4_(a4, 3)
        K.fill_fp4_(b4, 4)
        a6, b6 = (torch.empty(n, n, device=dev, dtype=torch.uint8) for _ in range(2))
        K.fill_fp6_(a6, 5)
        K.fill_fp6_(b6, 6)
        sa, sb = (torch.empty(n, 8, device=dev, dtype=torch.uint8) for _ in range(2))
        K.fill_e8m0_(sa, 7)
        K.fill_e8m0_(sb, 8)
        runs = {
            "fp8_e4m3": lambda: K.gemm_fp8_nt(a8, b8, out=out),
            "fp4_e2m1": lambda: K.gemm_fp4_nt(a4, b4, out=out),
            "fp6_e2m3": lambda: K.gemm_fp6_nt(a6, b6, out=out),
            "mxfp4": lambda: K.gemm_mxfp4_nt(a4, b4, sa, sb, out=out),
        }
        for name, fn in runs.items():
            fn()
            torch.cuda.synchronize()
            ms = timed(fn, a.iters, a.trials)
            print(json.dumps({"kernel": name, "n": n, "ms": round(ms, 4),
                              "tflops": round(2.0 * n ** 3 / (ms * 1e-3) / 1e12, 1)}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
