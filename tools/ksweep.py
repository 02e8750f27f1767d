"""Split a GEMM's time at M = N = ``--mn`` into a fixed part (launch,
prologue, epilogue) and a per-K part: the validator kernels at several K,
event-timed (fastest of ``--trials`` runs of ``--iters`` back-to-back
dispatches), then a least-squares line t(K) = fixed + K * slope per kernel.

  python tools/ksweep.py --mn 4096 --k 1024 2048 4096 8192 16384
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
    ap.add_argument("--mn", type=int, default=4096)
    ap.add_argument("--k", type=int, nargs="+", default=[1024, 2048, 4096, 8192, 16384])
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--trials", type=int, default=5)
    a = ap.parse_args()
    n = a.mn
    out = torch.empty(n, n, device="cuda", dtype=torch.bfloat16)
    rows: dict[str, list] = {}
    for k in a.k:
        ab = torch.randn(n, k, device="cuda").to(torch.bfloat16)
        bb = torch.randn(n, k, device="cuda").to(torch.bfloat16)
        a8, b8 = (torch.empty(n, k, device="cuda", dtype=torch.uint8) for _ in range(2))
        K.fill_fp8_(a8, 1)
        K.fill_fp8_(b8, 2)
        a4, b4 = (torch.empty(n, k // 2, device="cuda", dtype=torch.uint8) for _ in range(2))
        K.fill_fp4_(a4, 3)
        K.fill_fp4_(b4, 4)
        runs = {"bf16": lambda: K.gemm_bf16_nt(ab, bb, out=out),
                "fp8": lambda: K.gemm_fp8_nt(a8, b8, out=out),
                "fp4": lambda: K.gemm_fp4_nt(a4, b4, out=out)}
        for name, fn in runs.items():
            fn()
            torch.cuda.synchronize()
            ms = timed(fn, a.iters, a.trials)
            rows.setdefault(name, []).append((k, ms))
            print(json.dumps({"kernel": name, "m": n, "n": n, "k": k, "us": round(ms * 1000, 2),
                              "tflops": round(2.0 * n * n * k / (ms * 1e-3) / 1e12, 1)}), flush=True)
        del ab, bb, a8, b8, a4, b4
    for name, pts in rows.items():
        xs = [p[0] for p in pts]
        ys = [p[1] * 1000 for p in pts]
        mx, my = sum(xs) / len(xs), sum(ys) / len(ys)
        slope = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sum((x - mx) ** 2 for x in xs)
        fixed = my - slope * mx
        steady = 2.0 * n * n / (slope * 1e-6) / 1e12  # TF/s of the K loop alone
        print(json.dumps({"kernel": name, "fit": "t_us = fixed + k * slope", "fixed_us": round(fixed, 2),
                          "slope_us_per_k": round(slope, 5), "k_loop_tflops": round(steady, 1)}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
