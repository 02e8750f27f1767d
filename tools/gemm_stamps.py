"""Segment timing of the ping-pong GEMM from a diagnostic build
(build/libavk_stamps.so, -DAVK_STAMPS): s_memtime at six points per slice for
the 8 waves of the first 4 workgroups.  Prints median cycles per segment."""

import ctypes
import json
import os
import statistics
import sys

import torch

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = ctypes.CDLL(os.path.join(R, "build/libavk_stamps.so"))
P, I, S = ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p
lib.avk_gemm_bf16_nt_variant.argtypes = [P, P, P, I, I, I, I, I, S]
lib.avk_fill_uniform_bf16.argtypes = [P, ctypes.c_int64, ctypes.c_uint64, ctypes.c_float, ctypes.c_float, S]
lib.avk_stamps_read.argtypes = [P, I]
BLOCKS, WAVES, SLICES, POINTS = 4, 8, 32, 6


def run(n, variant):
    a = torch.empty(n, n, device="cuda", dtype=torch.bfloat16)
    b = torch.empty(n, n, device="cuda", dtype=torch.bfloat16)
    c = torch.empty(n, n, device="cuda", dtype=torch.bfloat16)
    st = torch.cuda.current_stream().cuda_stream
    lib.avk_fill_uniform_bf16(a.data_ptr(), a.numel(), 1, -1.0, 1.0, st)
    lib.avk_fill_uniform_bf16(b.data_ptr(), b.numel(), 2, -1.0, 1.0, st)
    for _ in range(20):  # warm clocks
        assert lib.avk_gemm_bf16_nt_variant(a.data_ptr(), b.data_ptr(), c.data_ptr(), 0, n, n, n, variant, st) == 0
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * (BLOCKS * WAVES * SLICES * POINTS))()
    assert lib.avk_stamps_read(buf, len(buf)) == 0
    v = list(buf)

    def at(blk, w, t, k):
        return v[((blk * WAVES + w) * SLICES + t) * POINTS + k]

    segs = {"read": (0, 1), "vmwait_r": (1, 2), "barrier_a": (2, 3), "mfma": (3, 4), "vmwait_m": (4, 5)}
    out = {}
    for grp, waves in (("group0", range(0, 4)), ("group1", range(4, 8))):
        d = {k: [] for k in segs}
        d["barrier_b"] = []
        d["slice"] = []
        for blk in range(BLOCKS):
            for w in waves:
                for t in range(8, SLICES - 1):
                    for name, (x, y) in segs.items():
                        d[name].append(at(blk, w, t, y) - at(blk, w, t, x))
                    d["barrier_b"].append(at(blk, w, t + 1, 0) - at(blk, w, t, 5))
                    d["slice"].append(at(blk, w, t + 1, 0) - at(blk, w, t, 0))
        out[grp] = {k: statistics.median(x) for k, x in d.items()}
    # absolute timeline of block 0, waves 0 and 4 (same SIMD), slices 8..11
    t0 = at(0, 0, 8, 0)
    out["timeline"] = {f"w{w}": [[at(0, w, t, k) - t0 for k in range(POINTS)] for t in range(8, 12)] for w in (0, 1, 4, 5)}
    return out


if __name__ == "__main__":
    res = {f"n{n}_v{v}": run(n, v) for n in (8192,) for v in (0,)}
    print(json.dumps(res, indent=1))
