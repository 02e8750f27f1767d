"""Micro-benchmarks of the validator kernels vs the vendor libraries.

Interleaved rounds in ONE process (cdna_hip_programming.md §5.4 rule 24), random
uniform [-1, 1) operands (rule 25).  Prints one JSON document.
"""

import argparse
import json
import statistics
import time

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from amdgpu_operator.ops import kernels as K  # noqa: E402


def time_ms(fn, iters):
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


GEMM_VARIANTS = {6: "default_8phase", 0: "ring_pingpong", 1: "dbuf", 2: "ring", 3: "w4", 4: "pp_load_in_r", 5: "pp_5slot",
                 7: "8phase_load_in_m", 8: "8phase_bal_load_in_r", 9: "8phase_bal_load_in_m",
                 10: "8phase_group_m8", 11: "8phase_group_m16", 12: "8phase_group_m2",
                 13: "8phase_lab_copy", 14: "4wave_builtin", 15: "4wave_asm",
                 16: "4wave_asm_no_glds", 17: "4wave_asm_no_barrier", 18: "4wave_asm_early_rotate",
                 19: "4wave_asm_no_dsread", 20: "4wave_asm_fixed_m0", 21: "4wave_asm_vgpr_loads",
                 22: "4wave_asm_piece_pairs", 23: "4wave_asm_piece_burst", 24: "4wave_asm_sched2", 25: "4wave_asm_sched3", 26: "4wave_asm_sched4", 27: "4wave_asm_sched4b", 28: "4wave_asm_sched4c", 29: "4wave_asm_sched4c_epi16", 30: "4wave_asm_sched4c_epi16_nt"}


def bench_gemm(n, rounds, iters, variants=None):
    """Every K2 variant (or the ``variants`` subset; all but the default need
    ``make -C native lab``) and hipBLASLt, interleaved
    round by round on the same random operands (cdna_hip_programming.md §5.4
    rules 24-25)."""
    sel = {v: GEMM_VARIANTS[v] for v in (variants if variants is not None else GEMM_VARIANTS)}
    a = torch.empty(n, n, device="cuda", dtype=torch.bfloat16)
    bt = torch.empty(n, n, device="cuda", dtype=torch.bfloat16)
    K.fill_uniform_(a, 1)
    K.fill_uniform_(bt, 2)
    c = torch.empty(n, n, device="cuda", dtype=torch.bfloat16)
    c2 = torch.empty_like(c)
    b = bt.t()
    times = {v: [] for v in sel}
    lib = []
    for _ in range(3):
        for v in sel:
            K.gemm_bf16_nt(a, bt, out=c, variant=v)
        torch.matmul(a, b, out=c2)
    for _ in range(rounds):
        for v in sel:
            times[v].append(time_ms(lambda: K.gemm_bf16_nt(a, bt, out=c, variant=v), iters))
        lib.append(time_ms(lambda: torch.matmul(a, b, out=c2), iters))
    fl = 2.0 * n ** 3
    K.gemm_bf16_nt(a, bt, out=c)
    err = (c.float() - c2.float()).abs().max().item()
    out = {"n": n}
    for v, name in sel.items():
        out[f"{name}_tflops"] = fl / statistics.median(times[v]) / 1e9
    ours = times[next(iter(sel))]
    out.update({
        "ours_ms_median": statistics.median(ours),
        "ours_tflops": fl / statistics.median(ours) / 1e9,
        "ours_tflops_best": fl / min(ours) / 1e9,
        "hipblaslt_ms_median": statistics.median(lib),
        "hipblaslt_tflops": fl / statistics.median(lib) / 1e9,
        "max_abs_diff_vs_hipblaslt": err,
    })
    return out


def bench_fp8(n, rounds, iters):
    """K2b (OCP e4m3 on v_mfma_f32_16x16x128_f8f6f4, bf16 out) against
    torch._scaled_mm (hipBLASLt's fp8 GEMM, unit scales, bf16 out) and the
    bf16 kernel, interleaved on the same random operands; TF/s also against
    the ~5 PF dense fp8 peak (MI355X_MICROARCH.md)."""
    a = torch.empty(n, n, device="cuda", dtype=torch.float8_e4m3fn)
    bt = torch.empty(n, n, device="cuda", dtype=torch.float8_e4m3fn)
    K.fill_fp8_(a, 11)
    K.fill_fp8_(bt, 12)
    c = torch.empty(n, n, device="cuda", dtype=torch.bfloat16)
    one = torch.ones((), device="cuda", dtype=torch.float32)
    a4 = torch.empty(n, n // 2, device="cuda", dtype=torch.uint8)
    b4 = torch.empty(n, n // 2, device="cuda", dtype=torch.uint8)
    K.fill_fp4_(a4, 13)
    K.fill_fp4_(b4, 14)
    c4 = torch.empty_like(c)
    arms = {"ours_fp8": lambda: K.gemm_fp8_nt(a, bt, out=c), "ours_fp4": lambda: K.gemm_fp4_nt(a4, b4, out=c4)}
    lib_err = None
    try:
        ref = torch._scaled_mm(a, bt.t(), scale_a=one, scale_b=one, out_dtype=torch.bfloat16)
        arms["scaled_mm_fp8"] = lambda: torch._scaled_mm(a, bt.t(), scale_a=one, scale_b=one, out_dtype=torch.bfloat16)
    except Exception as e:  # noqa: BLE001 - no fp8 GEMM in this torch build: report against the peak only
        ref, lib_err = None, f"{type(e).__name__}: {e}"[:300]
    ab, bb = a.to(torch.bfloat16), bt.to(torch.bfloat16)
    c16 = torch.empty_like(c)
    arms["ours_bf16_same_values"] = lambda: K.gemm_bf16_nt(ab, bb, out=c16)
    for fn in arms.values():
        fn()
    samples = {k: [] for k in arms}
    for _ in range(rounds):
        for k, fn in arms.items():
            samples[k].append(time_ms(fn, iters))
    fl = 2.0 * n ** 3
    out = {"n": n}
    for k, v in samples.items():
        out[k + "_tflops"] = fl / statistics.median(v) / 1e9
        out[k + "_tflops_best"] = fl / min(v) / 1e9
    out["ours_fp8_of_dense_peak"] = out["ours_fp8_tflops"] / 5000.0
    out["ours_fp4_of_dense_peak"] = out["ours_fp4_tflops"] / 10000.0  # FP4/FP6: 2x the fp8 rate on gfx950
    K.gemm_fp8_nt(a, bt, out=c)
    exact = a.float() @ bt.float().t()
    out["ours_fp8_max_rel_err_vs_fp32"] = ((c.float() - exact).abs().max() / exact.abs().max()).item()
    if ref is not None:
        out["scaled_mm_max_rel_err_vs_fp32"] = ((ref.float() - exact).abs().max() / exact.abs().max()).item()
        out["ours_over_scaled_mm"] = out["ours_fp8_tflops"] / out["scaled_mm_fp8_tflops"]
    else:
        out["scaled_mm_error"] = lib_err
    return out


def bench_hbm(nbytes, rounds, iters):
    src = torch.empty(nbytes // 4, device="cuda")
    dst = torch.empty_like(src)
    K.fill_uniform_(src, 3)
    res = {"bytes": nbytes}
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    arms = {
        "ours_plain": lambda: K.hbm_copy(src, dst, cus, 0),
        "ours_nt": lambda: K.hbm_copy(src, dst, cus, 1),
        "torch_copy": lambda: dst.copy_(src),
    }
    samples = {k: [] for k in arms}
    for fn in arms.values():
        fn()
    for _ in range(rounds):
        for k, fn in arms.items():
            samples[k].append(time_ms(fn, iters))
    for k, v in samples.items():
        res[k + "_gbps"] = 2 * nbytes / statistics.median(v) / 1e6
    return res


def bench_vecadd(n, iters):
    a = torch.empty(n, device="cuda")
    b = torch.empty(n, device="cuda")
    c = torch.empty(n, device="cuda")
    K.fill_uniform_(a, 1)
    K.fill_uniform_(b, 2)
    ms = time_ms(lambda: K.vector_add(a, b, c), iters)
    ms_t = time_ms(lambda: torch.add(a, b, out=c), iters)
    return {"n": n, "ours_gbps": 12 * n / ms / 1e6, "torch_gbps": 12 * n / ms_t / 1e6}


def bench_oneshot(n, peers, iters):
    ins = [torch.empty(n, device="cuda") for _ in range(peers)]
    for i, t in enumerate(ins):
        K.fill_uniform_(t, i)
    out = torch.empty(n, device="cuda")
    ms = time_ms(lambda: K.allreduce_oneshot(ins, out), iters)
    return {"n": n, "peers": peers, "ms": ms, "read_gbps": (peers + 1) * 4 * n / ms / 1e6}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--gemm-variants", type=int, nargs="+", default=None,
                    help="GEMM A/B only: these variants (the first is reported as ours) vs hipBLASLt")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--fp8", action="store_true", help="the fp8 GEMM vs torch._scaled_mm only (4096^3, 8192^3)")
    args = ap.parse_args()
    t0 = time.time()
    out = {"device": torch.cuda.get_device_name(0)}
    if args.fp8:
        out["fp8"] = [bench_fp8(n, args.rounds, 10) for n in (4096, 8192)]
    elif args.gemm_variants:
        out["gemm"] = [bench_gemm(n, args.rounds, 10, args.gemm_variants) for n in (4096, 8192)]
    elif args.quick:
        out["gemm"] = [bench_gemm(4096, 2, 5)]
        out["hbm"] = bench_hbm(1 << 30, 2, 5)
    else:
        out["gemm"] = [bench_gemm(n, 5, 10) for n in (4096, 8192)]
        out["hbm"] = bench_hbm(4 << 30, 5, 5)
        out["vecadd"] = bench_vecadd(1 << 26, 20)
        out["oneshot"] = bench_oneshot(1 << 24, 8, 10)
    out["wall_s"] = time.time() - t0
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
