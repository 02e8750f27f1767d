"""Python bindings for the hand-written gfx950 validator kernels (K1-K4).

Thin :mod:`ctypes` layer over ``libamdgpu_validator.so``
(``native/validator/validator_kernels.hip``).  Tensors are PyTorch-ROCm device
tensors; every call is enqueued on the current HIP stream.  Host-side shape
checks mirror the kernel's assumptions, and the C launchers check them again
(they return ``hipErrorInvalidValue`` instead of launching), so a bad shape
never reaches the GPU.

There is deliberately no eager-PyTorch fallback: if the library is missing
:class:`amdgpu_operator.native.NativeUnavailable` is raised.
"""

from __future__ import annotations

import ctypes
from dataclasses import dataclass

from .. import native

LIB_NAME = "libamdgpu_validator.so"
# every GEMM variant of rounds 1-2, for A/B runs: `make -C native lab` (not shipped)
LAB_LIB_NAME = "lab/libamdgpu_validator_lab.so"

GEMM_BM = 256
GEMM_BN = 256
GEMM_BK = 64

_c_i64 = ctypes.c_int64
_c_ptr = ctypes.c_void_p


class KernelError(RuntimeError):
    pass


def _lib(name: str = LIB_NAME) -> ctypes.CDLL:
    lib = native.load(name)
    if getattr(lib, "_avk_typed", False):
        return lib
    P, I, I64, U64, F, S = _c_ptr, ctypes.c_int, _c_i64, ctypes.c_uint64, ctypes.c_float, _c_ptr
    sig = {
        "avk_abi_version": ([], I),
        "avk_fill_uniform_f32": ([P, I64, U64, F, F, S], I),
        "avk_fill_uniform_bf16": ([P, I64, U64, F, F, S], I),
        "avk_vector_add_f32": ([P, P, P, I64, S], I),
        "avk_vector_add_verify_f32": ([P, P, P, I64, P, S], I),
        "avk_gemm_bf16_nt": ([P, P, P, I, I, I, I, S], I),
        "avk_gemm_bf16_nt_variant": ([P, P, P, I, I, I, I, I, S], I),
        "avk_gemv_rows": ([P, I, P, P, I, I, S], I),
        "avk_gemm_fp8_nt": ([P, P, P, I, I, I, I, S], I),
        "avk_fill_fp8": ([P, I64, U64, S], I),
        "avk_gemm_fp4_nt": ([P, P, P, I, I, I, I, S], I),
        "avk_fill_fp4": ([P, I64, U64, S], I),
        "avk_gemv_rows_fp8": ([P, P, P, I, I, S], I),
        "avk_gemv_cols_fp8": ([P, P, P, I, I, S], I),
        "avk_gemv_cols_bf16": ([P, P, P, I, I, S], I),
        "avk_gemv_rows_fp4": ([P, P, P, I, I, S], I),
        "avk_gemv_cols_fp4": ([P, P, P, I, I, S], I),
        "avk_gemm_fp6_nt": ([P, P, P, I, I, I, I, S], I),
        "avk_fill_fp6": ([P, I64, U64, S], I),
        "avk_gemv_rows_fp6": ([P, P, P, I, I, S], I),
        "avk_gemv_cols_fp6": ([P, P, P, I, I, S], I),
        "avk_gemm_mxfp4_nt": ([P, P, P, P, P, I, I, I, I, S], I),
        "avk_fill_e8m0": ([P, I64, U64, I, I, S], I),
        "avk_gemv_rows_mxfp4": ([P, P, P, P, I, I, S], I),
        "avk_gemv_cols_mxfp4": ([P, P, P, P, I, I, S], I),
        "avk_hbm_copy": ([P, P, I64, I, I, S], I),
        "avk_checksum": ([P, I64, P, S], I),
        "avk_max_abs_diff_f32": ([P, P, I64, P, S], I),
        "avk_allreduce_oneshot_f32": ([ctypes.POINTER(P), I, P, I64, S], I),
        "avk_allreduce_twoshot_f32": ([ctypes.POINTER(P), ctypes.POINTER(P), I, I, I64, S], I),
        "avk_fill_const": ([P, I64, I, ctypes.c_float, S], I),
        "avk_check_blocks": ([P, I64, I, I64, ctypes.c_float, ctypes.c_float, P, S], I),
        "avk_mfma_probe_count": ([], I),
        "avk_mfma_probe_name": ([I], ctypes.c_char_p),
        "avk_mfma_probe": ([I, U64, ctypes.POINTER(I), S], I),
    }
    for name, (args, res) in sig.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    lib._avk_typed = True
    return lib


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise KernelError(f"{what} failed with hipError {rc}")


def _stream(stream=None) -> int:
    import torch

    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream


def _require(t, dtype, name: str, numel_multiple: int = 1, aligned: bool = True) -> None:
    import torch

    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor")
    if not t.is_cuda:
        raise ValueError(f"{name} must be a GPU tensor")
    if t.dtype != dtype:
        raise ValueError(f"{name} must be {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    if aligned and t.data_ptr() % 16:
        raise ValueError(f"{name} must be 16-byte aligned")
    if t.numel() % numel_multiple:
        raise ValueError(f"{name}.numel() must be a multiple of {numel_multiple}")


def abi_version() -> int:
    return _lib().avk_abi_version()


def fill_uniform_(t, seed: int, lo: float = -1.0, hi: float = 1.0, stream=None):
    """Deterministic device-side uniform fill (fp32 or bf16)."""
    import torch

    seed &= (1 << 64) - 1
    if t.dtype == torch.float32:
        _require(t, torch.float32, "t")
        _check(_lib().avk_fill_uniform_f32(t.data_ptr(), t.numel(), seed, lo, hi, _stream(stream)), "fill_f32")
    elif t.dtype == torch.bfloat16:
        _require(t, torch.bfloat16, "t", 8)
        _check(_lib().avk_fill_uniform_bf16(t.data_ptr(), t.numel(), seed, lo, hi, _stream(stream)), "fill_bf16")
    else:
        raise ValueError(f"unsupported dtype {t.dtype}")
    return t


def vector_add(a, b, out=None, stream=None):
    """K1: ``out = a + b`` (fp32)."""
    import torch

    _require(a, torch.float32, "a")
    _require(b, torch.float32, "b")
    if a.numel() != b.numel():
        raise ValueError("a and b differ in size")
    if out is None:
        out = torch.empty_like(a)
    _require(out, torch.float32, "out")
    _check(_lib().avk_vector_add_f32(a.data_ptr(), b.data_ptr(), out.data_ptr(), a.numel(), _stream(stream)), "vector_add")
    return out


def vector_add_verify(a, b, c, stream=None) -> int:
    """K1 check on the device: number of i with ``c[i] != a[i] + b[i]``."""
    import torch

    for t, n in ((a, "a"), (b, "b"), (c, "c")):
        _require(t, torch.float32, n)
    if not a.numel() == b.numel() == c.numel():
        raise ValueError("size mismatch")
    bad = torch.empty(1, device=a.device, dtype=torch.int64)
    _check(_lib().avk_vector_add_verify_f32(a.data_ptr(), b.data_ptr(), c.data_ptr(), a.numel(), bad.data_ptr(),
                                            _stream(stream)), "vector_add_verify")
    return int(bad.item())


GEMM_DEFAULT_VARIANT = 29   # 4 waves x 128x128, generated main loop (schedule 4c), 16-B bf16 stores (K % 256 == 0)
GEMM_FALLBACK_VARIANT = 6   # 8-phase, 8 waves (K a multiple of 64)
GEMM_DEFAULT_K_MULTIPLE = 256
# variants in the shipped library; the rest need `make -C native lab`
SHIPPED_GEMM_VARIANTS = (6, 29)


def gemm_bf16_nt(a, bt, out=None, out_dtype=None, stream=None, variant: int | None = None):
    """K2: ``out[M,N] = a[M,K] @ bt[N,K].T`` on MFMA (bf16 in, fp32 accumulate).

    M and N must be multiples of 256 and K of 64 (the kernels have no edge
    tiles; the validator picks its shapes accordingly).  ``variant=None`` runs
    what the native validator runs: the 4-wave kernel (GEMM_DEFAULT_VARIANT)
    when K is a multiple of 256, else the 8-phase kernel
    (GEMM_FALLBACK_VARIANT).  The other generated schedules of the 4-wave
    kernel (15, 24-28, 30) and the A/B kernels of rounds 1-3 are served from
    the tools build (``make -C native lab``).
    """
    import torch

    _require(a, torch.bfloat16, "a")
    _require(bt, torch.bfloat16, "bt")
    if a.dim() != 2 or bt.dim() != 2 or a.shape[1] != bt.shape[1]:
        raise ValueError(f"bad GEMM operands {tuple(a.shape)} x {tuple(bt.shape)}^T")
    M, K = a.shape
    N = bt.shape[0]
    if M % GEMM_BM or N % GEMM_BN or K % GEMM_BK:
        raise ValueError(f"GEMM shape {M}x{N}x{K} must be multiples of {GEMM_BM}x{GEMM_BN}x{GEMM_BK}")
    if out is None:
        out = torch.empty((M, N), device=a.device, dtype=out_dtype or torch.bfloat16)
    if out.shape != (M, N) or out.dtype not in (torch.bfloat16, torch.float32):
        raise ValueError("bad GEMM output")
    _require(out, out.dtype, "out")
    if variant is None:
        variant = GEMM_DEFAULT_VARIANT if K % GEMM_DEFAULT_K_MULTIPLE == 0 else GEMM_FALLBACK_VARIANT
    lib = _lib() if variant in SHIPPED_GEMM_VARIANTS else _lib(LAB_LIB_NAME)
    rc = lib.avk_gemm_bf16_nt_variant(a.data_ptr(), bt.data_ptr(), out.data_ptr(), int(out.dtype == torch.float32),
                                      M, N, K, variant, _stream(stream))
    _check(rc, "gemm_bf16_nt")
    return out


FP8_K_MULTIPLE = 256


def _fp8_bytes(t, name: str):
    """An OCP e4m3 operand as its bytes: ``torch.float8_e4m3fn`` or uint8."""
    import torch

    if t.dtype == torch.float8_e4m3fn:
        t = t.view(torch.uint8)
    _require(t, torch.uint8, name)
    return t


def fill_fp8_(t, seed: int, stream=None):
    """Deterministic random finite e4m3 values (|x| <= 3.75) into a
    ``float8_e4m3fn`` / uint8 tensor (the fp8 rate step's operands)."""
    b = _fp8_bytes(t, "t")
    _check(_lib().avk_fill_fp8(b.data_ptr(), b.numel(), seed & ((1 << 64) - 1), _stream(stream)), "fill_fp8")
    return t


def gemm_fp8_nt(a, bt, out=None, out_dtype=None, stream=None):
    """K2b: ``out[M,N] = a[M,K] @ bt[N,K].T`` with OCP e4m3 operands
    (``torch.float8_e4m3fn`` or their uint8 bytes) on
    ``v_mfma_f32_16x16x128_f8f6f4``, fp32 accumulation, bf16 or fp32 out.
    M and N multiples of 256, K of 256 (the kernel has no edge tiles)."""
    import torch

    ab, bb = _fp8_bytes(a, "a"), _fp8_bytes(bt, "bt")
    if ab.dim() != 2 or bb.dim() != 2 or ab.shape[1] != bb.shape[1]:
        raise ValueError(f"bad GEMM operands {tuple(ab.shape)} x {tuple(bb.shape)}^T")
    M, K = ab.shape
    N = bb.shape[0]
    if M % GEMM_BM or N % GEMM_BN or K % FP8_K_MULTIPLE:
        raise ValueError(f"fp8 GEMM shape {M}x{N}x{K} must be multiples of {GEMM_BM}x{GEMM_BN}x{FP8_K_MULTIPLE}")
    if out is None:
        out = torch.empty((M, N), device=ab.device, dtype=out_dtype or torch.bfloat16)
    if out.shape != (M, N) or out.dtype not in (torch.bfloat16, torch.float32):
        raise ValueError("bad GEMM output")
    _require(out, out.dtype, "out")
    _check(_lib().avk_gemm_fp8_nt(ab.data_ptr(), bb.data_ptr(), out.data_ptr(), int(out.dtype == torch.float32),
                                  M, N, K, _stream(stream)), "gemm_fp8_nt")
    return out


FP4_K_MULTIPLE = 256
FP4_K_MIN = 512
# e2m1 code -> value (OCP FP4: 1 sign, 2 exponent (bias 1), 1 mantissa bit)
FP4_VALUES = (0.0, 0.5, 1.0, 1.5, 2.0, 3.0, 4.0, 6.0, -0.0, -0.5, -1.0, -1.5, -2.0, -3.0, -4.0, -6.0)


def fp4_to_float(t):
    """FP4 pairs (uint8 [..., K/2], element 2k in the low nibble) -> float32 [..., K]."""
    import torch

    lut = torch.tensor(FP4_VALUES, dtype=torch.float32, device=t.device)
    b = t.view(torch.uint8).long()
    return torch.stack((lut[b & 15], lut[b >> 4]), dim=-1).flatten(-2)


def fill_fp4_(t, seed: int, stream=None):
    """Deterministic random FP4 bytes (two e2m1 codes each, all finite) into
    a uint8 tensor."""
    import torch

    _require(t, torch.uint8, "t")
    _check(_lib().avk_fill_fp4(t.data_ptr(), t.numel(), seed & ((1 << 64) - 1), _stream(stream)), "fill_fp4")
    return t


def gemm_fp4_nt(a, bt, out=None, out_dtype=None, stream=None):
    """K2c: ``out[M,N] = A[M,K] @ Bt[N,K].T`` with OCP FP4 operands (e2m1
    pairs in uint8 ``[M, K/2]`` / ``[N, K/2]``, element 2k in the low nibble)
    on ``v_mfma_f32_16x16x128_f8f6f4 cbsz:4 blgp:4``, fp32 accumulation, bf16
    or fp32 out.  M, N multiples of 256; K a multiple of 256, at least 512."""
    import torch

    _require(a, torch.uint8, "a")
    _require(bt, torch.uint8, "bt")
    if a.dim() != 2 or bt.dim() != 2 or a.shape[1] != bt.shape[1]:
        raise ValueError(f"bad GEMM operands {tuple(a.shape)} x {tuple(bt.shape)}^T")
    M, K = a.shape[0], 2 * a.shape[1]
    N = bt.shape[0]
    if M % GEMM_BM or N % GEMM_BN or K % FP4_K_MULTIPLE or K < FP4_K_MIN:
        raise ValueError(f"fp4 GEMM shape {M}x{N}x{K} must be multiples of {GEMM_BM}x{GEMM_BN}x{FP4_K_MULTIPLE}, "
                         f"K >= {FP4_K_MIN}")
    if out is None:
        out = torch.empty((M, N), device=a.device, dtype=out_dtype or torch.bfloat16)
    if out.shape != (M, N) or out.dtype not in (torch.bfloat16, torch.float32):
        raise ValueError("bad GEMM output")
    _require(out, out.dtype, "out")
    _check(_lib().avk_gemm_fp4_nt(a.data_ptr(), bt.data_ptr(), out.data_ptr(), int(out.dtype == torch.float32),
                                  M, N, K, _stream(stream)), "gemm_fp4_nt")
    return out


# ----------------------------------------------------------------- fp6 (e2m3)
# The validator's fp6 storage: each 32-element k-block of a row is a 32-B slot
# with the 32 six-bit codes packed little-endian in its first 24 B (element j
# at bits 6j .. 6j+5, the f8f6f4 MFMA's operand order) and 8 B of zeros, so a
# row of K fp6 is K bytes (validator_kernels.hip gemm_fp6_nt_kernel).
FP6_K_MULTIPLE = 256


def e2m3_values():
    """code (0..63) -> value of OCP FP6 e2m3 (1 sign, 2 exponent bits with
    bias 1, 3 mantissa bits)."""
    out = []
    for c in range(64):
        e, m = (c >> 3) & 3, c & 7
        mag = m / 8 if e == 0 else (1 + m / 8) * 2.0 ** (e - 1)
        out.append(-mag if c & 0x20 else mag)
    return tuple(out)


FP6_VALUES = e2m3_values()


def fp6_to_float(t):
    """fp6 storage (uint8 [..., K], K a multiple of 32) -> float32 [..., K]."""
    import torch

    lut = torch.tensor(FP6_VALUES, dtype=torch.float32, device=t.device)
    slots = t.view(torch.uint8).reshape(*t.shape[:-1], t.shape[-1] // 32, 32)[..., :24].long()
    bits = torch.stack([(slots >> b) & 1 for b in range(8)], dim=-1).flatten(-2)  # [..., slots, 192] little-endian
    w = torch.tensor([1 << b for b in range(6)], device=t.device)
    codes = (bits.view(*bits.shape[:-1], 32, 6) * w).sum(-1)
    return lut[codes].flatten(-2)


def float_to_fp6(x):
    """float values in the e2m3 set [..., K] -> fp6 storage uint8 [..., K]."""
    import torch

    table = {v: i for i, v in enumerate(FP6_VALUES) if not (v == 0 and i == 32)}
    codes = torch.tensor([table[float(v)] for v in x.flatten().tolist()], dtype=torch.long)
    codes = codes.view(*x.shape[:-1], x.shape[-1] // 32, 32)
    bits = torch.stack([(codes >> b) & 1 for b in range(6)], dim=-1).flatten(-2)  # [..., slots, 192]
    byte = (bits.view(*bits.shape[:-1], 24, 8) * torch.tensor([1 << b for b in range(8)])).sum(-1)
    out = torch.zeros(*codes.shape[:-1], 32, dtype=torch.uint8)
    out[..., :24] = byte.to(torch.uint8)
    return out.flatten(-2)


def fill_fp6_(t, seed: int, stream=None):
    """Deterministic random fp6 storage (every e2m3 code, slots padded) into a
    uint8 tensor whose size is a multiple of 32."""
    import torch

    _require(t, torch.uint8, "t")
    _check(_lib().avk_fill_fp6(t.data_ptr(), t.numel(), seed & ((1 << 64) - 1), _stream(stream)), "fill_fp6")
    return t


def gemm_fp6_nt(a, bt, out=None, out_dtype=None, stream=None):
    """K2d: ``out[M,N] = A[M,K] @ Bt[N,K].T`` with OCP FP6 e2m3 operands in the
    fp6 storage (uint8 ``[M, K]`` / ``[N, K]``) on ``v_mfma_f32_16x16x128_f8f6f4
    cbsz:2 blgp:2``, fp32 accumulation, bf16 or fp32 out.  M, N multiples of
    256, K of 256."""
    import torch

    _require(a, torch.uint8, "a")
    _require(bt, torch.uint8, "bt")
    if a.dim() != 2 or bt.dim() != 2 or a.shape[1] != bt.shape[1]:
        raise ValueError(f"bad GEMM operands {tuple(a.shape)} x {tuple(bt.shape)}^T")
    M, K = a.shape
    N = bt.shape[0]
    if M % GEMM_BM or N % GEMM_BN or K % FP6_K_MULTIPLE:
        raise ValueError(f"fp6 GEMM shape {M}x{N}x{K} must be multiples of {GEMM_BM}x{GEMM_BN}x{FP6_K_MULTIPLE}")
    if out is None:
        out = torch.empty((M, N), device=a.device, dtype=out_dtype or torch.bfloat16)
    if out.shape != (M, N) or out.dtype not in (torch.bfloat16, torch.float32):
        raise ValueError("bad GEMM output")
    _require(out, out.dtype, "out")
    _check(_lib().avk_gemm_fp6_nt(a.data_ptr(), bt.data_ptr(), out.data_ptr(), int(out.dtype == torch.float32),
                                  M, N, K, _stream(stream)), "gemm_fp6_nt")
    return out


def gemv_fp6(x, v, transpose: bool = False, out=None, stream=None):
    """The fp6 step's Freivalds GEMVs on fp6 storage ``[R, C]``."""
    import torch

    _require(x, torch.uint8, "x", 16)
    _require(v, torch.float32, "v")
    R, C = x.shape
    if v.numel() != (R if transpose else C) or C % 32:
        raise ValueError("gemv_fp6 shape mismatch")
    if transpose:
        out = torch.zeros(C, device=x.device, dtype=torch.float32) if out is None else out.zero_()
        _check(_lib().avk_gemv_cols_fp6(x.data_ptr(), v.data_ptr(), out.data_ptr(), R, C, _stream(stream)), "gemv")
    else:
        out = torch.empty(R, device=x.device, dtype=torch.float32) if out is None else out
        _check(_lib().avk_gemv_rows_fp6(x.data_ptr(), v.data_ptr(), out.data_ptr(), R, C, _stream(stream)), "gemv")
    return out


# ------------------------------------------------------------ MXFP4 (scaled)
# Block-scaled OCP MXFP4: e2m1 pairs as gemm_fp4_nt's with one E8M0 scale
# (2^(s - 127)) per row and 32-element k-block, periodic in k with 8 blocks:
# scales uint8 [rows, 8], block b of row r scaled by S[r, b % 8].
MX_SCALE_PERIOD = 8


def fill_e8m0_(t, seed: int, lo: int = 124, hi: int = 130, stream=None):
    """Random E8M0 scales in [lo, hi] (default 2^-3 .. 2^3) into a uint8 tensor."""
    import torch

    _require(t, torch.uint8, "t", 1)
    _check(_lib().avk_fill_e8m0(t.data_ptr(), t.numel(), seed & ((1 << 64) - 1), lo, hi, _stream(stream)), "fill_e8m0")
    return t


def mxfp4_to_float(x, scales):
    """MXFP4 operand (pairs uint8 [R, K/2], scales uint8 [R, 8]) -> the
    dequantized float64 [R, K]."""
    import torch

    v = fp4_to_float(x).double()
    R, K = v.shape
    blk = (torch.arange(K, device=x.device) // 32) % MX_SCALE_PERIOD
    sc = torch.pow(2.0, scales.long().double() - 127.0)[:, blk]
    return v * sc


def gemm_mxfp4_nt(a, bt, sa, sb, out=None, out_dtype=None, stream=None):
    """K2e: ``out = (2^(SA-127) A) @ (2^(SB-127) Bt).T`` on
    ``v_mfma_scale_f32_16x16x128_f8f6f4 cbsz:4 blgp:4`` (MXFP4 with E8M0 block
    scales ``sa`` [M, 8] / ``sb`` [N, 8] uint8, see MX_SCALE_PERIOD)."""
    import torch

    for t, n in ((a, "a"), (bt, "bt")):
        _require(t, torch.uint8, n)
    for t, n in ((sa, "sa"), (sb, "sb")):
        _require(t, torch.uint8, n, 1)
    if a.dim() != 2 or bt.dim() != 2 or a.shape[1] != bt.shape[1]:
        raise ValueError(f"bad GEMM operands {tuple(a.shape)} x {tuple(bt.shape)}^T")
    M, K = a.shape[0], 2 * a.shape[1]
    N = bt.shape[0]
    if tuple(sa.shape) != (M, MX_SCALE_PERIOD) or tuple(sb.shape) != (N, MX_SCALE_PERIOD):
        raise ValueError("MX scales must be [rows, 8] uint8")
    if M % GEMM_BM or N % GEMM_BN or K % FP4_K_MULTIPLE or K < FP4_K_MIN:
        raise ValueError(f"mxfp4 GEMM shape {M}x{N}x{K} must be multiples of {GEMM_BM}x{GEMM_BN}x{FP4_K_MULTIPLE}, "
                         f"K >= {FP4_K_MIN}")
    if out is None:
        out = torch.empty((M, N), device=a.device, dtype=out_dtype or torch.bfloat16)
    if out.shape != (M, N) or out.dtype not in (torch.bfloat16, torch.float32):
        raise ValueError("bad GEMM output")
    _require(out, out.dtype, "out")
    _check(_lib().avk_gemm_mxfp4_nt(a.data_ptr(), bt.data_ptr(), sa.data_ptr(), sb.data_ptr(), out.data_ptr(),
                                    int(out.dtype == torch.float32), M, N, K, _stream(stream)), "gemm_mxfp4_nt")
    return out


def gemv_mxfp4(x, scales, v, transpose: bool = False, out=None, stream=None):
    """The MXFP4 step's Freivalds GEMVs on the dequantized operand."""
    import torch

    _require(x, torch.uint8, "x", 8)
    _require(scales, torch.uint8, "scales", 1)
    _require(v, torch.float32, "v")
    R, C = x.shape[0], 2 * x.shape[1]
    if v.numel() != (R if transpose else C) or C % 16:
        raise ValueError("gemv_mxfp4 shape mismatch")
    if transpose:
        out = torch.zeros(C, device=x.device, dtype=torch.float32) if out is None else out.zero_()
        _check(_lib().avk_gemv_cols_mxfp4(x.data_ptr(), scales.data_ptr(), v.data_ptr(), out.data_ptr(), R, C,
                                          _stream(stream)), "gemv")
    else:
        out = torch.empty(R, device=x.device, dtype=torch.float32) if out is None else out
        _check(_lib().avk_gemv_rows_mxfp4(x.data_ptr(), scales.data_ptr(), v.data_ptr(), out.data_ptr(), R, C,
                                          _stream(stream)), "gemv")
    return out


def gemv_rows(x, v, out=None, stream=None):
    """``out[r] = sum_c x[r, c] * v[c]`` (x bf16 or fp32)."""
    import torch

    R, C = x.shape
    _require(x, x.dtype, "x", 8)
    _require(v, torch.float32, "v")
    if C % 8 or v.numel() != C:
        raise ValueError("gemv_rows shape mismatch")
    if out is None:
        out = torch.empty(R, device=x.device, dtype=torch.float32)
    _check(_lib().avk_gemv_rows(x.data_ptr(), int(x.dtype == torch.bfloat16), v.data_ptr(), out.data_ptr(), R, C,
                                _stream(stream)), "gemv_rows")
    return out


def gemv_cols_bf16(x, v, out=None, stream=None):
    """``out[c] = sum_r x[r, c] * v[r]`` (x bf16)."""
    import torch

    R, C = x.shape
    _require(x, torch.bfloat16, "x", 8)
    _require(v, torch.float32, "v")
    if C % 8 or v.numel() != R:
        raise ValueError("gemv_cols shape mismatch")
    if out is None:
        out = torch.zeros(C, device=x.device, dtype=torch.float32)
    else:
        out.zero_()
    _check(_lib().avk_gemv_cols_bf16(x.data_ptr(), v.data_ptr(), out.data_ptr(), R, C, _stream(stream)), "gemv_cols")
    return out


def gemv_fp4(x, v, transpose: bool = False, out=None, stream=None):
    """The fp4 step's Freivalds GEMVs, x FP4 pairs uint8 ``[R, C/2]``:
    ``out[r] = sum_c x[r, c] v[c]``, or with ``transpose`` ``out[c] = sum_r
    x[r, c] v[r]`` (fp32).  C a multiple of 16."""
    import torch

    _require(x, torch.uint8, "x", 8)
    _require(v, torch.float32, "v")
    if x.dim() != 2:
        raise ValueError("gemv_fp4 shape mismatch")
    R, C = x.shape[0], 2 * x.shape[1]
    if C % 16 or v.numel() != (R if transpose else C):
        raise ValueError("gemv_fp4 shape mismatch")
    n = C if transpose else R
    if out is None:
        out = torch.zeros(n, device=x.device, dtype=torch.float32)
    elif transpose:
        out.zero_()
    fn = _lib().avk_gemv_cols_fp4 if transpose else _lib().avk_gemv_rows_fp4
    _check(fn(x.data_ptr(), v.data_ptr(), out.data_ptr(), R, C, _stream(stream)), "gemv_fp4")
    return out


def gemv_fp8(x, v, transpose: bool = False, out=None, stream=None):
    """The fp8 step's Freivalds GEMVs, x e4m3 bytes uint8 ``[R, C]``:
    ``out[r] = sum_c x[r, c] v[c]``, or with ``transpose`` ``out[c] = sum_r
    x[r, c] v[r]`` (fp32).  C a multiple of 8."""
    import torch

    _require(x, torch.uint8, "x", 8)
    _require(v, torch.float32, "v")
    if x.dim() != 2:
        raise ValueError("gemv_fp8 shape mismatch")
    R, C = x.shape
    if C % 8 or v.numel() != (R if transpose else C):
        raise ValueError("gemv_fp8 shape mismatch")
    n = C if transpose else R
    if out is None:
        out = torch.zeros(n, device=x.device, dtype=torch.float32)
    elif transpose:
        out.zero_()
    fn = _lib().avk_gemv_cols_fp8 if transpose else _lib().avk_gemv_rows_fp8
    _check(fn(x.data_ptr(), v.data_ptr(), out.data_ptr(), R, C, _stream(stream)), "gemv_fp8")
    return out


def hbm_copy(src, dst, num_cus: int = 256, variant: int = 0, stream=None):
    """K3: streaming copy of ``src`` into ``dst`` (any dtype, 16-B multiple)."""
    nbytes = src.numel() * src.element_size()
    if dst.numel() * dst.element_size() != nbytes or nbytes % 16:
        raise ValueError("hbm_copy size mismatch")
    if not (src.is_cuda and dst.is_cuda and src.is_contiguous() and dst.is_contiguous()):
        raise ValueError("hbm_copy needs contiguous GPU tensors")
    _check(_lib().avk_hbm_copy(src.data_ptr(), dst.data_ptr(), nbytes, num_cus, variant, _stream(stream)), "hbm_copy")
    return dst


def checksum(t, scratch=None, stream=None) -> int:
    import torch

    nbytes = t.numel() * t.element_size()
    if scratch is None:
        scratch = torch.empty(1, device=t.device, dtype=torch.int64)
    _check(_lib().avk_checksum(t.data_ptr(), nbytes, scratch.data_ptr(), _stream(stream)), "checksum")
    return int(scratch.item()) & ((1 << 64) - 1)


def max_abs_diff(a, b, stream=None) -> float:
    import torch

    _require(a, torch.float32, "a", aligned=False)  # the kernel takes a scalar path when unaligned
    _require(b, torch.float32, "b", aligned=False)
    if a.numel() != b.numel():
        raise ValueError("size mismatch")
    out = torch.empty(1, device=a.device, dtype=torch.int32)
    _check(_lib().avk_max_abs_diff_f32(a.data_ptr(), b.data_ptr(), a.numel(), out.data_ptr(), _stream(stream)), "max_abs_diff")
    return float(out.view(torch.float32).item())


def _ptr_array(ptrs):
    arr = (_c_ptr * len(ptrs))()
    for i, p in enumerate(ptrs):
        arr[i] = p
    return arr


def allreduce_oneshot(inputs_or_ptrs, out, count: int | None = None, stream=None):
    """K4 one-shot: ``out = sum(inputs)``; inputs are tensors or raw peer pointers."""
    import torch

    _require(out, torch.float32, "out", 4)
    ptrs = [x.data_ptr() if isinstance(x, torch.Tensor) else int(x) for x in inputs_or_ptrs]
    n = count if count is not None else out.numel()
    if not 1 <= len(ptrs) <= 8:
        raise ValueError("1..8 peers supported")
    _check(_lib().avk_allreduce_oneshot_f32(_ptr_array(ptrs), len(ptrs), out.data_ptr(), n, _stream(stream)), "allreduce_oneshot")
    return out


def allreduce_twoshot_slice(in_ptrs, out_ptrs, rank: int, count: int, stream=None):
    """K4 two-shot: reduce this rank's slice and write it into every peer output."""
    if len(in_ptrs) != len(out_ptrs) or not 1 <= len(in_ptrs) <= 8:
        raise ValueError("bad peer tables")
    _check(_lib().avk_allreduce_twoshot_f32(_ptr_array([int(p) for p in in_ptrs]), _ptr_array([int(p) for p in out_ptrs]),
                                            len(in_ptrs), rank, count, _stream(stream)), "allreduce_twoshot")


def _f32_or_bf16(x, name: str) -> int:
    import torch

    _require(x, x.dtype if x.dtype in (torch.float32, torch.bfloat16) else torch.float32, name)
    return int(x.dtype == torch.bfloat16)


def fill_const(x, value: float, stream=None) -> None:
    """Fill an fp32 or bf16 tensor with ``value`` on the device (RCCL-step operands)."""
    bf16 = _f32_or_bf16(x, "x")
    _check(_lib().avk_fill_const(x.data_ptr(), x.numel(), bf16, float(value), _stream(stream)), "fill_const")


def check_blocks(x, block: int, base: float, step: float, stream=None) -> int:
    """Count elements with x[i] != base + (i // block) * step (device-side check)."""
    import torch

    bf16 = _f32_or_bf16(x, "x")
    bad = torch.zeros(1, dtype=torch.int64, device=x.device)
    _check(_lib().avk_check_blocks(x.data_ptr(), x.numel(), bf16, int(block), float(base), float(step),
                                   bad.data_ptr(), _stream(stream)), "check_blocks")
    return int(bad.item())


def mfma_probe(seed: int = 1, stream=None) -> dict[str, int]:
    """K5: one MFMA tile per CDNA4 matrix data type, checked exactly against an
    integer reference; returns ``{dtype: mismatching outputs}`` (0 = works)."""
    lib = _lib()
    out = {}
    for kind in range(lib.avk_mfma_probe_count()):
        bad = ctypes.c_int(-1)
        _check(lib.avk_mfma_probe(kind, seed & ((1 << 64) - 1), ctypes.byref(bad), _stream(stream)), "mfma_probe")
        out[lib.avk_mfma_probe_name(kind).decode()] = bad.value
    return out


@dataclass
class GemmShape:
    m: int
    n: int
    k: int

    @property
    def flops(self) -> float:
        return 2.0 * self.m * self.n * self.k
