"""Numerics of the hand-written gfx950 validator kernels vs plain PyTorch fp32.

Every test here runs the native HIP path (``libamdgpu_validator.so``); there is
no fallback, so a missing library fails the test instead of passing on eager
PyTorch.
"""

import pytest

torch = pytest.importorskip("torch")

from amdgpu_operator.ops import kernels as K  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def test_abi_version():
    assert K.abi_version() == 1


@pytest.mark.parametrize("n", [1, 7, 1024, (1 << 20) + 3])
def test_vector_add_exact(n):
    a = torch.randn(n, device=DEV)
    b = torch.randn(n, device=DEV)
    if a.data_ptr() % 16 or b.data_ptr() % 16:
        pytest.skip("allocator returned unaligned block")
    c = K.vector_add(a, b)
    assert torch.equal(c, a + b)


_SHAPES = [(256, 256, 64), (512, 768, 320), (1024, 1024, 1024), (2048, 1024, 4096),
           (256, 512, 192), (512, 256, 128), (256, 256, 256), (768, 512, 2304)]
# None: the validator's dispatch (4-wave kernel when K % 256 == 0, else the
# 8-phase fallback); the 4-wave variant itself only takes K % 256 (its refusal
# of other K is test_gemm_rejects_bad_shapes).
_GEMM_CASES = [(v, s) for v in (None, K.GEMM_FALLBACK_VARIANT, K.GEMM_DEFAULT_VARIANT) for s in _SHAPES
               if v in (None, K.GEMM_FALLBACK_VARIANT) or s[2] % K.GEMM_DEFAULT_K_MULTIPLE == 0]


@pytest.mark.parametrize("out_dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("variant,shape", _GEMM_CASES)
def test_gemm_vs_fp32_reference(shape, out_dtype, variant):
    M, N, Kd = shape
    g = torch.Generator(device=DEV).manual_seed(M + N + Kd)
    a = (torch.rand(M, Kd, device=DEV, generator=g) * 2 - 1).to(torch.bfloat16)
    bt = (torch.rand(N, Kd, device=DEV, generator=g) * 2 - 1).to(torch.bfloat16)
    ref = a.float() @ bt.float().t()
    out = K.gemm_bf16_nt(a, bt, out_dtype=out_dtype, variant=variant)
    err = (out.float() - ref).abs().max().item()
    scale = ref.abs().max().item()
    tol = 1e-5 * Kd if out_dtype == torch.float32 else 8e-3 * scale
    assert err <= tol, (err, tol)


@pytest.mark.parametrize("variant,Kd", [(v, k) for v in (None, K.GEMM_FALLBACK_VARIANT, K.GEMM_DEFAULT_VARIANT)
                                         for k in (128, 512)
                                         if v in (None, K.GEMM_FALLBACK_VARIANT) or k % K.GEMM_DEFAULT_K_MULTIPLE == 0])
def test_gemm_exact_integer_asymmetric(variant, Kd):
    # A = small integers, B asymmetric: a transposed C-write or a swapped
    # fragment map changes the result; all sums are exact in fp32.
    M, N = 512, 256
    i = torch.arange(M, device=DEV).view(M, 1)
    k = torch.arange(Kd, device=DEV).view(1, Kd)
    a = ((i * 3 + k * 7) % 5 - 2).to(torch.bfloat16)
    n = torch.arange(N, device=DEV).view(N, 1)
    bt = ((n * 11 + k * 2 + (n > k).long()) % 7 - 3).to(torch.bfloat16)
    ref = a.double() @ bt.double().t()
    out = K.gemm_bf16_nt(a, bt, out_dtype=torch.float32, variant=variant)
    assert torch.equal(out.double(), ref)


@pytest.mark.parametrize("variant", [15, 24, 25, 26, 27, 28, 30])
def test_gemm_lab_schedules_vs_fp32_reference(variant):
    """The other generated schedules of the 4-wave kernel (tools build)."""
    from amdgpu_operator import native

    # build() makes the lab library; a GPU run without it is a build error, not a skip
    assert native.artefact(K.LAB_LIB_NAME).exists(), "lab library missing: make -C native lab"
    M, N, Kd = 512, 768, 2304
    g = torch.Generator(device=DEV).manual_seed(variant)
    a = (torch.rand(M, Kd, device=DEV, generator=g) * 2 - 1).to(torch.bfloat16)
    bt = (torch.rand(N, Kd, device=DEV, generator=g) * 2 - 1).to(torch.bfloat16)
    ref = a.float() @ bt.float().t()
    out = K.gemm_bf16_nt(a, bt, out_dtype=torch.float32, variant=variant)
    assert (out - ref).abs().max().item() <= 1e-5 * Kd
    out = K.gemm_bf16_nt(a, bt, out_dtype=torch.bfloat16, variant=variant)
    assert (out.float() - ref).abs().max().item() <= 8e-3 * ref.abs().max().item()


def test_gemm_identity_asymmetric():
    N = 256
    a = torch.eye(N, device=DEV, dtype=torch.bfloat16)
    bt = (torch.arange(N * N, device=DEV).view(N, N) % 97).to(torch.bfloat16)
    out = K.gemm_bf16_nt(a, bt, out_dtype=torch.float32)
    assert torch.equal(out, bt.float().t())


def test_gemm_rejects_bad_shapes():
    a = torch.zeros(100, 64, device=DEV, dtype=torch.bfloat16)
    bt = torch.zeros(256, 64, device=DEV, dtype=torch.bfloat16)
    with pytest.raises(ValueError):
        K.gemm_bf16_nt(a, bt)
    a = torch.zeros(256, 192, device=DEV, dtype=torch.bfloat16)
    bt = torch.zeros(256, 192, device=DEV, dtype=torch.bfloat16)
    with pytest.raises(K.KernelError):  # the 4-wave kernel refuses K % 256 != 0 (no silent fallback)
        K.gemm_bf16_nt(a, bt, variant=K.GEMM_DEFAULT_VARIANT)


def test_fill_uniform_deterministic_and_bounded():
    t1 = K.fill_uniform_(torch.empty(1 << 16, device=DEV), 42, -1, 1)
    t2 = K.fill_uniform_(torch.empty(1 << 16, device=DEV), 42, -1, 1)
    assert torch.equal(t1, t2)
    assert t1.min() >= -1 and t1.max() < 1 and t1.std() > 0.5
    b = K.fill_uniform_(torch.empty(1 << 16, device=DEV, dtype=torch.bfloat16), 7, 0, 2)
    assert b.float().min() >= 0 and b.float().max() <= 2


def test_gemv_rows_cols():
    R, C = 384, 512
    x = (torch.rand(R, C, device=DEV) * 2 - 1).to(torch.bfloat16)
    v = torch.randn(C, device=DEV)
    w = torch.randn(R, device=DEV)
    torch.testing.assert_close(K.gemv_rows(x, v), x.float() @ v, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(K.gemv_cols_bf16(x, w), x.float().t() @ w, rtol=1e-4, atol=1e-3)
    xf = x.float()
    torch.testing.assert_close(K.gemv_rows(xf, v), xf @ v, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("nbytes", [16, 4096, 3 << 20, (1 << 26) + 16])
@pytest.mark.parametrize("variant", [0, 1])
def test_hbm_copy_and_checksum(nbytes, variant):
    src = torch.randint(0, 255, (nbytes,), device=DEV, dtype=torch.uint8)
    dst = torch.zeros_like(src)
    K.hbm_copy(src, dst, variant=variant)
    assert torch.equal(src, dst)
    assert K.checksum(src) == K.checksum(dst)
    dst[nbytes // 2] ^= 1
    assert K.checksum(src) != K.checksum(dst)


def test_max_abs_diff():
    a = torch.zeros(10000, device=DEV)
    b = torch.zeros(10000, device=DEV)
    b[1234] = -3.5
    assert K.max_abs_diff(a, b) == 3.5
    b[5] = float("nan")
    assert K.max_abs_diff(a, b) == float("inf")


@pytest.mark.parametrize("n,offset", [(1, 0), (7, 1), (1 << 20, 0), ((1 << 22) + 3, 1), ((1 << 24) + 5, 2)])
def test_max_abs_diff_matches_torch(n, offset):
    """Against the fp32 PyTorch reference, including unaligned starts (scalar
    path) and tails past the last float4."""
    base_a = torch.randn(n + offset, device=DEV)
    base_b = base_a + 1e-3 * torch.randn(n + offset, device=DEV)
    a, b = base_a[offset:], base_b[offset:]
    want = (a - b).abs().max().item()
    assert K.max_abs_diff(a, b) == want


@pytest.mark.parametrize("nbytes", [16, 4096, (1 << 20) + 48, 1 << 26])
def test_checksum_matches_reference(nbytes):
    """sum over 16-byte words i of (x + 3y + 5z + 7w + i mod 65536) mod 2^64."""
    import numpy as np

    src = torch.randint(0, 256, (nbytes,), device=DEV, dtype=torch.uint8)
    w = src.cpu().numpy().view(np.uint32).reshape(-1, 4).astype(np.uint64)
    idx = np.arange(w.shape[0], dtype=np.uint64) & np.uint64(0xFFFF)
    with np.errstate(over="ignore"):
        want = int((w[:, 0] + 3 * w[:, 1] + 5 * w[:, 2] + 7 * w[:, 3] + idx).sum(dtype=np.uint64))
    assert K.checksum(src) == want


@pytest.mark.parametrize("peers", [1, 2, 3, 4, 8])
def test_allreduce_oneshot_emulated(peers):
    n = 1 << 18
    ins = [torch.randn(n, device=DEV) for _ in range(peers)]
    out = torch.empty(n, device=DEV)
    K.allreduce_oneshot(ins, out)
    torch.testing.assert_close(out, torch.stack(ins).sum(0), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("peers", [2, 4, 8])
def test_allreduce_twoshot_emulated(peers):
    n = (1 << 16) + 4 * 3
    ins = [torch.randn(n, device=DEV) for _ in range(peers)]
    outs = [torch.zeros(n, device=DEV) for _ in range(peers)]
    for r in range(peers):
        K.allreduce_twoshot_slice([t.data_ptr() for t in ins], [t.data_ptr() for t in outs], r, n)
    ref = torch.stack(ins).sum(0)
    for o in outs:
        torch.testing.assert_close(o, ref, rtol=1e-5, atol=1e-5)


def test_workload_quick_end_to_end():
    from amdgpu_operator.validator.workload import ValidatorWorkload, WorkloadConfig

    rep = ValidatorWorkload(0, WorkloadConfig.quick()).run()
    assert rep.ok, rep.as_dict()
    names = [s.name for s in rep.steps]
    assert names == list(ValidatorWorkload.STEPS)


def test_workload_detects_bad_gemm(monkeypatch):
    from amdgpu_operator.validator import workload as W

    real = K.gemm_bf16_nt

    def broken(a, bt, out=None, out_dtype=None, stream=None):
        o = real(a, bt, out=out, out_dtype=out_dtype, stream=stream)
        o[17, 3:40] += 10.0  # corrupt part of one tile
        return o

    monkeypatch.setattr(W.K, "gemm_bf16_nt", broken)
    wl = W.ValidatorWorkload(0, W.WorkloadConfig.quick())
    with pytest.raises(W.ValidationFailed):
        wl.step_gemm()


def test_workload_rccl_collectives_single_rank(tmp_path):
    import json
    import os
    import subprocess
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = (
        "import json, torch, torch.distributed as dist\n"
        "from amdgpu_operator.validator.workload import ValidatorWorkload, WorkloadConfig\n"
        "torch.cuda.set_device(0)\n"
        "dist.init_process_group('nccl', rank=0, world_size=1, init_method='tcp://127.0.0.1:29617',"
        " device_id=torch.device('cuda', 0))\n"
        "r = ValidatorWorkload(0, WorkloadConfig.quick()).step_rccl()\n"
        "dist.destroy_process_group()\n"
        "print(json.dumps({'ok': r.ok, **r.metrics}))\n")
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240, cwd=repo,
                       env={**os.environ, "PYTHONPATH": repo})
    assert p.returncode == 0, p.stderr[-3000:]
    rep = json.loads(p.stdout.strip().splitlines()[-1])
    assert rep["ok"] and rep["world"] == 1
    assert set(rep["collectives"]) == {"allreduce_f32", "allreduce_bf16", "allgather_f32", "reducescatter_f32"}


def test_vector_add_verify_counts_corruption():
    n = (1 << 20) + 3
    a = torch.empty(n, device="cuda")
    b = torch.empty(n, device="cuda")
    K.fill_uniform_(a, 5)
    K.fill_uniform_(b, 6)
    c = K.vector_add(a, b)
    assert K.vector_add_verify(a, b, c) == 0
    c[5] += 1.0
    c[n - 1] = float("nan")
    assert K.vector_add_verify(a, b, c) == 2


@pytest.mark.parametrize("seed", [1, 7])
def test_mfma_probe_every_cdna4_dtype_exact(seed):
    # K5: f16, bf16, OCP fp8/bf8, int8, block-scaled fp8/fp6/fp4 (scale 1), f32, f64
    res = K.mfma_probe(seed)
    assert set(res) == {"f16", "bf16", "fp8", "bf8", "i8", "mxfp8", "mxfp6", "mxfp4", "f32", "f64"}
    assert all(v == 0 for v in res.values()), res


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
def test_fill_const_and_block_check_match_torch(dtype):
    # RCCL-step operand fill and result check (device side) vs a PyTorch reference
    dt = getattr(torch, dtype)
    per, blocks = 4096 + 3, 64  # values 1..64: exact in bf16
    n = per * blocks
    x = torch.empty(n, dtype=dt, device="cuda")
    K.fill_const(x, 3.0)
    assert torch.equal(x.float().cpu(), torch.full((n,), 3.0))
    assert K.check_blocks(x, n, 3.0, 0.0) == 0
    y = (1.0 + torch.div(torch.arange(n, device="cuda"), per, rounding_mode="floor")).to(dt)  # all-gather pattern
    assert K.check_blocks(y, per, 1.0, 1.0) == 0
    assert K.check_blocks(y, per, 1.0, 2.0) == int((y.float() != 1.0 + 2.0 * torch.div(
        torch.arange(n, device="cuda"), per, rounding_mode="floor")).sum())
    y[5] += 1
    y[n - 1] = float("nan")
    assert K.check_blocks(y, per, 1.0, 1.0) == 2


# ---------------------------------------------------------- K2b fp8 GEMM ----
_FP8_SHAPES = [(256, 256, 256), (512, 768, 512), (1024, 1024, 1024), (2048, 1024, 4096), (768, 512, 2304),
               (256, 512, 768)]


def _fp8_pair(M, N, Kd, seed):
    a = torch.empty(M, Kd, device=DEV, dtype=torch.float8_e4m3fn)
    bt = torch.empty(N, Kd, device=DEV, dtype=torch.float8_e4m3fn)
    K.fill_fp8_(a, seed)
    K.fill_fp8_(bt, seed + 1)
    return a, bt


def test_fp8_fill_is_finite_ocp_e4m3_and_deterministic():
    a = torch.empty(1 << 16, device=DEV, dtype=torch.float8_e4m3fn)
    K.fill_fp8_(a, 5)
    x = a.float()
    assert torch.isfinite(x).all() and x.abs().max().item() <= 3.75 and x.unique().numel() > 100
    b = torch.empty_like(a)
    K.fill_fp8_(b, 5)
    assert torch.equal(a.view(torch.uint8), b.view(torch.uint8))


@pytest.mark.parametrize("out_dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", _FP8_SHAPES)
def test_fp8_gemm_vs_fp32_reference(shape, out_dtype):
    """The e4m3 GEMM against the fp64 product of the dequantized operands
    and against hipBLASLt's fp8 GEMM (torch._scaled_mm, unit scales).  The
    f8f6f4 MFMA does not keep a full fp32 sum inside one instruction: on
    gfx950 both kernels land ~5e-5 of the output's scale from the exact
    result (profiles/r5_fp8/diag.json), where an fp32 GEMM lands ~1e-6.  So
    the check against the exact product is loose, and the one against
    hipBLASLt, which runs the same instruction in another order, is tight."""
    M, N, Kd = shape
    a, bt = _fp8_pair(M, N, Kd, M + N + Kd)
    ref = a.double() @ bt.double().t()
    out = K.gemm_fp8_nt(a, bt, out_dtype=out_dtype)
    scale = ref.abs().max().item()
    err = (out.double() - ref).abs().max().item()
    assert err <= (2e-4 if out_dtype == torch.float32 else 8e-3) * scale, (err, scale)
    one = torch.ones((), device=DEV)
    lt = torch._scaled_mm(a, bt.t(), scale_a=one, scale_b=one, out_dtype=out_dtype)
    err_lt = (out.double() - lt.double()).abs().max().item()
    assert err_lt <= (1e-5 if out_dtype == torch.float32 else 8e-3) * scale, (err_lt, scale)


def test_fp8_gemm_one_k_block_matches_hipblaslt():
    """One MFMA's worth of K per output (A zero beyond k = 128): the rest of
    the sum adds zeros, so the result is hipBLASLt's to within a rounding of
    the order it adds its partial sums in (bit-equal at 1024 x 1024 x 4096 in
    profiles/r5_fp8/diag.json)."""
    a, bt = _fp8_pair(512, 256, 512, 77)
    a = a.view(torch.uint8).clone()
    a[:, 128:] = 0
    a = a.view(torch.float8_e4m3fn)
    one = torch.ones((), device=DEV)
    lt = torch._scaled_mm(a, bt.t(), scale_a=one, scale_b=one, out_dtype=torch.float32)
    out = K.gemm_fp8_nt(a, bt, out_dtype=torch.float32)
    assert (out - lt).abs().max().item() <= 2e-6 * lt.abs().max().item()


@pytest.mark.parametrize("Kd", [256, 1024])
def test_fp8_gemm_exact_integer_asymmetric(Kd):
    """Small integers (exact in e4m3), asymmetric B: a transposed C-write,
    a swapped fragment half or a wrong LDS swizzle changes the result; every
    sum is exact in fp32."""
    M, N = 512, 256
    i = torch.arange(M, device=DEV).view(M, 1)
    k = torch.arange(Kd, device=DEV).view(1, Kd)
    a = ((i * 3 + k * 7) % 5 - 2).float().to(torch.float8_e4m3fn)
    n = torch.arange(N, device=DEV).view(N, 1)
    bt = ((n * 11 + k * 2 + (n > k).long()) % 7 - 3).float().to(torch.float8_e4m3fn)
    ref = a.double() @ bt.double().t()
    out = K.gemm_fp8_nt(a, bt, out_dtype=torch.float32)
    assert torch.equal(out.double(), ref)
    eye = torch.eye(256, device=DEV).to(torch.float8_e4m3fn)
    bt2 = ((torch.arange(256 * Kd, device=DEV).view(256, Kd) % 9) - 4).float().to(torch.float8_e4m3fn)
    assert torch.equal(K.gemm_fp8_nt(bt2, eye[:, :Kd] if Kd == 256 else torch.cat(
        [eye, torch.zeros(256, Kd - 256, device=DEV).to(torch.float8_e4m3fn)], 1), out_dtype=torch.float32),
        bt2.float()[:, :256])


def test_fp8_gemm_rejects_bad_shapes():
    a = torch.zeros(256, 128, device=DEV, dtype=torch.float8_e4m3fn)
    with pytest.raises(ValueError):
        K.gemm_fp8_nt(a, a)
    with pytest.raises(ValueError):
        K.gemm_fp8_nt(torch.zeros(256, 256, device=DEV, dtype=torch.bfloat16), a)


# ---------------------------------------------------------- K2c fp4 GEMM ----
_FP4_SHAPES = [(256, 256, 512), (512, 768, 1024), (1024, 1024, 2048), (768, 512, 768), (256, 512, 4096)]


def _fp4_pair(M, N, Kd, seed):
    a = torch.empty(M, Kd // 2, device=DEV, dtype=torch.uint8)
    bt = torch.empty(N, Kd // 2, device=DEV, dtype=torch.uint8)
    K.fill_fp4_(a, seed)
    K.fill_fp4_(bt, seed + 1)
    return a, bt


def _to_fp4(x):
    """float values in the e2m1 set -> packed uint8 pairs (element 2k low)."""
    codes = {v: i for i, v in enumerate(K.FP4_VALUES) if not (v == 0 and i == 8)}
    flat = x.flatten().tolist()
    c = torch.tensor([codes[float(v)] for v in flat], dtype=torch.uint8).view(*x.shape[:-1], x.shape[-1] // 2, 2)
    return (c[..., 0] | (c[..., 1] << 4)).to(DEV)


def test_fp4_fill_is_deterministic_and_spans_the_codes():
    a = torch.empty(1 << 16, device=DEV, dtype=torch.uint8)
    K.fill_fp4_(a, 3)
    b = torch.empty_like(a)
    K.fill_fp4_(b, 3)
    assert torch.equal(a, b) and K.fp4_to_float(a).unique().numel() == 15  # +0 and -0 compare equal


@pytest.mark.parametrize("out_dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", _FP4_SHAPES)
def test_fp4_gemm_vs_exact_product(shape, out_dtype):
    """Every e2m1 value and product is exact; the MFMA's own sum is held to
    the fp8 instruction's measured accuracy (profiles/r5_fp8/diag.json)."""
    M, N, Kd = shape
    a, bt = _fp4_pair(M, N, Kd, M + N + Kd)
    ref = K.fp4_to_float(a).double() @ K.fp4_to_float(bt).double().t()
    out = K.gemm_fp4_nt(a, bt, out_dtype=out_dtype)
    scale = ref.abs().max().item()
    err = (out.double() - ref).abs().max().item()
    assert err <= (2e-4 if out_dtype == torch.float32 else 8e-3) * scale, (err, scale)


def test_fp4_gemm_exact_small_integers_and_identity():
    """Values in {0, +-1, +-2, +-4} with an asymmetric B: sums are small
    integers, exact; an identity B returns A.  A swapped k-step, nibble or
    fragment half changes the result."""
    M, N, Kd = 512, 256, 1024
    i = torch.arange(M).view(M, 1)
    k = torch.arange(Kd).view(1, Kd)
    vals = torch.tensor([0.0, 1.0, -1.0, 2.0, -2.0, 4.0, -4.0])
    a = vals[(i * 3 + k * 5) % 7]
    n = torch.arange(N).view(N, 1)
    b = vals[(n * 11 + k * 2 + (n > k).long()) % 7]
    out = K.gemm_fp4_nt(_to_fp4(a), _to_fp4(b), out_dtype=torch.float32)
    assert torch.equal(out.double().cpu(), a.double() @ b.double().t())
    eye = torch.zeros(256, Kd)
    eye[:, :256] = torch.eye(256)
    out = K.gemm_fp4_nt(_to_fp4(a), _to_fp4(eye), out_dtype=torch.float32)
    assert torch.equal(out.cpu(), a[:, :256])


def test_fp4_gemm_rejects_bad_shapes():
    a = torch.zeros(256, 128, device=DEV, dtype=torch.uint8)  # K = 256 < 512
    with pytest.raises(ValueError):
        K.gemm_fp4_nt(a, a)
    with pytest.raises(ValueError):
        K.gemm_fp4_nt(torch.zeros(256, 320, device=DEV, dtype=torch.uint8), torch.zeros(256, 320, device=DEV,
                                                                                      dtype=torch.uint8))  # K = 640


@pytest.mark.parametrize("shape", [(4096, 4096), (512, 1024), (300, 1040), (7, 16)])
def test_fp4_gemvs_vs_fp32(shape):
    """The fp4 step's Freivalds GEMVs against fp32 torch on the dequantized
    matrix: x v (one wave per row) and x^T v (column blocks of 1024, four row
    streams per block meeting in LDS, one atomic per column per block)."""
    R, C = shape
    x = torch.empty(R, C // 2, device=DEV, dtype=torch.uint8)
    K.fill_fp4_(x, R * 7 + C)
    xf = K.fp4_to_float(x)
    g = torch.Generator(device="cpu").manual_seed(R + C)
    vr = torch.rand(R, generator=g).mul_(2).sub_(1).to(DEV)
    vc = torch.rand(C, generator=g).mul_(2).sub_(1).to(DEV)
    ref_cols = (xf.double().t() @ vr.double())
    ref_rows = (xf.double() @ vc.double())
    cols = K.gemv_fp4(x, vr, transpose=True)
    rows = K.gemv_fp4(x, vc)
    for got, ref in ((cols, ref_cols), (rows, ref_rows)):
        scale = ref.abs().max().item()
        assert (got.double() - ref).abs().max().item() <= 1e-5 * max(scale, 1.0) * (1 + (R + C) / 1024)
    # accumulates into a given output only after zeroing it (the caller's z)
    z = torch.full((C,), 123.0, device=DEV)
    assert torch.allclose(K.gemv_fp4(x, vr, transpose=True, out=z).double(), ref_cols, atol=1e-3)


@pytest.mark.parametrize("shape", [(4096, 4096), (512, 1024), (300, 1032), (5, 8)])
def test_fp8_gemvs_vs_fp32(shape):
    """The fp8 step's Freivalds GEMVs (8-byte loads per lane, column blocks
    reduced in LDS) against fp32 torch on the dequantized e4m3 matrix."""
    R, C = shape
    x = torch.empty(R, C, device=DEV, dtype=torch.float8_e4m3fn)
    K.fill_fp8_(x, R * 5 + C)
    xf = x.float()
    g = torch.Generator(device="cpu").manual_seed(R * C)
    vr = torch.rand(R, generator=g).mul_(2).sub_(1).to(DEV)
    vc = torch.rand(C, generator=g).mul_(2).sub_(1).to(DEV)
    xb = x.view(torch.uint8)
    for got, ref in ((K.gemv_fp8(xb, vr, transpose=True), xf.double().t() @ vr.double()),
                     (K.gemv_fp8(xb, vc), xf.double() @ vc.double())):
        scale = ref.abs().max().item()
        assert (got.double() - ref).abs().max().item() <= 1e-5 * max(scale, 1.0) * (1 + (R + C) / 1024)


# ----------------------------------------------- fp6 (e2m3) and MXFP4 (scaled)
_FP6_SHAPES = [(256, 256, 256), (512, 768, 1024), (1024, 1024, 2048), (256, 512, 4096)]


def _fp6_pair(M, N, Kd, seed):
    a = torch.empty(M, Kd, device=DEV, dtype=torch.uint8)
    bt = torch.empty(N, Kd, device=DEV, dtype=torch.uint8)
    K.fill_fp6_(a, seed)
    K.fill_fp6_(bt, seed + 1)
    return a, bt


def test_fp6_fill_spans_the_codes_and_pads_its_slots():
    a = torch.empty(1 << 16, device=DEV, dtype=torch.uint8)
    K.fill_fp6_(a, 5)
    b = torch.empty_like(a)
    K.fill_fp6_(b, 5)
    assert torch.equal(a, b)
    assert K.fp6_to_float(a).unique().numel() == 63  # 64 codes, +0 and -0 compare equal
    assert int(a.view(-1, 32)[:, 24:].abs().sum()) == 0  # the 8 B of padding per slot


@pytest.mark.parametrize("out_dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", _FP6_SHAPES)
def test_fp6_gemm_vs_exact_product(shape, out_dtype):
    """e2m3 values (|x| <= 7.5) and their products are exact; the sum is the
    MFMA's fp32 accumulation, checked against the fp64 product of the decoded
    operands."""
    M, N, Kd = shape
    a, bt = _fp6_pair(M, N, Kd, M + 2 * N + Kd)
    ref = K.fp6_to_float(a).double() @ K.fp6_to_float(bt).double().t()
    out = K.gemm_fp6_nt(a, bt, out_dtype=out_dtype)
    scale = ref.abs().max().item()
    err = (out.double() - ref).abs().max().item()
    assert err <= (2e-4 if out_dtype == torch.float32 else 8e-3) * scale, (err, scale)


def test_fp6_gemm_exact_small_integers_and_identity():
    """Values in {0, +-1, +-2, +-4} with an asymmetric B: exact integer sums;
    an identity B returns A.  A swapped 6-bit field, slot or fragment half
    changes the result."""
    M, N, Kd = 512, 256, 512
    i = torch.arange(M).view(M, 1)
    k = torch.arange(Kd).view(1, Kd)
    vals = torch.tensor([0.0, 1.0, -1.0, 2.0, -2.0, 4.0, -4.0, 0.5])
    a = vals[(i * 3 + k * 5) % 8]
    n = torch.arange(N).view(N, 1)
    b = vals[(n * 11 + k * 2 + (n > k).long()) % 8]
    out = K.gemm_fp6_nt(K.float_to_fp6(a).to(DEV), K.float_to_fp6(b).to(DEV), out_dtype=torch.float32)
    assert torch.equal(out.double().cpu(), a.double() @ b.double().t())
    eye = torch.zeros(256, Kd)
    eye[:, :256] = torch.eye(256)
    out = K.gemm_fp6_nt(K.float_to_fp6(a).to(DEV), K.float_to_fp6(eye).to(DEV), out_dtype=torch.float32)
    assert torch.equal(out.cpu(), a[:, :256])


@pytest.mark.parametrize("shape", [(4096, 4096), (512, 1024), (300, 1056), (7, 32)])
def test_fp6_gemvs_vs_fp32(shape):
    R, C = shape
    x = torch.empty(R, C, device=DEV, dtype=torch.uint8)
    K.fill_fp6_(x, R * 5 + C)
    xf = K.fp6_to_float(x).double()
    g = torch.Generator(device="cpu").manual_seed(R + C)
    vr = torch.rand(R, generator=g).mul_(2).sub_(1).to(DEV)
    vc = torch.rand(C, generator=g).mul_(2).sub_(1).to(DEV)
    for got, ref in ((K.gemv_fp6(x, vr, transpose=True), xf.t() @ vr.double()), (K.gemv_fp6(x, vc), xf @ vc.double())):
        scale = ref.abs().max().item()
        assert (got.double() - ref).abs().max().item() <= 1e-5 * max(scale, 1.0) * (1 + (R + C) / 1024)


def _mx_operands(M, N, Kd, seed, lo=124, hi=130):
    a = torch.empty(M, Kd // 2, device=DEV, dtype=torch.uint8)
    bt = torch.empty(N, Kd // 2, device=DEV, dtype=torch.uint8)
    sa = torch.empty(M, 8, device=DEV, dtype=torch.uint8)
    sb = torch.empty(N, 8, device=DEV, dtype=torch.uint8)
    K.fill_fp4_(a, seed)
    K.fill_fp4_(bt, seed + 1)
    K.fill_e8m0_(sa, seed + 2, lo, hi)
    K.fill_e8m0_(sb, seed + 3, lo, hi)
    return a, bt, sa, sb


@pytest.mark.parametrize("out_dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", _FP4_SHAPES)
def test_mxfp4_gemm_vs_exact_product_with_non_unit_scales(shape, out_dtype):
    """Block-scaled MXFP4 with E8M0 scales 2^-3 .. 2^3 per row and k-block:
    against the fp64 product of the dequantized, scaled operands."""
    M, N, Kd = shape
    a, bt, sa, sb = _mx_operands(M, N, Kd, 3 * M + N + Kd)
    assert sa.unique().numel() == 7 and sb.unique().numel() == 7
    ref = K.mxfp4_to_float(a, sa) @ K.mxfp4_to_float(bt, sb).t()
    out = K.gemm_mxfp4_nt(a, bt, sa, sb, out_dtype=out_dtype)
    scale = ref.abs().max().item()
    err = (out.double() - ref).abs().max().item()
    assert err <= (2e-4 if out_dtype == torch.float32 else 8e-3) * scale, (err, scale)


def test_mxfp4_scales_are_per_row_and_block():
    """Unit scales give the plain fp4 GEMM bit for bit; doubling one row's
    scale of one k-block changes exactly that block's contribution (a scale
    taken from the wrong lane, fragment or byte fails this)."""
    M, N, Kd = 256, 256, 512
    a, bt, sa, sb = _mx_operands(M, N, Kd, 77, 127, 127)
    plain = K.gemm_fp4_nt(a, bt, out_dtype=torch.float32)
    assert torch.equal(K.gemm_mxfp4_nt(a, bt, sa, sb, out_dtype=torch.float32), plain)
    for r, blk in ((0, 0), (37, 5), (200, 7), (129, 3)):
        sa2 = sa.clone()
        sa2[r, blk] = 128  # x2 for row r, k-blocks blk, blk + 8, ...
        sb2 = sb.clone()
        sb2[(r * 7) % N, (blk + 1) % 8] = 125  # x1/4 for one B row, another block
        ref = K.mxfp4_to_float(a, sa2) @ K.mxfp4_to_float(bt, sb2).t()
        out = K.gemm_mxfp4_nt(a, bt, sa2, sb2, out_dtype=torch.float32)
        assert (out.double() - ref).abs().max().item() <= 2e-4 * ref.abs().max().item()


@pytest.mark.parametrize("shape", [(4096, 4096), (512, 1024), (300, 1040), (7, 16)])
def test_mxfp4_gemvs_vs_fp32(shape):
    R, C = shape
    x = torch.empty(R, C // 2, device=DEV, dtype=torch.uint8)
    s = torch.empty(R, 8, device=DEV, dtype=torch.uint8)
    K.fill_fp4_(x, R + 3 * C)
    K.fill_e8m0_(s, R + C)
    xf = K.mxfp4_to_float(x, s)
    g = torch.Generator(device="cpu").manual_seed(R * C)
    vr = torch.rand(R, generator=g).mul_(2).sub_(1).to(DEV)
    vc = torch.rand(C, generator=g).mul_(2).sub_(1).to(DEV)
    for got, ref in ((K.gemv_mxfp4(x, s, vr, transpose=True), xf.t() @ vr.double()),
                     (K.gemv_mxfp4(x, s, vc), xf @ vc.double())):
        scale = ref.abs().max().item()
        assert (got.double() - ref).abs().max().item() <= 1e-5 * max(scale, 1.0) * (1 + (R + C) / 1024)
