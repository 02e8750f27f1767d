"""fp8 GEMM accuracy diagnostics: our kernel and torch._scaled_mm vs an fp64 reference."""
import json
import torch
from amdgpu_operator.ops import kernels as K

dev = "cuda"
out = {}


def ref64(a, bt):
    return a.double() @ bt.double().t()


def errs(name, a, bt):
    r = ref64(a, bt)
    ours = K.gemm_fp8_nt(a, bt, out_dtype=torch.float32).double()
    one = torch.ones((), device=dev)
    sm = torch._scaled_mm(a, bt.t(), scale_a=one, scale_b=one, out_dtype=torch.float32).double()
    f32 = (a.float() @ bt.float().t()).double()
    sc = r.abs().max().item()
    out[name] = {"scale": sc, "ours": (ours - r).abs().max().item(), "scaled_mm": (sm - r).abs().max().item(),
                 "torch_f32": (f32 - r).abs().max().item(), "ours_vs_scaled_mm": (ours - sm).abs().max().item(),
                 "ours_eq_scaled_mm": bool(torch.equal(ours, sm))}


for (M, N, Kd) in [(256, 256, 128 * 2), (256, 256, 1024), (1024, 1024, 4096)]:
    a = torch.empty(M, Kd, device=dev, dtype=torch.float8_e4m3fn)
    bt = torch.empty(N, Kd, device=dev, dtype=torch.float8_e4m3fn)
    K.fill_fp8_(a, 1)
    K.fill_fp8_(bt, 2)
    errs(f"fill_{M}x{N}x{Kd}", a, bt)
    # no subnormals: exponent field >= 1
    au, bu = a.view(torch.uint8), bt.view(torch.uint8)
    a2 = (au | 0x08).view(torch.float8_e4m3fn)
    b2 = (bu | 0x08).view(torch.float8_e4m3fn)
    errs(f"normal_{M}x{N}x{Kd}", a2, b2)
    # only K slice 0..127 nonzero in A: one MFMA's worth
    a3 = a.float().clone(); a3[:, 128:] = 0
    errs(f"k128_{M}x{N}x{Kd}", a3.to(torch.float8_e4m3fn), bt)
    # small integers: exact everywhere
    g = torch.Generator(device=dev).manual_seed(3)
    ai = torch.randint(-8, 9, (M, Kd), device=dev, generator=g).float().to(torch.float8_e4m3fn)
    bi = torch.randint(-8, 9, (N, Kd), device=dev, generator=g).float().to(torch.float8_e4m3fn)
    errs(f"int_{M}x{N}x{Kd}", ai, bi)
    # subnormals only in A
    a4 = (au & 0x87).view(torch.float8_e4m3fn)
    errs(f"subnA_{M}x{N}x{Kd}", a4, b2)
print(json.dumps(out, indent=1))
