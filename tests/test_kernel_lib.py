"""The shipped validator kernels carry the GEMMs the validator runs: the
default 4-wave kernel with the generated main loop (variant 29, what the
native validator and its AQL counter gate dispatch when K % 256 == 0, named
in native/include/gemm_default.h) and the 8-phase fallback for the other K
(6).  The other generated schedules and the A/B kernels of rounds 1-3 live
in the tools build (``make -C native lab``) only."""

import pathlib
import re
import subprocess

from amdgpu_operator import native
from amdgpu_operator.ops import kernels as K

READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"


def _gemm_kernels(path):
    out = subprocess.run([READELF, "-s", "--wide", str(path)], capture_output=True, text=True, timeout=60).stdout
    return sorted(set(re.findall(r"(gemm_bf16_nt_\w+?_kernelI\w+?)EEv", out)))


def test_shipped_code_object_has_only_the_default_gemm():
    assert (K.GEMM_DEFAULT_VARIANT, K.GEMM_FALLBACK_VARIANT) == (29, 6)
    # variant 29: <OUT_F32 = false, LOOP = 13, EPI = 1> and its f32 twin <true, 13, 0>;
    # variant 6: <OUT_F32, LOAD_IN_M = false, BAL = false, GROUP_M = 4>
    assert _gemm_kernels(native.artefact("validator_kernels.co")) == [
        "gemm_bf16_nt_4wa_kernelILb0ELi13ELi1E", "gemm_bf16_nt_4wa_kernelILb1ELi13ELi0E",
        "gemm_bf16_nt_8p_kernelILb0ELb0ELb0ELi4E", "gemm_bf16_nt_8p_kernelILb1ELb0ELb0ELi4E"]


def test_the_gate_dispatches_the_default_kernel():
    """gemm_default.h's symbol (the AQL gate's prefix match) names exactly one
    kernel of the code object: variant 29's bf16-out instance."""
    hdr = (pathlib.Path(__file__).resolve().parents[1] / "native" / "include" / "gemm_default.h").read_text()
    sym = re.search(r'kGemmSymbol = "(\w+)"', hdr).group(1)
    assert [n for n in _gemm_kernels(native.artefact("validator_kernels.co")) if sym.startswith(n)] == \
        ["gemm_bf16_nt_4wa_kernelILb0ELi13ELi1E"]
    assert int(re.search(r"kGemmThreads = (\d+);", hdr).group(1)) == 64 * int(
        re.search(r"kGemmWavesPerTile = (\d+);", hdr).group(1)) == 256


def test_lab_variants_are_served_from_the_tools_build():
    assert K.LAB_LIB_NAME.startswith("lab/")
    lab = native.artefact(K.LAB_LIB_NAME)
    if lab.exists():  # built by `make -C native lab`
        names = _gemm_kernels(lab)
        assert any("ring" in n for n in names) and any("w4" in n for n in names)
