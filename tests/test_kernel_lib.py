"""The shipped validator kernels carry one GEMM: the default 8-phase MFMA
kernel (variant 6) that the native validator and its AQL counter gate
dispatch.  The nine A/B kernels of rounds 1-2 live in the tools build
(``make -C native lab``) only."""

import re
import subprocess

from amdgpu_operator import native
from amdgpu_operator.ops import kernels as K

READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"


def _gemm_kernels(path):
    out = subprocess.run([READELF, "-s", "--wide", str(path)], capture_output=True, text=True, timeout=60).stdout
    return sorted(set(re.findall(r"(gemm_bf16_nt_\w+?_kernelI\w+?)EEv", out)))


def test_shipped_code_object_has_only_the_default_gemm():
    assert K.GEMM_DEFAULT_VARIANT == 6
    # <OUT_F32 = false / true, LOAD_IN_M = false, BAL = false, GROUP_M = 4>: the AQL gate's kGemmSymbol
    # (a prefix match, native/prof/aql_gate.cpp) and its f32 twin
    assert _gemm_kernels(native.artefact("validator_kernels.co")) == ["gemm_bf16_nt_8p_kernelILb0ELb0ELb0ELi4E",
                                                                      "gemm_bf16_nt_8p_kernelILb1ELb0ELb0ELi4E"]


def test_lab_variants_are_served_from_the_tools_build():
    assert K.LAB_LIB_NAME.startswith("lab/")
    lab = native.artefact(K.LAB_LIB_NAME)
    if lab.exists():  # built by `make -C native lab`
        names = _gemm_kernels(lab)
        assert any("ring" in n for n in names) and any("w4" in n for n in names)
