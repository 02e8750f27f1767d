// The validator's default bf16 GEMM, as the launch sites outside the HIP
// runtime see it: the N7 AQL gate (prof/aql_gate.cpp) dispatches it from
// validator_kernels.co on its own HSA queue, and the gate policy
// (gate_policy.h) derives SQ_WAVES from its waves per tile.  One place, so the
// kernel the HIP path runs (validator_kernels.hip, kDefaultGemmVariant) and
// the one the gate counts cannot drift apart (tests/test_kernel_lib.py reads
// the code object's symbols against this file).
#pragma once

namespace avk {

// gemm_bf16_nt_4wa_kernel<OUT_F32=false, LOOP=13, EPI=1> (variant 29):
// 256x256 tile, 4 waves of 128x128, the generated main loop of schedule 4c
// (validator/gen_gemm4w_asm.py: 64-deep stages in 128-B LDS rows), bf16
// epilogue in 16-B stores
constexpr const char* kGemmSymbol = "gemm_bf16_nt_4wa_kernelILb0ELi13ELi1EE";
constexpr int kGemmThreads = 256;      // workgroup size
constexpr int kGemmWavesPerTile = 4;   // kGemmThreads / 64
constexpr int kGemmTile = 256;         // M and N multiple
constexpr int kGemmKMultiple = 256;    // K multiple

// gemm_fp8_nt_kernel<OUT_F32=false, EPI=1>: the e4m3 GEMM of the mfma-rate
// step, same 256x256 tile and 4 waves, the generated main loop of schedule 8
// (v_mfma_f32_16x16x128_f8f6f4, 128-deep stages)
constexpr const char* kGemmFp8Symbol = "gemm_fp8_nt_kernelILb0ELi1EE";

// gemm_fp4_nt_kernel<OUT_F32=false, EPI=1>: the OCP FP4 GEMM of the
// mfma-rate step (schedule 9: v_mfma_f32_16x16x128_f8f6f4 cbsz:4 blgp:4)
constexpr const char* kGemmFp4Symbol = "gemm_fp4_nt_kernelILb0ELi1EE";

// gemm_fp6_nt_kernel<false, 1>: the OCP FP6 (e2m3) GEMM of the mfma-rate step
// (schedule 10: cbsz:2 blgp:2, fp6 in 32-B slots per 32 elements)
constexpr const char* kGemmFp6Symbol = "gemm_fp6_nt_kernelILb0ELi1EE";

// gemm_mxfp4_nt_kernel<false, 1>: block-scaled MXFP4 (schedule 11:
// v_mfma_scale_f32_16x16x128_f8f6f4, E8M0 scales per row and k-block)
constexpr const char* kGemmMxFp4Symbol = "gemm_mxfp4_nt_kernelILb0ELi1EE";

}  // namespace avk
