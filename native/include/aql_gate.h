// N7 counter gate without a profiler runtime: PMC counters of one dispatch of
// the validator's own GEMM, read through AQL profiling packets on a private
// HSA queue (native/prof/aql_gate.cpp).
#pragma once

#include <cstdint>

#define AVK_AQL_GATE_COUNTERS 4
#define AVK_AQL_GATE_BF16 0  // gemm_default.h kGemmSymbol, SQ_INSTS_VALU_MFMA_MOPS_BF16
#define AVK_AQL_GATE_FP8 1   // gemm_default.h kGemmFp8Symbol, SQ_INSTS_VALU_MFMA_MOPS_F8
#define AVK_AQL_GATE_FP4 2   // gemm_default.h kGemmFp4Symbol, SQ_INSTS_VALU_MFMA_MOPS_F6F4
#define AVK_AQL_GATE_FP6 3   // gemm_default.h kGemmFp6Symbol, SQ_INSTS_VALU_MFMA_MOPS_F6F4
#define AVK_AQL_GATE_MXFP4 4 // gemm_default.h kGemmMxFp4Symbol (E8M0 scales), SQ_INSTS_VALU_MFMA_MOPS_F6F4
#define AVK_AQL_GATE_DTYPES 5

struct avk_aql_gate_result {
  // SQ_INSTS_VALU_MFMA_MOPS_{BF16|F8}, SQ_VALU_MFMA_BUSY_CYCLES, SQ_WAVES, GRBM_GUI_ACTIVE
  double values[AVK_AQL_GATE_COUNTERS];
  int samples[AVK_AQL_GATE_COUNTERS];  // per-instance samples summed into each value
  double setup_s;                      // aqlprofile load, queue, code object, buffers
  double dispatch_s;                   // start packet -> stop packet completion
};

extern "C" {
// Counter names in the order of avk_aql_gate_result::values.
const char* avk_aql_gate_counter_name(int i);
const char* avk_aql_gate_counter_name_dtype(int dtype, int i);

// Dispatch the default GEMM (gemm_default.h: C = A * Bt^T, bf16 out)
// from the code object at `code_object` on the GPU at `pci_bus_id`
// ("dddd:bb:dd.f", hipDeviceGetPCIBusId; `agent_ordinal` picks among the GPU
// agents at that address - the compute partitions of one GPU share it, and HIP
// numbers them in the HSA agents' order), bracketed by aqlprofile start/stop
// packets on a private queue, and sum every per-instance counter sample.  A,
// Bt and C are device pointers (hipMalloc); M, N and K are multiples of 256
// (the kernel's tile).  Waits at most timeout_s for the stop packet.  Returns
// 0, or -1 with a message in err.  The HSA state of the gate (aqlprofile,
// the loaded code object, a private queue, the counter buffers) is set up on
// the first call for a GPU agent and kept for the process's life, so a
// process's later gates (retries, the fp8 GEMM's) cost their dispatch only;
// setup_s is ~0 on those.
int avk_aql_gate_gemm(const char* pci_bus_id, int agent_ordinal, const void* A, const void* Bt, void* C, int M,
                      int N, int K, const char* code_object, double timeout_s, avk_aql_gate_result* out, char* err,
                      int errlen);

// The same for the GEMM of `dtype` (AVK_AQL_GATE_BF16, _FP8: gemm_fp8_nt_kernel,
// A and Bt e4m3 bytes, or _FP4: gemm_fp4_nt_kernel, A and Bt e2m1 pairs; bf16
// out, same grid and kernargs).
int avk_aql_gate_gemm_dtype(int dtype, const char* pci_bus_id, int agent_ordinal, const void* A, const void* Bt,
                            void* C, int M, int N, int K, const char* code_object, double timeout_s,
                            avk_aql_gate_result* out, char* err, int errlen);

// The same for a block-scaled GEMM (AVK_AQL_GATE_MXFP4: kernargs A, Bt, C, M,
// N, K, then the E8M0 scale arrays SA [M][8] and SB [N][8]); SA / SB are
// ignored (may be null) for the other dtypes.
int avk_aql_gate_gemm_scaled(int dtype, const char* pci_bus_id, int agent_ordinal, const void* A, const void* Bt,
                             void* C, int M, int N, int K, const void* SA, const void* SB, const char* code_object,
                             double timeout_s, avk_aql_gate_result* out, char* err, int errlen);

// Set up the gate's HSA state for a GPU agent ahead of its first gate: the
// session above and the counter profiles of every dtype.  It dispatches
// nothing, so it can run on another thread while the process's other kernels
// run; a gate call meanwhile waits for it.  Returns 0, or -1 with a message in
// err (the gate call then reports the failure itself).
int avk_aql_gate_prepare(const char* pci_bus_id, int agent_ordinal, const char* code_object, char* err, int errlen);
}
