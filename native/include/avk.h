// avk.h - C ABI of the validator kernels (validator_kernels.hip) and the N7
// counter gate (prof/counter_gate.cpp).
#ifndef AVK_H_
#define AVK_H_

#include <hip/hip_runtime.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

int avk_abi_version(void);
int avk_fill_uniform_f32(float* p, int64_t n, uint64_t seed, float lo, float hi, hipStream_t s);
int avk_fill_uniform_bf16(void* p, int64_t n, uint64_t seed, float lo, float hi, hipStream_t s);
int avk_vector_add_f32(const float* a, const float* b, float* c, int64_t n, hipStream_t s);
int avk_vector_add_verify_f32(const float* a, const float* b, const float* c, int64_t n, unsigned long long* bad_dev,
                              hipStream_t s);
int avk_gemm_bf16_nt(const void* A, const void* Bt, void* C, int out_f32, int M, int N, int K, hipStream_t s);
int avk_gemv_rows(const void* X, int x_is_bf16, const float* v, float* y, int R, int C, hipStream_t s);
int avk_gemm_fp8_nt(const void* A, const void* Bt, void* C, int out_f32, int M, int N, int K, hipStream_t s);
int avk_fill_fp8(void* p, int64_t n, uint64_t seed, hipStream_t s);
int avk_gemm_fp4_nt(const void* A, const void* Bt, void* C, int out_f32, int M, int N, int K, hipStream_t s);
int avk_fill_fp4(void* p, int64_t nbytes, uint64_t seed, hipStream_t s);
int avk_gemv_rows_fp4(const void* X, const float* v, float* y, int R, int C, hipStream_t s);
int avk_gemv_cols_fp4(const void* X, const float* v, float* z, int R, int C, hipStream_t s);
int avk_gemm_fp6_nt(const void* A, const void* Bt, void* C, int out_f32, int M, int N, int K, hipStream_t s);
int avk_fill_fp6(void* p, int64_t nbytes, uint64_t seed, hipStream_t s);
int avk_gemv_rows_fp6(const void* X, const float* v, float* y, int R, int C, hipStream_t s);
int avk_gemv_cols_fp6(const void* X, const float* v, float* z, int R, int C, hipStream_t s);
int avk_gemm_mxfp4_nt(const void* A, const void* Bt, const void* SA, const void* SB, void* C, int out_f32, int M,
                      int N, int K, hipStream_t s);
int avk_fill_e8m0(void* p, int64_t n, uint64_t seed, int lo, int hi, hipStream_t s);
int avk_gemv_rows_mxfp4(const void* X, const void* S, const float* v, float* y, int R, int C, hipStream_t s);
int avk_gemv_cols_mxfp4(const void* X, const void* S, const float* v, float* z, int R, int C, hipStream_t s);
int avk_gemv_rows_fp8(const void* X, const float* v, float* y, int R, int C, hipStream_t s);
int avk_gemv_cols_fp8(const void* X, const float* v, float* z, int R, int C, hipStream_t s);
int avk_gemv_cols_bf16(const void* X, const float* v, float* z, int R, int C, hipStream_t s);
int avk_hbm_copy(const void* src, void* dst, int64_t bytes, int num_cus, int variant, hipStream_t s);
int avk_checksum(const void* p, int64_t bytes, unsigned long long* out_dev, hipStream_t s);
int avk_max_abs_diff_f32(const float* a, const float* b, int64_t n, unsigned int* out_dev, hipStream_t s);
int avk_allreduce_oneshot_f32(const float* const* ptrs, int np, float* out, int64_t count, hipStream_t s);
int avk_allreduce_twoshot_f32(const float* const* in_ptrs, float* const* out_ptrs, int np, int rank, int64_t count,
                              hipStream_t s);
int avk_fill_const(void* x, int64_t n, int is_bf16, float value, hipStream_t s);
int avk_check_blocks(const void* x, int64_t n, int is_bf16, int64_t block, float base, float step,
                     unsigned long long* bad_dev, hipStream_t s);
int avk_mfma_probe_count(void);
const char* avk_mfma_probe_name(int kind);
int avk_mfma_probe(int kind, uint64_t seed, int* mismatches, hipStream_t s);

// N7 counter gate: exported by libamdgpu_counter_gate.so (a rocprofiler-sdk
// tool), resolved at run time by the validator (validator_main.cpp, Gate)
int avk_prof_active(void);
void avk_prof_arm(const char* kernel_substr);
void avk_prof_disarm(void);
int avk_prof_dispatches(void);
double avk_prof_value(const char* counter);

#ifdef __cplusplus
}
#endif

#endif  // AVK_H_
