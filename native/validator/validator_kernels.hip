// Operator-validator GPU workload for MI355X (gfx950 / CDNA4).
//
// Capability parity: the reference's "Running or Completed" validator pods
// (/root/reference/README.md:199) run an upstream CUDA vectorAdd sample.  This
// file is the MI355X-native replacement described in SURVEY.md §2.D:
//   K1 vector_add      - fp32 c = a + b, 16 B/lane, grid-stride
//   K2 gemm_bf16_nt    - bf16 MFMA GEMM (v_mfma_f32_16x16x32_bf16), 256x256x64
//                        block tile, 8 waves in two ping-pong groups, 8-phase
//                        quadrant pipeline, global_load_lds staging into an
//                        XOR-swizzled LDS image, XCD-aware tile order
//   K3 hbm_copy        - float4 streaming copy (HBM3E bandwidth check)
//   K4 allreduce_*     - one-shot / two-shot sum over n peer buffers (peer
//                        pointers over xGMI, or n emulated buffers on one GPU)
//   K5 mfma_probe      - one MFMA tile per CDNA4 matrix data type (f16, bf16,
//                        fp8, bf8, int8, block-scaled fp8/fp6/fp4, f32, f64),
//                        checked exactly on the host
// plus helpers for the correctness gates (device RNG fill, Freivalds GEMV
// check, checksum, max-abs-diff).
//
// Everything is exported through a C ABI (avk_*) so the same library serves
// the Python control plane (ctypes, torch tensors) and the standalone
// C++ validator binary (validator_main.cpp).  Every launcher validates the
// shapes its kernel assumes and returns hipErrorInvalidValue instead of
// launching an out-of-bounds grid.

#include <hip/hip_runtime.h>
#include <utility>
#include "gemm_default.h"
#include <stdint.h>
#include <string.h>

#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));

#define AVK_API extern "C" __attribute__((visibility("default")))

namespace {

constexpr int kNumXcd = 8;

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// uniform in [lo, hi) from a 24-bit mantissa
__device__ __forceinline__ float u01(uint64_t h) {
  return (float)(h >> 40) * (1.0f / 16777216.0f);
}

// ---------------------------------------------------------------- fills ----

__global__ __launch_bounds__(256) void fill_uniform_f32_kernel(float* __restrict__ p, int64_t n,
                                                               uint64_t seed, float lo, float hi) {
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  int64_t stride = (int64_t)gridDim.x * 256;
  float scale = hi - lo;
  for (; i < n; i += stride) p[i] = lo + scale * u01(splitmix64(seed ^ (uint64_t)i * 0xD1B54A32D192ED03ull));
}

__global__ __launch_bounds__(256) void fill_uniform_bf16_kernel(__bf16* __restrict__ p, int64_t n8,
                                                                uint64_t seed, float lo, float hi) {
  // n8 = number of 8-element (16 B) groups
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  int64_t stride = (int64_t)gridDim.x * 256;
  float scale = hi - lo;
  for (; i < n8; i += stride) {
    bf16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      uint64_t idx = (uint64_t)(i * 8 + j);
      v[j] = (__bf16)(lo + scale * u01(splitmix64(seed ^ idx * 0xD1B54A32D192ED03ull)));
    }
    reinterpret_cast<bf16x8*>(p)[i] = v;
  }
}

// ------------------------------------------------------------ K1 vector add ----

// U float4s per lane per iteration, nontemporal (streamed once) - the K3
// sweep's best copy shape (profiles/r1_hbm)
template <int U>
__global__ __launch_bounds__(256) void vector_add_kernel(const f32x4* __restrict__ a, const f32x4* __restrict__ b,
                                                         f32x4* __restrict__ c, int64_t n4) {
  const int64_t stride = (int64_t)gridDim.x * 256 * U;
  int64_t i = (int64_t)blockIdx.x * 256 * U + threadIdx.x;
  for (; i + (U - 1) * 256 < n4; i += stride) {
    f32x4 x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      x[u] = __builtin_nontemporal_load(a + i + u * 256);
      y[u] = __builtin_nontemporal_load(b + i + u * 256);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) __builtin_nontemporal_store(x[u] + y[u], c + i + u * 256);
  }
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (i + u * 256 < n4) c[i + u * 256] = a[i + u * 256] + b[i + u * 256];
}

// The in-container GPU check (native/validator/gpu_check.cpp) dispatches this
// through HSA directly: one element per lane, no loop and no implicit kernel
// arguments (grid and block sizes are not read), so a raw AQL packet with the
// explicit arguments alone runs it correctly and it always terminates.
extern "C" __global__ __launch_bounds__(256) void avk_gpu_check_add(const float* __restrict__ a,
                                                                   const float* __restrict__ b,
                                                                   float* __restrict__ c, int n) {
  const int i = (int)blockIdx.x * 256 + (int)threadIdx.x;
  if (i < n) c[i] = a[i] + b[i];
}

__global__ void vector_add_tail_kernel(const float* a, const float* b, float* c, int64_t start, int64_t n) {
  int64_t i = start + threadIdx.x;
  if (i < n) c[i] = a[i] + b[i];
}

// K1 check: counts c[i] != a[i] + b[i] on the device (the validator also
// spot-checks a prefix on the host), so the 16M-element check costs one
// stream over HBM instead of a 192 MB device-to-host copy
__global__ __launch_bounds__(256) void vector_add_verify_kernel(const float* __restrict__ a,
                                                                const float* __restrict__ b,
                                                                const float* __restrict__ c, int64_t n,
                                                                unsigned long long* __restrict__ bad) {
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * 256;
  unsigned long long m = 0;
  for (; i < n; i += stride) m += c[i] != a[i] + b[i];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) m += __shfl_xor(m, off, 64);
  if ((threadIdx.x & 63) == 0 && m) atomicAdd(bad, m);
}

// ------------------------------------------- collective operand fill / check ----
// The RCCL step's operands are filled and checked on the device: rank r fills
// r+1, and element i of a result must equal base + (i / block) * step (a
// constant for all-reduce / reduce-scatter, the source rank's value for
// all-gather).  No host round trip of the 64 MB buffers.
template <typename T>
__global__ __launch_bounds__(256) void fill_const_kernel(T* __restrict__ x, int64_t n, T v) {
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (; i < n; i += stride) x[i] = v;
}

// f32: exact compare; bf16 (is_bf16): compare the bit pattern of the expected
// value rounded to bf16 (exact for the small integers used)
template <bool kBf16>
__global__ __launch_bounds__(256) void check_blocks_kernel(const void* __restrict__ x, int64_t n, int64_t block,
                                                           float base, float step, unsigned long long* __restrict__ bad) {
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * 256;
  unsigned long long m = 0;
  for (; i < n; i += stride) {
    const float want = base + (float)(i / block) * step;
    if constexpr (kBf16) {
      m += static_cast<const uint16_t*>(x)[i] != (uint16_t)(__float_as_uint(want) >> 16);
    } else {
      m += static_cast<const float*>(x)[i] != want;
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) m += __shfl_xor(m, off, 64);
  if ((threadIdx.x & 63) == 0 && m) atomicAdd(bad, m);
}

// --------------------------------------------------------- K2 bf16 MFMA GEMM ----
//
// C[M][N] = A[M][K] · Bt[N][K]^T   (both operands K-contiguous, "NT")
//
// Block tile 256x256, K-step 64, 512 threads = 8 waves arranged 2 (M) x 4 (N);
// each wave owns a 128x64 output = 8x4 tiles of v_mfma_f32_16x16x32_bf16.
// LDS holds two stages of {A 256x64, B 256x64} bf16 = 2 x 64 KiB.  Each stage
// is filled by global_load_lds_dwordx4: one wave-instruction writes 1 KiB =
// 8 rows x 128 B lane-linearly; the bank swizzle lives on the SOURCE address
// (logical 16-B chunk = physical chunk ^ ((row >> 1) & 7)) and the same XOR is
// applied on the ds_read_b128 side, which makes every 16-lane ds_read_b128
// group of a fragment read hit 16 distinct 16-B slots (conflict-free).

namespace gemm {
constexpr int BM = 256, BN = 256, BK = 64;   // every variant's block tile (the launcher's shape check)
#if AVK_GEMM_LAB
constexpr int TILE_BYTES = BM * BK * 2;      // 32 KiB (A or B of one stage)
constexpr int STAGE_BYTES = 2 * TILE_BYTES;  // 64 KiB
constexpr int NTHR = 512;
constexpr int LDS_BYTES = 2 * STAGE_BYTES;   // 128 KiB
constexpr int GROUP_M = 4;                   // tile rows per L2 band
#endif
}  // namespace gemm

typedef __attribute__((address_space(3))) void* lds_void_ptr;

// Diagnostic build only (-DAVK_STAMPS, tools/gemm_stamps.py): s_memtime at
// the segment boundaries of the ping-pong GEMM for the first workgroups, to
// split a slice into read / wait / barrier / MFMA time.  The shipped library
// compiles every AVK_STAMP away.
#ifdef AVK_STAMPS
constexpr int kStampBlocks = 4, kStampSlices = 32, kStampPoints = 6;
__device__ unsigned long long g_stamps[kStampBlocks * 8 * kStampSlices * kStampPoints];
#define AVK_STAMP(t, k)                                                                              \
  do {                                                                                               \
    if (blockIdx.x < kStampBlocks && (t) < kStampSlices && (threadIdx.x & 63) == 0)                 \
      g_stamps[((blockIdx.x * 8 + (threadIdx.x >> 6)) * kStampSlices + (t)) * kStampPoints + (k)] = \
          __builtin_amdgcn_s_memtime();                                                              \
  } while (0)
#else
#define AVK_STAMP(t, k) \
  do {                  \
  } while (0)
#endif

#if AVK_GEMM_LAB
#include "gemm_lab_1.inc"
#endif  // AVK_GEMM_LAB

__device__ __forceinline__ void wg_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

#if AVK_GEMM_LAB
#include "gemm_lab_2.inc"
#endif  // AVK_GEMM_LAB

// ------------------- K2 GEMM, 8-phase quadrant pipeline (BK = 64, 2 buffers) ----
//
// Same 256x256 block, 8 waves (2M x 4N, 128x64 per wave, 16x16x32 MFMA) and
// two-group ping-pong as gemm_bf16_nt_pp_kernel, but the unit of work is a
// wave QUADRANT (64 rows x 32 cols x K 64 = 16 MFMAs) and the unit of staging
// a HALF-TILE (16 KiB) that is refilled as soon as its fragments are in
// registers (cdna_hip_programming.md §5 "The 256² 8-phase template").
//
// A K-tile (64 deep) lives in one of two 64 KiB buffers as four half-tiles:
//   A0 / A1  = quadrant rows 0..63 / 64..127 of BOTH row groups (128 rows)
//   B0 / B1  = quadrant cols 0..31 / 32..63 of all four column groups
// (128-B rows, source-side XOR swizzle chunk ^ ((row >> 1) & 7): every 16-lane
// ds_read_b128 group hits 16 distinct bank slots).  Phases of K-tile t:
//   phase  reads (regs)         MFMAs     refill issued (LDS slot freed)
//   0      A0 -> a, B0 -> b0    Q(0,0)    A1 of K-tile t+1 (other buffer)
//   1      B1 -> b1             Q(0,1)    A0 of K-tile t+2 (read in phase 0)
//   2      A1 -> a              Q(1,1)    B0 of K-tile t+2 (read in phase 0)
//   3      -                    Q(1,0)    B1 of K-tile t+2 (read in phase 1)
// so every half-tile is issued 6-7 phases before it is read, and at every
// wait five younger half-tiles (10 LDS-DMAs per wave) may stay in flight.
// A phase = read segment | barrier | MFMA segment | barrier; group 1 (waves
// 4-7) passes one extra barrier up front, so each SIMD alternates one wave
// reading with one wave issuing MFMAs.  Barrier b separates segments b, b+1;
// group 0 reads phase R in segment 2R, group 1 in 2R+1.
//   RAW  data read in phase R was issued by phase R-6; every wave retires it
//        before barrier 2R-1 (group 0 at the end of its MFMA segment R-1,
//        group 1 at the end of its read segment R-1) with vmcnt(10) - or
//        vmcnt(8) for group 1 when the refill sits in the MFMA segment
//        (LOAD_IN_M: issued only through R-2 at that point).
//   WAR  a slot is refilled one phase after its last read; those reads were
//        retired by lgkmcnt(0) BEFORE the reading phase's first barrier, which
//        every wave passes before it issues the refill.
// Past the last K-tile the refills re-read K-tile nk-1 into slots no one reads
// again, which keeps every wait count constant; vmcnt(0) drains them at exit.
namespace g8 {
constexpr int BM = 256, BN = 256, BK = 64, NTHR = 512;
constexpr int HT_BYTES = 128 * BK * 2;    // 16 KiB half-tile: 128 rows x 128 B
constexpr int BUF_BYTES = 4 * HT_BYTES;   // 64 KiB: A0 A1 B0 B1
constexpr int LDS_BYTES = 2 * BUF_BYTES;  // 128 KiB
constexpr int GROUP_M = 4;  // tile rows per L2 band (8 / 16 / 2: lab variants 10-12; profiles/r3_gemm)
constexpr int HA0 = 0, HA1 = 1, HB0 = 2, HB1 = 3;
}  // namespace g8

// this wave's 2 pieces (8 rows x 128 B each) of half-tile HT of K-tile kt
template <int HT>
__device__ __forceinline__ void g8_issue(const __bf16* __restrict__ A, const __bf16* __restrict__ Bt, int K, int m0,
                                         int n0, int kt, char* buf, int wave, int lane) {
  using namespace g8;
  const int rsub = lane >> 3, pc = lane & 7;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int p = wave * 2 + i;   // piece 0..15
    const int lr = p * 8 + rsub;  // half-tile row 0..127
    const int lc = pc ^ ((lr >> 1) & 7);
    const __bf16* src;
    if constexpr (HT == HA0 || HT == HA1)
      src = A + (size_t)(m0 + (lr >> 6) * 128 + (HT == HA1 ? 64 : 0) + (lr & 63)) * K;
    else
      src = Bt + (size_t)(n0 + (lr >> 5) * 64 + (HT == HB1 ? 32 : 0) + (lr & 31)) * K;
    __builtin_amdgcn_global_load_lds(src + kt * BK + lc * 8, (lds_void_ptr)(buf + HT * HT_BYTES + p * 1024), 16, 0, 0);
  }
}

// A quadrant fragments: 4 row tiles x 2 k-halves (8 x ds_read_b128)
__device__ __forceinline__ void g8_read_a(bf16x8 (&a)[4][2], const char* ht, int wm, int lane) {
  const int fr = lane & 15, fq = lane >> 4, fsw = fr >> 1;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int s = 0; s < 2; ++s)
      a[i][s] = *reinterpret_cast<const bf16x8*>(ht + (wm * 64 + i * 16 + fr) * 128 + (((s * 4 + fq) ^ fsw) << 4));
}

// B quadrant fragments: 2 col tiles x 2 k-halves (4 x ds_read_b128)
__device__ __forceinline__ void g8_read_b(bf16x8 (&b)[2][2], const char* ht, int wn, int lane) {
  const int fr = lane & 15, fq = lane >> 4, fsw = fr >> 1;
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int s = 0; s < 2; ++s)
      b[j][s] = *reinterpret_cast<const bf16x8*>(ht + (wn * 32 + j * 16 + fr) * 128 + (((s * 4 + fq) ^ fsw) << 4));
}

template <int N>
__device__ __forceinline__ void g8_vmwait() {
  if constexpr (N == 6)
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if constexpr (N == 8)
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (N == 10)
    asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
  else
    static_assert(N == 6 || N == 8 || N == 10, "vmcnt");
}

// One phase from the first barrier on: MFMAs of quadrant (MQ, NQ) and the
// refill of half-tile HT (K-tile kt into buf).  VM_LEAD / VM_LAG are the
// vmcnt counts of group 0 (end of MFMA segment) and group 1 (end of read
// segment).  EARLY_LGKM retires this phase's ds_reads before the first
// barrier (needed when the next phase refills a slot read here); otherwise
// the compiler's own lgkmcnt waits land between the MFMAs.
template <int MQ, int NQ, int HT, bool LOAD_IN_M, int VM_LEAD, int VM_LAG, bool EARLY_LGKM>
__device__ __forceinline__ void g8_phase(f32x4 (&acc)[8][4], const bf16x8 (&a)[4][2], const bf16x8 (&b)[2][2],
                                         const __bf16* __restrict__ A, const __bf16* __restrict__ Bt, int K, int m0,
                                         int n0, int kt, char* buf, int wave, int lane, bool lag, bool skip_last) {
  if constexpr (!LOAD_IN_M) g8_issue<HT>(A, Bt, K, m0, n0, kt, buf, wave, lane);
  if constexpr (EARLY_LGKM) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (lag) g8_vmwait<VM_LAG>();
  wg_barrier();
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[MQ * 4 + i][NQ * 2 + j] =
            __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j][s], a[i][s], acc[MQ * 4 + i][NQ * 2 + j], 0, 0, 0);
  if constexpr (LOAD_IN_M) {
    g8_issue<HT>(A, Bt, K, m0, n0, kt, buf, wave, lane);
    __builtin_amdgcn_sched_group_barrier(0x008, 6, 0);  // MFMA
    __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // one LDS-DMA piece
    __builtin_amdgcn_sched_group_barrier(0x008, 6, 0);
    __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
  }
  __builtin_amdgcn_s_setprio(0);
  if (!lag) g8_vmwait<VM_LEAD>();
  if (!skip_last) wg_barrier();
}

// BAL (balanced reads, 8/4/8/4 ds_read_b128 per phase instead of 12/4/8/0):
// phase 3 of K-tile t also reads B0 of K-tile t+1 into a second register set
// (b0n), which phase 0 then takes over.  That read is 5 phases after its
// issue (4t-2 -> 4t+3), so one fewer half-tile may stay in flight: vmcnt(8),
// or vmcnt(6) for group 1 with LOAD_IN_M.  B0's slot is now last read 3
// phases before its refill, so only phase 0 (A0, refilled in phase 1) retires
// its reads before the first barrier.
template <bool OUT_F32, bool LOAD_IN_M, bool BAL, int GM = g8::GROUP_M>
__global__ __launch_bounds__(g8::NTHR, 2) void gemm_bf16_nt_8p_kernel(const __bf16* __restrict__ A,
                                                                     const __bf16* __restrict__ Bt,
                                                                     void* __restrict__ Cv, int M, int N, int K) {
  using namespace g8;
  constexpr int VM_LEAD = BAL ? 8 : 10;
  constexpr int VM_LAG = LOAD_IN_M ? VM_LEAD - 2 : VM_LEAD;
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const bool lag = wm == 1;  // wave-uniform

  const int tiles_m = M / BM, tiles_n = N / BN;
  const int nwg = tiles_m * tiles_n;
  const int bid = blockIdx.x;
  const int xcd = bid % kNumXcd;
  const int q = nwg / kNumXcd, rr = nwg % kNumXcd;
  const int wgid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + bid / kNumXcd;
  const int per_group = GM * tiles_n;  // GM tile rows per L2 band (lab variants 10-12 vary it)
  const int first_m = (wgid / per_group) * GM;
  const int gsize = min(tiles_m - first_m, GM);
  const int in_group = wgid % per_group;
  const int m0 = (first_m + in_group % gsize) * BM;
  const int n0 = (in_group / gsize) * BN;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nk = K / BK;
  // prologue = the issues the steady state makes in phases -7..-1:
  // K-tile 0 complete, K-tile 1 without A1 (issued by phase 0)
  const int k1 = min(1, nk - 1);
  g8_issue<HA0>(A, Bt, K, m0, n0, 0, smem, wave, lane);
  g8_issue<HB0>(A, Bt, K, m0, n0, 0, smem, wave, lane);
  g8_issue<HB1>(A, Bt, K, m0, n0, 0, smem, wave, lane);
  g8_issue<HA1>(A, Bt, K, m0, n0, 0, smem, wave, lane);
  g8_issue<HA0>(A, Bt, K, m0, n0, k1, smem + BUF_BYTES, wave, lane);
  g8_issue<HB0>(A, Bt, K, m0, n0, k1, smem + BUF_BYTES, wave, lane);
  g8_issue<HB1>(A, Bt, K, m0, n0, k1, smem + BUF_BYTES, wave, lane);
  asm volatile("s_waitcnt vmcnt(10)" ::: "memory");  // A0, B0 of K-tile 0 landed
  wg_barrier();
  if (lag) wg_barrier();

  bf16x8 a[4][2], b0[2][2], b1[2][2], b0n[2][2];
  if constexpr (BAL) g8_read_b(b0n, smem + HB0 * HT_BYTES, wn, lane);
  for (int t = 0; t < nk; ++t) {
    char* cur = smem + (t & 1) * BUF_BYTES;
    char* nxt = smem + ((t + 1) & 1) * BUF_BYTES;
    const int kn1 = min(t + 1, nk - 1), kn2 = min(t + 2, nk - 1);
    g8_read_a(a, cur + HA0 * HT_BYTES, wm, lane);
    if constexpr (BAL) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int s = 0; s < 2; ++s) b0[j][s] = b0n[j][s];
    } else {
      g8_read_b(b0, cur + HB0 * HT_BYTES, wn, lane);
    }
    g8_phase<0, 0, HA1, LOAD_IN_M, VM_LEAD, VM_LAG, true>(acc, a, b0, A, Bt, K, m0, n0, kn1, nxt, wave, lane, lag,
                                                          false);
    g8_read_b(b1, cur + HB1 * HT_BYTES, wn, lane);
    g8_phase<0, 1, HA0, LOAD_IN_M, VM_LEAD, VM_LAG, !BAL>(acc, a, b1, A, Bt, K, m0, n0, kn2, cur, wave, lane, lag,
                                                          false);
    g8_read_a(a, cur + HA1 * HT_BYTES, wm, lane);
    g8_phase<1, 1, HB0, LOAD_IN_M, VM_LEAD, VM_LAG, !BAL>(acc, a, b1, A, Bt, K, m0, n0, kn2, cur, wave, lane, lag,
                                                          false);
    if constexpr (BAL) g8_read_b(b0n, nxt + HB0 * HT_BYTES, wn, lane);  // unused past the last K-tile
    g8_phase<1, 0, HB1, LOAD_IN_M, VM_LEAD, VM_LAG, !BAL>(acc, a, b0, A, Bt, K, m0, n0, kn2, cur, wave, lane, lag,
                                                          lag && t == nk - 1);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may outlive the workgroup
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");

  const int crow = m0 + wm * 128 + (lane & 15);
  const int ccol = n0 + wn * 64 + (lane >> 4) * 4;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const size_t idx = (size_t)(crow + i * 16) * N + ccol + j * 16;
      if constexpr (OUT_F32) {
        *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(Cv) + idx) = acc[i][j];
      } else {
        typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
        bf16x4 v = {(__bf16)acc[i][j][0], (__bf16)acc[i][j][1], (__bf16)acc[i][j][2], (__bf16)acc[i][j][3]};
        *reinterpret_cast<bf16x4*>(reinterpret_cast<__bf16*>(Cv) + idx) = v;
      }
    }
}

// ------------- K2 GEMM, 4 waves x 128x128, 5-slot LDS-DMA ring (variant 14) ----
//
// Same 256x256 block tile, but 4 waves (2M x 2N), each owning 128x128 of the
// output = 8x8 tiles of v_mfma_f32_16x16x32_bf16 (256 accumulators, the AGPR
// half of the register file; one wave per SIMD).  Against the 8-wave
// kernels' 128x64 wave tile this halves the LDS reads per MFMA (16
// ds_read_b128 per 64 MFMAs instead of 12 per 32: 0.25 vs 0.375), which the
// round-1/3 counters name as the cost (profiles/r3_gemm: MFMA util 0.66,
// SQ_WAIT_ANY 29 %; hipBLASLt's MT256x256x64 4-wave kernel 0.88 / 5 %).
// With no partner wave on the SIMD to hide behind, the wave pipelines
// itself:
//   * K is consumed in 32-deep slices (A 256x32 + B 256x32 = 32 KiB) through a
//     5-slot ring (all 160 KiB of LDS) filled by global_load_lds_dwordx4;
//     slice s+5 is issued right after barrier s into the slot slice s just
//     left, so every slice has four barrier intervals (~4 K cycles) to land;
//   * two fragment register sets (2 x 64 VGPRs): the MFMAs of slice s run on
//     one while slice s+1's 16 ds_read_b128 fill the other, spread over the
//     first 48 MFMAs, and the 8 LDS-DMA pieces of slice s+5 sit between
//     MFMAs too (sched_group_barrier pins the interleave);
//   * one raw barrier per slice (1,024 MFMA cycles), behind a counted
//     vmcnt(24) - three slices stay in flight across it - and lgkmcnt(0).
//   RAW  slice x is read during slice x-1, after barrier x-1; every wave's
//        pieces of it were waited for (vmcnt) before that barrier.
//   WAR  slot s%5 is refilled after barrier s; every wave retired its reads
//        of slice s (issued during slice s-1) before reaching barrier s.
// LDS image of one operand slice: row r at r*64 B, 16-B chunk c at
// (c ^ ((-(r >> 2)) & 3)) * 16 - with the ds_read_b128 lane groups
// ({0-3,12-15,20-27}, {4-11,16-19,28-31}, ... MI355X_MICROARCH.md §LDS) every
// fragment read of a 16-row tile hits 16 distinct 16-B bank slots; the XOR is
// applied to the glds SOURCE address (the LDS side is lane-linear) and on
// the read.  Past the last slice the refills re-read slice nk-1 into slots no
// one reads, which keeps the wait counts constant; vmcnt(0) drains them.
namespace g4 {
constexpr int BM = 256, BN = 256, BKS = 32, NTHR = 256, NSLOT = 5;
constexpr int OP_BYTES = BM * BKS * 2;          // 16 KiB: one operand's slice, 256 rows x 64 B
constexpr int SLOT_BYTES = 2 * OP_BYTES;        // 32 KiB
constexpr int LDS_BYTES = NSLOT * SLOT_BYTES;   // 160 KiB
constexpr int GROUP_M = 4;                      // tile rows per L2 band
constexpr int VM_INFLIGHT = (NSLOT - 2) * 8;    // pieces per wave of the slices that may stay in flight
}  // namespace g4

__device__ __forceinline__ int g4_chunk_xor(int row) { return (-(row >> 2)) & 3; }

template <int N>
__device__ __forceinline__ void g4_vmwait() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Slice s's MFMAs (row-major: MFMA m = 8i + j updates acc[i][j]) on fa / cb;
// slice s+1's fragments from rslot: A fragment i into fa[i] right after its
// last use (MFMA 8i+7) - one A register set - and the B fragments into the
// second set nb early in the slice; this wave's 8 pieces of slice `kload`
// into wslot between MFMAs.
__device__ __forceinline__ constexpr bool g4_bread(int m) { return m % 3 == 1 && m / 3 < 8; }
__device__ __forceinline__ constexpr bool g4_aread(int m) { return m % 8 == 7; }
__device__ __forceinline__ constexpr bool g4_glds(int m) { return m % 8 == 4; }

__device__ __forceinline__ void g4_slice(f32x4 (&acc)[8][8], bf16x8 (&fa)[8], const bf16x8 (&cb)[8], bf16x8 (&nb)[8],
                                         const char* rslot, char* wslot, const __bf16* __restrict__ ga,
                                         const __bf16* __restrict__ gb, size_t piece_stride, int kload, int a_off,
                                         int b_off, int wave) {
  using namespace g4;
  // pin every accumulator to the AGPR file at the slice boundary (an empty
  // asm, no instruction): the register allocator otherwise parks some of the
  // 256 in VGPRs and shuffles them through v_accvgpr_read/write every slice
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) asm volatile("" : "+a"(acc[i][j]));
#pragma unroll
  for (int m = 0; m < 64; ++m) {
    const int i = m >> 3, j = m & 7;
    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cb[j], fa[i], acc[i][j], 0, 0, 0);
    if (g4_bread(m)) nb[m / 3] = *reinterpret_cast<const bf16x8*>(rslot + b_off + (m / 3) * 1024);
    if (g4_aread(m)) fa[i] = *reinterpret_cast<const bf16x8*>(rslot + a_off + i * 1024);
    if (g4_glds(m)) {
      const int q = m / 8;  // piece: operand q >> 2, row block wave*4 + (q & 3)
      const __bf16* src = (q < 4 ? ga : gb) + (q & 3) * piece_stride + kload;
      __builtin_amdgcn_global_load_lds(src, (lds_void_ptr)(wslot + (q < 4 ? 0 : OP_BYTES) + (wave * 4 + (q & 3)) * 1024),
                                       16, 0, 0);
    }
  }
#pragma unroll
  for (int m = 0; m < 64; ++m) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
    if (g4_bread(m)) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
    if (g4_aread(m)) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    if (g4_glds(m)) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // LDS-DMA piece
  }
}

__device__ __forceinline__ void g4_stage(const __bf16* __restrict__ ga, const __bf16* __restrict__ gb,
                                         size_t piece_stride, int k0, char* slot, int wave) {
  using namespace g4;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const __bf16* src = (q < 4 ? ga : gb) + (q & 3) * piece_stride + k0;
    __builtin_amdgcn_global_load_lds(src, (lds_void_ptr)(slot + (q < 4 ? 0 : OP_BYTES) + (wave * 4 + (q & 3)) * 1024),
                                     16, 0, 0);
  }
}

template <bool OUT_F32>
__global__ __launch_bounds__(g4::NTHR, 1) void gemm_bf16_nt_4w_kernel(const __bf16* __restrict__ A,
                                                                     const __bf16* __restrict__ Bt,
                                                                     void* __restrict__ Cv, int M, int N, int K) {
  using namespace g4;
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;

  const int tiles_m = M / BM, tiles_n = N / BN;
  const int nwg = tiles_m * tiles_n;
  const int bid = blockIdx.x;
  const int xcd = bid % kNumXcd;
  const int q = nwg / kNumXcd, rr = nwg % kNumXcd;
  const int wgid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + bid / kNumXcd;
  const int per_group = GROUP_M * tiles_n;
  const int first_m = (wgid / per_group) * GROUP_M;
  const int gsize = min(tiles_m - first_m, GROUP_M);
  const int in_group = wgid % per_group;
  const int m0 = (first_m + in_group % gsize) * BM;
  const int n0 = (in_group / gsize) * BN;

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // glds source of this lane: row (wave*4 + i)*16 + lane/4 of the operand
  // tile, logical chunk (lane & 3) ^ xor(row) (the XOR depends on lane/16 only)
  const int srow = wave * 64 + (lane >> 2);
  const int schunk = (lane & 3) ^ g4_chunk_xor(lane >> 2);
  const __bf16* ga = A + (size_t)(m0 + srow) * K + schunk * 8;
  const __bf16* gb = Bt + (size_t)(n0 + srow) * K + schunk * 8;
  const size_t piece_stride = (size_t)16 * K;
  // ds_read_b128 fragment addresses: row (w*128 + i*16 + lane%16), chunk lane/16
  const int fr = lane & 15;
  const int fch = ((lane >> 4) ^ g4_chunk_xor(fr)) * 16;
  const int a_off = (wm * 128 + fr) * 64 + fch;
  const int b_off = OP_BYTES + (wn * 128 + fr) * 64 + fch;

  const int nk = K / BKS;  // even (K % 256 == 0)
#pragma unroll
  for (int s = 0; s < NSLOT; ++s) g4_stage(ga, gb, piece_stride, min(s, nk - 1) * BKS, smem + s * SLOT_BYTES, wave);
  g4_vmwait<VM_INFLIGHT>();  // slices 0 and 1 landed (own pieces)
  wg_barrier();
  bf16x8 fa[8], fb0[8], fb1[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    fa[r] = *reinterpret_cast<const bf16x8*>(smem + a_off + r * 1024);
    fb0[r] = *reinterpret_cast<const bf16x8*>(smem + b_off + r * 1024);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  wg_barrier();  // every wave's reads of slot 0 retired: it may be refilled

  for (int s = 0; s < nk; s += 2) {
    g4_slice(acc, fa, fb0, fb1, smem + ((s + 1) % NSLOT) * SLOT_BYTES, smem + (s % NSLOT) * SLOT_BYTES, ga, gb,
             piece_stride, min(s + NSLOT, nk - 1) * BKS, a_off, b_off, wave);
    g4_vmwait<VM_INFLIGHT>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    wg_barrier();
    g4_slice(acc, fa, fb1, fb0, smem + ((s + 2) % NSLOT) * SLOT_BYTES, smem + ((s + 1) % NSLOT) * SLOT_BYTES,
             ga, gb, piece_stride, min(s + 1 + NSLOT, nk - 1) * BKS, a_off, b_off, wave);
    g4_vmwait<VM_INFLIGHT>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    wg_barrier();
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may outlive the workgroup

  // D = Bfrag x Afrag: lane holds row (lane & 15), columns 4*(lane >> 4) + 0..3
  const int crow = m0 + wm * 128 + fr;
  const int ccol = n0 + wn * 128 + (lane >> 4) * 4;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const size_t idx = (size_t)(crow + i * 16) * N + ccol + j * 16;
      if constexpr (OUT_F32) {
        *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(Cv) + idx) = acc[i][j];
      } else {
        typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
        bf16x4 v = {(__bf16)acc[i][j][0], (__bf16)acc[i][j][1], (__bf16)acc[i][j][2], (__bf16)acc[i][j][3]};
        *reinterpret_cast<bf16x4*>(reinterpret_cast<__bf16*>(Cv) + idx) = v;
      }
    }
}

// Variant 15: the same 4-wave tile and 5-slot ring, with the main loop as one
// generated asm statement (gemm4w_asm.inc, native/validator/gen_gemm4w_asm.py):
// every accumulator stays in its AGPR and every fragment in its VGPR, and the
// interleave of MFMAs, fragment reads and LDS-DMA pieces is exactly the
// generator's schedule (hipcc's register allocation of the builtin version
// above moves accumulators through VGPRs every slice).
#include "gemm4w_asm.inc"

// schedule 4's image: physical 16-B chunk p of a 128-B row r holds logical chunk p ^ g4_swz128(r % 8)
__device__ __forceinline__ int g4_swz128(int r) { return ((r & 2) << 1) | ((r & 4) >> 1); }

template <int T>
__device__ __forceinline__ f32x4 g4_acc() {
  float x0, x1, x2, x3;
  asm volatile("v_accvgpr_read_b32 %0, a%c4\n\tv_accvgpr_read_b32 %1, a%c5\n\t"
               "v_accvgpr_read_b32 %2, a%c6\n\tv_accvgpr_read_b32 %3, a%c7"
               : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)
               : "i"(4 * T), "i"(4 * T + 1), "i"(4 * T + 2), "i"(4 * T + 3));
  return (f32x4){x0, x1, x2, x3};
}

template <bool OUT_F32, int T>
__device__ __forceinline__ void g4_store_tile(void* __restrict__ Cv, int N, int crow, int ccol) {
  constexpr int i = T >> 3, j = T & 7;
  const f32x4 v = g4_acc<T>();
  const size_t idx = (size_t)(crow + i * 16) * N + ccol + j * 16;
  if constexpr (OUT_F32) {
    *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(Cv) + idx) = v;
  } else {
    typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
    bf16x4 h = {(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
    *reinterpret_cast<bf16x4*>(reinterpret_cast<__bf16*>(Cv) + idx) = h;
  }
}

template <bool OUT_F32, int... T>
__device__ __forceinline__ void g4_store_all(void* __restrict__ Cv, int N, int crow, int ccol,
                                             std::integer_sequence<int, T...>) {
  (g4_store_tile<OUT_F32, T>(Cv, N, crow, ccol), ...);
}

// bf16 epilogue in 16-B stores: tiles (i, 2p) = X and (i, 2p + 1) = Y packed
// to bf16 pairs, then v_permlane16_swap trades X's odd 16-lane rows for Y's
// even ones, so lane-row q holds 8 consecutive columns of one output row:
// q 0 / 2 -> X columns 0-7 / 8-15, q 1 / 3 -> Y columns 0-7 / 8-15; a store
// instruction covers 16 rows x 64 B (the 8-B form: 16 rows x 32 B, twice the
// instructions).
template <int P, bool NT = false>
__device__ __forceinline__ void g4_store_pair_bf16(__bf16* __restrict__ C, int N, int crow, int ccol16, int q) {
  constexpr int i = P >> 2, jx = 2 * (P & 3);
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  const f32x4 x = g4_acc<8 * i + jx>(), y = g4_acc<8 * i + jx + 1>();
  const unsigned x0 = __builtin_bit_cast(unsigned, (bf16x2){(__bf16)x[0], (__bf16)x[1]});
  const unsigned x1 = __builtin_bit_cast(unsigned, (bf16x2){(__bf16)x[2], (__bf16)x[3]});
  const unsigned y0 = __builtin_bit_cast(unsigned, (bf16x2){(__bf16)y[0], (__bf16)y[1]});
  const unsigned y1 = __builtin_bit_cast(unsigned, (bf16x2){(__bf16)y[2], (__bf16)y[3]});
  const auto s0 = __builtin_amdgcn_permlane16_swap(x0, y0, false, false);
  const auto s1 = __builtin_amdgcn_permlane16_swap(x1, y1, false, false);
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 v = {s0[0], s1[0], s0[1], s1[1]};
  const size_t idx = (size_t)(crow + i * 16) * N + ccol16 + 16 * (jx + (q & 1)) + 8 * (q >> 1);
  if constexpr (NT) __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(C + idx));
  else *reinterpret_cast<u32x4*>(C + idx) = v;
}

template <bool NT, int... P>
__device__ __forceinline__ void g4_store_pairs_bf16(__bf16* __restrict__ C, int N, int crow, int ccol16, int q,
                                                    std::integer_sequence<int, P...>) {
  (g4_store_pair_bf16<P, NT>(C, N, crow, ccol16, q), ...);
}

template <bool OUT_F32, int LOOP = 0, int EPI = 0>
__global__ __launch_bounds__(g4::NTHR, 1) void gemm_bf16_nt_4wa_kernel(const __bf16* __restrict__ A,
                                                                      const __bf16* __restrict__ Bt,
                                                                      void* __restrict__ Cv, int M, int N, int K) {
  using namespace g4;
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;

  const int tiles_m = M / BM, tiles_n = N / BN;
  const int nwg = tiles_m * tiles_n;
  const int bid = blockIdx.x;
  const int xcd = bid % kNumXcd;
  const int q = nwg / kNumXcd, rr = nwg % kNumXcd;
  const int wgid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + bid / kNumXcd;
  const int per_group = GROUP_M * tiles_n;
  const int first_m = (wgid / per_group) * GROUP_M;
  const int gsize = min(tiles_m - first_m, GROUP_M);
  const int in_group = wgid % per_group;
  const int m0 = (first_m + in_group % gsize) * BM;
  const int n0 = (in_group / gsize) * BN;

  // this wave's first piece: operand rows wave*64 .. +15 (the 4 pieces of a
  // slice are 16 rows apart); each lane moves 16 B of it: row lane/4, logical
  // chunk (lane & 3) ^ xor(row) (the XOR depends on lane/16 only)
  const uint64_t a0 = reinterpret_cast<uint64_t>(A + (size_t)(m0 + wave * 64) * K);
  const uint64_t b0 = reinterpret_cast<uint64_t>(Bt + (size_t)(n0 + wave * 64) * K);
  const unsigned g_off = (unsigned)(((lane >> 2) * K + ((lane & 3) ^ g4_chunk_xor(lane >> 2)) * 8) * 2);
  const unsigned lds = (unsigned)(uintptr_t)smem;
  const int fr = lane & 15;
  const int fch = ((lane >> 4) ^ g4_chunk_xor(fr)) * 16;
  const unsigned a_off = lds + (wm * 128 + fr) * 64 + fch;
  const unsigned b_off = lds + OP_BYTES + (wn * 128 + fr) * 64 + fch;
  const int nk = K / BKS;  // >= 8 and even (K % 256 == 0)
#define AVK_G4_ARGS                                                                                          \
  __builtin_amdgcn_readfirstlane((unsigned)a0), __builtin_amdgcn_readfirstlane((unsigned)(a0 >> 32)),       \
      __builtin_amdgcn_readfirstlane((unsigned)b0), __builtin_amdgcn_readfirstlane((unsigned)(b0 >> 32)),   \
      (unsigned)(16 * K * 2), __builtin_amdgcn_readfirstlane(lds + wave * 4 * 1024), nk - 6,                 \
      (unsigned)((nk - 2) / 2), a_off, b_off, g_off
  if constexpr (LOOP == 0) avk_g4_mainloop(AVK_G4_ARGS);
  else if constexpr (LOOP == 1) avk_g4_mainloop_noglds(AVK_G4_ARGS);
  else if constexpr (LOOP == 2) avk_g4_mainloop_nobar(AVK_G4_ARGS);
  else if constexpr (LOOP == 3) avk_g4_mainloop_early(AVK_G4_ARGS);
  else if constexpr (LOOP == 4) avk_g4_mainloop_nods(AVK_G4_ARGS);
  else if constexpr (LOOP == 5) avk_g4_mainloop_fixm0(AVK_G4_ARGS);
  else if constexpr (LOOP == 6) avk_g4_mainloop_vgpr(AVK_G4_ARGS);
  else if constexpr (LOOP == 7) avk_g4_mainloop_pairs(AVK_G4_ARGS);
  else if constexpr (LOOP == 8) avk_g4_mainloop_burst(AVK_G4_ARGS);
  else if constexpr (LOOP == 9)
    avk_g4_mainloop2(__builtin_amdgcn_readfirstlane((unsigned)a0), __builtin_amdgcn_readfirstlane((unsigned)(a0 >> 32)),
                     __builtin_amdgcn_readfirstlane((unsigned)b0), __builtin_amdgcn_readfirstlane((unsigned)(b0 >> 32)),
                     (unsigned)(16 * K * 2), __builtin_amdgcn_readfirstlane(lds + wave * 4 * 1024), (unsigned)nk, a_off,
                     b_off, g_off);
  else if constexpr (LOOP >= 11 && LOOP <= 13) {
    // schedule 4: 8-row x 128-B pieces, rows of the [rows][128 B] image swizzled by g4_swz128
    const int pr = lane >> 3;
    const unsigned g4off = (unsigned)((pr * K + ((lane & 7) ^ g4_swz128(pr)) * 8) * 2);
    const unsigned fch0 = (unsigned)((((lane >> 4) ^ g4_swz128(fr & 7))) * 16);
    const unsigned fch1 = fch0 ^ 64u;  // k-half 1: logical chunk + 4
    const unsigned la = lds + (wm * 128 + fr) * 128, lb = lds + (wn * 128 + fr) * 128;
#define AVK_G4_ARGS4                                                                                         \
  __builtin_amdgcn_readfirstlane((unsigned)a0), __builtin_amdgcn_readfirstlane((unsigned)(a0 >> 32)),       \
      __builtin_amdgcn_readfirstlane((unsigned)b0), __builtin_amdgcn_readfirstlane((unsigned)(b0 >> 32)),   \
      (unsigned)(8 * K * 2), __builtin_amdgcn_readfirstlane(lds + wave * 8 * 1024), (unsigned)(K / 64),      \
      la + fch0, la + fch1, lb + fch0, lb + fch1, g4off
    if constexpr (LOOP == 11) avk_g4_mainloop4(AVK_G4_ARGS4);
    else if constexpr (LOOP == 12) avk_g4_mainloop4b(AVK_G4_ARGS4);
    else avk_g4_mainloop4c(AVK_G4_ARGS4);
#undef AVK_G4_ARGS4
  } else
    avk_g4_mainloop3(__builtin_amdgcn_readfirstlane((unsigned)a0), __builtin_amdgcn_readfirstlane((unsigned)(a0 >> 32)),
                     __builtin_amdgcn_readfirstlane((unsigned)b0), __builtin_amdgcn_readfirstlane((unsigned)(b0 >> 32)),
                     (unsigned)(16 * K * 2), __builtin_amdgcn_readfirstlane(lds + wave * 4 * 1024), (unsigned)nk, a_off,
                     b_off, g_off);
#undef AVK_G4_ARGS

  // D = Bfrag x Afrag: lane holds row (lane & 15), columns 4*(lane >> 4) + 0..3
  if constexpr (!OUT_F32 && EPI >= 1)
    g4_store_pairs_bf16<EPI == 2>(reinterpret_cast<__bf16*>(Cv), N, m0 + wm * 128 + fr, n0 + wn * 128, lane >> 4,
                                  std::make_integer_sequence<int, 32>{});
  else
    g4_store_all<OUT_F32>(Cv, N, m0 + wm * 128 + fr, n0 + wn * 128 + (lane >> 4) * 4,
                          std::make_integer_sequence<int, 64>{});
}

// ------------------------------------------------ K2b fp8 (e4m3) GEMM ----
// The MI355X's fp8 rate (2x bf16 per clock on the f8f6f4 MFMA, ~5 PF dense):
// C = A . Bt^T with A [M][K], Bt [N][K] OCP e4m3 (row-major bytes), f32
// accumulation, bf16 or f32 out.  The 4-wave 256x256 tile and schedule 4b's
// data movement with schedule 8's main loop (gen_gemm4w_asm.py): 64
// v_mfma_f32_16x16x128_f8f6f4 per 128-deep stage per wave, every fragment in
// one register set, the image swizzled by g8_swz.  Same epilogues as the bf16
// kernel (the 16x16 C/D layout does not depend on the data type).
__device__ __forceinline__ int g8_swz(int r) { return ((r >> 1) & 1) | (((r >> 2) & 1) << 2); }

template <bool OUT_F32, int EPI = 1>
__global__ __launch_bounds__(g4::NTHR, 1) void gemm_fp8_nt_kernel(const uint8_t* __restrict__ A,
                                                                 const uint8_t* __restrict__ Bt,
                                                                 void* __restrict__ Cv, int M, int N, int K) {
  using namespace g4;
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;

  const int tiles_m = M / BM, tiles_n = N / BN;
  const int nwg = tiles_m * tiles_n;
  const int bid = blockIdx.x;
  const int xcd = bid % kNumXcd;
  const int q = nwg / kNumXcd, rr = nwg % kNumXcd;
  const int wgid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + bid / kNumXcd;
  const int per_group = GROUP_M * tiles_n;
  const int first_m = (wgid / per_group) * GROUP_M;
  const int gsize = min(tiles_m - first_m, GROUP_M);
  const int in_group = wgid % per_group;
  const int m0 = (first_m + in_group % gsize) * BM;
  const int n0 = (in_group / gsize) * BN;

  // this wave's pieces: 8 rows x 128 B (128 k) each, rows wave*64 + 8j; lane
  // l moves 16 B: row l >> 3, logical chunk (l & 7) ^ g8_swz(row)
  const uint64_t a0 = reinterpret_cast<uint64_t>(A + (size_t)(m0 + wave * 64) * K);
  const uint64_t b0 = reinterpret_cast<uint64_t>(Bt + (size_t)(n0 + wave * 64) * K);
  const int pr = lane >> 3;
  const unsigned g_off = (unsigned)(pr * K + ((lane & 7) ^ g8_swz(pr)) * 16);
  const unsigned lds = (unsigned)(uintptr_t)smem;
  // fragment i: rows 16i + (lane & 15) of the wave's 128, logical chunks
  // 2 (lane >> 4) and 2 (lane >> 4) + 1 of the 128-B row (32 fp8 of k)
  const int fr = lane & 15;
  const unsigned c0 = (unsigned)(((2 * (lane >> 4)) ^ g8_swz(fr & 7)) * 16);
  const unsigned c1 = (unsigned)(((2 * (lane >> 4) + 1) ^ g8_swz(fr & 7)) * 16);
  const unsigned la = lds + (wm * 128 + fr) * 128, lb = lds + (wn * 128 + fr) * 128;
  avk_g8_mainloop(__builtin_amdgcn_readfirstlane((unsigned)a0), __builtin_amdgcn_readfirstlane((unsigned)(a0 >> 32)),
                  __builtin_amdgcn_readfirstlane((unsigned)b0), __builtin_amdgcn_readfirstlane((unsigned)(b0 >> 32)),
                  (unsigned)(8 * K), __builtin_amdgcn_readfirstlane(lds + wave * 8 * 1024), (unsigned)(K / 128),
                  la + c0, la + c1, lb + c0, lb + c1, g_off);

  if constexpr (!OUT_F32 && EPI >= 1)
    g4_store_pairs_bf16<EPI == 2>(reinterpret_cast<__bf16*>(Cv), N, m0 + wm * 128 + fr, n0 + wn * 128, lane >> 4,
                                  std::make_integer_sequence<int, 32>{});
  else
    g4_store_all<OUT_F32>(Cv, N, m0 + wm * 128 + fr, n0 + wn * 128 + (lane >> 4) * 4,
                          std::make_integer_sequence<int, 64>{});
}

// K2c: C[M][N] = A[M][K] * Bt[N][K]^T with OCP FP4 (e2m1, two per byte, element
// 2k in the low nibble) operands, fp32 accumulation: the 4-wave tile of the
// fp8 kernel with schedule 9's main loop (gen_gemm4w_asm.py: the same 128-B
// LDS rows, here 256 k = two v_mfma_f32_16x16x128_f8f6f4 cbsz:4 blgp:4 steps
// per row; lane group g reads chunk g for k-step 0 and g + 4 for k-step 1,
// under the bf16 kernel's swizzle).  K % 256 == 0, K >= 512.
__device__ __forceinline__ int g9_swz(int r) { return ((r & 2) << 1) | ((r & 4) >> 1); }

template <bool OUT_F32, int EPI = 1>
__global__ __launch_bounds__(g4::NTHR, 1) void gemm_fp4_nt_kernel(const uint8_t* __restrict__ A,
                                                                 const uint8_t* __restrict__ Bt,
                                                                 void* __restrict__ Cv, int M, int N, int K) {
  using namespace g4;
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;

  const int tiles_m = M / BM, tiles_n = N / BN;
  const int nwg = tiles_m * tiles_n;
  const int bid = blockIdx.x;
  const int xcd = bid % kNumXcd;
  const int q = nwg / kNumXcd, rr = nwg % kNumXcd;
  const int wgid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + bid / kNumXcd;
  const int per_group = GROUP_M * tiles_n;
  const int first_m = (wgid / per_group) * GROUP_M;
  const int gsize = min(tiles_m - first_m, GROUP_M);
  const int in_group = wgid % per_group;
  const int m0 = (first_m + in_group % gsize) * BM;
  const int n0 = (in_group / gsize) * BN;

  const int kb = K / 2;  // bytes per row
  const uint64_t a0 = reinterpret_cast<uint64_t>(A + (size_t)(m0 + wave * 64) * kb);
  const uint64_t b0 = reinterpret_cast<uint64_t>(Bt + (size_t)(n0 + wave * 64) * kb);
  const int pr = lane >> 3;
  const unsigned g_off = (unsigned)(pr * kb + ((lane & 7) ^ g9_swz(pr)) * 16);
  const unsigned lds = (unsigned)(uintptr_t)smem;
  const int fr = lane & 15;
  const unsigned c0 = (unsigned)(((lane >> 4) ^ g9_swz(fr & 7)) * 16);
  const unsigned c1 = (unsigned)((((lane >> 4) + 4) ^ g9_swz(fr & 7)) * 16);
  const unsigned la = lds + (wm * 128 + fr) * 128, lb = lds + (wn * 128 + fr) * 128;
  avk_g9_mainloop(__builtin_amdgcn_readfirstlane((unsigned)a0), __builtin_amdgcn_readfirstlane((unsigned)(a0 >> 32)),
                  __builtin_amdgcn_readfirstlane((unsigned)b0), __builtin_amdgcn_readfirstlane((unsigned)(b0 >> 32)),
                  (unsigned)(8 * kb), __builtin_amdgcn_readfirstlane(lds + wave * 8 * 1024), (unsigned)(K / 256),
                  la + c0, la + c1, lb + c0, lb + c1, g_off);

  if constexpr (!OUT_F32 && EPI >= 1)
    g4_store_pairs_bf16<EPI == 2>(reinterpret_cast<__bf16*>(Cv), N, m0 + wm * 128 + fr, n0 + wn * 128, lane >> 4,
                                  std::make_integer_sequence<int, 32>{});
  else
    g4_store_all<OUT_F32>(Cv, N, m0 + wm * 128 + fr, n0 + wn * 128 + (lane >> 4) * 4,
                          std::make_integer_sequence<int, 64>{});
}

// K2d: C = A . Bt^T with OCP FP6 (e2m3) operands in the validator's fp6
// storage: each 32-element k-block of a row is a 32-B slot holding the 32
// 6-bit codes packed little-endian (element j at bits 6j .. 6j + 5 of the
// slot, the f8f6f4 MFMA's operand order) in its first 24 B and 8 B of zeros,
// so a row of K fp6 is K bytes - the fp8 kernel's data movement unchanged,
// with schedule 10's main loop (v_mfma_f32_16x16x128_f8f6f4 cbsz:2 blgp:2,
// which reads the first six VGPRs of each fragment: the fp4 rate per clock).
template <bool OUT_F32, int EPI = 1>
__global__ __launch_bounds__(g4::NTHR, 1) void gemm_fp6_nt_kernel(const uint8_t* __restrict__ A,
                                                                 const uint8_t* __restrict__ Bt,
                                                                 void* __restrict__ Cv, int M, int N, int K) {
  using namespace g4;
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;

  const int tiles_m = M / BM, tiles_n = N / BN;
  const int nwg = tiles_m * tiles_n;
  const int bid = blockIdx.x;
  const int xcd = bid % kNumXcd;
  const int q = nwg / kNumXcd, rr = nwg % kNumXcd;
  const int wgid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + bid / kNumXcd;
  const int per_group = GROUP_M * tiles_n;
  const int first_m = (wgid / per_group) * GROUP_M;
  const int gsize = min(tiles_m - first_m, GROUP_M);
  const int in_group = wgid % per_group;
  const int m0 = (first_m + in_group % gsize) * BM;
  const int n0 = (in_group / gsize) * BN;

  const uint64_t a0 = reinterpret_cast<uint64_t>(A + (size_t)(m0 + wave * 64) * K);
  const uint64_t b0 = reinterpret_cast<uint64_t>(Bt + (size_t)(n0 + wave * 64) * K);
  const int pr = lane >> 3;
  const unsigned g_off = (unsigned)(pr * K + ((lane & 7) ^ g8_swz(pr)) * 16);
  const unsigned lds = (unsigned)(uintptr_t)smem;
  const int fr = lane & 15;
  const unsigned c0 = (unsigned)(((2 * (lane >> 4)) ^ g8_swz(fr & 7)) * 16);
  const unsigned c1 = (unsigned)(((2 * (lane >> 4) + 1) ^ g8_swz(fr & 7)) * 16);
  const unsigned la = lds + (wm * 128 + fr) * 128, lb = lds + (wn * 128 + fr) * 128;
  avk_g10_mainloop(__builtin_amdgcn_readfirstlane((unsigned)a0), __builtin_amdgcn_readfirstlane((unsigned)(a0 >> 32)),
                   __builtin_amdgcn_readfirstlane((unsigned)b0), __builtin_amdgcn_readfirstlane((unsigned)(b0 >> 32)),
                   (unsigned)(8 * K), __builtin_amdgcn_readfirstlane(lds + wave * 8 * 1024), (unsigned)(K / 128),
                   la + c0, la + c1, lb + c0, lb + c1, g_off);

  if constexpr (!OUT_F32 && EPI >= 1)
    g4_store_pairs_bf16<EPI == 2>(reinterpret_cast<__bf16*>(Cv), N, m0 + wm * 128 + fr, n0 + wn * 128, lane >> 4,
                                  std::make_integer_sequence<int, 32>{});
  else
    g4_store_all<OUT_F32>(Cv, N, m0 + wm * 128 + fr, n0 + wn * 128 + (lane >> 4) * 4,
                          std::make_integer_sequence<int, 64>{});
}

// K2e: block-scaled MXFP4.  C = (2^(SA - 127) . A) (2^(SB - 127) . Bt)^T with A,
// Bt OCP FP4 pairs as gemm_fp4_nt_kernel's and one E8M0 scale per row and
// 32-element k-block, periodic in k with 8 blocks (SA[M][8], SB[N][8]: block
// b of row r has scale S[r][b % 8] - every block of a 256-deep stage its own
// scale, the same in every stage).  Schedule 11's main loop
// (v_mfma_scale_f32_16x16x128_f8f6f4): a lane's scales are one byte per
// fragment and k-step, loaded here before the loop into four VGPRs per
// operand (fragment i, k-step t at byte 2i + t; k-step t of lane group g
// reads k-block g + 4t of the stage, gemm_fp4_nt_kernel).
template <bool OUT_F32, int EPI = 1>
__global__ __launch_bounds__(g4::NTHR, 1) void gemm_mxfp4_nt_kernel(const uint8_t* __restrict__ A,
                                                                   const uint8_t* __restrict__ Bt,
                                                                   void* __restrict__ Cv, int M, int N, int K,
                                                                   const uint8_t* __restrict__ SA,
                                                                   const uint8_t* __restrict__ SB) {
  using namespace g4;
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;

  const int tiles_m = M / BM, tiles_n = N / BN;
  const int nwg = tiles_m * tiles_n;
  const int bid = blockIdx.x;
  const int xcd = bid % kNumXcd;
  const int q = nwg / kNumXcd, rr = nwg % kNumXcd;
  const int wgid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + bid / kNumXcd;
  const int per_group = GROUP_M * tiles_n;
  const int first_m = (wgid / per_group) * GROUP_M;
  const int gsize = min(tiles_m - first_m, GROUP_M);
  const int in_group = wgid % per_group;
  const int m0 = (first_m + in_group % gsize) * BM;
  const int n0 = (in_group / gsize) * BN;

  const int fr = lane & 15, g = lane >> 4;
  unsigned sa[4] = {0, 0, 0, 0}, sb[4] = {0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int byte = 2 * i + t;
      sa[byte >> 2] |= (unsigned)SA[(size_t)(m0 + wm * 128 + 16 * i + fr) * 8 + g + 4 * t] << (8 * (byte & 3));
      sb[byte >> 2] |= (unsigned)SB[(size_t)(n0 + wn * 128 + 16 * i + fr) * 8 + g + 4 * t] << (8 * (byte & 3));
    }

  const int kb = K / 2;
  const uint64_t a0 = reinterpret_cast<uint64_t>(A + (size_t)(m0 + wave * 64) * kb);
  const uint64_t b0 = reinterpret_cast<uint64_t>(Bt + (size_t)(n0 + wave * 64) * kb);
  const int pr = lane >> 3;
  const unsigned g_off = (unsigned)(pr * kb + ((lane & 7) ^ g9_swz(pr)) * 16);
  const unsigned lds = (unsigned)(uintptr_t)smem;
  const unsigned c0 = (unsigned)((g ^ g9_swz(fr & 7)) * 16);
  const unsigned c1 = (unsigned)(((g + 4) ^ g9_swz(fr & 7)) * 16);
  const unsigned la = lds + (wm * 128 + fr) * 128, lb = lds + (wn * 128 + fr) * 128;
  avk_g11_mainloop(__builtin_amdgcn_readfirstlane((unsigned)a0), __builtin_amdgcn_readfirstlane((unsigned)(a0 >> 32)),
                   __builtin_amdgcn_readfirstlane((unsigned)b0), __builtin_amdgcn_readfirstlane((unsigned)(b0 >> 32)),
                   (unsigned)(8 * kb), __builtin_amdgcn_readfirstlane(lds + wave * 8 * 1024), (unsigned)(K / 256),
                   la + c0, la + c1, lb + c0, lb + c1, g_off, sa[0], sa[1], sa[2], sa[3], sb[0], sb[1], sb[2], sb[3]);

  if constexpr (!OUT_F32 && EPI >= 1)
    g4_store_pairs_bf16<EPI == 2>(reinterpret_cast<__bf16*>(Cv), N, m0 + wm * 128 + fr, n0 + wn * 128, lane >> 4,
                                  std::make_integer_sequence<int, 32>{});
  else
    g4_store_all<OUT_F32>(Cv, N, m0 + wm * 128 + fr, n0 + wn * 128 + (lane >> 4) * 4,
                          std::make_integer_sequence<int, 64>{});
}

// four OCP e4m3 bytes (1 sign, 4 exponent bits with bias 7, 3 mantissa bits;
// gfx950's fp8, not MI300's fnuz) -> floats on the conversion unit
// (v_cvt_pk_f32_fp8): a tenth of the VALU work of a bit decode, which had
// made the column GEMV decode-bound (profiles/r5_kernels)
__device__ __forceinline__ void e4m3x4_to_f32(uint32_t x, float* out) {
  const auto lo = __builtin_amdgcn_cvt_pk_f32_fp8((int)x, false);
  const auto hi = __builtin_amdgcn_cvt_pk_f32_fp8((int)x, true);
  out[0] = lo[0];
  out[1] = lo[1];
  out[2] = hi[0];
  out[3] = hi[1];
}

// random finite e4m3 bytes: sign, exponent field 0..8, any mantissa (|x| <= 3.75)
__global__ __launch_bounds__(256) void fill_fp8_kernel(uint8_t* __restrict__ p, int64_t n, uint64_t seed) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    uint64_t h = (uint64_t)i * 0x9E3779B97F4A7C15ull ^ seed * 0xD1B54A32D192ED03ull;
    h ^= h >> 31;
    h *= 0xBF58476D1CE4E5B9ull;
    h ^= h >> 29;
    const unsigned mag = (unsigned)((h >> 8) % 72u);  // exponent 0..8 x mantissa 0..7
    p[i] = (uint8_t)(((h & 1u) << 7) | ((mag >> 3) << 3) | (mag & 7u));
  }
}

// random FP4 bytes: every e2m1 code is finite (+-{0, 0.5, 1, 1.5, 2, 3, 4, 6})
__global__ __launch_bounds__(256) void fill_fp4_kernel(uint8_t* __restrict__ p, int64_t n, uint64_t seed) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    uint64_t h = (uint64_t)i * 0x9E3779B97F4A7C15ull ^ seed * 0xD1B54A32D192ED03ull;
    h ^= h >> 31;
    h *= 0xBF58476D1CE4E5B9ull;
    h ^= h >> 29;
    p[i] = (uint8_t)(h >> 24);
  }
}

// eight OCP FP4 e2m1 codes (1 sign, 2 exponent bits with bias 1, 1 mantissa
// bit; four bytes, element 2k in the low nibble) -> floats on gfx950's
// conversion unit (v_cvt_scalef32_pk_f32_fp4, scale 1)
__device__ __forceinline__ void e2m1x8_to_f32(uint32_t x, float* out) {
  const auto p0 = __builtin_amdgcn_cvt_scalef32_pk_f32_fp4(x, 1.0f, 0);
  const auto p1 = __builtin_amdgcn_cvt_scalef32_pk_f32_fp4(x, 1.0f, 1);
  const auto p2 = __builtin_amdgcn_cvt_scalef32_pk_f32_fp4(x, 1.0f, 2);
  const auto p3 = __builtin_amdgcn_cvt_scalef32_pk_f32_fp4(x, 1.0f, 3);
  out[0] = p0[0];
  out[1] = p0[1];
  out[2] = p1[0];
  out[3] = p1[1];
  out[4] = p2[0];
  out[5] = p2[1];
  out[6] = p3[0];
  out[7] = p3[1];
}

// OCP FP6 e2m3 (1 sign, 2 exponent bits with bias 1, 3 mantissa bits; every
// code finite, |x| <= 7.5) -> float
__device__ __forceinline__ float e2m3_to_f32(unsigned c) {
  const unsigned e = (c >> 3) & 3u, m = c & 7u;
  const float mag = e == 0 ? (float)m * 0.125f : (float)(8u + m) * 0.125f * (float)(1u << (e - 1));
  return (c & 0x20u) ? -mag : mag;
}

// one 32-B fp6 slot (32 codes in its first 24 B) -> 32 floats
__device__ __forceinline__ void fp6_slot_to_f32(const uint8_t* slot, float* out) {
  const uint4 lo = *reinterpret_cast<const uint4*>(slot);
  const uint2 hi = *reinterpret_cast<const uint2*>(slot + 16);
  const uint32_t w[6] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y};
#pragma unroll
  for (int j = 0; j < 32; ++j) {
    const int bit = 6 * j, wi = bit >> 5, sh = bit & 31;
    unsigned c = w[wi] >> sh;
    if (sh > 26) c |= w[wi + 1] << (32 - sh);
    out[j] = e2m3_to_f32(c & 0x3Fu);
  }
}

// random fp6 storage: per 32-B slot 32 random e2m3 codes, packed, 8 B of zeros
__global__ __launch_bounds__(256) void fill_fp6_kernel(uint8_t* __restrict__ p, int64_t slots, uint64_t seed) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < slots; i += (int64_t)gridDim.x * 256) {
    uint32_t w[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t h = (uint64_t)i * 0x9E3779B97F4A7C15ull ^ seed * 0xD1B54A32D192ED03ull;
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      if ((j & 7) == 0) {
        h ^= h >> 31;
        h *= 0xBF58476D1CE4E5B9ull;
        h ^= h >> 29;
      }
      const unsigned c = (unsigned)(h >> (6 * (j & 7) + 8)) & 0x3Fu;
      const int bit = 6 * j, wi = bit >> 5, sh = bit & 31;
      w[wi] |= c << sh;
      if (sh > 26) w[wi + 1] |= c >> (32 - sh);
    }
    uint4* d = reinterpret_cast<uint4*>(p + i * 32);
    d[0] = make_uint4(w[0], w[1], w[2], w[3]);
    d[1] = make_uint4(w[4], w[5], 0u, 0u);
  }
}

// random E8M0 scales in [lo, hi] (2^(lo - 127) .. 2^(hi - 127))
__global__ __launch_bounds__(256) void fill_e8m0_kernel(uint8_t* __restrict__ p, int64_t n, uint64_t seed, int lo,
                                                        int span) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    uint64_t h = (uint64_t)i * 0x9E3779B97F4A7C15ull ^ seed * 0xD1B54A32D192ED03ull;
    h ^= h >> 31;
    h *= 0xBF58476D1CE4E5B9ull;
    h ^= h >> 29;
    p[i] = (uint8_t)(lo + (int)((h >> 16) % (uint64_t)span));
  }
}

__device__ __forceinline__ float e8m0_to_f32(uint8_t s) { return __uint_as_float((unsigned)s << 23); }

// y[r] = sum_c X[r][c] v[c], X fp6 storage [R][C] bytes (a wave per row, a slot per lane step)
__global__ __launch_bounds__(256) void gemv_rows_fp6_kernel(const uint8_t* __restrict__ X, const float* __restrict__ v,
                                                            float* __restrict__ y, int R, int C) {
  const int wave = (blockIdx.x * 256 + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (wave >= R) return;
  const uint8_t* row = X + (size_t)wave * C;
  float s = 0.f;
  for (int c = lane * 32; c < C; c += 64 * 32) {
    float f[32];
    fp6_slot_to_f32(row + c, f);
#pragma unroll
    for (int j = 0; j < 32; ++j) s += f[j] * v[c + j];
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if (lane == 0) y[wave] = s;
}

// y[r] = sum_c 2^(S[r][(c / 32) % 8] - 127) X[r][c] v[c], X FP4 pairs [R][C/2]
__global__ __launch_bounds__(256) void gemv_rows_mxfp4_kernel(const uint8_t* __restrict__ X,
                                                              const uint8_t* __restrict__ S,
                                                              const float* __restrict__ v, float* __restrict__ y,
                                                              int R, int C) {
  const int wave = (blockIdx.x * 256 + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (wave >= R) return;
  const uint8_t* row = X + (size_t)wave * (C / 2);
  float s = 0.f;
  for (int c = lane * 16; c < C; c += 64 * 16) {
    const uint64_t x = *reinterpret_cast<const uint64_t*>(row + c / 2);
    float f[16];
    e2m1x8_to_f32((uint32_t)x, f);
    e2m1x8_to_f32((uint32_t)(x >> 32), f + 8);
    float p = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) p += f[j] * v[c + j];
    s += p * e8m0_to_f32(S[(size_t)wave * 8 + ((c >> 5) & 7)]);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if (lane == 0) y[wave] = s;
}

// y[r] = sum_c X[r][c] * v[c], X FP4 pairs [R][C/2] (one wave per row, 16 values per lane step)
__global__ __launch_bounds__(256) void gemv_rows_fp4_kernel(const uint8_t* __restrict__ X, const float* __restrict__ v,
                                                            float* __restrict__ y, int R, int C) {
  const int wave = (blockIdx.x * 256 + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (wave >= R) return;
  const uint8_t* row = X + (size_t)wave * (C / 2);
  float s = 0.f;
  for (int c = lane * 16; c < C; c += 64 * 16) {
    const uint64_t x = *reinterpret_cast<const uint64_t*>(row + c / 2);
    float f[16];
    e2m1x8_to_f32((uint32_t)x, f);
    e2m1x8_to_f32((uint32_t)(x >> 32), f + 8);
#pragma unroll
    for (int j = 0; j < 16; ++j) s += f[j] * v[c + j];
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if (lane == 0) y[wave] = s;
}

// Column GEMVs of the Freivalds checks: z[c] += sum_{r in slice} X[r][c] v[r],
// X row-major.  A block covers 64 * Dec::kCols columns (one 8- or 16-byte load
// per lane per row), its 4 waves take every 4th row of the slice (4 row
// streams in flight per block), and their partial sums meet in LDS, so each
// column gets one atomic per block.  (A wave per block-row with kCols atomics
// per lane made the fp4 one 121 us at 4096^2: profiles/r5_kernels.)
struct DecFp4 {  // FP4 pairs [R][C/2]: 16 columns in 8 bytes
  static constexpr int kCols = 16;
  __device__ static void load(const void* X, const void*, int r, int C, int c0, float* out) {
    const uint64_t x = *reinterpret_cast<const uint64_t*>(static_cast<const uint8_t*>(X) + (size_t)r * (C / 2) + c0 / 2);
    e2m1x8_to_f32((uint32_t)x, out);
    e2m1x8_to_f32((uint32_t)(x >> 32), out + 8);
  }
};
struct DecFp8 {  // e4m3 [R][C]: 8 columns in 8 bytes
  static constexpr int kCols = 8;
  __device__ static void load(const void* X, const void*, int r, int C, int c0, float* out) {
    const uint64_t x = *reinterpret_cast<const uint64_t*>(static_cast<const uint8_t*>(X) + (size_t)r * C + c0);
    e4m3x4_to_f32((uint32_t)x, out);
    e4m3x4_to_f32((uint32_t)(x >> 32), out + 4);
  }
};
struct DecBf16 {  // bf16 [R][C]: 8 columns in 16 bytes
  static constexpr int kCols = 8;
  __device__ static void load(const void* X, const void*, int r, int C, int c0, float* out) {
    const bf16x8 x = *reinterpret_cast<const bf16x8*>(static_cast<const __bf16*>(X) + (size_t)r * C + c0);
#pragma unroll
    for (int j = 0; j < 8; ++j) out[j] = (float)x[j];
  }
};

struct DecFp6 {  // fp6 storage [R][C] bytes: 32 columns in one 32-B slot
  static constexpr int kCols = 32;
  __device__ static void load(const void* X, const void*, int r, int C, int c0, float* out) {
    fp6_slot_to_f32(static_cast<const uint8_t*>(X) + (size_t)r * C + c0, out);
  }
};
struct DecMxFp4 {  // FP4 pairs [R][C/2] with E8M0 scales S[R][8] (block c / 32 mod 8): 16 columns in 8 bytes
  static constexpr int kCols = 16;
  __device__ static void load(const void* X, const void* S, int r, int C, int c0, float* out) {
    DecFp4::load(X, nullptr, r, C, c0, out);
    const float sc = e8m0_to_f32(static_cast<const uint8_t*>(S)[(size_t)r * 8 + ((c0 >> 5) & 7)]);
#pragma unroll
    for (int j = 0; j < 16; ++j) out[j] *= sc;
  }
};

template <typename Dec>
__global__ __launch_bounds__(256) void gemv_cols_kernel(const void* __restrict__ X, const float* __restrict__ v,
                                                        float* __restrict__ z, int R, int C, int rows_per_slice,
                                                        const void* __restrict__ aux) {
  constexpr int W = 64 * Dec::kCols;  // columns per block
  __shared__ float red[4][W];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int cb = blockIdx.x * W;
  const int c0 = cb + lane * Dec::kCols;
  const int r0 = blockIdx.y * rows_per_slice;
  const int r1 = min(R, r0 + rows_per_slice);
  float s[Dec::kCols] = {};
  if (c0 < C) {
    for (int r = r0 + w; r < r1; r += 4) {
      float x[Dec::kCols];
      Dec::load(X, aux, r, C, c0, x);
      const float vr = v[r];
#pragma unroll
      for (int j = 0; j < Dec::kCols; ++j) s[j] += x[j] * vr;
    }
  }
#pragma unroll
  for (int j = 0; j < Dec::kCols; ++j) red[w][lane * Dec::kCols + j] = s[j];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < W / 256; ++k) {
    const int col = k * 256 + threadIdx.x;
    if (cb + col < C) atomicAdd(z + cb + col, red[0][col] + red[1][col] + red[2][col] + red[3][col]);
  }
}

template <typename Dec>
int launch_gemv_cols(const void* X, const float* v, float* z, int R, int C, hipStream_t s,
                     const void* aux = nullptr) {
  constexpr int W = 64 * Dec::kCols;
  const int bx = (C + W - 1) / W;
  int slices = 512 / bx;  // ~2048 waves in all at 4096^2 (4 per block), each over a stream of rows
  if (slices < 1) slices = 1;
  if (slices > R) slices = R;
  const int rows_per_slice = (R + slices - 1) / slices;
  dim3 grid(bx, (R + rows_per_slice - 1) / rows_per_slice);
  gemv_cols_kernel<Dec><<<grid, 256, 0, s>>>(X, v, z, R, C, rows_per_slice, aux);
  return hipGetLastError();
}

// y[r] = sum_c X[r][c] v[c], X e4m3 [R][C] (one wave per row, 8 bytes per lane step)
__global__ __launch_bounds__(256) void gemv_rows_fp8_kernel(const uint8_t* __restrict__ X, const float* __restrict__ v,
                                                            float* __restrict__ y, int R, int C) {
  const int wave = (blockIdx.x * 256 + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (wave >= R) return;
  const uint8_t* row = X + (size_t)wave * C;
  float s = 0.f;
  for (int c = lane * 8; c < C; c += 64 * 8) {
    const uint64_t x = *reinterpret_cast<const uint64_t*>(row + c);
    float f[8];
    e4m3x4_to_f32((uint32_t)x, f);
    e4m3x4_to_f32((uint32_t)(x >> 32), f + 4);
#pragma unroll
    for (int j = 0; j < 8; ++j) s += f[j] * v[c + j];
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if (lane == 0) y[wave] = s;
}

// ------------------------------------------------- Freivalds check GEMVs ----
// y[r] = sum_c X[r][c] * v[c]   (X bf16 or f32, row-major, one wave per row)
template <typename T>
__global__ __launch_bounds__(256) void gemv_rows_kernel(const T* __restrict__ X, const float* __restrict__ v,
                                                        float* __restrict__ y, int R, int C) {
  const int wave = (blockIdx.x * 256 + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (wave >= R) return;
  const T* row = X + (size_t)wave * C;
  float s = 0.f;
  for (int c = lane * 8; c < C; c += 64 * 8) {
#pragma unroll
    for (int j = 0; j < 8; ++j) s += (float)row[c + j] * v[c + j];
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if (lane == 0) y[wave] = s;
}

// ------------------------------------------------------------ K3 HBM copy ----
template <int U, bool NT>
__global__ __launch_bounds__(256) void hbm_copy_kernel(const f32x4* __restrict__ s, f32x4* __restrict__ d,
                                                       int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * 256 * U;
  int64_t i = (int64_t)blockIdx.x * 256 * U + threadIdx.x;
  for (; i + (U - 1) * 256 < n; i += stride) {
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = NT ? __builtin_nontemporal_load(s + i + u * 256) : s[i + u * 256];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if constexpr (NT) __builtin_nontemporal_store(v[u], d + i + u * 256);
      else d[i + u * 256] = v[u];
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (i + u * 256 < n) d[i + u * 256] = s[i + u * 256];
}

// 64-bit wrapping sum of 32-bit words (copy integrity check)
// Block-wide reductions for the two check kernels below: wave shuffles, then
// the 4 wave partials through LDS, then ONE global atomic per block.  (One
// atomic per wave on a single address serialised 16 K atomics per call:
// the 1 GiB checksum ran at 3.4 TB/s and the 16 M-element max|a-b| at
// 0.17 TB/s, profiles/r2_kernels/rocprof_validator_kernel_stats_final.csv.)
template <typename T, typename Op>
__device__ __forceinline__ T block_reduce_256(T v, Op op) {
  __shared__ T part[4];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = op(v, __shfl_xor(v, off, 64));
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = v;
  __syncthreads();
  return op(op(part[0], part[1]), op(part[2], part[3]));
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned long long checksum_term(u32x4 v, int64_t i) {
  return (unsigned long long)v.x * 1u + (unsigned long long)v.y * 3u + (unsigned long long)v.z * 5u +
         (unsigned long long)v.w * 7u + (unsigned long long)(i & 0xffff);
}

// sum over 16-byte words i of (x + 3y + 5z + 7w + (i mod 65536)) mod 2^64;
// four independent non-temporal loads in flight per thread
__global__ __launch_bounds__(256) void checksum_kernel(const u32x4* __restrict__ p, int64_t n4,
                                                       unsigned long long* __restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  unsigned long long s = 0;
  for (; i + 3 * stride < n4; i += 4 * stride) {
    const u32x4 v0 = __builtin_nontemporal_load(p + i);
    const u32x4 v1 = __builtin_nontemporal_load(p + i + stride);
    const u32x4 v2 = __builtin_nontemporal_load(p + i + 2 * stride);
    const u32x4 v3 = __builtin_nontemporal_load(p + i + 3 * stride);
    s += checksum_term(v0, i) + checksum_term(v1, i + stride) + checksum_term(v2, i + 2 * stride) +
         checksum_term(v3, i + 3 * stride);
  }
  for (; i < n4; i += stride) s += checksum_term(__builtin_nontemporal_load(p + i), i);
  s = block_reduce_256(s, [](unsigned long long x, unsigned long long y) { return x + y; });
  if (threadIdx.x == 0) atomicAdd(out, s);
}

__device__ __forceinline__ float absdiff_nan_inf(float x, float y) {
  const float d = fabsf(x - y);
  return (d != d) ? __int_as_float(0x7f800000) : d;  // NaN -> +inf so the gate fails
}

// max |a-b| over fp32 arrays; result written as float bits via atomicMax on
// uint (non-negative floats order like their bit patterns).  float4 loads
// when both arrays are 16-byte aligned, a scalar tail otherwise.
__global__ __launch_bounds__(256) void max_abs_diff_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                           int64_t n, unsigned int* __restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  float m = 0.f;
  int64_t done = 0;
  if ((((uintptr_t)a | (uintptr_t)b) & 15) == 0) {
    const int64_t n4 = n / 4;
    const f32x4* a4 = reinterpret_cast<const f32x4*>(a);
    const f32x4* b4 = reinterpret_cast<const f32x4*>(b);
    for (int64_t i = t; i < n4; i += stride) {
      const f32x4 x = __builtin_nontemporal_load(a4 + i), y = __builtin_nontemporal_load(b4 + i);
      m = fmaxf(m, fmaxf(fmaxf(absdiff_nan_inf(x.x, y.x), absdiff_nan_inf(x.y, y.y)),
                         fmaxf(absdiff_nan_inf(x.z, y.z), absdiff_nan_inf(x.w, y.w))));
    }
    done = n4 * 4;
  }
  for (int64_t i = done + t; i < n; i += stride) m = fmaxf(m, absdiff_nan_inf(a[i], b[i]));
  m = block_reduce_256(m, [](float x, float y) { return fmaxf(x, y); });
  if (threadIdx.x == 0) atomicMax(out, __float_as_uint(m));
}

// ------------------------------------------------------- K4 all-reduce ----
// Peer pointer table lives in kernel arguments (<= 8 peers).
struct PeerPtrs {
  const float* p[8];
};
struct PeerPtrsMut {
  float* p[8];
};

// one-shot: out[i] = sum_r in_r[i] for every i (each rank reads every peer).
// Every peer's float4 is loaded before the first add (NP loads in flight per
// lane; over xGMI each peer sits behind its own link), streamed nontemporal.
template <int NP>
__global__ __launch_bounds__(256) void allreduce_oneshot_f32_kernel(PeerPtrs in, float* __restrict__ out,
                                                                    int64_t n4, int np_runtime) {
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * 256;
  if constexpr (NP > 0) {
    for (; i < n4; i += stride) {
      f32x4 v[NP];
#pragma unroll
      for (int r = 0; r < NP; ++r) v[r] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(in.p[r]) + i);
#pragma unroll
      for (int r = 1; r < NP; ++r) v[0] += v[r];
      __builtin_nontemporal_store(v[0], reinterpret_cast<f32x4*>(out) + i);
    }
  } else {
    for (; i < n4; i += stride) {
      f32x4 acc = reinterpret_cast<const f32x4*>(in.p[0])[i];
      for (int r = 1; r < np_runtime; ++r) acc += reinterpret_cast<const f32x4*>(in.p[r])[i];
      reinterpret_cast<f32x4*>(out)[i] = acc;
    }
  }
}

// two-shot phase 1 (reduce-scatter): rank `rank` reduces slice [lo, hi) of the
// float4 index space from every peer and writes the sum into EVERY peer's
// output buffer (remote writes over xGMI) -> after phase 1 on all ranks plus a
// cross-device barrier, every output holds the full result.
__global__ __launch_bounds__(256) void allreduce_twoshot_f32_kernel(PeerPtrs in, PeerPtrsMut out, int np,
                                                                    int64_t lo, int64_t hi) {
  int64_t i = lo + (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (; i < hi; i += stride) {
    float4 s = reinterpret_cast<const float4*>(in.p[0])[i];
    for (int r = 1; r < np; ++r) {
      float4 v = reinterpret_cast<const float4*>(in.p[r])[i];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    for (int r = 0; r < np; ++r) reinterpret_cast<float4*>(out.p[r])[i] = s;
  }
}

// ------------------------------------------------ K5 MFMA data-type probe ----
// One wave, one 16x16 output tile per matrix-core data type the node's GFD
// labels advertise for CDNA4 (amd.com/gpu.mfma.*): f16, bf16, OCP fp8 and bf8,
// int8, the block-scaled f8f6f4 forms with fp8 / fp6 / fp4 operands (scale 1),
// f32 and f64.  The host lays out each lane's operand fragment (lane-major:
// fragment of lane l at byte l * FRAG), so the kernel only loads, issues the
// MFMA and stores each lane's 4 accumulators; avk_mfma_probe checks the tile
// exactly against an integer reference.
template <int KIND>
__global__ __launch_bounds__(64) void mfma_probe_kernel(const void* __restrict__ A, const void* __restrict__ B,
                                                        void* __restrict__ D) {
  typedef int i32x4 __attribute__((ext_vector_type(4)));
  typedef int i32x8 __attribute__((ext_vector_type(8)));
  typedef double f64x4 __attribute__((ext_vector_type(4)));
  typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
  const int l = threadIdx.x;
  const f32x4 z = {0.f, 0.f, 0.f, 0.f};
  if constexpr (KIND == 0) {
    reinterpret_cast<f32x4*>(D)[l] = __builtin_amdgcn_mfma_f32_16x16x32_f16(
        reinterpret_cast<const f16x8*>(A)[l], reinterpret_cast<const f16x8*>(B)[l], z, 0, 0, 0);
  } else if constexpr (KIND == 1) {
    reinterpret_cast<f32x4*>(D)[l] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
        reinterpret_cast<const bf16x8*>(A)[l], reinterpret_cast<const bf16x8*>(B)[l], z, 0, 0, 0);
  } else if constexpr (KIND == 2) {
    reinterpret_cast<f32x4*>(D)[l] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(
        reinterpret_cast<const long*>(A)[l], reinterpret_cast<const long*>(B)[l], z, 0, 0, 0);
  } else if constexpr (KIND == 3) {
    reinterpret_cast<f32x4*>(D)[l] = __builtin_amdgcn_mfma_f32_16x16x32_bf8_bf8(
        reinterpret_cast<const long*>(A)[l], reinterpret_cast<const long*>(B)[l], z, 0, 0, 0);
  } else if constexpr (KIND == 4) {
    reinterpret_cast<i32x4*>(D)[l] = __builtin_amdgcn_mfma_i32_16x16x64_i8(
        reinterpret_cast<const i32x4*>(A)[l], reinterpret_cast<const i32x4*>(B)[l], (i32x4){0, 0, 0, 0}, 0, 0, 0);
  } else if constexpr (KIND >= 5 && KIND <= 7) {
    // operand formats (cbsz / blgp): 0 fp8 e4m3, 2 fp6 e2m3, 4 fp4 e2m1; E8M0 scale 127 = 1.0
    constexpr int FMT = KIND == 5 ? 0 : (KIND == 6 ? 2 : 4);
    reinterpret_cast<f32x4*>(D)[l] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
        reinterpret_cast<const i32x8*>(A)[l], reinterpret_cast<const i32x8*>(B)[l], z, FMT, FMT, 0, 127, 0, 127);
  } else if constexpr (KIND == 8) {
    reinterpret_cast<f32x4*>(D)[l] = __builtin_amdgcn_mfma_f32_16x16x4f32(
        reinterpret_cast<const float*>(A)[l], reinterpret_cast<const float*>(B)[l], z, 0, 0, 0);
  } else {
    reinterpret_cast<f64x4*>(D)[l] = __builtin_amdgcn_mfma_f64_16x16x4f64(
        reinterpret_cast<const double*>(A)[l], reinterpret_cast<const double*>(B)[l], (f64x4){0., 0., 0., 0.}, 0, 0,
        0);
  }
}

inline int grid_for(int64_t work_items, int per_block, int max_blocks) {
  int64_t g = (work_items + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > max_blocks) g = max_blocks;
  return (int)g;
}

}  // namespace

// ============================================================== C ABI ====

AVK_API int avk_abi_version() { return 1; }

#ifdef AVK_STAMPS
AVK_API int avk_stamps_read(unsigned long long* host, int n) {
  const int total = kStampBlocks * 8 * kStampSlices * kStampPoints;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * (n < total ? n : total));
}
#endif

AVK_API int avk_fill_uniform_f32(float* p, int64_t n, uint64_t seed, float lo, float hi, hipStream_t s) {
  if (!p || n < 0) return hipErrorInvalidValue;
  if (n == 0) return hipSuccess;
  fill_uniform_f32_kernel<<<grid_for(n, 256, 8192), 256, 0, s>>>(p, n, seed, lo, hi);
  return hipGetLastError();
}

AVK_API int avk_fill_uniform_bf16(void* p, int64_t n, uint64_t seed, float lo, float hi, hipStream_t s) {
  if (!p || n < 0 || (n % 8) != 0 || ((uintptr_t)p % 16) != 0) return hipErrorInvalidValue;
  if (n == 0) return hipSuccess;
  fill_uniform_bf16_kernel<<<grid_for(n / 8, 256, 8192), 256, 0, s>>>((__bf16*)p, n / 8, seed, lo, hi);
  return hipGetLastError();
}

AVK_API int avk_vector_add_f32(const float* a, const float* b, float* c, int64_t n, hipStream_t s) {
  if (!a || !b || !c || n < 0) return hipErrorInvalidValue;
  if (((uintptr_t)a | (uintptr_t)b | (uintptr_t)c) % 16 != 0) return hipErrorInvalidValue;
  const int64_t n4 = n / 4;
  if (n4 > 0)
    vector_add_kernel<4><<<grid_for(n4, 256 * 4, 4096), 256, 0, s>>>((const f32x4*)a, (const f32x4*)b, (f32x4*)c, n4);
  if (n4 * 4 < n) vector_add_tail_kernel<<<1, 64, 0, s>>>(a, b, c, n4 * 4, n);
  return hipGetLastError();
}

// Variants (interleaved A/B on uniform random bf16, one process, same box;
// profiles/r1_gemm/kernel_bench_8phase.json, 15 rounds each):
//                                                                   4096^3  8192^3 TF/s
//   6 8-phase quadrant pipeline, refill in the read segment (DEFAULT) 1323    1367
//   0 ring + ping-pong, LDS-DMA issued in the MFMA segment            1275    1362
//   8 as 6 with balanced reads (8/4/8/4 per phase)                    1263    1309
//   7 / 9 as 6 / 8 with the refill in the MFMA segment                1186    1354 (7)
//   1 2-stage double buffer, one barrier per K-step                   1183    1275
//   2 4-slot ring without the ping-pong                               1127    1237
//   3 4 waves x 128x128 (one wave per SIMD)                           1125    1261
//   4 ring + ping-pong, LDS-DMA issued in the read segment            1248    1336
//   5 as 0 with a 5-slot (160 KiB) ring                               1225    1334
//   hipBLASLt (torch.matmul) on the same operands                     1548    1672
// A finer split of the ring (two 16-MFMA phases per slice, 4 barriers)
// measured 1308 at 8192^3: not kept.
// Round 4: the 4-wave kernel with the generated main loop is the default for
// K a multiple of 256, the 8-phase kernel the fallback for the other K (a
// multiple of 64).  The AQL gate dispatches the same default (gemm_default.h).
// Interleaved A/B in one process, uniform random operands, TF/s
// (profiles/r4_gemm/kernel_bench_*.json; hipBLASLt varies by box):
//                                                          4096^3  8192^3  hipBLASLt
//   6 8-phase, 8 waves (round 1-3 default, fallback)        1222*   1367*
//  15 schedule 1 (32-deep, 64-B rows)                       1246    1429    1476 / 1646
//  24 schedule 2 (unrolled, constant addresses)             1273    1430    same box
//  25 schedule 3 (slice-pair loads)                         1387    1544    1454 / 1593
//  26 schedule 4 (64-deep stages, 128-B rows)               1416    1574    same box
//  27 schedule 4b (barrier after even sub-slices only)      1417    1577    1440 / 1595
//  28 schedule 4c (4b, B units' pieces early)               1418    1578    same box
//  29 4c + bf16 epilogue in 16-B stores (DEFAULT)            1521    1654    1522 / 1654
//  30 29 with non-temporal stores                            1516    1656    same box
//  (* BENCH_r03 / round 1 figures)  MFMA utilisation at 8192^3: schedule 4c 0.84,
//  schedule 2 0.75, hipBLASLt 0.87 (profiles/r4_gemm/pmc_summary_*).
constexpr int kDefaultGemmVariant = 29;
constexpr int kFallbackGemmVariant = 6;
static_assert(avk::kGemmThreads == g4::NTHR && avk::kGemmWavesPerTile * 64 == g4::NTHR &&
                  avk::kGemmTile == g4::BM && avk::kGemmTile == g4::BN && avk::kGemmKMultiple == 256,
              "gemm_default.h describes the default kernel");

AVK_API int avk_vector_add_verify_f32(const float* a, const float* b, const float* c, int64_t n,
                                      unsigned long long* bad_dev, hipStream_t s) {
  if (!a || !b || !c || !bad_dev || n <= 0) return hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(bad_dev, 0, sizeof(unsigned long long), s);
  if (e != hipSuccess) return e;
  vector_add_verify_kernel<<<grid_for(n, 256, 4096), 256, 0, s>>>(a, b, c, n, bad_dev);
  return hipGetLastError();
}

AVK_API int avk_fill_const(void* x, int64_t n, int is_bf16, float value, hipStream_t s) {
  if (!x || n <= 0) return hipErrorInvalidValue;
  if (is_bf16)
    fill_const_kernel<uint16_t><<<grid_for(n, 256, 4096), 256, 0, s>>>(static_cast<uint16_t*>(x), n,
                                                                       (uint16_t)(__builtin_bit_cast(uint32_t, value) >> 16));
  else
    fill_const_kernel<float><<<grid_for(n, 256, 4096), 256, 0, s>>>(static_cast<float*>(x), n, value);
  return hipGetLastError();
}

AVK_API int avk_check_blocks(const void* x, int64_t n, int is_bf16, int64_t block, float base, float step,
                             unsigned long long* bad_dev, hipStream_t s) {
  if (!x || !bad_dev || n <= 0 || block <= 0) return hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(bad_dev, 0, sizeof(unsigned long long), s);
  if (e != hipSuccess) return e;
  if (is_bf16)
    check_blocks_kernel<true><<<grid_for(n, 256, 4096), 256, 0, s>>>(x, n, block, base, step, bad_dev);
  else
    check_blocks_kernel<false><<<grid_for(n, 256, 4096), 256, 0, s>>>(x, n, block, base, step, bad_dev);
  return hipGetLastError();
}

AVK_API int avk_gemm_bf16_nt_variant(const void* A, const void* Bt, void* C, int out_f32, int M, int N, int K,
                                     int variant, hipStream_t s) {
  using namespace gemm;
  if (!A || !Bt || !C || M <= 0 || N <= 0 || K <= 0) return hipErrorInvalidValue;
  if (M % BM || N % BN || K % BK) return hipErrorInvalidValue;
  if (((uintptr_t)A | (uintptr_t)Bt | (uintptr_t)C) % 16 != 0) return hipErrorInvalidValue;
  const int nwg = (M / BM) * (N / BN);
  const __bf16* a = (const __bf16*)A;
  const __bf16* b = (const __bf16*)Bt;
#define AVK_G8(V, LIM, BAL)                                                                       \
    case V:                                                                                     \
      if (out_f32) gemm_bf16_nt_8p_kernel<true, LIM, BAL><<<nwg, g8::NTHR, 0, s>>>(a, b, C, M, N, K); \
      else gemm_bf16_nt_8p_kernel<false, LIM, BAL><<<nwg, g8::NTHR, 0, s>>>(a, b, C, M, N, K);        \
      break;
  switch (variant) {
    AVK_G8(6, false, false)  // kFallbackGemmVariant: 8 waves, K a multiple of 64
#define AVK_G4A(V, L)                                                                            \
    case V:                                                                                      \
      if (K % 256) return hipErrorInvalidValue;                                                  \
      if (out_f32) gemm_bf16_nt_4wa_kernel<true, L><<<nwg, g4::NTHR, 0, s>>>(a, b, C, M, N, K);  \
      else gemm_bf16_nt_4wa_kernel<false, L><<<nwg, g4::NTHR, 0, s>>>(a, b, C, M, N, K);         \
      break;
    // 4 waves x 128x128 per 256x256 tile, 5-unit LDS ring (K: a multiple of 256)
    case 29:  // kDefaultGemmVariant: schedule 4c, the bf16 epilogue in 16-B stores (permlane16_swap pairs)
      if (K % 256) return hipErrorInvalidValue;
      if (out_f32) gemm_bf16_nt_4wa_kernel<true, 13><<<nwg, g4::NTHR, 0, s>>>(a, b, C, M, N, K);
      else gemm_bf16_nt_4wa_kernel<false, 13, 1><<<nwg, g4::NTHR, 0, s>>>(a, b, C, M, N, K);
      break;
#if AVK_GEMM_LAB
    AVK_G4A(28, 13)  // 4c with the 8-B bf16 epilogue
    case 30:  // 29 with non-temporal stores (no difference: profiles/r4_gemm/kernel_bench_epilogue16_nt_vs_28.json)
      if (K % 256) return hipErrorInvalidValue;
      if (out_f32) gemm_bf16_nt_4wa_kernel<true, 13><<<nwg, g4::NTHR, 0, s>>>(a, b, C, M, N, K);
      else gemm_bf16_nt_4wa_kernel<false, 13, 2><<<nwg, g4::NTHR, 0, s>>>(a, b, C, M, N, K);
      break;
    // the other generated schedules (gen_gemm4w_asm.py; profiles/r4_gemm/)
    AVK_G4A(15, 0)   // 1: 32-deep slices in 64-B rows, rotating slot registers
    AVK_G4A(24, 9)   // 2: 10-slice unrolled body, constant addresses, one filler per MFMA gap
    AVK_G4A(25, 10)  // 3: 2 with the loads in slice pairs (whole 128-B lines back to back)
    AVK_G4A(26, 11)  // 4: 64-deep stages in 128-B rows, 8-row x 128-B pieces
    AVK_G4A(27, 12)  // 4b: 4 with a barrier after even sub-slices only
    case 14:  // the 4-wave kernel in builtins (hipcc moves accumulators through VGPRs, spills)
      if (K % 256) return hipErrorInvalidValue;
      if (out_f32) gemm_bf16_nt_4w_kernel<true><<<nwg, g4::NTHR, 0, s>>>(a, b, C, M, N, K);
      else gemm_bf16_nt_4w_kernel<false><<<nwg, g4::NTHR, 0, s>>>(a, b, C, M, N, K);
      break;
    AVK_G4A(16, 1)  // ablations of 15 (wrong results by design, timing only): no LDS-DMA
    AVK_G4A(17, 2)  // no barrier
    AVK_G4A(18, 3)  // the slice change's SALU work among the last MFMAs (correct)
    AVK_G4A(19, 4)  // no fragment reads
    AVK_G4A(20, 5)  // one M0 for every piece (wrong LDS image): the cost of the per-piece M0 set-up
    AVK_G4A(21, 6)  // the loads into VGPRs instead of LDS (wrong results): glds vs a plain load
    AVK_G4A(22, 7)  // pieces in pairs (wrong results: M0 / base rewritten before the previous piece read it)
    AVK_G4A(23, 8)  // pieces in one burst after the barrier (wrong results, as 22)
#endif
#undef AVK_G4A
#if AVK_GEMM_LAB
    case 0:
      if (out_f32) gemm_bf16_nt_pp_kernel<true, true><<<nwg, NTHR, 0, s>>>(a, b, C, M, N, K);
      else gemm_bf16_nt_pp_kernel<false, true><<<nwg, NTHR, 0, s>>>(a, b, C, M, N, K);
      break;
    case 1:
      if (out_f32) gemm_bf16_nt_kernel<true><<<nwg, NTHR, 0, s>>>(a, b, C, M, N, K);
      else gemm_bf16_nt_kernel<false><<<nwg, NTHR, 0, s>>>(a, b, C, M, N, K);
      break;
    case 2:
      if (out_f32) gemm_bf16_nt_ring_kernel<true><<<nwg, NTHR, 0, s>>>(a, b, C, M, N, K);
      else gemm_bf16_nt_ring_kernel<false><<<nwg, NTHR, 0, s>>>(a, b, C, M, N, K);
      break;
    case 3:
      if (out_f32) gemm_bf16_nt_w4_kernel<true><<<nwg, gw4::NTHR, 0, s>>>(a, b, C, M, N, K);
      else gemm_bf16_nt_w4_kernel<false><<<nwg, gw4::NTHR, 0, s>>>(a, b, C, M, N, K);
      break;
    case 4:
      if (out_f32) gemm_bf16_nt_pp_kernel<true, false><<<nwg, NTHR, 0, s>>>(a, b, C, M, N, K);
      else gemm_bf16_nt_pp_kernel<false, false><<<nwg, NTHR, 0, s>>>(a, b, C, M, N, K);
      break;
    case 5:
      if (out_f32) gemm_bf16_nt_pp_kernel<true, true, 5><<<nwg, NTHR, 0, s>>>(a, b, C, M, N, K);
      else gemm_bf16_nt_pp_kernel<false, true, 5><<<nwg, NTHR, 0, s>>>(a, b, C, M, N, K);
      break;
    AVK_G8(7, true, false)
    AVK_G8(8, false, true)
    AVK_G8(9, true, true)
#define AVK_G8M(V, GM)                                                                                    \
    case V:                                                                                              \
      if (out_f32) gemm_bf16_nt_8p_kernel<true, false, false, GM><<<nwg, g8::NTHR, 0, s>>>(a, b, C, M, N, K); \
      else gemm_bf16_nt_8p_kernel<false, false, false, GM><<<nwg, g8::NTHR, 0, s>>>(a, b, C, M, N, K);        \
      break;
    AVK_G8M(10, 8)  // the default kernel with 8 / 16 / 2 tile rows per L2 band, and with the default 4 (13):
    AVK_G8M(11, 16)  // 13 is variant 6 built into the lab library, for same-library A/B (the two libraries'
    AVK_G8M(12, 2)   // copies of one kernel timed 1-4 % apart, profiles/r3_gemm)
    AVK_G8M(13, 4)
#undef AVK_G8M
#endif
#undef AVK_G8
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

AVK_API int avk_gemm_bf16_nt(const void* A, const void* Bt, void* C, int out_f32, int M, int N, int K,
                             hipStream_t s) {
  return avk_gemm_bf16_nt_variant(A, Bt, C, out_f32, M, N, K,
                                  K % avk::kGemmKMultiple == 0 ? kDefaultGemmVariant : kFallbackGemmVariant, s);
}

// C = A . Bt^T, OCP e4m3 operands (K a multiple of 256); the fp8 rate step and
// its counter gate (gate_policy.h, SQ_INSTS_VALU_MFMA_MOPS_F8)
AVK_API int avk_gemm_fp8_nt(const void* A, const void* Bt, void* C, int out_f32, int M, int N, int K, hipStream_t s) {
  if (!A || !Bt || !C || M <= 0 || N <= 0 || K <= 0) return hipErrorInvalidValue;
  if (M % avk::kGemmTile || N % avk::kGemmTile || K % 256) return hipErrorInvalidValue;
  if (((uintptr_t)A | (uintptr_t)Bt | (uintptr_t)C) % 16 != 0) return hipErrorInvalidValue;
  const int nwg = (M / g4::BM) * (N / g4::BN);
  const uint8_t* a = (const uint8_t*)A;
  const uint8_t* b = (const uint8_t*)Bt;
  if (out_f32) gemm_fp8_nt_kernel<true><<<nwg, g4::NTHR, 0, s>>>(a, b, C, M, N, K);
  else gemm_fp8_nt_kernel<false, 1><<<nwg, g4::NTHR, 0, s>>>(a, b, C, M, N, K);
  return hipGetLastError();
}

AVK_API int avk_fill_fp8(void* p, int64_t n, uint64_t seed, hipStream_t s) {
  if (!p || n < 0) return hipErrorInvalidValue;
  if (n == 0) return hipSuccess;
  fill_fp8_kernel<<<grid_for(n, 256, 8192), 256, 0, s>>>((uint8_t*)p, n, seed);
  return hipGetLastError();
}

// FP4 (e2m1 pairs): A [M][K/2], Bt [N][K/2] bytes; M, N % 256, K % 256, K >= 512
AVK_API int avk_gemm_fp4_nt(const void* A, const void* Bt, void* C, int out_f32, int M, int N, int K, hipStream_t s) {
  if (!A || !Bt || !C || M <= 0 || N <= 0 || K < 512) return hipErrorInvalidValue;
  if (M % avk::kGemmTile || N % avk::kGemmTile || K % 256) return hipErrorInvalidValue;
  if (((uintptr_t)A | (uintptr_t)Bt | (uintptr_t)C) % 16 != 0) return hipErrorInvalidValue;
  const int nwg = (M / g4::BM) * (N / g4::BN);
  const uint8_t* a = (const uint8_t*)A;
  const uint8_t* b = (const uint8_t*)Bt;
  if (out_f32) gemm_fp4_nt_kernel<true><<<nwg, g4::NTHR, 0, s>>>(a, b, C, M, N, K);
  else gemm_fp4_nt_kernel<false, 1><<<nwg, g4::NTHR, 0, s>>>(a, b, C, M, N, K);
  return hipGetLastError();
}

// C = A . Bt^T with fp6 (e2m3) operands in the validator's fp6 storage (32-B
// slot per 32 elements: K bytes per row); K a multiple of 256
AVK_API int avk_gemm_fp6_nt(const void* A, const void* Bt, void* C, int out_f32, int M, int N, int K, hipStream_t s) {
  if (!A || !Bt || !C || M <= 0 || N <= 0 || K <= 0) return hipErrorInvalidValue;
  if (M % avk::kGemmTile || N % avk::kGemmTile || K % 256) return hipErrorInvalidValue;
  if (((uintptr_t)A | (uintptr_t)Bt | (uintptr_t)C) % 16 != 0) return hipErrorInvalidValue;
  const int nwg = (M / g4::BM) * (N / g4::BN);
  const uint8_t* a = (const uint8_t*)A;
  const uint8_t* b = (const uint8_t*)Bt;
  if (out_f32) gemm_fp6_nt_kernel<true><<<nwg, g4::NTHR, 0, s>>>(a, b, C, M, N, K);
  else gemm_fp6_nt_kernel<false, 1><<<nwg, g4::NTHR, 0, s>>>(a, b, C, M, N, K);
  return hipGetLastError();
}

// nbytes: a multiple of 32 (one slot per 32 elements)
AVK_API int avk_fill_fp6(void* p, int64_t nbytes, uint64_t seed, hipStream_t s) {
  if (!p || nbytes <= 0 || nbytes % 32) return hipErrorInvalidValue;
  fill_fp6_kernel<<<grid_for(nbytes / 32, 256, 8192), 256, 0, s>>>((uint8_t*)p, nbytes / 32, seed);
  return hipGetLastError();
}

AVK_API int avk_gemv_rows_fp6(const void* X, const float* v, float* y, int R, int C, hipStream_t s) {
  if (!X || !v || !y || R <= 0 || C <= 0 || C % 32) return hipErrorInvalidValue;
  gemv_rows_fp6_kernel<<<(R + 3) / 4, 256, 0, s>>>((const uint8_t*)X, v, y, R, C);
  return hipGetLastError();
}

AVK_API int avk_gemv_cols_fp6(const void* X, const float* v, float* z, int R, int C, hipStream_t s) {
  if (!X || !v || !z || R <= 0 || C <= 0 || C % 32) return hipErrorInvalidValue;
  return launch_gemv_cols<DecFp6>(X, v, z, R, C, s);
}

// block-scaled MXFP4: C = (2^(SA-127) A)(2^(SB-127) Bt)^T, A / Bt FP4 pairs,
// SA [M][8] / SB [N][8] E8M0 (scale of row r, k-block b: S[r][b % 8]); K a
// multiple of 256, >= 512
AVK_API int avk_gemm_mxfp4_nt(const void* A, const void* Bt, const void* SA, const void* SB, void* C, int out_f32,
                              int M, int N, int K, hipStream_t s) {
  if (!A || !Bt || !SA || !SB || !C || M <= 0 || N <= 0 || K < 512) return hipErrorInvalidValue;
  if (M % avk::kGemmTile || N % avk::kGemmTile || K % 256) return hipErrorInvalidValue;
  if (((uintptr_t)A | (uintptr_t)Bt | (uintptr_t)C) % 16 != 0) return hipErrorInvalidValue;
  const int nwg = (M / g4::BM) * (N / g4::BN);
  const uint8_t* a = (const uint8_t*)A;
  const uint8_t* b = (const uint8_t*)Bt;
  const uint8_t* sa = (const uint8_t*)SA;
  const uint8_t* sb = (const uint8_t*)SB;
  if (out_f32) gemm_mxfp4_nt_kernel<true><<<nwg, g4::NTHR, 0, s>>>(a, b, C, M, N, K, sa, sb);
  else gemm_mxfp4_nt_kernel<false, 1><<<nwg, g4::NTHR, 0, s>>>(a, b, C, M, N, K, sa, sb);
  return hipGetLastError();
}

// n random E8M0 scales in [lo, hi]
AVK_API int avk_fill_e8m0(void* p, int64_t n, uint64_t seed, int lo, int hi, hipStream_t s) {
  if (!p || n <= 0 || lo < 1 || hi > 254 || hi < lo) return hipErrorInvalidValue;
  fill_e8m0_kernel<<<grid_for(n, 256, 8192), 256, 0, s>>>((uint8_t*)p, n, seed, lo, hi - lo + 1);
  return hipGetLastError();
}

AVK_API int avk_gemv_rows_mxfp4(const void* X, const void* S, const float* v, float* y, int R, int C, hipStream_t s) {
  if (!X || !S || !v || !y || R <= 0 || C <= 0 || C % 16) return hipErrorInvalidValue;
  gemv_rows_mxfp4_kernel<<<(R + 3) / 4, 256, 0, s>>>((const uint8_t*)X, (const uint8_t*)S, v, y, R, C);
  return hipGetLastError();
}

AVK_API int avk_gemv_cols_mxfp4(const void* X, const void* S, const float* v, float* z, int R, int C, hipStream_t s) {
  if (!X || !S || !v || !z || R <= 0 || C <= 0 || C % 16) return hipErrorInvalidValue;
  return launch_gemv_cols<DecMxFp4>(X, v, z, R, C, s, S);
}

AVK_API int avk_fill_fp4(void* p, int64_t nbytes, uint64_t seed, hipStream_t s) {
  if (!p || nbytes < 0) return hipErrorInvalidValue;
  if (nbytes == 0) return hipSuccess;
  fill_fp4_kernel<<<grid_for(nbytes, 256, 8192), 256, 0, s>>>((uint8_t*)p, nbytes, seed);
  return hipGetLastError();
}

// y = X v, X FP4 pairs [R][C/2] (C % 16 == 0)
AVK_API int avk_gemv_rows_fp4(const void* X, const float* v, float* y, int R, int C, hipStream_t s) {
  if (!X || !v || !y || R <= 0 || C <= 0 || C % 16 || ((uintptr_t)X % 8)) return hipErrorInvalidValue;
  gemv_rows_fp4_kernel<<<(R + 3) / 4, 256, 0, s>>>((const uint8_t*)X, v, y, R, C);
  return hipGetLastError();
}

// z = X^T v accumulated into z (caller zeroes z); X FP4 pairs [R][C/2], C % 16 == 0
AVK_API int avk_gemv_cols_fp4(const void* X, const float* v, float* z, int R, int C, hipStream_t s) {
  if (!X || !v || !z || R <= 0 || C <= 0 || C % 16 || ((uintptr_t)X % 8)) return hipErrorInvalidValue;
  return launch_gemv_cols<DecFp4>(X, v, z, R, C, s);
}

// y = X v, X e4m3 [R][C] (C % 8 == 0)
AVK_API int avk_gemv_rows_fp8(const void* X, const float* v, float* y, int R, int C, hipStream_t s) {
  if (!X || !v || !y || R <= 0 || C <= 0 || C % 8 || ((uintptr_t)X % 8)) return hipErrorInvalidValue;
  gemv_rows_fp8_kernel<<<(R + 3) / 4, 256, 0, s>>>((const uint8_t*)X, v, y, R, C);
  return hipGetLastError();
}

// z = X^T v accumulated into z (caller zeroes z); X e4m3 [R][C], C % 8 == 0
AVK_API int avk_gemv_cols_fp8(const void* X, const float* v, float* z, int R, int C, hipStream_t s) {
  if (!X || !v || !z || R <= 0 || C <= 0 || C % 8 || ((uintptr_t)X % 8)) return hipErrorInvalidValue;
  return launch_gemv_cols<DecFp8>(X, v, z, R, C, s);
}

// y = X v ; X is [R][C] row-major (bf16 when x_is_bf16, else f32); C % 8 == 0
AVK_API int avk_gemv_rows(const void* X, int x_is_bf16, const float* v, float* y, int R, int C, hipStream_t s) {
  if (!X || !v || !y || R <= 0 || C <= 0 || C % 8) return hipErrorInvalidValue;
  const int blocks = (R + 3) / 4;
  if (x_is_bf16)
    gemv_rows_kernel<__bf16><<<blocks, 256, 0, s>>>((const __bf16*)X, v, y, R, C);
  else
    gemv_rows_kernel<float><<<blocks, 256, 0, s>>>((const float*)X, v, y, R, C);
  return hipGetLastError();
}

// z = X^T v accumulated into z (caller zeroes z); X bf16 [R][C], C % 8 == 0
AVK_API int avk_gemv_cols_bf16(const void* X, const float* v, float* z, int R, int C, hipStream_t s) {
  if (!X || !v || !z || R <= 0 || C <= 0 || C % 8 || ((uintptr_t)X % 16)) return hipErrorInvalidValue;
  return launch_gemv_cols<DecBf16>(X, v, z, R, C, s);
}

// variant: 0 = plain loads/stores, 1 = nontemporal
// variant bit 0: nontemporal loads/stores; bits 1-2: float4s per lane per
// iteration (0 -> 4, 1 -> 8, 2 -> 2, 3 -> 1).  Grid = num_cus * 16 blocks of
// 256: the sweep in profiles/r1_hbm (1 GiB, read + write counted) peaks at
// 6.30 TB/s for nontemporal x4 at 16 blocks/CU vs 6.10 at 8 and 5.08 for
// torch's copy_.
AVK_API int avk_hbm_copy(const void* src, void* dst, int64_t bytes, int num_cus, int variant, hipStream_t s) {
  if (!src || !dst || bytes <= 0 || bytes % 16 || (((uintptr_t)src | (uintptr_t)dst) % 16)) return hipErrorInvalidValue;
  if (variant < 0 || variant > 7) return hipErrorInvalidValue;
  const int64_t n = bytes / 16;
  const int blocks = (num_cus > 0 ? num_cus : 256) * 16;
  const bool nt = variant & 1;
  const int u = (const int[]){4, 8, 2, 1}[(variant >> 1) & 3];
  const int g = grid_for(n, 256 * u, blocks);
  const f32x4* a = (const f32x4*)src;
  f32x4* d = (f32x4*)dst;
#define AVK_COPY(U)                                                      \
  if (nt)                                                                \
    hbm_copy_kernel<U, true><<<g, 256, 0, s>>>(a, d, n);                 \
  else                                                                   \
    hbm_copy_kernel<U, false><<<g, 256, 0, s>>>(a, d, n);
  switch (u) {
    case 8: AVK_COPY(8) break;
    case 2: AVK_COPY(2) break;
    case 1: AVK_COPY(1) break;
    default: AVK_COPY(4) break;
  }
#undef AVK_COPY
  return hipGetLastError();
}

AVK_API int avk_checksum(const void* p, int64_t bytes, unsigned long long* out_dev, hipStream_t s) {
  if (!p || !out_dev || bytes <= 0 || bytes % 16 || ((uintptr_t)p % 16)) return hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(out_dev, 0, sizeof(unsigned long long), s);
  if (e != hipSuccess) return e;
  checksum_kernel<<<grid_for(bytes / 16, 256 * 4, 2048), 256, 0, s>>>((const u32x4*)p, bytes / 16, out_dev);
  return hipGetLastError();
}

AVK_API int avk_max_abs_diff_f32(const float* a, const float* b, int64_t n, unsigned int* out_dev, hipStream_t s) {
  if (!a || !b || !out_dev || n <= 0) return hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(out_dev, 0, sizeof(unsigned int), s);
  if (e != hipSuccess) return e;
  max_abs_diff_kernel<<<grid_for(n / 4 + 1, 256, 2048), 256, 0, s>>>(a, b, n, out_dev);
  return hipGetLastError();
}

// ptrs: host array of np device pointers (peer-mapped or local); count % 4 == 0
AVK_API int avk_allreduce_oneshot_f32(const float* const* ptrs, int np, float* out, int64_t count, hipStream_t s) {
  if (!ptrs || !out || np < 1 || np > 8 || count <= 0 || count % 4) return hipErrorInvalidValue;
  PeerPtrs pp{};
  for (int r = 0; r < np; ++r) {
    if (!ptrs[r] || ((uintptr_t)ptrs[r] % 16)) return hipErrorInvalidValue;
    pp.p[r] = ptrs[r];
  }
  const int64_t n4 = count / 4;
  const int g = grid_for(n4, 256, 256 * 16);
  switch (np) {
    case 2: allreduce_oneshot_f32_kernel<2><<<g, 256, 0, s>>>(pp, out, n4, np); break;
    case 4: allreduce_oneshot_f32_kernel<4><<<g, 256, 0, s>>>(pp, out, n4, np); break;
    case 8: allreduce_oneshot_f32_kernel<8><<<g, 256, 0, s>>>(pp, out, n4, np); break;
    default: allreduce_oneshot_f32_kernel<0><<<g, 256, 0, s>>>(pp, out, n4, np); break;
  }
  return hipGetLastError();
}

// two-shot slice for `rank`: reduce slice of the float4 space, broadcast into all outs
AVK_API int avk_allreduce_twoshot_f32(const float* const* in_ptrs, float* const* out_ptrs, int np, int rank,
                                      int64_t count, hipStream_t s) {
  if (!in_ptrs || !out_ptrs || np < 1 || np > 8 || rank < 0 || rank >= np || count <= 0 || count % 4)
    return hipErrorInvalidValue;
  PeerPtrs pi{};
  PeerPtrsMut po{};
  for (int r = 0; r < np; ++r) {
    if (!in_ptrs[r] || !out_ptrs[r]) return hipErrorInvalidValue;
    pi.p[r] = in_ptrs[r];
    po.p[r] = out_ptrs[r];
  }
  const int64_t n4 = count / 4;
  const int64_t per = (n4 + np - 1) / np;
  const int64_t lo = per * rank;
  const int64_t hi = lo + per < n4 ? lo + per : n4;
  if (hi <= lo) return hipSuccess;
  allreduce_twoshot_f32_kernel<<<grid_for(hi - lo, 256, 256 * 8), 256, 0, s>>>(pi, po, np, lo, hi);
  return hipGetLastError();
}

// ---------------------------------------------------------- K5 host side ----
namespace {
struct ProbeKind {
  const char* name;
  int k;          // K of one MFMA
  int elem_bits;  // operand element width
  int frag;       // bytes per lane fragment in the lane-major buffer
  bool fp64;      // f64 C/D layout
};
constexpr ProbeKind kProbe[] = {
    {"f16", 32, 16, 16, false},   {"bf16", 32, 16, 16, false}, {"fp8", 32, 8, 8, false},
    {"bf8", 32, 8, 8, false},     {"i8", 64, 8, 16, false},    {"mxfp8", 128, 8, 32, false},
    {"mxfp6", 128, 6, 32, false}, {"mxfp4", 128, 4, 32, false}, {"f32", 4, 32, 4, false},
    {"f64", 4, 64, 8, true},
};
constexpr int kProbeKinds = sizeof(kProbe) / sizeof(kProbe[0]);

// bit pattern of a small integer v in [-2, 2] in each operand format
uint64_t probe_encode(int kind, int v) {
  const int a = v < 0 ? -v : v;
  const bool neg = v < 0;
  switch (kind) {
    case 0: return (neg ? 0x8000 : 0) | (a == 0 ? 0 : a == 1 ? 0x3C00 : 0x4000);  // f16
    case 1: return (neg ? 0x8000 : 0) | (a == 0 ? 0 : a == 1 ? 0x3F80 : 0x4000);  // bf16
    case 2: case 5: return (neg ? 0x80 : 0) | (a == 0 ? 0 : a == 1 ? 0x38 : 0x40);  // e4m3
    case 3: return (neg ? 0x80 : 0) | (a == 0 ? 0 : a == 1 ? 0x3C : 0x40);  // e5m2
    case 4: return (uint64_t)(uint8_t)(int8_t)v;                           // int8
    case 6: return (neg ? 0x20 : 0) | (a == 0 ? 0 : a == 1 ? 0x08 : 0x10);  // fp6 e2m3
    case 7: return (neg ? 0x8 : 0) | (a == 0 ? 0 : a == 1 ? 0x2 : 0x4);     // fp4 e2m1
    case 8: { float f = (float)v; uint32_t u; memcpy(&u, &f, 4); return u; }
    default: { double f = (double)v; uint64_t u; memcpy(&u, &f, 8); return u; }
  }
}

void put_bits(uint8_t* p, int bit, int width, uint64_t v) {
  for (int b = 0; b < width; ++b)
    if ((v >> b) & 1) p[(bit + b) >> 3] |= (uint8_t)(1u << ((bit + b) & 7));
}

// lane l holds X[row l & 15][k = (l >> 4) * E + j], j < E (E = K / 4 elements)
void probe_fragments(int kind, const std::vector<int>& X, std::vector<uint8_t>* out) {
  const ProbeKind& pk = kProbe[kind];
  const int E = pk.k / 4;
  out->assign(64 * pk.frag, 0);
  for (int l = 0; l < 64; ++l)
    for (int j = 0; j < E; ++j)
      put_bits(out->data() + l * pk.frag, j * pk.elem_bits, pk.elem_bits,
               probe_encode(kind, X[(l & 15) * pk.k + (l >> 4) * E + j]));
}
}  // namespace

AVK_API int avk_mfma_probe_count() { return kProbeKinds; }

AVK_API const char* avk_mfma_probe_name(int kind) {
  return kind >= 0 && kind < kProbeKinds ? kProbe[kind].name : "";
}

// Runs probe `kind` on the current device; *mismatches = output elements that
// differ from the exact integer reference (0 = the data type works).
AVK_API int avk_mfma_probe(int kind, uint64_t seed, int* mismatches, hipStream_t s) {
  if (kind < 0 || kind >= kProbeKinds || !mismatches) return hipErrorInvalidValue;
  const ProbeKind& pk = kProbe[kind];
  std::vector<int> a(16 * pk.k), bt(16 * pk.k);  // A[16][K], Bt[16][K] (= B^T)
  uint64_t h = seed * 0x9E3779B97F4A7C15ull + (uint64_t)kind;
  auto next = [&h]() {
    h ^= h >> 33;
    h *= 0xff51afd7ed558ccdull;
    h ^= h >> 29;
    return (int)(h % 5) - 2;
  };
  for (int& v : a) v = next();
  for (int& v : bt) v = next();
  std::vector<uint8_t> fa, fb;
  probe_fragments(kind, a, &fa);
  probe_fragments(kind, bt, &fb);
  const size_t dbytes = 64 * 4 * (pk.fp64 ? 8 : 4);
  void *da = nullptr, *db = nullptr, *dd = nullptr;
  hipError_t e = hipMalloc(&da, fa.size());
  if (e == hipSuccess) e = hipMalloc(&db, fb.size());
  if (e == hipSuccess) e = hipMalloc(&dd, dbytes);
  if (e == hipSuccess) e = hipMemcpyAsync(da, fa.data(), fa.size(), hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipMemcpyAsync(db, fb.data(), fb.size(), hipMemcpyHostToDevice, s);
  if (e == hipSuccess) {
    switch (kind) {
#define AVK_PROBE(K) case K: mfma_probe_kernel<K><<<1, 64, 0, s>>>(da, db, dd); break;
      AVK_PROBE(0) AVK_PROBE(1) AVK_PROBE(2) AVK_PROBE(3) AVK_PROBE(4)
      AVK_PROBE(5) AVK_PROBE(6) AVK_PROBE(7) AVK_PROBE(8) AVK_PROBE(9)
#undef AVK_PROBE
    }
    e = hipGetLastError();
  }
  std::vector<uint8_t> out(dbytes);
  if (e == hipSuccess) e = hipMemcpyAsync(out.data(), dd, dbytes, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  for (void* p : {da, db, dd})
    if (p) (void)hipFree(p);
  if (e != hipSuccess) return e;
  int bad = 0;
  for (int l = 0; l < 64; ++l)
    for (int i = 0; i < 4; ++i) {
      // C/D maps (cdna_hip_programming.md §3): col = lane & 15; row = 4*(lane>>4) + i, f64: (lane>>4) + 4*i
      const int col = l & 15, row = pk.fp64 ? (l >> 4) + 4 * i : 4 * (l >> 4) + i;
      long long ref = 0;
      for (int k = 0; k < pk.k; ++k) ref += (long long)a[row * pk.k + k] * bt[col * pk.k + k];
      double got;
      if (pk.fp64) {
        memcpy(&got, out.data() + (l * 4 + i) * 8, 8);
      } else if (kind == 4) {
        int32_t v;
        memcpy(&v, out.data() + (l * 4 + i) * 4, 4);
        got = v;
      } else {
        float v;
        memcpy(&v, out.data() + (l * 4 + i) * 4, 4);
        got = v;
      }
      bad += got != (double)ref;
    }
  *mismatches = bad;
  return hipSuccess;
}
