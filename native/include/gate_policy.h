// N7 counter-gate policy: the verdict on one counted dispatch of the
// validator's default MFMA GEMM (gemm_default.h: 256x256 tiles,
// kGemmWavesPerTile waves per workgroup, v_mfma_f32_16x16x32_bf16).
//
// The counters of that dispatch are not noisy measurements but exact
// functions of the launch (BASELINE.md "Round 2: ... AQL-packet gate",
// profiles/r2_gate/aql_v2.json at 4096^3):
//   SQ_INSTS_VALU_MFMA_MOPS_BF16 * 512 == 2 * M * N * K   (1 MOP = 512 FLOP)
//   SQ_WAVES == (M/256) * (N/256) * kGemmWavesPerTile
// A GPU that drops or duplicates work (a dead CU that never retires its
// waves, a mis-scheduled dispatch, a corrupted code object) breaks the
// equalities even when the output checksum happens to match.  The third
// condition is time-based: MFMA busy cycles over elapsed GPU cycles per SIMD,
// SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE per XCD * SIMDs).  At 4096^3 on
// a healthy MI355X it read ~0.49 with round 3's 8-wave kernel; a starved matrix pipe (HBM stack running
// slow, CUs fenced off, the GEMM waiting on a throttled fabric) pulls it down.
// The floor scales with how many CUs the launch can occupy (tiles / CUs,
// capped at 1), so a 1024^3 plugin-pod GEMM (16 tiles on 256 CUs) is held to
// 1/16 of it.  Clock speed cancels out of the ratio: low clocks are caught by
// the TF/s floor instead (validator_main.cpp --min-gemm-tflops).
//
// Header-only so the validator binary and its --check-gate mode (the CPU
// tests, tests/test_gate_policy.py) run the same code.
#pragma once

#include <cmath>
#include <cstdio>
#include <string>

#include "gemm_default.h"

namespace avk {

struct GateCounters {
  double mops = 0;         // SQ_INSTS_VALU_MFMA_MOPS_<dtype>, summed over instances
  double busy = 0;         // SQ_VALU_MFMA_BUSY_CYCLES, summed over instances
  double waves = 0;        // SQ_WAVES, summed over instances
  double gui = 0;          // GRBM_GUI_ACTIVE, summed over instances (one per XCD)
  int gui_samples = 0;     // GRBM instances summed into gui
  bool output_matches = true;  // the counted dispatch reproduced the HIP run's output
};

struct GateVerdict {
  bool ok = false;
  std::string reason;      // empty when ok; else the first failed condition
  double expected_mops = 0;
  double expected_waves = 0;
  double mfma_util = 0;    // busy / (gui per instance * SIMDs)
  double util_floor = 0;   // the floor applied (min_util * occupancy)
};

// `mops_name` / `flop_per_mop`: the MOPS counter of the GEMM's data type
// (SQ_INSTS_VALU_MFMA_MOPS_BF16 for the default GEMM, _F8 for the mfma-rate
// step's e4m3 GEMM; profiles/r5_fp8 measured the same 512 FLOP per MOP).
inline GateVerdict gate_verdict(long long m, long long n, long long k, int cus, const GateCounters& c,
                                double min_util, const char* mops_name = "SQ_INSTS_VALU_MFMA_MOPS_BF16",
                                double flop_per_mop = 512.0) {
  GateVerdict v;
  char buf[256];
  v.expected_mops = 2.0 * (double)m * (double)n * (double)k / flop_per_mop;
  const long long tiles = (m / 256) * (n / 256);
  v.expected_waves = (double)tiles * kGemmWavesPerTile;
  const double simds = 4.0 * (cus > 0 ? cus : 0);
  const double gui_per = c.gui_samples > 0 ? c.gui / c.gui_samples : 0.0;
  v.mfma_util = (gui_per > 0 && simds > 0) ? c.busy / (gui_per * simds) : 0.0;
  const double occupancy = cus > 0 ? std::fmin(1.0, (double)tiles / cus) : 0.0;
  v.util_floor = min_util > 0 ? min_util * occupancy : 0.0;
  if (m <= 0 || n <= 0 || k <= 0 || m % 256 || n % 256 || k % 256) {
    v.reason = "shape is not a multiple of the 256x256 tile";
  } else if (cus <= 0) {
    v.reason = "unknown CU count";
  } else if (!c.output_matches) {
    v.reason = "counted dispatch output differs from the HIP run";
  } else if (!(c.mops == v.expected_mops)) {
    snprintf(buf, sizeof(buf), "%s %.0f != 2MNK/%.0f = %.0f", mops_name, c.mops, flop_per_mop, v.expected_mops);
    v.reason = buf;
  } else if (!(c.waves == v.expected_waves)) {
    snprintf(buf, sizeof(buf), "SQ_WAVES %.0f != tiles*%d = %.0f", c.waves, kGemmWavesPerTile, v.expected_waves);
    v.reason = buf;
  } else if (!(c.busy > 0) || !(c.gui > 0) || c.gui_samples <= 0) {
    v.reason = "MFMA busy / GUI active cycles not counted";
  } else if (v.mfma_util > 1.0 + 1e-9) {
    snprintf(buf, sizeof(buf), "MFMA utilisation %.3f > 1: inconsistent counters", v.mfma_util);
    v.reason = buf;
  } else if (v.mfma_util < v.util_floor) {
    snprintf(buf, sizeof(buf), "MFMA utilisation %.4f below floor %.4f", v.mfma_util, v.util_floor);
    v.reason = buf;
  }
  v.ok = v.reason.empty();
  return v;
}

// Whether a failed verdict may be counted again (validator_main.cpp aql_gate,
// at most kGateAttempts in all).  The counters are device-wide, so a window
// that overlapped someone else's work is not evidence against this GPU:
//   "preempted"    - output and op count exact, waves above the launch's
//                    (a queue remap saved and restored ours) or exact waves
//                    with the utilisation under its floor (our dispatch
//                    waited while the GPU stayed busy);
//   "foreign_mfma" - output exact, op count above 2MNK, waves not below the
//                    launch's: another process's MFMA kernel of the same data
//                    type ran in the window.  Its waves count only if they
//                    started inside it: a co-tenant's GEMM whose waves were
//                    already resident added 2.08x our ops with our waves
//                    exact (tests/test_native_gpu.py, a PyTorch bf16 loop).
// Everything else is the GPU's own: a wrong output, an op count short of
// 2MNK (other work only adds), missing waves.  A retry never passes by
// itself - a pass needs every equality exact on one attempt - so a truncated
// dispatch hidden under foreign work, or a kernel that itself issues extra
// MFMAs, is counted again and fails after the last attempt, not accepted.
// Returns "" when the failure is final.
inline const char* gate_retry_kind(const GateCounters& c, const GateVerdict& v) {
  if (v.ok || !c.output_matches) return "";
  if (c.mops == v.expected_mops &&
      (c.waves > v.expected_waves || (c.waves == v.expected_waves && v.mfma_util < v.util_floor)))
    return "preempted";
  if (c.mops > v.expected_mops && c.waves >= v.expected_waves) return "foreign_mfma";
  return "";
}

// Floors given for a whole MI355X (256 CUs) apply pro rata to a compute
// partition (DPX 128, QPX 64, CPX 32 CUs).
inline double scale_floor_by_cus(double floor_full_gpu, int cus) {
  return floor_full_gpu > 0 && cus > 0 ? floor_full_gpu * std::fmin(1.0, cus / 256.0) : floor_full_gpu;
}

}  // namespace avk
