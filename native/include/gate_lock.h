// N7 gate lock: a node-local, per-GPU advisory lock that makes the counter
// gate's verdict independent of the operator's own concurrent GPU work.
//
// The AQL counters the gate reads are device-wide: any kernel another process
// runs on the GPU during the counted dispatch adds its waves and MFMA ops, and
// the gate's exact equalities (gate_policy.h) fail.  Round 5 met that with a
// retry loop (a plugin-validation pod's code-object upload landed inside the
// counted window on a CPU-throttled box, profiles/r5_final/gate_retry).  The
// operator's own GPU processes now take turns instead:
//
//   * the validator holds  gate-<bdf>.lock  EXCLUSIVELY around each counted
//     dispatch only (~1-5 ms);
//   * everything else the operator runs on that GPU - the plugin-validation
//     pod's code-object load and kernel (amdgpu-gpu-check), the RCCL
//     collectives of the validator's own processes - holds it SHARED around
//     its GPU work.
//
// The lock files live in the node's validations hostPath (the directory in
// AMDGPU_GATE_LOCK_DIR; unset: no locking), which the validator pods and the
// plugin-validation pod already mount.  flock(2) locks belong to the open file
// description, so two holders in one process (the gate and an RCCL thread)
// exclude each other like two processes, and a crashed holder's lock goes
// with its descriptor.  Acquisition polls with LOCK_NB and gives up after a
// bound (a wedged holder must not hang the validation): the caller then runs
// unlocked and reports it, and the gate's own verdict stays exact.
//
// Header-only: the validator, the pod check and the CPU tests
// (tests/test_gate_lock.py through amdgpu-validator --gate-lock-probe) share it.
#pragma once

#include <fcntl.h>
#include <sys/file.h>
#include <unistd.h>

#include <cctype>
#include <chrono>
#include <cstdlib>
#include <string>
#include <thread>
#include <utility>

namespace avk {

constexpr const char* kGateLockEnv = "AMDGPU_GATE_LOCK_DIR";

// "0000:75:00.0" (any case) -> "gate-0000-75-00-0.lock"
inline std::string gate_lock_name(const std::string& bdf) {
  std::string s = "gate-";
  for (char c : bdf) s += (c == ':' || c == '.') ? '-' : (char)std::tolower((unsigned char)c);
  return s + ".lock";
}

class GateLock {
 public:
  enum Mode { kShared, kExclusive };
  GateLock() = default;
  // Acquire the lock of GPU `bdf` in `dir` (empty: the AMDGPU_GATE_LOCK_DIR
  // env; none: a no-op lock).  Waits at most `timeout_s`.
  GateLock(const std::string& bdf, Mode mode, double timeout_s = 2.0, std::string dir = "") {
    if (dir.empty()) {
      const char* e = getenv(kGateLockEnv);
      if (!e || !*e) return;
      dir = e;
    }
    enabled_ = true;
    const std::string path = dir + "/" + gate_lock_name(bdf);
    fd_ = ::open(path.c_str(), O_RDWR | O_CREAT | O_CLOEXEC, 0666);
    if (fd_ < 0) return;
    const auto t0 = std::chrono::steady_clock::now();
    const int op = (mode == kExclusive ? LOCK_EX : LOCK_SH) | LOCK_NB;
    for (;;) {
      if (::flock(fd_, op) == 0) {
        held_ = true;
        break;
      }
      wait_s_ = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (wait_s_ >= timeout_s) break;
      std::this_thread::sleep_for(std::chrono::microseconds(100));
    }
    wait_s_ = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
  GateLock(const GateLock&) = delete;
  GateLock& operator=(const GateLock&) = delete;
  GateLock(GateLock&& o) noexcept { *this = std::move(o); }
  GateLock& operator=(GateLock&& o) noexcept {
    release();
    fd_ = o.fd_, held_ = o.held_, enabled_ = o.enabled_, wait_s_ = o.wait_s_;
    o.fd_ = -1, o.held_ = false;
    return *this;
  }
  ~GateLock() { release(); }

  void release() {
    if (fd_ >= 0) {
      if (held_) ::flock(fd_, LOCK_UN);
      ::close(fd_);
    }
    fd_ = -1;
    held_ = false;
  }
  bool enabled() const { return enabled_; }
  bool held() const { return held_; }
  double wait_s() const { return wait_s_; }
  // "off" (no lock dir), "held", or "timeout" (ran unlocked)
  const char* state() const { return !enabled_ ? "off" : held_ ? "held" : "timeout"; }

 private:
  int fd_ = -1;
  bool held_ = false;
  bool enabled_ = false;
  double wait_s_ = 0;
};

}  // namespace avk
