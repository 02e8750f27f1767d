// amdgpu-gpu-check: the plugin-validation pod's GPU check, on the HSA runtime
// alone.
//
// The pod proves the device-plugin path: the kubelet allocated the GPUs
// through the plugin, the runtime (OCI hook / CDI / device specs) put their
// device nodes into the container, and each one runs a kernel from inside it.
// The reference's equivalent is a CUDA vectorAdd sample pod
// (/root/reference/README.md:199).  The full HIP + MFMA + HBM + RCCL check of
// every GPU already ran outside the pod (amdgpu-validator); here a kernel
// launch per device is the point, and the HIP runtime's start-up (comgr, the
// runtime's own blit kernels, a context per device) is not: this binary links
// libhsa-runtime64 only, loads the validator's own gfx950 code object
// (validator_kernels.co, next to the binary) and per visible GPU agent
//
//   creates a queue, dispatches avk_gpu_check_add on 64 Ki floats in
//   fine-grained system memory the GPU was granted, waits (bounded) and checks
//   every element on the host.
//
// The devices are checked concurrently, one thread each: a pod holding all 8
// GPUs of a node (one pod per resource, validator/validate.py) would
// otherwise load the code object and create a queue 8 times in a row
// (~10 ms each on MI355X) on the bring-up's critical path.
//
// Output: one JSON line in the validator's report shape ({"ok", "seconds",
// "steps": [{"name": "hsa" | "vecadd", "device": d, ...}]}); exit 0 when every
// device passed.  A dispatch that does not complete within --timeout fails
// the check; its queue, signal, code object and buffers are left to the
// process exit.
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <unistd.h>

#include "gate_lock.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <fstream>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

namespace {

using Clock = std::chrono::steady_clock;
double secs(Clock::time_point t0) { return std::chrono::duration<double>(Clock::now() - t0).count(); }

const char* kKernel = "avk_gpu_check_add";

struct Fail {
  std::string msg;
};

void check(hsa_status_t st, const char* what) {
  if (st != HSA_STATUS_SUCCESS && st != HSA_STATUS_INFO_BREAK) {
    const char* s = nullptr;
    hsa_status_string(st, &s);
    throw Fail{std::string(what) + ": " + (s ? s : "hsa error")};
  }
}

struct Agents {
  std::vector<hsa_agent_t> gpus;
  hsa_agent_t cpu{};
  bool cpu_ok = false;
};

hsa_status_t find_agents(hsa_agent_t a, void* d) {
  auto* s = static_cast<Agents*>(d);
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
  if (t == HSA_DEVICE_TYPE_GPU) s->gpus.push_back(a);
  if (t == HSA_DEVICE_TYPE_CPU && !s->cpu_ok) {
    s->cpu = a;
    s->cpu_ok = true;
  }
  return HSA_STATUS_SUCCESS;
}

// fine-grained system memory (the CPU agent's kernarg pool): kernel arguments
// and the check's operands, which the host fills and verifies directly
hsa_status_t find_fine_pool(hsa_amd_memory_pool_t p, void* d) {
  hsa_amd_segment_t seg;
  if (hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg) != HSA_STATUS_SUCCESS ||
      seg != HSA_AMD_SEGMENT_GLOBAL)
    return HSA_STATUS_SUCCESS;
  uint32_t flags = 0;
  hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
  if (flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_KERNARG_INIT) {
    *static_cast<hsa_amd_memory_pool_t*>(d) = p;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

struct Kernel {
  uint64_t object = 0;
  uint32_t kernarg_size = 0, group_size = 0, private_size = 0;
};

hsa_status_t find_kernel(hsa_executable_t, hsa_agent_t, hsa_executable_symbol_t sym, void* d) {
  auto* k = static_cast<Kernel*>(d);
  hsa_symbol_kind_t kind;
  if (hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_TYPE, &kind) != HSA_STATUS_SUCCESS ||
      kind != HSA_SYMBOL_KIND_KERNEL)
    return HSA_STATUS_SUCCESS;
  uint32_t len = 0;
  hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_NAME_LENGTH, &len);
  std::string name(len, '\0');
  hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_NAME, name.data());
  if (name != std::string(kKernel) + ".kd" && name != kKernel) return HSA_STATUS_SUCCESS;
  hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &k->object);
  hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &k->kernarg_size);
  hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &k->group_size);
  hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &k->private_size);
  return HSA_STATUS_INFO_BREAK;
}

void* alloc(hsa_amd_memory_pool_t pool, hsa_agent_t gpu, size_t bytes) {
  void* p = nullptr;
  bytes = (bytes + 4095) & ~size_t(4095);
  check(hsa_amd_memory_pool_allocate(pool, bytes, 0, &p), "pool allocate");
  check(hsa_amd_agents_allow_access(1, &gpu, nullptr, p), "allow access");
  return p;
}

std::string exe_dir() {
  char buf[4096];
  ssize_t n = readlink("/proc/self/exe", buf, sizeof(buf) - 1);
  if (n <= 0) return "./";
  buf[n] = 0;
  std::string s(buf);
  return s.substr(0, s.rfind('/') + 1);
}

std::string fmt_step(const char* name, int dev, bool ok, double s, const std::string& detail) {
  char b[256];
  snprintf(b, sizeof b, "{\"name\": \"%s\", \"device\": %d, \"ok\": %s, \"seconds\": %.4f", name, dev,
           ok ? "true" : "false", s);
  return std::string(b) + (detail.empty() ? "" : ", " + detail) + "}";
}

// the agent's PCI address, as the validator names it (hipDeviceGetPCIBusId)
std::string agent_bdf(hsa_agent_t gpu) {
  uint32_t bdf = 0, domain = 0;
  hsa_agent_get_info(gpu, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_BDFID), &bdf);
  hsa_agent_get_info(gpu, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_DOMAIN), &domain);
  char b[32];
  snprintf(b, sizeof b, "%04x:%02x:%02x.%x", domain & 0xffff, (bdf >> 8) & 0xff, (bdf >> 3) & 0x1f, bdf & 0x7);
  return b;
}

// What one device's check holds until its teardown (DeviceRes::release),
// which runs after the report is out: the queue, the executable and the
// buffers, and the GPU's gate lock (gate_lock.h) taken before the code-object
// load.  The lock covers the upload, the queue creation and the kernel - the
// pod's GPU work a counted window of the validator must not see - and is let
// go before the teardown: a queue destruction in a counted window shows as
// the preemption signature and that attempt is counted again
// (validator_main.cpp aql_gate), which costs less than every first gate
// waiting out the teardown (interleaved A/B, 40 pairs: time-to-Ready median
// 0.2415 against 0.2517 s, the validator process 0.140 against 0.153 s, gate
// retries 18 against 9 of 200, none past a second attempt:
// profiles/r6_unlock).  AMDGPU_GPU_CHECK_LOCK_TEARDOWN=1 keeps the lock
// through the teardown (the A/B's other arm).
struct DeviceRes {
  avk::GateLock lock;
  hsa_code_object_reader_t reader{0};
  hsa_executable_t exe{0};
  hsa_queue_t* queue = nullptr;
  hsa_signal_t done{0};
  std::vector<void*> allocs;
  bool dispatched = false, finished = false;

  // A dispatch that did not finish may still be running (slow, not dead): its
  // queue, completion signal, code object and buffers all stay until the
  // process exit, so the kernel never runs from freed code or signals freed
  // memory.  (A failure before the dispatch left nothing in flight.)
  void release(bool unlock_first) {
    if (unlock_first) lock.release();
    if (!(dispatched && !finished)) {
      if (queue) hsa_queue_destroy(queue);
      if (done.handle) hsa_signal_destroy(done);
      if (exe.handle) hsa_executable_destroy(exe);
      if (reader.handle) hsa_code_object_reader_destroy(reader);
      for (void* q : allocs) hsa_amd_memory_pool_free(q);
    }
    queue = nullptr;
    done.handle = exe.handle = reader.handle = 0;
    allocs.clear();
    lock.release();  // (a no-op once let go above)
  }
};

// one device: queue, dispatch, verify; appends its step records and leaves
// what it holds in `res` for DeviceRes::release.  `loop_s` > 0 (tests): keep
// dispatching the kernel for that long, the lock released between dispatches.
bool check_device(int d, hsa_agent_t gpu, hsa_amd_memory_pool_t pool, const std::vector<char>& co, int n,
                  double timeout_s, std::vector<std::string>* steps, std::string* error, double loop_s,
                  DeviceRes* res) {
  const auto t0 = Clock::now();
  const std::string bdf = agent_bdf(gpu);
  avk::GateLock& lock = res->lock;
  lock = avk::GateLock(bdf, avk::GateLock::kShared, 2.0);
  hsa_code_object_reader_t& reader = res->reader;
  hsa_executable_t& exe = res->exe;
  hsa_queue_t*& queue = res->queue;
  hsa_signal_t& done = res->done;
  std::vector<void*>& allocs = res->allocs;
  bool& dispatched = res->dispatched;
  bool& finished = res->finished;
  bool ok = false;
  char agent_name[64] = {0};
  try {
    hsa_agent_get_info(gpu, HSA_AGENT_INFO_NAME, agent_name);
    check(hsa_code_object_reader_create_from_memory(co.data(), co.size(), &reader), "code object reader");
    check(hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr, &exe),
          "executable create");
    check(hsa_executable_load_agent_code_object(exe, gpu, reader, nullptr, nullptr), "load code object");
    check(hsa_executable_freeze(exe, nullptr), "executable freeze");
    const double co_load_s = secs(t0);
    Kernel k;
    check(hsa_executable_iterate_agent_symbols(exe, gpu, find_kernel, &k), "kernel symbols");
    if (!k.object) throw Fail{std::string(kKernel) + " not in the code object for " + agent_name};
    if (k.kernarg_size < 28) throw Fail{"unexpected kernarg layout"};
    const auto tq = Clock::now();
    check(hsa_queue_create(gpu, 64, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &queue),
          "queue create");
    const double queue_s = secs(tq);
    check(hsa_signal_create(1, 0, nullptr, &done), "signal create");
    auto* a = static_cast<float*>(alloc(pool, gpu, n * 4));
    auto* b = static_cast<float*>(alloc(pool, gpu, n * 4));
    auto* c = static_cast<float*>(alloc(pool, gpu, n * 4));
    char* karg = static_cast<char*>(alloc(pool, gpu, k.kernarg_size));
    allocs = {a, b, c, karg};
    for (int i = 0; i < n; ++i) {
      a[i] = (float)(i % 1024) * 0.5f;
      b[i] = (float)(d + 1) * 0.25f;
      c[i] = -1.0f;
    }
    memset(karg, 0, k.kernarg_size);
    memcpy(karg + 0, &a, 8);
    memcpy(karg + 8, &b, 8);
    memcpy(karg + 16, &c, 8);
    memcpy(karg + 24, &n, 4);
    char tdet[160];
    snprintf(tdet, sizeof tdet, "\"co_load_s\": %.4f, \"queue_s\": %.4f, \"gate_lock\": \"%s\", \"gate_lock_wait_s\": %.4f, ",
             co_load_s, queue_s, lock.state(), lock.wait_s());
    steps->push_back(fmt_step("hsa", d, true, secs(t0), std::string(tdet) + "\"bdf\": \"" + bdf + "\", \"agent\": \"" +
                                                            agent_name + "\""));

    const auto t1 = Clock::now();
    int dispatches = 0;
    for (;;) {
      ++dispatches;
      const uint64_t idx = hsa_queue_add_write_index_relaxed(queue, 1);
      auto* p = reinterpret_cast<hsa_kernel_dispatch_packet_t*>(static_cast<char*>(queue->base_address) +
                                                                (idx & (queue->size - 1)) * 64);
      memset(reinterpret_cast<char*>(p) + 4, 0, 60);
      p->workgroup_size_x = 256;
      p->workgroup_size_y = 1;
      p->workgroup_size_z = 1;
      p->grid_size_x = static_cast<uint32_t>((n + 255) / 256) * 256u;
      p->grid_size_y = 1;
      p->grid_size_z = 1;
      p->private_segment_size = k.private_size;
      p->group_segment_size = k.group_size;
      p->kernel_object = k.object;
      p->kernarg_address = karg;
      p->completion_signal = done;
      const uint16_t hdr = static_cast<uint16_t>((HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                                                 (1 << HSA_PACKET_HEADER_BARRIER) |
                                                 (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                                                 (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE));
      __atomic_store_n(reinterpret_cast<uint32_t*>(p),
                       static_cast<uint32_t>(hdr) |
                           (static_cast<uint32_t>(1u << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS) << 16),
                       __ATOMIC_RELEASE);
      hsa_signal_store_screlease(queue->doorbell_signal, static_cast<hsa_signal_value_t>(idx));
      dispatched = true;
      while (hsa_signal_wait_scacquire(done, HSA_SIGNAL_CONDITION_LT, 1, 1000000, HSA_WAIT_STATE_BLOCKED) >= 1)
        if (secs(t1) > timeout_s + loop_s) throw Fail{"dispatch did not complete within the timeout"};
      if (secs(t1) >= loop_s) break;
      // --loop-seconds: the lock is released between dispatches, so a gate waits one kernel at most
      lock.release();
      std::this_thread::sleep_for(std::chrono::microseconds(500));
      lock = avk::GateLock(bdf, avk::GateLock::kShared, 2.0);
      hsa_signal_store_relaxed(done, 1);
    }
    finished = true;
    int bad = 0;
    for (int i = 0; i < n; ++i)
      if (c[i] != a[i] + b[i]) ++bad;
    ok = bad == 0;
    char det[96];
    snprintf(det, sizeof det, "\"elems\": %d, \"mismatches\": %d, \"dispatches\": %d", n, bad, dispatches);
    steps->push_back(fmt_step("vecadd", d, ok, secs(t1), det));
    if (!ok) *error = "device " + std::to_string(d) + ": " + std::to_string(bad) + " wrong elements";
  } catch (const Fail& f) {
    *error = "device " + std::to_string(d) + ": " + f.msg;
    steps->push_back(fmt_step("vecadd", d, false, secs(t0), ""));
  }
  return ok;
}

}  // namespace

int main(int argc, char** argv) {
  const auto t0 = Clock::now();
  double timeout_s = 10.0;
  int elems = 1 << 16;
  int expect = -1;  // --expect-devices: the GPUs the kubelet allocated to this pod
  std::string result_file;  // --result-file: the report, also written here (validate.py reads it)
  double loop_s = 0;  // --loop-seconds (tests): dispatch continuously for this long
  for (int i = 1; i < argc; ++i) {
    std::string k = argv[i];
    if (k == "--timeout" && i + 1 < argc) timeout_s = atof(argv[++i]);
    else if (k == "--result-file" && i + 1 < argc) result_file = argv[++i];
    else if (k == "--elems" && i + 1 < argc) elems = atoi(argv[++i]);
    else if (k == "--expect-devices" && i + 1 < argc) expect = atoi(argv[++i]);
    else if (k == "--loop-seconds" && i + 1 < argc) loop_s = atof(argv[++i]);
    else if (k == "--help" || k == "-h") {
      fprintf(stderr, "usage: amdgpu-gpu-check [--timeout S] [--elems N] [--expect-devices N] [--result-file PATH]"
                      " [--loop-seconds S]   (every visible GPU; gate locks in $AMDGPU_GATE_LOCK_DIR)\n");
      return 2;
    }
    // other flags (the validator's pod arguments) are accepted and ignored
  }
  if (elems < 256 || elems > (1 << 24) || loop_s < 0 || loop_s > 600) {
    fprintf(stderr, "amdgpu-gpu-check: --elems must be in [256, 2^24], --loop-seconds in [0, 600]\n");
    return 2;
  }
  std::vector<std::string> steps;
  std::string error;
  bool ok = true;
  int ngpu = 0;
  std::vector<DeviceRes> dev_res;  // each GPU's queue, executable, buffers and gate lock (check_device)
  double hsa_init_s = -1;
  try {
    const auto th = Clock::now();
    check(hsa_init(), "hsa_init");
    hsa_init_s = secs(th);
    Agents ag;
    check(hsa_iterate_agents(find_agents, &ag), "iterate agents");
    ngpu = (int)ag.gpus.size();
    if (ag.gpus.empty()) throw Fail{"no GPU agent visible in this container"};
    // every allocated device must have been put into the container: a device
    // the runtime hook or CDI spec left out is a failed check, not a pass on
    // the ones that are there
    if (expect >= 0 && ngpu != expect)
      throw Fail{std::to_string(expect) + " GPU(s) allocated to the pod, " + std::to_string(ngpu) + " visible"};
    if (!ag.cpu_ok) throw Fail{"no CPU agent"};
    hsa_amd_memory_pool_t pool{0};
    check(hsa_amd_agent_iterate_memory_pools(ag.cpu, find_fine_pool, &pool), "memory pools");
    if (!pool.handle) throw Fail{"no fine-grained system memory pool"};
    const std::string path = exe_dir() + "validator_kernels.co";
    std::ifstream f(path, std::ios::binary);
    std::stringstream ss;
    ss << f.rdbuf();
    const std::string text = ss.str();
    if (!f || text.empty()) throw Fail{"cannot read " + path};
    const std::vector<char> co(text.begin(), text.end());
    std::vector<std::vector<std::string>> dev_steps(ngpu);
    std::vector<std::string> dev_error(ngpu);
    std::vector<char> dev_ok(ngpu, 0);
    dev_res.resize(ngpu);
    std::vector<std::thread> threads;
    threads.reserve(ngpu);
    for (int d = 0; d < ngpu; ++d)
      threads.emplace_back([&, d] {
        try {  // nothing may leave a thread (std::terminate): an unexpected error fails this device only
          dev_ok[d] = check_device(d, ag.gpus[d], pool, co, elems, timeout_s, &dev_steps[d], &dev_error[d], loop_s,
                                   &dev_res[d]);
        } catch (const std::exception& e) {
          dev_error[d] = "device " + std::to_string(d) + ": " + e.what();
        } catch (...) {
          dev_error[d] = "device " + std::to_string(d) + ": unexpected error";
        }
      });
    for (auto& t : threads) t.join();
    for (int d = 0; d < ngpu; ++d) {  // report in device order; the first failing device names the error
      steps.insert(steps.end(), dev_steps[d].begin(), dev_steps[d].end());
      if (!dev_ok[d] && ok) {
        ok = false;
        error = dev_error[d];
      }
    }
  } catch (const Fail& f) {
    ok = false;
    error = f.msg;
  }
  std::string out = "{\"ok\": " + std::string(ok ? "true" : "false") + ", \"devices\": " + std::to_string(ngpu);
  char b[96];
  // t_main: CLOCK_MONOTONIC at main (steady_clock), comparable with a parent's time.monotonic()
  snprintf(b, sizeof b, ", \"seconds\": %.4f, \"hsa_init_s\": %.4f, \"t_main\": %.6f", secs(t0), hsa_init_s,
           std::chrono::duration<double>(t0.time_since_epoch()).count());
  out += b;
  if (!error.empty()) {
    std::string esc;
    for (char c : error) esc += (c == '"' || c == '\\') ? '\'' : c;
    out += ", \"error\": \"" + esc + "\"";
  }
  out += ", \"steps\": [";
  for (size_t i = 0; i < steps.size(); ++i) out += (i ? ", " : "") + steps[i];
  out += "]}";
  puts(out.c_str());
  fflush(stdout);
  // --result-file: the same report in a file of the node's validation
  // directory (a hostPath the validator watches), published by rename.  The
  // pod's exit - the kernel releasing this process's GPU state, ~50 ms
  // (pod_exit_probe) - is then no longer between the check and
  // the validator seeing its result; the kubelet still reports the pod's end.
  if (!result_file.empty()) {
    const std::string tmp = result_file + ".tmp";
    if (FILE* rf = fopen(tmp.c_str(), "w")) {
      const bool wrote = fputs(out.c_str(), rf) >= 0;
      if (fclose(rf) == 0 && wrote) rename(tmp.c_str(), result_file.c_str());
    }
  }
  // The report is out: now each device's queue, executable and buffers go
  // (DeviceRes::release; ~7.5 ms a device, which the report no longer waits
  // for), the gate lock let go first.  Devices in parallel, as their checks ran.
  {
    std::vector<std::thread> rel;
    rel.reserve(dev_res.size());
    const char* lt = getenv("AMDGPU_GPU_CHECK_LOCK_TEARDOWN");
    const bool unlock_first = !(lt && lt[0] == '1');
    for (auto& r : dev_res) rel.emplace_back([&r, unlock_first] { r.release(unlock_first); });
    for (auto& t : rel) t.join();
  }
  // the report is the result: the runtime's teardown is left to the exit
  // (AMDGPU_GPU_CHECK_SHUTDOWN=1: hsa_shut_down first - tools/pod_exit_probe.py
  // A/B).  Holding the gate locks through hsa_shut_down kept its queue
  // unmaps out of the validator's counted windows, but made the first gate
  // wait 21-42 ms for it (+30 ms time-to-Ready, profiles/r6_gate_lock): the
  // gate retries a window with evidence of preemption instead
  // (validator_main.cpp aql_gate)
  if (const char* e = getenv("AMDGPU_GPU_CHECK_SHUTDOWN"); ok && e && e[0] == '1') hsa_shut_down();
  _exit(ok ? 0 : 1);
}
