// N7 counter gate on AQL profiling packets (no profiler runtime in the process).
//
// The validator decides a node is Ready from correctness AND hardware
// evidence that the MFMA pipes executed.  The
// rocprofiler-sdk path (counter_gate.cpp) costs a gated process ~0.2 s before
// main and opens /dev/kfd as it loads (profiles/r2_ttr/startup_probe.json).
// This path asks the hardware directly, the way a profiler does underneath:
//
//   * the validator's own GEMM code object (the same default kernel the HIP
//     path launches, gemm_default.h; built device-only next to the binary) is
//     loaded into an HSA executable;
//   * libhsa-amd-aqlprofile64 builds the PM4 start/stop command buffers for
//     the four gfx950 counters of the gate (SQ_INSTS_VALU_MFMA_MOPS_BF16 =
//     SQ event 52, SQ_VALU_MFMA_BUSY_CYCLES = SQ 93, SQ_WAVES = SQ 4,
//     GRBM_GUI_ACTIVE = GRBM 2: one pass, the ids of ROCm 7.2's gfx950
//     counter definitions);
//   * one private HSA queue (profiling enabled) carries [PM4 start] [GEMM
//     dispatch] [PM4 stop] [PM4 read]; the read packet has the CP copy the
//     counters into the output buffer (without it every sample reads 0 on
//     gfx950), which aqlprofile's iterator then returns per block instance
//     (32 SQ samples, 8 GRBM samples on MI355X).
//
// Every packet is written before its header is published (release store),
// and the wait on the stop packet's signal is bounded: a gate that does not
// complete fails closed instead of blocking the validator.

#include "../include/aql_gate.h"
#include "../include/gemm_default.h"

#include <dlfcn.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <hsa/hsa_ven_amd_aqlprofile.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <algorithm>
#include <fstream>
#include <atomic>
#include <map>
#include <mutex>
#include <sstream>
#include <string>
#include <vector>

namespace {

using Clock = std::chrono::steady_clock;

double secs(Clock::time_point t0) { return std::chrono::duration<double>(Clock::now() - t0).count(); }

// Per gated GEMM (AVK_AQL_GATE_BF16 / _FP8): the kernel and the MOPS counter
// of its data type; the other three counters are the same.  Event ids of
// ROCm 7.2's gfx950 counter definitions (rocprofiler-sdk counter_defs.yaml):
// SQ_INSTS_VALU_MFMA_MOPS_BF16 52, SQ_INSTS_VALU_MFMA_MOPS_F8 56, _F6F4 57.
struct GateSpec {
  const char* symbol;
  const char* names[AVK_AQL_GATE_COUNTERS];
  hsa_ven_amd_aqlprofile_event_t events[AVK_AQL_GATE_COUNTERS];
};
const GateSpec kSpecs[AVK_AQL_GATE_DTYPES] = {
    {avk::kGemmSymbol,
     {"SQ_INSTS_VALU_MFMA_MOPS_BF16", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_WAVES", "GRBM_GUI_ACTIVE"},
     {{HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_SQ, 0, 52},
      {HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_SQ, 0, 93},
      {HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_SQ, 0, 4},
      {HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_GRBM, 0, 2}}},
    {avk::kGemmFp8Symbol,
     {"SQ_INSTS_VALU_MFMA_MOPS_F8", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_WAVES", "GRBM_GUI_ACTIVE"},
     {{HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_SQ, 0, 56},
      {HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_SQ, 0, 93},
      {HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_SQ, 0, 4},
      {HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_GRBM, 0, 2}}},
    {avk::kGemmFp4Symbol,
     {"SQ_INSTS_VALU_MFMA_MOPS_F6F4", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_WAVES", "GRBM_GUI_ACTIVE"},
     {{HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_SQ, 0, 57},
      {HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_SQ, 0, 93},
      {HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_SQ, 0, 4},
      {HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_GRBM, 0, 2}}},
    {avk::kGemmFp6Symbol,
     {"SQ_INSTS_VALU_MFMA_MOPS_F6F4", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_WAVES", "GRBM_GUI_ACTIVE"},
     {{HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_SQ, 0, 57},
      {HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_SQ, 0, 93},
      {HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_SQ, 0, 4},
      {HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_GRBM, 0, 2}}},
    {avk::kGemmMxFp4Symbol,
     {"SQ_INSTS_VALU_MFMA_MOPS_F6F4", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_WAVES", "GRBM_GUI_ACTIVE"},
     {{HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_SQ, 0, 57},
      {HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_SQ, 0, 93},
      {HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_SQ, 0, 4},
      {HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_GRBM, 0, 2}}},
};

struct Api {
  decltype(&hsa_ven_amd_aqlprofile_validate_event) validate_event = nullptr;
  decltype(&hsa_ven_amd_aqlprofile_start) start = nullptr;
  decltype(&hsa_ven_amd_aqlprofile_stop) stop = nullptr;
  decltype(&hsa_ven_amd_aqlprofile_read) read = nullptr;
  decltype(&hsa_ven_amd_aqlprofile_get_info) get_info = nullptr;
  decltype(&hsa_ven_amd_aqlprofile_iterate_data) iterate_data = nullptr;
  decltype(&hsa_ven_amd_aqlprofile_error_string) error_string = nullptr;

  bool load(std::string* err) {
    void* h = dlopen("libhsa-amd-aqlprofile64.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("/opt/rocm/lib/libhsa-amd-aqlprofile64.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) {
      *err = std::string("dlopen aqlprofile: ") + dlerror();
      return false;
    }
    validate_event = reinterpret_cast<decltype(validate_event)>(dlsym(h, "hsa_ven_amd_aqlprofile_validate_event"));
    start = reinterpret_cast<decltype(start)>(dlsym(h, "hsa_ven_amd_aqlprofile_start"));
    stop = reinterpret_cast<decltype(stop)>(dlsym(h, "hsa_ven_amd_aqlprofile_stop"));
    read = reinterpret_cast<decltype(read)>(dlsym(h, "hsa_ven_amd_aqlprofile_read"));
    get_info = reinterpret_cast<decltype(get_info)>(dlsym(h, "hsa_ven_amd_aqlprofile_get_info"));
    iterate_data = reinterpret_cast<decltype(iterate_data)>(dlsym(h, "hsa_ven_amd_aqlprofile_iterate_data"));
    error_string = reinterpret_cast<decltype(error_string)>(dlsym(h, "hsa_ven_amd_aqlprofile_error_string"));
    if (!validate_event || !start || !stop || !read || !get_info || !iterate_data) {
      *err = "aqlprofile: missing entry points";
      return false;
    }
    return true;
  }
};

struct AgentSearch {
  uint32_t domain = 0, bdfid = 0;
  int ordinal = 0;  // which of the GPU agents at this PCI address (compute partitions share it)
  int seen = 0;
  hsa_agent_t gpu{}, cpu{};
  bool gpu_ok = false, cpu_ok = false;
};

hsa_status_t find_agents(hsa_agent_t a, void* d) {
  auto* s = static_cast<AgentSearch*>(d);
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
  if (t == HSA_DEVICE_TYPE_CPU && !s->cpu_ok) {
    s->cpu = a;
    s->cpu_ok = true;
  } else if (t == HSA_DEVICE_TYPE_GPU && !s->gpu_ok) {
    uint32_t bdf = 0, dom = 0;
    hsa_agent_get_info(a, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_BDFID), &bdf);
    hsa_agent_get_info(a, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_DOMAIN), &dom);
    if (bdf == s->bdfid && dom == s->domain && s->seen++ == s->ordinal) {
      s->gpu = a;
      s->gpu_ok = true;
    }
  }
  return HSA_STATUS_SUCCESS;
}

// the CPU agent's kernarg pool: fine-grained system memory the CP reads (and,
// once the GPU is granted access, writes) coherently
hsa_status_t find_kernarg_pool(hsa_amd_memory_pool_t p, void* d) {
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
  const char* symbol = nullptr;  // substring of the mangled name to find
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
  if (name.find(k->symbol) == std::string::npos) return HSA_STATUS_SUCCESS;
  hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &k->object);
  hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &k->kernarg_size);
  hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &k->group_size);
  hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &k->private_size);
  return HSA_STATUS_INFO_BREAK;
}

struct Sums {
  const hsa_ven_amd_aqlprofile_event_t* events = nullptr;
  double values[AVK_AQL_GATE_COUNTERS] = {};
  int samples[AVK_AQL_GATE_COUNTERS] = {};
};

hsa_status_t collect(hsa_ven_amd_aqlprofile_info_type_t type, hsa_ven_amd_aqlprofile_info_data_t* info, void* d) {
  if (type != HSA_VEN_AMD_AQLPROFILE_INFO_PMC_DATA) return HSA_STATUS_SUCCESS;
  auto* s = static_cast<Sums*>(d);
  for (int i = 0; i < AVK_AQL_GATE_COUNTERS; ++i) {
    if (info->pmc_data.event.block_name == s->events[i].block_name &&
        info->pmc_data.event.counter_id == s->events[i].counter_id) {
      s->values[i] += static_cast<double>(info->pmc_data.result);
      s->samples[i] += 1;
    }
  }
  return HSA_STATUS_SUCCESS;
}

// AQL header of a packet with a barrier and system-scope fences
uint16_t header(hsa_packet_type_t type) {
  return static_cast<uint16_t>((type << HSA_PACKET_HEADER_TYPE) | (1 << HSA_PACKET_HEADER_BARRIER) |
                               (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                               (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE));
}

// publish a packet: its first 32 bits (header + next 16 bits) last, with release order
void publish(void* slot, uint16_t hdr, uint16_t next16) {
  __atomic_store_n(static_cast<uint32_t*>(slot), static_cast<uint32_t>(hdr) | (static_cast<uint32_t>(next16) << 16),
                   __ATOMIC_RELEASE);
}

bool read_file(const char* path, std::vector<char>* out) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return false;
  std::stringstream ss;
  ss << f.rdbuf();
  const std::string s = ss.str();
  out->assign(s.begin(), s.end());
  return !out->empty();
}

struct Fail {
  std::string msg;
};

decltype(&hsa_ven_amd_aqlprofile_error_string) g_aql_error = nullptr;

void check(hsa_status_t st, const char* what) {
  if (st != HSA_STATUS_SUCCESS && st != HSA_STATUS_INFO_BREAK) {
    const char* s = nullptr;
    hsa_status_string(st, &s);
    std::string msg = std::string(what) + ": " + (s ? s : "hsa error");
    const char* detail = nullptr;
    if (g_aql_error && g_aql_error(&detail) == HSA_STATUS_SUCCESS && detail && *detail)
      msg += std::string(" (aqlprofile: ") + detail + ")";
    throw Fail{msg};
  }
}

void* pool_alloc(hsa_amd_memory_pool_t pool, hsa_agent_t gpu, size_t bytes) {
  void* p = nullptr;
  bytes = (bytes + 4095) & ~size_t(4095);
  check(hsa_amd_memory_pool_allocate(pool, bytes, 0, &p), "pool allocate");
  check(hsa_amd_agents_allow_access(1, &gpu, nullptr, p), "allow access");
  memset(p, 0, bytes);
  return p;
}

// One per GPU agent (and code object), kept for the life of the process:
// aqlprofile, the agent lookup, the loaded executable with both gated GEMMs,
// the private queue and the counter buffers.  The validator gates the bf16
// GEMM, then the fp8 one (and retries a polluted count), so only the first
// gate of a process pays the set-up (~5 ms); the rest cost their dispatch.
// The queue is left to the process exit, like HIP's own.
struct Session {
  std::mutex m;
  // a dispatch that never completed: the queue is not reused.  Written under
  // the session's lock, read under g_sessions_m by session_for: atomic
  std::atomic<bool> broken{false};
  Api api;
  AgentSearch as;
  hsa_amd_memory_pool_t kpool{0};
  hsa_executable_t exe{0};
  hsa_code_object_reader_t reader{0};
  Kernel kern[AVK_AQL_GATE_DTYPES];
  hsa_queue_t* queue = nullptr;
  hsa_signal_t done{0};
  char* karg = nullptr;
  hsa_ven_amd_aqlprofile_profile_t prof[AVK_AQL_GATE_DTYPES]{};

  void open(const char* pci_bus_id, int agent_ordinal, const char* code_object) {
    unsigned dom = 0, bus = 0, dev = 0, fn = 0;
    if (!pci_bus_id || sscanf(pci_bus_id, "%x:%x:%x.%x", &dom, &bus, &dev, &fn) != 4)
      throw Fail{std::string("bad PCI bus id '") + (pci_bus_id ? pci_bus_id : "") + "'"};
    std::string e;
    if (!api.load(&e)) throw Fail{e};
    g_aql_error = api.error_string;
    check(hsa_init(), "hsa_init");  // reference-counted: HIP holds the runtime already
    as.domain = dom;
    as.bdfid = (bus << 8) | (dev << 3) | fn;
    as.ordinal = agent_ordinal;
    check(hsa_iterate_agents(find_agents, &as), "iterate agents");
    if (!as.gpu_ok || !as.cpu_ok) throw Fail{std::string("no HSA agent for ") + pci_bus_id};
    check(hsa_amd_agent_iterate_memory_pools(as.cpu, find_kernarg_pool, &kpool), "memory pools");
    if (!kpool.handle) throw Fail{"no kernarg memory pool"};
    // the GEMM kernels from the validator's device code object
    std::vector<char> co;
    if (!read_file(code_object, &co)) throw Fail{std::string("cannot read ") + code_object};
    check(hsa_code_object_reader_create_from_memory(co.data(), co.size(), &reader), "code object reader");
    check(hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr, &exe),
          "executable create");
    check(hsa_executable_load_agent_code_object(exe, as.gpu, reader, nullptr, nullptr), "load code object");
    check(hsa_executable_freeze(exe, nullptr), "executable freeze");
    uint32_t karg_size = 0;
    for (int d = 0; d < AVK_AQL_GATE_DTYPES; ++d) {
      kern[d].symbol = kSpecs[d].symbol;
      check(hsa_executable_iterate_agent_symbols(exe, as.gpu, find_kernel, &kern[d]), "kernel symbols");
      if (!kern[d].object) throw Fail{std::string("GEMM kernel ") + kSpecs[d].symbol + " not in the code object"};
      if (kern[d].kernarg_size < 36) throw Fail{"unexpected GEMM kernarg layout"};
      karg_size = std::max(karg_size, kern[d].kernarg_size);
    }
    karg = static_cast<char*>(pool_alloc(kpool, as.gpu, karg_size));
    check(hsa_queue_create(as.gpu, 64, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &queue),
          "queue create");
    check(hsa_amd_profiling_set_profiler_enabled(queue, 1), "queue profiling");
    check(hsa_signal_create(1, 0, nullptr, &done), "signal create");
  }

  // the counter profile of `d` (command and output buffers), on first use
  hsa_ven_amd_aqlprofile_profile_t& profile(int d) {
    auto& p = prof[d];
    if (p.command_buffer.ptr) return p;
    const auto* ev = kSpecs[d].events;
    for (int i = 0; i < AVK_AQL_GATE_COUNTERS; ++i) {
      bool ok = false;
      check(api.validate_event(as.gpu, &ev[i], &ok), "validate event");
      if (!ok) throw Fail{std::string("aqlprofile rejects ") + kSpecs[d].names[i] + " on this agent"};
    }
    p.agent = as.gpu;
    p.type = HSA_VEN_AMD_AQLPROFILE_EVENT_TYPE_PMC;
    p.events = ev;
    p.event_count = AVK_AQL_GATE_COUNTERS;
    uint32_t cmd_size = 0, out_size = 0;
    check(api.get_info(&p, HSA_VEN_AMD_AQLPROFILE_INFO_COMMAND_BUFFER_SIZE, &cmd_size), "command buffer size");
    check(api.get_info(&p, HSA_VEN_AMD_AQLPROFILE_INFO_PMC_DATA_SIZE, &out_size), "output buffer size");
    // gfx950, ROCm 7.2: start() refuses the four-counter profile with the
    // sizes get_info reports (any one or two counters pass); 4x both is
    // accepted, and costs 56 KiB of host memory
    cmd_size *= 4;
    out_size *= 4;
    p.command_buffer.ptr = pool_alloc(kpool, as.gpu, cmd_size);
    p.command_buffer.size = cmd_size;
    p.output_buffer.ptr = pool_alloc(kpool, as.gpu, out_size);
    p.output_buffer.size = out_size;
    return p;
  }

  // aqlprofile refused the profile: name the counters (and pairs) it refuses
  std::string refused(int d, const hsa_ven_amd_aqlprofile_profile_t& p) {
    const auto* ev = kSpecs[d].events;
    std::string bad;
    for (int i = 0; i < AVK_AQL_GATE_COUNTERS; ++i) {
      hsa_ven_amd_aqlprofile_profile_t one = p;
      one.events = &ev[i];
      one.event_count = 1;
      hsa_ext_amd_aql_pm4_packet_t pk{};
      if (api.start(&one, &pk) != HSA_STATUS_SUCCESS) bad += std::string(bad.empty() ? "" : ",") + kSpecs[d].names[i];
    }
    std::string pairs;
    for (int i = 0; i < AVK_AQL_GATE_COUNTERS; ++i)
      for (int j = i + 1; j < AVK_AQL_GATE_COUNTERS; ++j) {
        hsa_ven_amd_aqlprofile_event_t two[2] = {ev[i], ev[j]};
        hsa_ven_amd_aqlprofile_profile_t p2 = p;
        p2.events = two;
        p2.event_count = 2;
        hsa_ext_amd_aql_pm4_packet_t pk{};
        if (api.start(&p2, &pk) != HSA_STATUS_SUCCESS)
          pairs += std::string(pairs.empty() ? "" : ",") + std::to_string(i) + "+" + std::to_string(j);
      }
    return "aqlprofile start refused the profile; single-counter profiles refused: " +
           (bad.empty() ? std::string("none") : bad) + "; pairs refused: " + (pairs.empty() ? "none" : pairs) +
           " (cmd " + std::to_string(p.command_buffer.size) + " B, out " + std::to_string(p.output_buffer.size) + " B)";
  }
};

std::mutex g_sessions_m;
std::map<std::string, Session*> g_sessions;  // by "bus/ordinal/code object"; never freed (process lifetime)

// The open session of an agent and code object, opened here on first use.
// A caller that finds the session being opened (avk_aql_gate_prepare on
// another thread) waits for it on the lock.
Session* session_for(const char* pci_bus_id, int agent_ordinal, const char* code_object) {
  const std::string key = std::string(pci_bus_id ? pci_bus_id : "") + "/" + std::to_string(agent_ordinal) + "/" +
                          (code_object ? code_object : "");
  std::lock_guard<std::mutex> l(g_sessions_m);
  auto it = g_sessions.find(key);
  if (it != g_sessions.end() && it->second->broken) g_sessions.erase(it), it = g_sessions.end();
  if (it == g_sessions.end()) {
    auto* fresh = new Session;
    try {
      fresh->open(pci_bus_id, agent_ordinal, code_object);
    } catch (...) {
      delete fresh;  // a half-open session is not kept (its HSA objects go with the process)
      throw;
    }
    it = g_sessions.emplace(key, fresh).first;
  }
  return it->second;
}

}  // namespace

extern "C" int avk_aql_gate_prepare(const char* pci_bus_id, int agent_ordinal, const char* code_object, char* err,
                                    int errlen) {
  try {
    Session* ss = session_for(pci_bus_id, agent_ordinal, code_object);
    std::lock_guard<std::mutex> l(ss->m);
    for (int d = 0; d < AVK_AQL_GATE_DTYPES; ++d) ss->profile(d);
    return 0;
  } catch (const Fail& f) {
    if (err && errlen > 0) snprintf(err, errlen, "%s", f.msg.c_str());
  }
  return -1;
}

extern "C" const char* avk_aql_gate_counter_name(int i) {
  return (i >= 0 && i < AVK_AQL_GATE_COUNTERS) ? kSpecs[0].names[i] : "";
}

extern "C" const char* avk_aql_gate_counter_name_dtype(int dtype, int i) {
  return (dtype >= 0 && dtype < AVK_AQL_GATE_DTYPES && i >= 0 && i < AVK_AQL_GATE_COUNTERS) ? kSpecs[dtype].names[i]
                                                                                            : "";
}

extern "C" int avk_aql_gate_gemm(const char* pci_bus_id, int agent_ordinal, const void* A, const void* Bt, void* C,
                                 int M, int N, int K, const char* code_object, double timeout_s,
                                 avk_aql_gate_result* out, char* err, int errlen) {
  return avk_aql_gate_gemm_dtype(AVK_AQL_GATE_BF16, pci_bus_id, agent_ordinal, A, Bt, C, M, N, K, code_object,
                                 timeout_s, out, err, errlen);
}

extern "C" int avk_aql_gate_gemm_dtype(int dtype, const char* pci_bus_id, int agent_ordinal, const void* A,
                                       const void* Bt, void* C, int M, int N, int K, const char* code_object,
                                       double timeout_s, avk_aql_gate_result* out, char* err, int errlen) {
  return avk_aql_gate_gemm_scaled(dtype, pci_bus_id, agent_ordinal, A, Bt, C, M, N, K, nullptr, nullptr, code_object,
                                  timeout_s, out, err, errlen);
}

extern "C" int avk_aql_gate_gemm_scaled(int dtype, const char* pci_bus_id, int agent_ordinal, const void* A,
                                        const void* Bt, void* C, int M, int N, int K, const void* SA, const void* SB,
                                        const char* code_object, double timeout_s, avk_aql_gate_result* out,
                                        char* err, int errlen) {
  const int d = dtype >= 0 && dtype < AVK_AQL_GATE_DTYPES ? dtype : 0;
  const auto t0 = Clock::now();
  memset(out, 0, sizeof(*out));
  try {
    if (M <= 0 || N <= 0 || K <= 0 || M % 256 || N % 256 || K % 256) throw Fail{"M, N, K must be multiples of 256"};
    Session* ss = session_for(pci_bus_id, agent_ordinal, code_object);
    std::lock_guard<std::mutex> l(ss->m);
    auto& prof = ss->profile(d);
    memset(prof.output_buffer.ptr, 0, prof.output_buffer.size);
    hsa_ext_amd_aql_pm4_packet_t start{}, stop{}, rd{};
    if (ss->api.start(&prof, &start) != HSA_STATUS_SUCCESS) throw Fail{ss->refused(d, prof)};
    check(ss->api.stop(&prof, &stop), "aqlprofile stop");
    check(ss->api.read(&prof, &rd), "aqlprofile read");
    const Kernel& kern = ss->kern[d];
    // kernel arguments: (const T* A, const T* Bt, void* C, int M, int N, int K)
    char* karg = ss->karg;
    memcpy(karg + 0, &A, 8);
    memcpy(karg + 8, &Bt, 8);
    memcpy(karg + 16, &C, 8);
    memcpy(karg + 24, &M, 4);
    memcpy(karg + 28, &N, 4);
    memcpy(karg + 32, &K, 4);
    if (d == AVK_AQL_GATE_MXFP4) {  // (..., int K, const uint8_t* SA, const uint8_t* SB)
      if (!SA || !SB || kern.kernarg_size < 56) throw Fail{"MX gate: scale arrays or kernarg layout missing"};
      memcpy(karg + 40, &SA, 8);
      memcpy(karg + 48, &SB, 8);
    }
    hsa_queue_t* queue = ss->queue;
    hsa_signal_store_relaxed(ss->done, 1);
    out->setup_s = secs(t0);

    // [PM4 start] [GEMM] [PM4 stop] [PM4 read -> done]: bodies first, headers last, in order
    const uint64_t npk = 4;
    const uint64_t idx = hsa_queue_add_write_index_relaxed(queue, npk);
    auto slot = [&](uint64_t i) {
      return static_cast<char*>(queue->base_address) + (i & (queue->size - 1)) * 64;
    };
    auto* p0 = reinterpret_cast<hsa_ext_amd_aql_pm4_packet_t*>(slot(idx));
    auto* p1 = reinterpret_cast<hsa_kernel_dispatch_packet_t*>(slot(idx + 1));
    auto* p2 = reinterpret_cast<hsa_ext_amd_aql_pm4_packet_t*>(slot(idx + 2));
    auto* p3 = reinterpret_cast<hsa_ext_amd_aql_pm4_packet_t*>(slot(idx + 3));
    memcpy(reinterpret_cast<char*>(p0) + 4, reinterpret_cast<char*>(&start) + 4, 60);
    p0->completion_signal.handle = 0;
    memset(reinterpret_cast<char*>(p1) + 4, 0, 60);
    const int nwg = (M / 256) * (N / 256);
    p1->workgroup_size_x = avk::kGemmThreads;
    p1->workgroup_size_y = 1;
    p1->workgroup_size_z = 1;
    p1->grid_size_x = static_cast<uint32_t>(nwg) * static_cast<uint32_t>(avk::kGemmThreads);
    p1->grid_size_y = 1;
    p1->grid_size_z = 1;
    p1->private_segment_size = kern.private_size;
    p1->group_segment_size = kern.group_size;
    p1->kernel_object = kern.object;
    p1->kernarg_address = karg;
    p1->completion_signal.handle = 0;
    memcpy(reinterpret_cast<char*>(p2) + 4, reinterpret_cast<char*>(&stop) + 4, 60);
    p2->completion_signal.handle = 0;
    memcpy(reinterpret_cast<char*>(p3) + 4, reinterpret_cast<char*>(&rd) + 4, 60);
    p3->completion_signal = ss->done;
    const auto t1 = Clock::now();
    publish(p0, header(HSA_PACKET_TYPE_VENDOR_SPECIFIC), start.pm4_command[0]);
    publish(p1, header(HSA_PACKET_TYPE_KERNEL_DISPATCH), 1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS);
    publish(p2, header(HSA_PACKET_TYPE_VENDOR_SPECIFIC), stop.pm4_command[0]);
    publish(p3, header(HSA_PACKET_TYPE_VENDOR_SPECIFIC), rd.pm4_command[0]);
    hsa_signal_store_screlease(queue->doorbell_signal, static_cast<hsa_signal_value_t>(idx + npk - 1));
    while (hsa_signal_wait_scacquire(ss->done, HSA_SIGNAL_CONDITION_LT, 1, 1000000, HSA_WAIT_STATE_BLOCKED) >= 1) {
      if (secs(t1) > timeout_s) {
        ss->broken = true;  // its packets may still run: a later gate opens a new session
        throw Fail{"counter gate: dispatch did not complete"};
      }
    }
    out->dispatch_s = secs(t1);
    Sums sums;
    sums.events = kSpecs[d].events;
    check(ss->api.iterate_data(&prof, collect, &sums), "iterate counter data");
    for (int i = 0; i < AVK_AQL_GATE_COUNTERS; ++i) {
      out->values[i] = sums.values[i];
      out->samples[i] = sums.samples[i];
    }
    return 0;
  } catch (const Fail& f) {
    snprintf(err, errlen, "%s", f.msg.c_str());
  }
  return -1;
}
