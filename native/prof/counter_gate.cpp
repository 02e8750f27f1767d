// N7: in-process rocprofiler-sdk counter gate for the validator binary.
//
// The validator decides a node is Ready from correctness AND hardware
// evidence that the MFMA pipes executed: it reads
// per-dispatch PMC counters of its own GEMM through the rocprofiler-sdk
// dispatch counting service.  Built as libamdgpu_counter_gate.so: a
// rocprofiler-sdk tool library loaded through ROCP_TOOL_LIBRARIES (the
// validator sets it for gated runs before its first HIP call; the operator
// sets it in the pod env).  Its `rocprofiler_configure` entry point activates
// the tool only when AMDGPU_VALIDATOR_COUNTERS=1 (otherwise it returns null
// and the process runs unprofiled, e.g. under an outer rocprofv3).
//
// gfx950 has no derived-counter XML in ROCm 7.2 (MI355X_MICROARCH.md
// §rocprofv3 PMC slots), so only raw counters are requested:
// SQ_INSTS_VALU_MFMA_MOPS_BF16, SQ_VALU_MFMA_BUSY_CYCLES, SQ_WAVES,
// GRBM_GUI_ACTIVE (SQ 3 slots + GRBM 1 slot: one pass).

#include <rocprofiler-sdk/registration.h>
#include <rocprofiler-sdk/rocprofiler.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#define GATE_API extern "C" __attribute__((visibility("default")))

// Start-up cost (validator process with the gate, profiles/r1_bench): the
// kernel-symbol tracing that maps kernel ids to names made rocprofiler-sdk
// walk every code object the process loads, and building the counter config
// (iterate + query every counter the agent supports) sat inside the gated
// dispatch.  Now the dispatch is identified by arming: the validator arms the
// gate, enqueues ONE GEMM on its only stream and waits for it, so the first
// dispatch seen while armed is that GEMM (one-shot arm; the name filter still
// applies when AMDGPU_GATE_KERNEL_NAMES=1 turns symbol tracing back on).  The
// per-agent counter configs are built on a helper thread started by
// tool_init, while the runtime finishes its own start-up and the validator
// runs its earlier steps; a dispatch that needs a config before the thread
// is done waits for it.

namespace {

using Clock = std::chrono::steady_clock;

const char* kCounters[] = {"SQ_INSTS_VALU_MFMA_MOPS_BF16", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_WAVES", "GRBM_GUI_ACTIVE"};

std::mutex g_mu;
std::atomic<bool> g_active{false};
std::atomic<bool> g_armed{false};
bool g_trace_names = false;
std::string g_filter;
std::map<uint64_t, std::string> g_kernel_names;                 // kernel_id -> name
std::map<uint64_t, rocprofiler_counter_config_id_t> g_configs;  // agent handle -> config
std::map<uint64_t, std::string> g_counter_names;                // counter id -> name
std::map<std::string, double> g_values;
int g_dispatches = 0;
rocprofiler_context_id_t g_ctx{};

// helper-thread state (configs for every GPU agent)
std::mutex g_cfg_mu;
std::condition_variable g_cfg_cv;
bool g_cfg_done = false;
double g_cfg_seconds = -1.0;
std::thread g_cfg_thread;

void code_object_cb(rocprofiler_callback_tracing_record_t record, rocprofiler_user_data_t*, void*) {
  if (record.kind == ROCPROFILER_CALLBACK_TRACING_CODE_OBJECT &&
      record.operation == ROCPROFILER_CODE_OBJECT_DEVICE_KERNEL_SYMBOL_REGISTER &&
      record.phase == ROCPROFILER_CALLBACK_PHASE_LOAD) {
    auto* d = static_cast<rocprofiler_callback_tracing_code_object_kernel_symbol_register_data_t*>(record.payload);
    std::lock_guard<std::mutex> lk(g_mu);
    g_kernel_names[d->kernel_id] = d->kernel_name ? d->kernel_name : "";
  }
}

struct CounterSearch {
  std::vector<rocprofiler_counter_id_t> found;
  std::map<uint64_t, std::string> names;
};

rocprofiler_status_t collect_counters(rocprofiler_agent_id_t, rocprofiler_counter_id_t* counters, size_t n, void* ud) {
  auto* s = static_cast<CounterSearch*>(ud);
  for (size_t i = 0; i < n; ++i) {
    rocprofiler_counter_info_v0_t info;
    if (rocprofiler_query_counter_info(counters[i], ROCPROFILER_COUNTER_INFO_VERSION_0, &info) != ROCPROFILER_STATUS_SUCCESS)
      continue;
    for (const char* want : kCounters) {
      if (info.name && strcmp(info.name, want) == 0) {
        s->found.push_back(counters[i]);
        s->names[counters[i].handle] = want;
      }
    }
  }
  return ROCPROFILER_STATUS_SUCCESS;
}

rocprofiler_counter_config_id_t make_config(rocprofiler_agent_id_t agent) {
  CounterSearch s;
  rocprofiler_iterate_agent_supported_counters(agent, collect_counters, &s);
  rocprofiler_counter_config_id_t cfg{};
  if (s.found.empty() ||
      rocprofiler_create_counter_config(agent, s.found.data(), s.found.size(), &cfg) != ROCPROFILER_STATUS_SUCCESS)
    cfg.handle = 0;
  std::lock_guard<std::mutex> lk(g_mu);
  g_counter_names.insert(s.names.begin(), s.names.end());
  return cfg;
}

rocprofiler_status_t gpu_agents(rocprofiler_agent_version_t, const void** agents, size_t n, void* ud) {
  auto* out = static_cast<std::vector<rocprofiler_agent_id_t>*>(ud);
  for (size_t i = 0; i < n; ++i) {
    const auto* a = static_cast<const rocprofiler_agent_v0_t*>(agents[i]);
    if (a->type == ROCPROFILER_AGENT_TYPE_GPU) out->push_back(a->id);
  }
  return ROCPROFILER_STATUS_SUCCESS;
}

void build_configs() {
  const auto t0 = Clock::now();
  std::vector<rocprofiler_agent_id_t> agents;
  rocprofiler_query_available_agents(ROCPROFILER_AGENT_INFO_VERSION_0, gpu_agents, sizeof(rocprofiler_agent_v0_t),
                                     &agents);
  std::map<uint64_t, rocprofiler_counter_config_id_t> built;
  for (auto ag : agents) built[ag.handle] = make_config(ag);
  {
    std::lock_guard<std::mutex> lk(g_mu);
    for (auto& kv : built) g_configs.emplace(kv.first, kv.second);
  }
  std::lock_guard<std::mutex> lk(g_cfg_mu);
  g_cfg_seconds = std::chrono::duration<double>(Clock::now() - t0).count();
  g_cfg_done = true;
  g_cfg_cv.notify_all();
}

void wait_configs() {
  std::unique_lock<std::mutex> lk(g_cfg_mu);
  g_cfg_cv.wait_for(lk, std::chrono::seconds(5), [] { return g_cfg_done; });
}

void dispatch_cb(rocprofiler_dispatch_counting_service_data_t data, rocprofiler_counter_config_id_t* config,
                 rocprofiler_user_data_t*, void*) {
  if (!g_armed.load()) return;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_trace_names && !g_filter.empty()) {
      auto it = g_kernel_names.find(data.dispatch_info.kernel_id);
      if (it == g_kernel_names.end() || it->second.find(g_filter) == std::string::npos) return;
    }
  }
  if (!g_armed.exchange(false)) return;  // one-shot: the first dispatch after arm
  wait_configs();
  const uint64_t agent = data.dispatch_info.agent_id.handle;
  rocprofiler_counter_config_id_t cfg{};
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto cit = g_configs.find(agent);
    if (cit != g_configs.end()) cfg = cit->second;
  }
  if (!cfg.handle) {  // agent the helper did not see: build it here
    cfg = make_config(data.dispatch_info.agent_id);
    std::lock_guard<std::mutex> lk(g_mu);
    g_configs[agent] = cfg;
  }
  if (cfg.handle) *config = cfg;
}

void record_cb(rocprofiler_dispatch_counting_service_data_t, rocprofiler_counter_record_t* recs, size_t n,
               rocprofiler_user_data_t, void*) {
  std::lock_guard<std::mutex> lk(g_mu);
  ++g_dispatches;
  for (size_t i = 0; i < n; ++i) {
    rocprofiler_counter_id_t cid{};
    if (rocprofiler_query_record_counter_id(recs[i].id, &cid) != ROCPROFILER_STATUS_SUCCESS) continue;
    auto nit = g_counter_names.find(cid.handle);
    if (nit != g_counter_names.end()) g_values[nit->second] += recs[i].counter_value;
  }
}

bool env_is(const char* name, const char* val) {
  const char* e = getenv(name);
  return e && strcmp(e, val) == 0;
}

int tool_init(rocprofiler_client_finalize_t, void*) {
  if (rocprofiler_create_context(&g_ctx) != ROCPROFILER_STATUS_SUCCESS) return -1;
  g_trace_names = env_is("AMDGPU_GATE_KERNEL_NAMES", "1");
  if (g_trace_names)
    rocprofiler_configure_callback_tracing_service(g_ctx, ROCPROFILER_CALLBACK_TRACING_CODE_OBJECT, nullptr, 0,
                                                   code_object_cb, nullptr);
  if (rocprofiler_configure_callback_dispatch_counting_service(g_ctx, dispatch_cb, nullptr, record_cb, nullptr) !=
      ROCPROFILER_STATUS_SUCCESS)
    return -1;
  if (rocprofiler_start_context(g_ctx) != ROCPROFILER_STATUS_SUCCESS) return -1;
  if (env_is("AMDGPU_GATE_LAZY_CONFIG", "1")) {
    std::lock_guard<std::mutex> lk(g_cfg_mu);
    g_cfg_done = true;  // dispatch_cb builds the config itself
  } else {
    g_cfg_thread = std::thread(build_configs);
  }
  g_active = true;
  return 0;
}

void tool_fini(void*) {
  g_active = false;
  if (g_cfg_thread.joinable()) g_cfg_thread.join();
}

rocprofiler_tool_configure_result_t g_cfg = {sizeof(rocprofiler_tool_configure_result_t), tool_init, tool_fini, nullptr};

}  // namespace

extern "C" rocprofiler_tool_configure_result_t* rocprofiler_configure(uint32_t, const char*, uint32_t,
                                                                      rocprofiler_client_id_t* id) {
  const char* e = getenv("AMDGPU_VALIDATOR_COUNTERS");
  if (!e || strcmp(e, "1") != 0) return nullptr;
  if (id) id->name = "amdgpu-validator-counter-gate";
  return &g_cfg;
}

// ---- C API used by validator_main.cpp -------------------------------------
GATE_API int avk_prof_active() { return g_active.load() ? 1 : 0; }

GATE_API void avk_prof_arm(const char* kernel_substr) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_filter = kernel_substr ? kernel_substr : "";
  g_values.clear();
  g_dispatches = 0;
  g_armed = true;
}

GATE_API void avk_prof_disarm() { g_armed = false; }

GATE_API int avk_prof_dispatches() {
  std::lock_guard<std::mutex> lk(g_mu);
  return g_dispatches;
}

GATE_API double avk_prof_value(const char* counter) {
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_values.find(counter ? counter : "");
  return it == g_values.end() ? -1.0 : it->second;
}

// seconds the helper thread took to build the counter configs (-1: not run)
GATE_API double avk_prof_config_seconds() {
  std::lock_guard<std::mutex> lk(g_cfg_mu);
  return g_cfg_seconds;
}
