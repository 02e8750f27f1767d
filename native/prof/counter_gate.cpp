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
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#define GATE_API extern "C" __attribute__((visibility("default")))

namespace {

const char* kCounters[] = {"SQ_INSTS_VALU_MFMA_MOPS_BF16", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_WAVES", "GRBM_GUI_ACTIVE"};

std::mutex g_mu;
std::atomic<bool> g_active{false};
std::atomic<bool> g_armed{false};
std::string g_filter;
std::map<uint64_t, std::string> g_kernel_names;                 // kernel_id -> name
std::map<uint64_t, rocprofiler_counter_config_id_t> g_configs;  // agent handle -> config
std::map<uint64_t, std::string> g_counter_names;                // counter id -> name
std::map<std::string, double> g_values;
int g_dispatches = 0;
rocprofiler_context_id_t g_ctx{};

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
        g_counter_names[counters[i].handle] = want;
      }
    }
  }
  return ROCPROFILER_STATUS_SUCCESS;
}

void dispatch_cb(rocprofiler_dispatch_counting_service_data_t data, rocprofiler_counter_config_id_t* config,
                 rocprofiler_user_data_t*, void*) {
  if (!g_armed.load()) return;
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_kernel_names.find(data.dispatch_info.kernel_id);
  if (!g_filter.empty() && (it == g_kernel_names.end() || it->second.find(g_filter) == std::string::npos)) return;
  const uint64_t agent = data.dispatch_info.agent_id.handle;
  auto cit = g_configs.find(agent);
  if (cit == g_configs.end()) {
    CounterSearch s;
    rocprofiler_iterate_agent_supported_counters(data.dispatch_info.agent_id, collect_counters, &s);
    rocprofiler_counter_config_id_t cfg{};
    if (s.found.empty() ||
        rocprofiler_create_counter_config(data.dispatch_info.agent_id, s.found.data(), s.found.size(), &cfg) !=
            ROCPROFILER_STATUS_SUCCESS)
      cfg.handle = 0;
    cit = g_configs.emplace(agent, cfg).first;
  }
  if (cit->second.handle) *config = cit->second;
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

int tool_init(rocprofiler_client_finalize_t, void*) {
  if (rocprofiler_create_context(&g_ctx) != ROCPROFILER_STATUS_SUCCESS) return -1;
  rocprofiler_configure_callback_tracing_service(g_ctx, ROCPROFILER_CALLBACK_TRACING_CODE_OBJECT, nullptr, 0,
                                                 code_object_cb, nullptr);
  if (rocprofiler_configure_callback_dispatch_counting_service(g_ctx, dispatch_cb, nullptr, record_cb, nullptr) !=
      ROCPROFILER_STATUS_SUCCESS)
    return -1;
  if (rocprofiler_start_context(g_ctx) != ROCPROFILER_STATUS_SUCCESS) return -1;
  g_active = true;
  return 0;
}

void tool_fini(void*) { g_active = false; }

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
