// How long a fresh process takes to run one kernel through ROCr (HSA) alone,
// without the HIP runtime on top (tools/hsa_init_probe.sh): hsa_init, agent
// and pool discovery, the validator's code object loaded and frozen, a queue,
// and one 64-lane vector_add_tail_kernel dispatch checked on the host.
// Wall-clock of each stage from main, one JSON line.
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <unistd.h>
#include <vector>

namespace {
using Clock = std::chrono::steady_clock;

struct Agents {
  hsa_agent_t gpu{}, cpu{};
  bool gpu_ok = false, cpu_ok = false;
};

hsa_status_t on_agent(hsa_agent_t a, void* d) {
  auto* s = static_cast<Agents*>(d);
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
  if (t == HSA_DEVICE_TYPE_CPU && !s->cpu_ok) {
    s->cpu = a;
    s->cpu_ok = true;
  } else if (t == HSA_DEVICE_TYPE_GPU && !s->gpu_ok) {
    s->gpu = a;
    s->gpu_ok = true;
  }
  return HSA_STATUS_SUCCESS;
}

hsa_status_t on_pool(hsa_amd_memory_pool_t p, void* d) {
  hsa_amd_segment_t seg;
  uint32_t flags = 0;
  if (hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg) != HSA_STATUS_SUCCESS ||
      seg != HSA_AMD_SEGMENT_GLOBAL)
    return HSA_STATUS_SUCCESS;
  hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
  if (flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_KERNARG_INIT) {
    *static_cast<hsa_amd_memory_pool_t*>(d) = p;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

struct Sym {
  const char* want;
  uint64_t object = 0;
  uint32_t kernarg = 0, group = 0, priv = 0;
};

hsa_status_t on_symbol(hsa_executable_t, hsa_agent_t, hsa_executable_symbol_t s, void* d) {
  auto* k = static_cast<Sym*>(d);
  hsa_symbol_kind_t kind;
  if (hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_TYPE, &kind) != HSA_STATUS_SUCCESS ||
      kind != HSA_SYMBOL_KIND_KERNEL)
    return HSA_STATUS_SUCCESS;
  uint32_t len = 0;
  hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_NAME_LENGTH, &len);
  std::string name(len, '\0');
  hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_NAME, name.data());
  if (name.find(k->want) == std::string::npos) return HSA_STATUS_SUCCESS;
  hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &k->object);
  hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &k->kernarg);
  hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &k->group);
  hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &k->priv);
  return HSA_STATUS_INFO_BREAK;
}

#define OK(x)                                                          \
  do {                                                                 \
    hsa_status_t st_ = (x);                                            \
    if (st_ != HSA_STATUS_SUCCESS && st_ != HSA_STATUS_INFO_BREAK) {   \
      const char* m_ = nullptr;                                        \
      hsa_status_string(st_, &m_);                                     \
      printf("{\"ok\": false, \"error\": \"%s: %s\"}\n", #x, m_ ? m_ : "?"); \
      fflush(stdout);                                                  \
      _exit(1);                                                        \
    }                                                                  \
  } while (0)
}  // namespace

int main(int argc, char** argv) {
  const auto t0 = Clock::now();
  auto ms = [&]() { return std::chrono::duration<double, std::milli>(Clock::now() - t0).count(); };
  std::string out = "{";
  auto mark = [&](const char* k) { out += "\"" + std::string(k) + "\": " + std::to_string(ms()) + ", "; };
  const char* co_path = argc > 1 ? argv[1] : "amdgpu_operator/_native/validator_kernels.co";

  OK(hsa_init());
  mark("hsa_init");
  Agents ag;
  OK(hsa_iterate_agents(on_agent, &ag));
  if (!ag.gpu_ok || !ag.cpu_ok) {
    puts("{\"ok\": false, \"error\": \"no GPU agent\"}");
    return 1;
  }
  hsa_amd_memory_pool_t pool{0};
  OK(hsa_amd_agent_iterate_memory_pools(ag.cpu, on_pool, &pool));
  mark("agents_pools");

  std::ifstream f(co_path, std::ios::binary);
  std::stringstream ss;
  ss << f.rdbuf();
  const std::string co = ss.str();
  if (co.empty()) {
    printf("{\"ok\": false, \"error\": \"cannot read %s\"}\n", co_path);
    return 1;
  }
  hsa_code_object_reader_t reader;
  hsa_executable_t exe;
  OK(hsa_code_object_reader_create_from_memory(co.data(), co.size(), &reader));
  OK(hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr, &exe));
  OK(hsa_executable_load_agent_code_object(exe, ag.gpu, reader, nullptr, nullptr));
  OK(hsa_executable_freeze(exe, nullptr));
  Sym k{"vector_add_tail_kernel"};
  OK(hsa_executable_iterate_agent_symbols(exe, ag.gpu, on_symbol, &k));
  if (!k.object) {
    puts("{\"ok\": false, \"error\": \"kernel not found\"}");
    return 1;
  }
  mark("code_object");

  const int64_t n = 64;
  float *a = nullptr, *b = nullptr, *c = nullptr;
  char* karg = nullptr;
  OK(hsa_amd_memory_pool_allocate(pool, 4096, 0, reinterpret_cast<void**>(&a)));
  OK(hsa_amd_memory_pool_allocate(pool, 4096, 0, reinterpret_cast<void**>(&b)));
  OK(hsa_amd_memory_pool_allocate(pool, 4096, 0, reinterpret_cast<void**>(&c)));
  OK(hsa_amd_memory_pool_allocate(pool, 4096, 0, reinterpret_cast<void**>(&karg)));
  for (void* p : {static_cast<void*>(a), static_cast<void*>(b), static_cast<void*>(c), static_cast<void*>(karg)})
    OK(hsa_amd_agents_allow_access(1, &ag.gpu, nullptr, p));
  for (int i = 0; i < n; ++i) {
    a[i] = float(i);
    b[i] = 2.0f * i;
    c[i] = -1.0f;
  }
  const int64_t start = 0;
  memcpy(karg, &a, 8);
  memcpy(karg + 8, &b, 8);
  memcpy(karg + 16, &c, 8);
  memcpy(karg + 24, &start, 8);
  memcpy(karg + 32, &n, 8);
  mark("buffers");

  hsa_queue_t* q = nullptr;
  hsa_signal_t done;
  OK(hsa_queue_create(ag.gpu, 64, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &q));
  OK(hsa_signal_create(1, 0, nullptr, &done));
  mark("queue");

  const uint64_t idx = hsa_queue_add_write_index_relaxed(q, 1);
  auto* pk = reinterpret_cast<hsa_kernel_dispatch_packet_t*>(static_cast<char*>(q->base_address) +
                                                             (idx & (q->size - 1)) * 64);
  memset(reinterpret_cast<char*>(pk) + 4, 0, 60);
  pk->workgroup_size_x = 64;
  pk->workgroup_size_y = pk->workgroup_size_z = 1;
  pk->grid_size_x = 64;
  pk->grid_size_y = pk->grid_size_z = 1;
  pk->private_segment_size = k.priv;
  pk->group_segment_size = k.group;
  pk->kernel_object = k.object;
  pk->kernarg_address = karg;
  pk->completion_signal = done;
  const uint16_t hdr = static_cast<uint16_t>((HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                                             (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                                             (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE));
  __atomic_store_n(reinterpret_cast<uint32_t*>(pk),
                   uint32_t(hdr) | (uint32_t(1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS) << 16),
                   __ATOMIC_RELEASE);
  hsa_signal_store_screlease(q->doorbell_signal, static_cast<hsa_signal_value_t>(idx));
  int spins = 0;
  while (hsa_signal_wait_scacquire(done, HSA_SIGNAL_CONDITION_LT, 1, 100000000, HSA_WAIT_STATE_BLOCKED) >= 1) {
    if (++spins > 50) {
      puts("{\"ok\": false, \"error\": \"dispatch timeout\"}");
      fflush(stdout);
      _exit(2);
    }
  }
  mark("kernel");
  int bad = 0;
  for (int i = 0; i < n; ++i) bad += c[i] != a[i] + b[i];
  out += "\"ok\": " + std::string(bad ? "false" : "true") + ", \"bad\": " + std::to_string(bad) + "}";
  puts(out.c_str());
  fflush(stdout);
  _exit(bad ? 1 : 0);
}
