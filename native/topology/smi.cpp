// N4: per-GPU metrics collector over libamd_smi (dlopen'ed), plus the
// partition get/set used by the partition manager (C10, the MIG-manager
// analog the reference disables at /root/reference/README.md:109).
//
// The collector is the MI355X replacement for DCGM behind dcgm-exporter
// (README.md:204,213): one call gathers every field for every GPU so the
// Python exporter does a single native round trip per scrape interval.

#include <dlfcn.h>

#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include <amd_smi/amdsmi.h>

#include "amdgpu_topo.h"
#include "smi_internal.h"

namespace at_smi {

Api g_api;
static std::mutex g_mu;
static int g_refs = 0;

template <typename F>
static bool sym(void* h, const char* name, F* fp) {
  *fp = reinterpret_cast<F>(dlsym(h, name));
  return *fp != nullptr;
}

static bool load_api(Api* a) {
  const char* names[] = {"libamd_smi.so", "libamd_smi.so.26", "/opt/rocm/lib/libamd_smi.so"};
  for (const char* n : names) {
    a->dl = dlopen(n, RTLD_NOW | RTLD_LOCAL);
    if (a->dl) break;
  }
  if (!a->dl) return false;
  bool ok = sym(a->dl, "amdsmi_init", &a->init) && sym(a->dl, "amdsmi_shut_down", &a->shut_down) &&
            sym(a->dl, "amdsmi_get_socket_handles", &a->get_socket_handles) &&
            sym(a->dl, "amdsmi_get_processor_handles", &a->get_processor_handles);
  if (!ok) return false;
  // optional entry points: a missing one just leaves its fields invalid
  sym(a->dl, "amdsmi_get_gpu_device_bdf", &a->get_bdf);
  sym(a->dl, "amdsmi_get_gpu_device_uuid", &a->get_uuid);
  sym(a->dl, "amdsmi_get_gpu_asic_info", &a->get_asic);
  sym(a->dl, "amdsmi_get_gpu_memory_total", &a->mem_total);
  sym(a->dl, "amdsmi_get_gpu_memory_usage", &a->mem_usage);
  sym(a->dl, "amdsmi_get_gpu_activity", &a->activity);
  sym(a->dl, "amdsmi_get_power_info", &a->power);
  sym(a->dl, "amdsmi_get_temp_metric", &a->temp);
  sym(a->dl, "amdsmi_get_clock_info", &a->clock);
  sym(a->dl, "amdsmi_get_energy_count", &a->energy);
  sym(a->dl, "amdsmi_get_gpu_total_ecc_count", &a->ecc);
  sym(a->dl, "amdsmi_get_gpu_xgmi_link_status", &a->xgmi_status);
  sym(a->dl, "amdsmi_get_gpu_bad_page_info", &a->bad_pages);
  sym(a->dl, "amdsmi_get_gpu_process_list", &a->procs);
  sym(a->dl, "amdsmi_get_gpu_driver_info", &a->driver);
  sym(a->dl, "amdsmi_get_gpu_compute_partition", &a->get_cpart);
  sym(a->dl, "amdsmi_get_gpu_memory_partition", &a->get_mpart);
  sym(a->dl, "amdsmi_set_gpu_compute_partition", &a->set_cpart);
  sym(a->dl, "amdsmi_set_gpu_memory_partition", &a->set_mpart);
  sym(a->dl, "amdsmi_init_gpu_event_notification", &a->evt_init);
  sym(a->dl, "amdsmi_set_gpu_event_notification_mask", &a->evt_mask);
  sym(a->dl, "amdsmi_get_gpu_event_notification", &a->evt_get);
  sym(a->dl, "amdsmi_stop_gpu_event_notification", &a->evt_stop);
  sym(a->dl, "amdsmi_get_gpu_metrics_info", &a->gpu_metrics);
  return true;
}

static bool enumerate(Api* a) {
  a->gpus.clear();
  uint32_t nsock = 0;
  if (a->get_socket_handles(&nsock, nullptr) != AMDSMI_STATUS_SUCCESS) return false;
  std::vector<amdsmi_socket_handle> socks(nsock);
  if (nsock && a->get_socket_handles(&nsock, socks.data()) != AMDSMI_STATUS_SUCCESS) return false;
  for (uint32_t s = 0; s < nsock; ++s) {
    uint32_t np = 0;
    if (a->get_processor_handles(socks[s], &np, nullptr) != AMDSMI_STATUS_SUCCESS) continue;
    std::vector<amdsmi_processor_handle> ph(np);
    if (np && a->get_processor_handles(socks[s], &np, ph.data()) != AMDSMI_STATUS_SUCCESS) continue;
    for (uint32_t i = 0; i < np; ++i) a->gpus.push_back(ph[i]);
  }
  return true;
}

}  // namespace at_smi

using namespace at_smi;

// PMFW table fields read all-ones when the firmware does not report them
static bool valid64(uint64_t v) { return v != UINT64_MAX; }
static uint64_t or0(uint64_t v) { return valid64(v) ? v : 0; }

// bounded copy that always NUL-terminates (amd-smi strings may exceed our fields)
static void copy_str(char* dst, size_t cap, const char* s) {
  if (cap == 0) return;
  const size_t n = s ? strnlen(s, cap - 1) : 0;
  if (n) memcpy(dst, s, n);
  dst[n] = '\0';
}

extern "C" {

AT_API int at_smi_open(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_refs > 0) {
    ++g_refs;
    return AT_OK;
  }
  if (!g_api.dl && !load_api(&g_api)) return AT_ERR_UNSUPPORTED;
  if (g_api.init(AMDSMI_INIT_AMD_GPUS) != AMDSMI_STATUS_SUCCESS) return AT_ERR_UNSUPPORTED;
  if (!enumerate(&g_api)) {
    g_api.shut_down();
    return AT_ERR_UNSUPPORTED;
  }
  g_refs = 1;
  return AT_OK;
}

AT_API void at_smi_close(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_refs > 0 && --g_refs == 0) g_api.shut_down();
}

AT_API int at_smi_count(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  return g_refs > 0 ? (int)g_api.gpus.size() : AT_ERR_UNSUPPORTED;
}

AT_API int at_smi_collect(at_metrics_t* out, int max, int* count) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_refs <= 0) return AT_ERR_UNSUPPORTED;
  if (!count || max < 0 || (max > 0 && !out)) return AT_ERR_INVAL;
  Api& a = g_api;
  *count = (int)a.gpus.size();
  const int n = std::min<int>(max, (int)a.gpus.size());
  for (int i = 0; i < n; ++i) {
    amdsmi_processor_handle h = a.gpus[i];
    at_metrics_t& m = out[i];
    memset(&m, 0, sizeof(m));
    m.index = i;
    if (a.get_bdf) {
      amdsmi_bdf_t b;
      if (a.get_bdf(h, &b) == AMDSMI_STATUS_SUCCESS)
        snprintf(m.bdf, sizeof(m.bdf), "%04x:%02x:%02x.%x", (unsigned)b.domain_number, (unsigned)b.bus_number,
                 (unsigned)b.device_number, (unsigned)b.function_number);
    }
    if (a.get_uuid) {
      unsigned len = sizeof(m.uuid);
      a.get_uuid(h, &len, m.uuid);
    }
    if (a.get_asic) {
      amdsmi_asic_info_t ai;
      if (a.get_asic(h, &ai) == AMDSMI_STATUS_SUCCESS) copy_str(m.market_name, sizeof(m.market_name), ai.market_name);
    }
    if (a.mem_total && a.mem_usage) {
      uint64_t t = 0, u = 0;
      if (a.mem_total(h, AMDSMI_MEM_TYPE_VRAM, &t) == AMDSMI_STATUS_SUCCESS &&
          a.mem_usage(h, AMDSMI_MEM_TYPE_VRAM, &u) == AMDSMI_STATUS_SUCCESS) {
        m.vram_total_bytes = t;
        m.vram_used_bytes = u;
        m.valid_mask |= AT_M_VRAM;
      }
    }
    if (a.activity) {
      amdsmi_engine_usage_t e;
      if (a.activity(h, &e) == AMDSMI_STATUS_SUCCESS) {
        m.gfx_activity_pct = e.gfx_activity;
        m.umc_activity_pct = e.umc_activity;
        m.mm_activity_pct = e.mm_activity;
        m.valid_mask |= AT_M_ACTIVITY;
      }
    }
    if (a.power) {
      amdsmi_power_info_t p;
      if (a.power(h, &p) == AMDSMI_STATUS_SUCCESS) {
        m.socket_power_w = p.current_socket_power ? p.current_socket_power : (double)p.average_socket_power;
        m.power_limit_w = p.power_limit;
        m.valid_mask |= AT_M_POWER;
      }
    }
    if (a.temp) {
      int64_t t = 0;
      bool any = false;
      if (a.temp(h, AMDSMI_TEMPERATURE_TYPE_HOTSPOT, AMDSMI_TEMP_CURRENT, &t) == AMDSMI_STATUS_SUCCESS) {
        m.temp_hotspot_c = (double)t;
        any = true;
      }
      if (a.temp(h, AMDSMI_TEMPERATURE_TYPE_VRAM, AMDSMI_TEMP_CURRENT, &t) == AMDSMI_STATUS_SUCCESS) {
        m.temp_mem_c = (double)t;
        any = true;
      }
      if (a.temp(h, AMDSMI_TEMPERATURE_TYPE_EDGE, AMDSMI_TEMP_CURRENT, &t) == AMDSMI_STATUS_SUCCESS) {
        m.temp_edge_c = (double)t;
        any = true;
      }
      if (any) m.valid_mask |= AT_M_TEMP;
    }
    if (a.clock) {
      amdsmi_clk_info_t c;
      bool any = false;
      if (a.clock(h, AMDSMI_CLK_TYPE_GFX, &c) == AMDSMI_STATUS_SUCCESS) {
        m.gfx_clk_mhz = c.clk;
        any = true;
      }
      if (a.clock(h, AMDSMI_CLK_TYPE_MEM, &c) == AMDSMI_STATUS_SUCCESS) {
        m.mem_clk_mhz = c.clk;
        any = true;
      }
      if (any) m.valid_mask |= AT_M_CLOCK;
    }
    if (a.energy) {
      uint64_t acc = 0, ts = 0;
      float res = 0;
      if (a.energy(h, &acc, &res, &ts) == AMDSMI_STATUS_SUCCESS) {
        m.energy_j = (double)acc * (double)res * 1e-6;  // resolution is in uJ per count
        m.valid_mask |= AT_M_ENERGY;
      }
    }
    if (a.ecc) {
      amdsmi_error_count_t ec;
      if (a.ecc(h, &ec) == AMDSMI_STATUS_SUCCESS) {
        m.ecc_correctable = ec.correctable_count;
        m.ecc_uncorrectable = ec.uncorrectable_count;
        m.ecc_deferred = ec.deferred_count;
        m.valid_mask |= AT_M_ECC;
      }
    }
    if (a.xgmi_status) {
      amdsmi_xgmi_link_status_t ls;
      memset(&ls, 0, sizeof(ls));
      if (a.xgmi_status(h, &ls) == AMDSMI_STATUS_SUCCESS) {
        m.xgmi_links_total = ls.total_links;
        for (uint32_t l = 0; l < ls.total_links && l < AMDSMI_MAX_NUM_XGMI_LINKS; ++l) {
          if (ls.status[l] == AMDSMI_XGMI_LINK_UP) ++m.xgmi_links_up;
          if (ls.status[l] != AMDSMI_XGMI_LINK_UP && ls.status[l] != AMDSMI_XGMI_LINK_DOWN &&
              ls.status[l] != AMDSMI_XGMI_LINK_DISABLE)
            ++m.xgmi_links_error;
        }
        m.valid_mask |= AT_M_XGMI;
      }
    }
    if (a.bad_pages) {
      uint32_t np = 0;
      if (a.bad_pages(h, &np, nullptr) == AMDSMI_STATUS_SUCCESS) {
        m.bad_pages = np;
        m.valid_mask |= AT_M_BADPAGES;
      }
    }
    if (a.procs) {
      uint32_t np = 0;
      amdsmi_status_t st = a.procs(h, &np, nullptr);
      if (st == AMDSMI_STATUS_SUCCESS || st == AMDSMI_STATUS_OUT_OF_RESOURCES) {
        m.num_processes = np;
        m.valid_mask |= AT_M_PROCS;
      }
    }
    if (a.gpu_metrics) {
      // one PMFW table read per GPU: xGMI traffic, PCIe health, throttle residency
      // (the MI355X counterparts of DCGM's NVLink / PCIe / violation fields)
      static thread_local amdsmi_gpu_metrics_t gm;
      memset(&gm, 0, sizeof(gm));
      if (a.gpu_metrics(h, &gm) == AMDSMI_STATUS_SUCCESS) {
        m.xgmi_read_bytes = m.xgmi_write_bytes = 0;
        for (int l = 0; l < AMDSMI_MAX_NUM_XGMI_LINKS; ++l) {
          if (valid64(gm.xgmi_read_data_acc[l])) m.xgmi_read_bytes += gm.xgmi_read_data_acc[l] * 1024ull;
          if (valid64(gm.xgmi_write_data_acc[l])) m.xgmi_write_bytes += gm.xgmi_write_data_acc[l] * 1024ull;
        }
        m.pcie_bandwidth_gbps = or0(gm.pcie_bandwidth_inst);
        m.pcie_replay_count = or0(gm.pcie_replay_count_acc);
        m.pcie_nak_sent = gm.pcie_nak_sent_count_acc == UINT32_MAX ? 0 : gm.pcie_nak_sent_count_acc;
        m.pcie_nak_rcvd = gm.pcie_nak_rcvd_count_acc == UINT32_MAX ? 0 : gm.pcie_nak_rcvd_count_acc;
        m.prochot_residency = or0(gm.prochot_residency_acc);
        m.ppt_residency = or0(gm.ppt_residency_acc);
        m.socket_thermal_residency = or0(gm.socket_thm_residency_acc);
        m.hbm_thermal_residency = or0(gm.hbm_thm_residency_acc);
        m.vram_max_bandwidth_gbps = or0(gm.vram_max_bandwidth);
        m.xgmi_link_speed_gbps = gm.xgmi_link_speed == UINT16_MAX ? 0 : gm.xgmi_link_speed;
        m.xgmi_link_width = gm.xgmi_link_width == UINT16_MAX ? 0 : gm.xgmi_link_width;
        m.pcie_link_width = gm.pcie_link_width == UINT16_MAX ? 0 : gm.pcie_link_width;
        m.pcie_link_speed_mts = gm.pcie_link_speed == UINT16_MAX ? 0 : gm.pcie_link_speed * 100u;
        m.throttle_status = gm.throttle_status == UINT32_MAX ? 0 : gm.throttle_status;
        m.valid_mask |= AT_M_GPU_METRICS;
      }
    }
  }
  return AT_OK;
}

AT_API int at_smi_driver_version(char* buf, int len) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_refs <= 0 || !g_api.driver || g_api.gpus.empty() || !buf || len <= 0) return AT_ERR_UNSUPPORTED;
  amdsmi_driver_info_t d;
  if (g_api.driver(g_api.gpus[0], &d) != AMDSMI_STATUS_SUCCESS) return AT_ERR_UNSUPPORTED;
  copy_str(buf, (size_t)len, d.driver_version);
  return AT_OK;
}

static int cpart_from_name(const char* s) {
  if (!strcmp(s, "SPX")) return AMDSMI_COMPUTE_PARTITION_SPX;
  if (!strcmp(s, "DPX")) return AMDSMI_COMPUTE_PARTITION_DPX;
  if (!strcmp(s, "TPX")) return AMDSMI_COMPUTE_PARTITION_TPX;
  if (!strcmp(s, "QPX")) return AMDSMI_COMPUTE_PARTITION_QPX;
  if (!strcmp(s, "CPX")) return AMDSMI_COMPUTE_PARTITION_CPX;
  return -1;
}

static int mpart_from_name(const char* s) {
  if (!strcmp(s, "NPS1")) return AMDSMI_MEMORY_PARTITION_NPS1;
  if (!strcmp(s, "NPS2")) return AMDSMI_MEMORY_PARTITION_NPS2;
  if (!strcmp(s, "NPS4")) return AMDSMI_MEMORY_PARTITION_NPS4;
  if (!strcmp(s, "NPS8")) return AMDSMI_MEMORY_PARTITION_NPS8;
  return -1;
}

AT_API int at_smi_set_compute_partition(int index, const char* mode) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_refs <= 0 || !g_api.set_cpart) return AT_ERR_UNSUPPORTED;
  if (!mode || index < 0 || index >= (int)g_api.gpus.size()) return AT_ERR_INVAL;
  int v = cpart_from_name(mode);
  if (v < 0) return AT_ERR_INVAL;
  amdsmi_status_t st = g_api.set_cpart(g_api.gpus[index], (amdsmi_compute_partition_type_t)v);
  return st == AMDSMI_STATUS_SUCCESS ? AT_OK : -(int)st - 1000;
}

AT_API int at_smi_set_memory_partition(int index, const char* mode) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_refs <= 0 || !g_api.set_mpart) return AT_ERR_UNSUPPORTED;
  if (!mode || index < 0 || index >= (int)g_api.gpus.size()) return AT_ERR_INVAL;
  int v = mpart_from_name(mode);
  if (v < 0) return AT_ERR_INVAL;
  amdsmi_status_t st = g_api.set_mpart(g_api.gpus[index], (amdsmi_memory_partition_type_t)v);
  return st == AMDSMI_STATUS_SUCCESS ? AT_OK : -(int)st - 1000;
}

AT_API int at_smi_get_partitions(int index, char* compute, int clen, char* memory, int mlen) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_refs <= 0) return AT_ERR_UNSUPPORTED;
  if (index < 0 || index >= (int)g_api.gpus.size()) return AT_ERR_INVAL;
  if (compute && clen > 0) {
    compute[0] = 0;
    if (g_api.get_cpart) g_api.get_cpart(g_api.gpus[index], compute, (uint32_t)clen);
  }
  if (memory && mlen > 0) {
    memory[0] = 0;
    if (g_api.get_mpart) g_api.get_mpart(g_api.gpus[index], memory, (uint32_t)mlen);
  }
  return AT_OK;
}

}  // extern "C"
