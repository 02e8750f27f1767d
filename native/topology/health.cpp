// N6: GPU health watcher for the device plugin's ListAndWatch stream.
//
// The NVIDIA device plugin marks a GPU Unhealthy on critical XID events
// (/root/reference/README.md:211 names the plugin; the mechanism is upstream
// behaviour).  On MI355X the equivalent signals are:
//   * amd-smi event notifications (amdsmi_init_gpu_event_notification /
//     amdsmi_get_gpu_event_notification): GPU pre-reset is critical, VM faults
//     and thermal throttling are reported but not critical (an application
//     fault must not take the device out of service);
//   * counter deltas between polls: uncorrectable ECC (critical), xGMI link
//     errors (critical), newly retired bad pages (reported), and a device that
//     stops answering (critical).

#include <cstdio>
#include <cstring>
#include <mutex>
#include <vector>

#include <amd_smi/amdsmi.h>

#include "amdgpu_topo.h"
#include "smi_internal.h"

namespace {

struct Prev {
  uint64_t ecc_uncorrectable = 0;
  uint32_t xgmi_links_error = 0;
  uint32_t bad_pages = 0;
  uint32_t valid = 0;
};

std::mutex g_hmu;
bool g_started = false;
bool g_events = false;
std::vector<Prev> g_prev;

void push(std::vector<at_event_t>& evs, int index, int kind, int critical, const char* msg) {
  at_event_t e;
  memset(&e, 0, sizeof(e));
  e.index = index;
  e.kind = kind;
  e.critical = critical;
  snprintf(e.message, sizeof(e.message), "%s", msg ? msg : "");
  evs.push_back(e);
}

}  // namespace

extern "C" {

AT_API int at_health_start(void) {
  std::lock_guard<std::mutex> lk(g_hmu);
  if (g_started) return AT_OK;
  int rc = at_smi_open();
  if (rc != AT_OK) return rc;
  at_smi::Api& a = at_smi::g_api;
  g_events = a.evt_init && a.evt_mask && a.evt_get;
  if (g_events) {
    const uint64_t mask = (1ull << (AMDSMI_EVT_NOTIF_VMFAULT - 1)) | (1ull << (AMDSMI_EVT_NOTIF_THERMAL_THROTTLE - 1)) |
                          (1ull << (AMDSMI_EVT_NOTIF_GPU_PRE_RESET - 1)) | (1ull << (AMDSMI_EVT_NOTIF_GPU_POST_RESET - 1));
    for (auto h : a.gpus) {
      if (a.evt_init(h) != AMDSMI_STATUS_SUCCESS || a.evt_mask(h, mask) != AMDSMI_STATUS_SUCCESS) g_events = false;
    }
  }
  // prime the counter baseline
  int n = at_smi_count();
  std::vector<at_metrics_t> m(n > 0 ? n : 0);
  int cnt = 0;
  if (n > 0) at_smi_collect(m.data(), n, &cnt);
  g_prev.assign(n > 0 ? n : 0, Prev());
  for (int i = 0; i < cnt; ++i) {
    g_prev[i].ecc_uncorrectable = m[i].ecc_uncorrectable;
    g_prev[i].xgmi_links_error = m[i].xgmi_links_error;
    g_prev[i].bad_pages = m[i].bad_pages;
    g_prev[i].valid = m[i].valid_mask;
  }
  g_started = true;
  return AT_OK;
}

AT_API void at_health_stop(void) {
  std::lock_guard<std::mutex> lk(g_hmu);
  if (!g_started) return;
  at_smi::Api& a = at_smi::g_api;
  if (g_events && a.evt_stop)
    for (auto h : a.gpus) a.evt_stop(h);
  g_started = false;
  at_smi_close();
}

AT_API int at_health_poll(int timeout_ms, at_event_t* out, int max, int* count) {
  std::lock_guard<std::mutex> lk(g_hmu);
  if (!g_started) return AT_ERR_UNSUPPORTED;
  if (!count || max < 0 || (max > 0 && !out)) return AT_ERR_INVAL;
  at_smi::Api& a = at_smi::g_api;
  std::vector<at_event_t> evs;

  if (g_events) {
    amdsmi_evt_notification_data_t data[32];
    uint32_t n = 32;
    if (a.evt_get(timeout_ms, &n, data) == AMDSMI_STATUS_SUCCESS) {
      for (uint32_t i = 0; i < n && i < 32; ++i) {
        int idx = -1;
        for (size_t g = 0; g < a.gpus.size(); ++g)
          if (a.gpus[g] == data[i].processor_handle) idx = (int)g;
        switch (data[i].event) {
          case AMDSMI_EVT_NOTIF_GPU_PRE_RESET: push(evs, idx, AT_EV_GPU_PRE_RESET, 1, data[i].message); break;
          case AMDSMI_EVT_NOTIF_GPU_POST_RESET: push(evs, idx, AT_EV_GPU_POST_RESET, 0, data[i].message); break;
          case AMDSMI_EVT_NOTIF_VMFAULT: push(evs, idx, AT_EV_VMFAULT, 0, data[i].message); break;
          case AMDSMI_EVT_NOTIF_THERMAL_THROTTLE: push(evs, idx, AT_EV_THERMAL_THROTTLE, 0, data[i].message); break;
          default: break;
        }
      }
    }
  }

  const int n = (int)g_prev.size();
  std::vector<at_metrics_t> m(n);
  int cnt = 0;
  if (n > 0 && at_smi_collect(m.data(), n, &cnt) == AT_OK) {
    for (int i = 0; i < n && i < cnt; ++i) {
      Prev& p = g_prev[i];
      char msg[128];
      if (m[i].valid_mask == 0 && p.valid != 0) push(evs, i, AT_EV_DEVICE_LOST, 1, "device stopped answering amd-smi queries");
      if ((m[i].valid_mask & AT_M_ECC) && m[i].ecc_uncorrectable > p.ecc_uncorrectable) {
        snprintf(msg, sizeof(msg), "uncorrectable ECC errors %llu -> %llu", (unsigned long long)p.ecc_uncorrectable,
                 (unsigned long long)m[i].ecc_uncorrectable);
        push(evs, i, AT_EV_ECC_UNCORRECTABLE, 1, msg);
      }
      if ((m[i].valid_mask & AT_M_XGMI) && m[i].xgmi_links_error > p.xgmi_links_error) {
        snprintf(msg, sizeof(msg), "xGMI links in error %u -> %u", p.xgmi_links_error, m[i].xgmi_links_error);
        push(evs, i, AT_EV_XGMI_LINK_ERROR, 1, msg);
      }
      if ((m[i].valid_mask & AT_M_BADPAGES) && m[i].bad_pages > p.bad_pages) {
        snprintf(msg, sizeof(msg), "retired pages %u -> %u", p.bad_pages, m[i].bad_pages);
        push(evs, i, AT_EV_BAD_PAGES, 0, msg);
      }
      if (m[i].valid_mask) {
        p.ecc_uncorrectable = m[i].ecc_uncorrectable;
        p.xgmi_links_error = m[i].xgmi_links_error;
        p.bad_pages = m[i].bad_pages;
      }
      p.valid = m[i].valid_mask;
    }
  }

  *count = (int)evs.size();
  const int k = std::min<int>(max, (int)evs.size());
  for (int i = 0; i < k; ++i) out[i] = evs[i];
  return (int)evs.size() > max ? AT_ERR_NOSPC : AT_OK;
}

}  // extern "C"
