// amdgpu_topo.h - C ABI of libamdgpu_topo.so (native N3/N4/N6 of SURVEY.md §2.C)
//
//   N3  device + topology enumeration from KFD sysfs (+ PCI/DRM sysfs):
//       the MI355X counterpart of the NVML device queries behind nvidia-smi
//       (/root/reference/README.md:152,158-167) and of the device plugin's
//       device discovery (/root/reference/README.md:211).
//   N4  metrics collector over libamd_smi (dlopen'ed at runtime): the
//       DCGM-equivalent behind the metrics exporter (README.md:204,213).
//   N6  health watcher: amd-smi event notifications + ECC / xGMI polling,
//       feeding ListAndWatch health (README.md:211).
//
// Every entry point takes a `root` prefix ("" or "/" = the real machine) so the
// whole library runs against captured or synthetic sysfs trees in tests.

#ifndef AMDGPU_TOPO_H_
#define AMDGPU_TOPO_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AT_API __attribute__((visibility("default")))

#define AT_OK 0
#define AT_ERR_NOENT -2
#define AT_ERR_INVAL -22
#define AT_ERR_NOSPC -28
#define AT_ERR_UNSUPPORTED -95

typedef struct {
  int32_t kfd_node;             // KFD topology node index
  uint32_t gpu_id;              // KFD gpu_id
  uint32_t gfx_target_version;  // e.g. 90500 for gfx950
  char arch[16];                // "gfx950"
  uint32_t simd_count;
  uint32_t simd_per_cu;
  uint32_t cu_count;
  uint32_t num_xcc;
  uint32_t max_waves_per_simd;
  uint32_t wave_front_size;
  uint32_t lds_size_kib;
  uint32_t max_engine_clk_mhz;
  uint64_t vram_bytes;          // frame-buffer heaps (public + private)
  uint32_t drm_render_minor;    // /dev/dri/renderD<minor>
  uint32_t domain;
  uint32_t location_id;         // bus << 8 | dev << 3 | fn
  char bdf[16];                 // "0000:05:00.0"
  uint32_t vendor_id;
  uint32_t device_id;
  uint64_t unique_id;
  uint64_t hive_id;
  uint32_t num_xgmi_links;      // xGMI io/p2p links to other GPU nodes
  int32_t numa_node;            // -1 when unknown
  int32_t physical_index;       // index of the physical GPU (grouped by BDF)
  int32_t partition_index;      // index inside the physical GPU (0 in SPX)
  int32_t partition_count;      // partitions of this physical GPU (1 in SPX)
  char compute_partition[8];    // SPX/DPX/QPX/CPX ("" when unknown)
  char memory_partition[8];     // NPS1/NPS2/... ("" when unknown)
} at_gpu_t;

#define AT_LINK_PCIE 2
#define AT_LINK_XGMI 11

typedef struct {
  int32_t from_gpu;   // index into the at_enumerate() array
  int32_t to_gpu;
  uint32_t type;      // AT_LINK_*
  uint32_t weight;    // KFD link weight (lower = closer)
  uint32_t min_bandwidth_mbps;
  uint32_t max_bandwidth_mbps;
} at_link_t;

// ---- N3 -------------------------------------------------------------------
AT_API int at_abi_version(void);
AT_API int at_enumerate(const char* root, at_gpu_t* out, int max, int* count);
AT_API int at_links(const char* root, at_link_t* out, int max, int* count);
// N1 readiness: fills `msg` with a human-readable reason; returns AT_OK when
// /dev/kfd, the amdgpu module, KFD GPU nodes and their render nodes are present.
AT_API int at_probe(const char* root, int expect_gpus, char* msg, int msg_len);

// ---- N4 -------------------------------------------------------------------
typedef struct {
  int32_t index;             // amd-smi processor index
  char bdf[16];
  char uuid[64];
  char market_name[64];
  uint64_t vram_total_bytes;
  uint64_t vram_used_bytes;
  uint32_t gfx_activity_pct;
  uint32_t umc_activity_pct;
  uint32_t mm_activity_pct;
  double socket_power_w;
  double power_limit_w;
  double temp_hotspot_c;
  double temp_mem_c;
  double temp_edge_c;
  uint32_t gfx_clk_mhz;
  uint32_t mem_clk_mhz;
  double energy_j;
  uint64_t ecc_correctable;
  uint64_t ecc_uncorrectable;
  uint64_t ecc_deferred;
  uint32_t xgmi_links_total;
  uint32_t xgmi_links_up;       // links whose status is "no errors"
  uint32_t xgmi_links_error;
  uint32_t bad_pages;
  uint32_t num_processes;
  // amdsmi_get_gpu_metrics_info (PMFW metrics table), AT_M_GPU_METRICS
  uint64_t xgmi_read_bytes;      // accumulated over every xGMI link (table: KB)
  uint64_t xgmi_write_bytes;
  uint64_t pcie_bandwidth_gbps;  // instantaneous PCIe bandwidth (GB/s)
  uint64_t pcie_replay_count;    // accumulated PCIe replays
  uint64_t pcie_nak_sent;
  uint64_t pcie_nak_rcvd;
  uint64_t prochot_residency;    // throttle residency accumulators (PMFW units)
  uint64_t ppt_residency;
  uint64_t socket_thermal_residency;
  uint64_t hbm_thermal_residency;
  uint64_t vram_max_bandwidth_gbps;
  uint32_t xgmi_link_speed_gbps;
  uint32_t xgmi_link_width;  // lanes per xGMI link (x16 on MI355X): link GB/s = speed x width / 8
  uint32_t pcie_link_width;
  uint32_t pcie_link_speed_mts;  // table: 0.1 GT/s
  uint32_t throttle_status;
  uint32_t valid_mask;          // AT_M_* bits for fields that were read
} at_metrics_t;

#define AT_M_VRAM (1u << 0)
#define AT_M_ACTIVITY (1u << 1)
#define AT_M_POWER (1u << 2)
#define AT_M_TEMP (1u << 3)
#define AT_M_CLOCK (1u << 4)
#define AT_M_ENERGY (1u << 5)
#define AT_M_ECC (1u << 6)
#define AT_M_XGMI (1u << 7)
#define AT_M_BADPAGES (1u << 8)
#define AT_M_PROCS (1u << 9)
#define AT_M_GPU_METRICS (1u << 10)

// Opens libamd_smi (dlopen) and initialises it; AT_ERR_UNSUPPORTED when the
// library or a GPU is unavailable.  Reference-counted, thread-safe.
AT_API int at_smi_open(void);
AT_API void at_smi_close(void);
AT_API int at_smi_count(void);
AT_API int at_smi_collect(at_metrics_t* out, int max, int* count);
AT_API int at_smi_driver_version(char* buf, int len);
AT_API int at_smi_set_compute_partition(int index, const char* mode);  // SPX/DPX/QPX/CPX
AT_API int at_smi_set_memory_partition(int index, const char* mode);   // NPS1/NPS2/...
AT_API int at_smi_get_partitions(int index, char* compute, int clen, char* memory, int mlen);

// ---- N6 -------------------------------------------------------------------
typedef struct {
  int32_t index;        // GPU index (amd-smi order)
  int32_t kind;         // AT_EV_*
  int32_t critical;     // 1 -> device must be reported Unhealthy
  char message[128];
} at_event_t;

#define AT_EV_NONE 0
#define AT_EV_VMFAULT 1
#define AT_EV_THERMAL_THROTTLE 2
#define AT_EV_GPU_PRE_RESET 3
#define AT_EV_GPU_POST_RESET 4
#define AT_EV_ECC_UNCORRECTABLE 100
#define AT_EV_XGMI_LINK_ERROR 101
#define AT_EV_DEVICE_LOST 102
#define AT_EV_BAD_PAGES 103

// Starts event notification on every GPU (best effort).
AT_API int at_health_start(void);
AT_API void at_health_stop(void);
// Waits up to timeout_ms for driver events, then polls ECC / xGMI / bad-page
// counters against the previous poll and reports increases as events.
AT_API int at_health_poll(int timeout_ms, at_event_t* out, int max, int* count);

#ifdef __cplusplus
}
#endif

#endif  // AMDGPU_TOPO_H_
