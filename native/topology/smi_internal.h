// Shared dlopen'ed libamd_smi function table (smi.cpp <-> health.cpp).
#ifndef AMDGPU_SMI_INTERNAL_H_
#define AMDGPU_SMI_INTERNAL_H_

#include <amd_smi/amdsmi.h>

#include <vector>

namespace at_smi {

struct Api {
  void* dl = nullptr;
  amdsmi_status_t (*init)(uint64_t) = nullptr;
  amdsmi_status_t (*shut_down)(void) = nullptr;
  amdsmi_status_t (*get_socket_handles)(uint32_t*, amdsmi_socket_handle*) = nullptr;
  amdsmi_status_t (*get_processor_handles)(amdsmi_socket_handle, uint32_t*, amdsmi_processor_handle*) = nullptr;
  amdsmi_status_t (*get_bdf)(amdsmi_processor_handle, amdsmi_bdf_t*) = nullptr;
  amdsmi_status_t (*get_uuid)(amdsmi_processor_handle, unsigned int*, char*) = nullptr;
  amdsmi_status_t (*get_asic)(amdsmi_processor_handle, amdsmi_asic_info_t*) = nullptr;
  amdsmi_status_t (*mem_total)(amdsmi_processor_handle, amdsmi_memory_type_t, uint64_t*) = nullptr;
  amdsmi_status_t (*mem_usage)(amdsmi_processor_handle, amdsmi_memory_type_t, uint64_t*) = nullptr;
  amdsmi_status_t (*activity)(amdsmi_processor_handle, amdsmi_engine_usage_t*) = nullptr;
  amdsmi_status_t (*power)(amdsmi_processor_handle, amdsmi_power_info_t*) = nullptr;
  amdsmi_status_t (*temp)(amdsmi_processor_handle, amdsmi_temperature_type_t, amdsmi_temperature_metric_t, int64_t*) = nullptr;
  amdsmi_status_t (*clock)(amdsmi_processor_handle, amdsmi_clk_type_t, amdsmi_clk_info_t*) = nullptr;
  amdsmi_status_t (*energy)(amdsmi_processor_handle, uint64_t*, float*, uint64_t*) = nullptr;
  amdsmi_status_t (*ecc)(amdsmi_processor_handle, amdsmi_error_count_t*) = nullptr;
  amdsmi_status_t (*xgmi_status)(amdsmi_processor_handle, amdsmi_xgmi_link_status_t*) = nullptr;
  amdsmi_status_t (*bad_pages)(amdsmi_processor_handle, uint32_t*, amdsmi_retired_page_record_t*) = nullptr;
  amdsmi_status_t (*procs)(amdsmi_processor_handle, uint32_t*, amdsmi_proc_info_t*) = nullptr;
  amdsmi_status_t (*driver)(amdsmi_processor_handle, amdsmi_driver_info_t*) = nullptr;
  amdsmi_status_t (*get_cpart)(amdsmi_processor_handle, char*, uint32_t) = nullptr;
  amdsmi_status_t (*get_mpart)(amdsmi_processor_handle, char*, uint32_t) = nullptr;
  amdsmi_status_t (*set_cpart)(amdsmi_processor_handle, amdsmi_compute_partition_type_t) = nullptr;
  amdsmi_status_t (*set_mpart)(amdsmi_processor_handle, amdsmi_memory_partition_type_t) = nullptr;
  amdsmi_status_t (*evt_init)(amdsmi_processor_handle) = nullptr;
  amdsmi_status_t (*evt_mask)(amdsmi_processor_handle, uint64_t) = nullptr;
  amdsmi_status_t (*evt_get)(int, uint32_t*, amdsmi_evt_notification_data_t*) = nullptr;
  amdsmi_status_t (*evt_stop)(amdsmi_processor_handle) = nullptr;
  amdsmi_status_t (*gpu_metrics)(amdsmi_processor_handle, amdsmi_gpu_metrics_t*) = nullptr;
  std::vector<amdsmi_processor_handle> gpus;
};

extern Api g_api;

}  // namespace at_smi

#endif  // AMDGPU_SMI_INTERNAL_H_
