// Run-time loader for libamd_smi: dlopen + dlsym into a typed function table.
//
// This is the MI355X equivalent of the reference's vendored libltdl.so.7 (SURVEY.md N1;
// /root/reference/Dockerfile:4): it decouples the exporter from the host's tool-library ABI.
// The exporter binary links against nothing from ROCm; a missing optional symbol disables the
// metric that needs it (NOT_SUPPORTED path) instead of failing the load. amdsmi.h is used for
// types only.
#pragma once

#include <amd_smi/amdsmi.h>

#include <string>

namespace gpumon {

#define GPUMON_SMI_REQUIRED(X)          \
  X(amdsmi_init)                        \
  X(amdsmi_shut_down)                   \
  X(amdsmi_get_socket_handles)          \
  X(amdsmi_get_processor_handles)

#define GPUMON_SMI_OPTIONAL(X)          \
  X(amdsmi_get_lib_version)             \
  X(amdsmi_get_processor_type)          \
  X(amdsmi_get_gpu_enumeration_info)    \
  X(amdsmi_get_gpu_device_uuid)         \
  X(amdsmi_get_gpu_device_bdf)          \
  X(amdsmi_get_gpu_asic_info)           \
  X(amdsmi_get_gpu_kfd_info)            \
  X(amdsmi_get_gpu_board_info)          \
  X(amdsmi_get_gpu_driver_info)         \
  X(amdsmi_get_gpu_compute_partition)   \
  X(amdsmi_get_gpu_memory_partition)    \
  X(amdsmi_get_gpu_metrics_info)        \
  X(amdsmi_get_gpu_vram_usage)          \
  X(amdsmi_get_gpu_activity)            \
  X(amdsmi_get_power_info)              \
  X(amdsmi_get_energy_count)            \
  X(amdsmi_get_gpu_process_list)        \
  X(amdsmi_get_link_metrics)            \
  X(amdsmi_get_temp_metric)             \
  X(amdsmi_get_clock_info)             \
  X(amdsmi_get_gpu_ecc_count)          \
  X(amdsmi_get_gpu_bad_page_info)

struct SmiTable {
  void* dl = nullptr;
  std::string path;
#define GPUMON_DECL(fn) decltype(&::fn) fn = nullptr;
  GPUMON_SMI_REQUIRED(GPUMON_DECL)
  GPUMON_SMI_OPTIONAL(GPUMON_DECL)
#undef GPUMON_DECL

  // Tries `explicit_path`, $GPUMON_AMDSMI_LIB, then the usual sonames/paths.
  bool load(const std::string& explicit_path, std::string* err);
  void unload();
  ~SmiTable() { unload(); }
};

const char* smi_status_str(int status);

}  // namespace gpumon
