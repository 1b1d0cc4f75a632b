// nos amd-smi backend: a C ABI over libamd_smi for the partition agent.
//
// Replaces the reference's NVML/cgo client (reference pkg/gpu/nvml/client.go:31-511). On MI355X a
// "partition change" is one amdsmi_set_gpu_compute_partition call per physical GPU (homogeneous
// SPX/DPX/QPX/CPX) plus an optional node-wide memory-partition (NPS) change, so the reference's
// GPU-instance/compute-instance bookkeeping and its n! creation-order search disappear.
//
// What does NOT disappear is re-enumeration: after SPX -> CPX amd-smi reports one processor per
// partition (8 per GPU), each with its own UUID, KFD node, render node and HIP ordinal, and the
// handles taken before the switch are stale. So this backend exposes *processors* (not GPUs), and
// nos_smi_enumerate(reinit=1) shuts the session down and re-initialises it before listing them
// again. Grouping processors into physical GPUs (by BDF) is done by the caller
// (walkai_nos_amd/device/topology.py). The reference reaches the same freshness by running
// nvml.Init/Shutdown around every call (client.go:46-57).
//
// Return codes: 0 ok, 1 generic, 2 permission, 3 not found, 4 busy. No HIP is linked or loaded.
#include <amd_smi/amdsmi.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

namespace {

std::mutex g_mu;
bool g_init = false;
std::vector<amdsmi_processor_handle> g_procs;
thread_local std::string g_err;

int map_status(amdsmi_status_t st, const char* what) {
  if (st == AMDSMI_STATUS_SUCCESS) return 0;
  const char* s = nullptr;
  amdsmi_status_code_to_string(st, &s);
  g_err = std::string(what) + ": " + (s ? s : "amdsmi error") + " (" + std::to_string(int(st)) + ")";
  switch (st) {
    case AMDSMI_STATUS_NO_PERM: return 2;
    case AMDSMI_STATUS_NOT_FOUND: return 3;
    case AMDSMI_STATUS_BUSY: return 4;
    default: return 1;
  }
}

int handle(uint32_t idx, amdsmi_processor_handle* h) {
  if (!g_init) { g_err = "amdsmi not initialised"; return 1; }
  if (idx >= g_procs.size()) { g_err = "processor index out of range (re-enumerate after a partition change)"; return 3; }
  *h = g_procs[idx];
  return 0;
}

// caller holds g_mu
int list_processors() {
  g_procs.clear();
  uint32_t nsock = 0;
  amdsmi_status_t st = amdsmi_get_socket_handles(&nsock, nullptr);
  if (st != AMDSMI_STATUS_SUCCESS) return map_status(st, "amdsmi_get_socket_handles");
  std::vector<amdsmi_socket_handle> socks(nsock);
  st = amdsmi_get_socket_handles(&nsock, socks.data());
  if (st != AMDSMI_STATUS_SUCCESS) return map_status(st, "amdsmi_get_socket_handles");
  for (uint32_t s = 0; s < nsock; ++s) {
    uint32_t n = 0;
    if (amdsmi_get_processor_handles(socks[s], &n, nullptr) != AMDSMI_STATUS_SUCCESS) continue;
    std::vector<amdsmi_processor_handle> hs(n);
    if (amdsmi_get_processor_handles(socks[s], &n, hs.data()) != AMDSMI_STATUS_SUCCESS) continue;
    for (uint32_t i = 0; i < n; ++i) {
      processor_type_t t;
      if (amdsmi_get_processor_type(hs[i], &t) == AMDSMI_STATUS_SUCCESS && t == AMDSMI_PROCESSOR_TYPE_AMD_GPU)
        g_procs.push_back(hs[i]);
    }
  }
  return 0;
}

// caller holds g_mu
int open_session() {
  amdsmi_status_t st = amdsmi_init(AMDSMI_INIT_AMD_GPUS);
  if (st != AMDSMI_STATUS_SUCCESS) return map_status(st, "amdsmi_init");
  g_init = true;
  return list_processors();
}

}  // namespace

extern "C" {

struct nos_proc_info {
  uint32_t ordinal;
  char uuid[64];
  char bdf[32];          // physical GPU, "dddd:bb:dd.f"
  char market_name[64];
  char hip_uuid[64];
  uint64_t bdf_id;       // KFD location id incl. partition bits [31:28]
  uint64_t kfd_id;
  uint64_t vram_bytes;
  uint32_t partition_id; // 0xFFFFFFFF if the driver does not report one
  int32_t kfd_node;
  int32_t hip_id;
  int32_t hsa_id;
  int32_t render_minor;
  uint32_t cu_count;
  uint32_t xcds;
};

const char* nos_smi_last_error() { return g_err.c_str(); }

int nos_smi_init() {
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_init) return 0;
  return open_session();
}

int nos_smi_shutdown() {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_init) return 0;
  g_procs.clear();
  g_init = false;
  return map_status(amdsmi_shut_down(), "amdsmi_shut_down");
}

// Re-list processors; with reinit the session is closed and reopened first, which is required
// after a compute/memory partition change. Returns the processor count, or -1.
int nos_smi_enumerate(int reinit) {
  std::lock_guard<std::mutex> lk(g_mu);
  int rc = 0;
  if (g_init && reinit) {
    g_procs.clear();
    g_init = false;
    amdsmi_shut_down();
  }
  rc = g_init ? list_processors() : open_session();
  return rc ? -1 : int(g_procs.size());
}

int nos_smi_proc_info(uint32_t idx, nos_proc_info* out) {
  std::lock_guard<std::mutex> lk(g_mu);
  amdsmi_processor_handle h;
  if (int rc = handle(idx, &h)) return rc;
  std::memset(out, 0, sizeof(*out));
  out->ordinal = idx;
  out->partition_id = 0xFFFFFFFFu;
  out->kfd_node = out->hip_id = out->hsa_id = out->render_minor = -1;
  unsigned int ulen = sizeof(out->uuid);
  amdsmi_get_gpu_device_uuid(h, &ulen, out->uuid);
  amdsmi_bdf_t bdf;
  if (amdsmi_get_gpu_device_bdf(h, &bdf) == AMDSMI_STATUS_SUCCESS) {
    std::snprintf(out->bdf, sizeof(out->bdf), "%04llx:%02llx:%02llx.%llx",
                  (unsigned long long)bdf.domain_number, (unsigned long long)bdf.bus_number,
                  (unsigned long long)bdf.device_number, (unsigned long long)bdf.function_number);
  }
  uint64_t bdfid = 0;
  if (amdsmi_get_gpu_bdf_id(h, &bdfid) == AMDSMI_STATUS_SUCCESS) out->bdf_id = bdfid;
  amdsmi_kfd_info_t kfd;
  if (amdsmi_get_gpu_kfd_info(h, &kfd) == AMDSMI_STATUS_SUCCESS) {
    out->kfd_id = kfd.kfd_id;
    if (kfd.node_id != 0xFFFFFFFFu) out->kfd_node = int32_t(kfd.node_id);
    out->partition_id = kfd.current_partition_id;
  }
  amdsmi_enumeration_info_t en;
  if (amdsmi_get_gpu_enumeration_info(h, &en) == AMDSMI_STATUS_SUCCESS) {
    out->hip_id = int32_t(en.hip_id);
    out->hsa_id = int32_t(en.hsa_id);
    out->render_minor = int32_t(en.drm_render);
    std::snprintf(out->hip_uuid, sizeof(out->hip_uuid), "%.63s", en.hip_uuid);
  }
  amdsmi_asic_info_t asic;
  if (amdsmi_get_gpu_asic_info(h, &asic) == AMDSMI_STATUS_SUCCESS) {
    std::snprintf(out->market_name, sizeof(out->market_name), "%.63s", asic.market_name);
    if (asic.num_of_compute_units != 0xFFFFFFFFu) out->cu_count = asic.num_of_compute_units;
  }
  uint64_t total = 0;
  if (amdsmi_get_gpu_memory_total(h, AMDSMI_MEM_TYPE_VRAM, &total) == AMDSMI_STATUS_SUCCESS) out->vram_bytes = total;
  uint16_t xcd = 0;
  if (amdsmi_get_gpu_xcd_counter(h, &xcd) == AMDSMI_STATUS_SUCCESS && xcd > 0) out->xcds = xcd;
  return 0;
}

int nos_smi_get_compute_partition(uint32_t idx, char* buf, uint32_t len) {
  std::lock_guard<std::mutex> lk(g_mu);
  amdsmi_processor_handle h;
  if (int rc = handle(idx, &h)) return rc;
  return map_status(amdsmi_get_gpu_compute_partition(h, buf, len), "amdsmi_get_gpu_compute_partition");
}

int nos_smi_get_memory_partition(uint32_t idx, char* buf, uint32_t len) {
  std::lock_guard<std::mutex> lk(g_mu);
  amdsmi_processor_handle h;
  if (int rc = handle(idx, &h)) return rc;
  return map_status(amdsmi_get_gpu_memory_partition(h, buf, len), "amdsmi_get_gpu_memory_partition");
}

int nos_smi_set_compute_partition(uint32_t idx, const char* mode) {
  std::lock_guard<std::mutex> lk(g_mu);
  amdsmi_processor_handle h;
  if (int rc = handle(idx, &h)) return rc;
  amdsmi_compute_partition_type_t t = AMDSMI_COMPUTE_PARTITION_INVALID;
  std::string m(mode);
  if (m == "SPX") t = AMDSMI_COMPUTE_PARTITION_SPX;
  else if (m == "DPX") t = AMDSMI_COMPUTE_PARTITION_DPX;
  else if (m == "TPX") t = AMDSMI_COMPUTE_PARTITION_TPX;
  else if (m == "QPX") t = AMDSMI_COMPUTE_PARTITION_QPX;
  else if (m == "CPX") t = AMDSMI_COMPUTE_PARTITION_CPX;
  else { g_err = "invalid compute partition " + m; return 1; }
  return map_status(amdsmi_set_gpu_compute_partition(h, t), "amdsmi_set_gpu_compute_partition");
}

int nos_smi_set_memory_partition(uint32_t idx, const char* mode) {
  std::lock_guard<std::mutex> lk(g_mu);
  amdsmi_processor_handle h;
  if (int rc = handle(idx, &h)) return rc;
  amdsmi_memory_partition_type_t t = AMDSMI_MEMORY_PARTITION_UNKNOWN;
  std::string m(mode);
  if (m == "NPS1") t = AMDSMI_MEMORY_PARTITION_NPS1;
  else if (m == "NPS2") t = AMDSMI_MEMORY_PARTITION_NPS2;
  else if (m == "NPS4") t = AMDSMI_MEMORY_PARTITION_NPS4;
  else if (m == "NPS8") t = AMDSMI_MEMORY_PARTITION_NPS8;
  else { g_err = "invalid memory partition " + m; return 1; }
  return map_status(amdsmi_set_gpu_memory_partition(h, t), "amdsmi_set_gpu_memory_partition");
}

// Processes with a KFD context on this processor (a compute-partition switch destroys them all).
int nos_smi_process_count(uint32_t idx) {
  std::lock_guard<std::mutex> lk(g_mu);
  amdsmi_processor_handle h;
  if (handle(idx, &h)) return -1;
  uint32_t n = 0;
  amdsmi_status_t st = amdsmi_get_gpu_process_list(h, &n, nullptr);
  if (st != AMDSMI_STATUS_SUCCESS && st != AMDSMI_STATUS_OUT_OF_RESOURCES) {
    map_status(st, "amdsmi_get_gpu_process_list");
    return -1;
  }
  return int(n);
}

// Per-process VRAM on this processor (the HBM budget guard's input): fills up to cap (pid, bytes)
// pairs and returns how many processes hold a context (may exceed cap), or -1.
int nos_smi_process_memory(uint32_t idx, uint32_t* pids, uint64_t* vram, uint32_t cap) {
  std::lock_guard<std::mutex> lk(g_mu);
  amdsmi_processor_handle h;
  if (handle(idx, &h)) return -1;
  uint32_t n = 0;
  amdsmi_status_t st = amdsmi_get_gpu_process_list(h, &n, nullptr);
  if (st != AMDSMI_STATUS_SUCCESS && st != AMDSMI_STATUS_OUT_OF_RESOURCES) {
    map_status(st, "amdsmi_get_gpu_process_list");
    return -1;
  }
  if (n == 0 || cap == 0) return int(n);
  std::vector<amdsmi_proc_info_t> list(n);
  uint32_t got = n;
  st = amdsmi_get_gpu_process_list(h, &got, list.data());
  if (st != AMDSMI_STATUS_SUCCESS && st != AMDSMI_STATUS_OUT_OF_RESOURCES) {
    map_status(st, "amdsmi_get_gpu_process_list");
    return -1;
  }
  uint32_t k = got < n ? got : n;
  for (uint32_t i = 0; i < k && i < cap; ++i) {
    pids[i] = uint32_t(list[i].pid);
    vram[i] = list[i].memory_usage.vram_mem ? list[i].memory_usage.vram_mem : list[i].mem;
  }
  return int(got);
}

// Per-process VRAM, CU occupancy and queue-eviction time on this processor (the slice guards'
// input): cu_occupancy is the KFD's CU-equivalents of the process's waves in flight (waves /
// waves-per-CU, sampled when read), evicted_ms the time its queues spent evicted (time-sliced
// out by the hardware scheduler). Fills up to cap entries; returns the process count, or -1.
int nos_smi_process_info(uint32_t idx, uint32_t* pids, uint64_t* vram, uint32_t* cu_occupancy,
                         uint32_t* evicted_ms, uint32_t cap) {
  std::lock_guard<std::mutex> lk(g_mu);
  amdsmi_processor_handle h;
  if (handle(idx, &h)) return -1;
  uint32_t n = 0;
  amdsmi_status_t st = amdsmi_get_gpu_process_list(h, &n, nullptr);
  if (st != AMDSMI_STATUS_SUCCESS && st != AMDSMI_STATUS_OUT_OF_RESOURCES) {
    map_status(st, "amdsmi_get_gpu_process_list");
    return -1;
  }
  if (n == 0 || cap == 0) return int(n);
  std::vector<amdsmi_proc_info_t> list(n);
  uint32_t got = n;
  st = amdsmi_get_gpu_process_list(h, &got, list.data());
  if (st != AMDSMI_STATUS_SUCCESS && st != AMDSMI_STATUS_OUT_OF_RESOURCES) {
    map_status(st, "amdsmi_get_gpu_process_list");
    return -1;
  }
  uint32_t k = got < n ? got : n;
  for (uint32_t i = 0; i < k && i < cap; ++i) {
    pids[i] = uint32_t(list[i].pid);
    vram[i] = list[i].memory_usage.vram_mem ? list[i].memory_usage.vram_mem : list[i].mem;
    cu_occupancy[i] = list[i].cu_occupancy;
    evicted_ms[i] = list[i].evicted_time;
  }
  return int(got);
}

int nos_smi_activity(uint32_t idx, uint32_t* gfx, uint32_t* umc, uint32_t* mm) {
  std::lock_guard<std::mutex> lk(g_mu);
  amdsmi_processor_handle h;
  if (int rc = handle(idx, &h)) return rc;
  amdsmi_engine_usage_t u;
  int rc = map_status(amdsmi_get_gpu_activity(h, &u), "amdsmi_get_gpu_activity");
  if (rc) return rc;
  *gfx = u.gfx_activity; *umc = u.umc_activity; *mm = u.mm_activity;
  return 0;
}

// Socket power (W), its limit (W) and the current / max GFX clock (MHz): a fully busy MI355X is
// power-capped and clocks its matrix pipes down (profiles/clock_under_mfma_load_r2.json), which
// is what bounds the aggregate throughput of concurrently busy partitions.
int nos_smi_power_clock(uint32_t idx, uint32_t* watts, uint32_t* limit_w, uint32_t* gfx_mhz, uint32_t* gfx_max_mhz) {
  std::lock_guard<std::mutex> lk(g_mu);
  amdsmi_processor_handle h;
  if (int rc = handle(idx, &h)) return rc;
  *watts = *limit_w = *gfx_mhz = *gfx_max_mhz = 0;
  amdsmi_power_info_t p;
  int rc = map_status(amdsmi_get_power_info(h, &p), "amdsmi_get_power_info");
  if (rc == 0) {
    *watts = p.current_socket_power != 0xFFFFFFFFu ? p.current_socket_power
                                                    : (p.average_socket_power != 0xFFFFFFFFu ? p.average_socket_power : 0);
    *limit_w = p.power_limit != 0xFFFFFFFFu ? p.power_limit : 0;
  }
  amdsmi_clk_info_t c;
  if (amdsmi_get_clock_info(h, AMDSMI_CLK_TYPE_GFX, &c) == AMDSMI_STATUS_SUCCESS) {
    *gfx_mhz = c.clk;
    *gfx_max_mhz = c.max_clk;
  }
  return rc;
}

int nos_smi_vram(uint32_t idx, uint64_t* total, uint64_t* used) {
  std::lock_guard<std::mutex> lk(g_mu);
  amdsmi_processor_handle h;
  if (int rc = handle(idx, &h)) return rc;
  int rc = map_status(amdsmi_get_gpu_memory_total(h, AMDSMI_MEM_TYPE_VRAM, total), "amdsmi_get_gpu_memory_total");
  if (rc) return rc;
  return map_status(amdsmi_get_gpu_memory_usage(h, AMDSMI_MEM_TYPE_VRAM, used), "amdsmi_get_gpu_memory_usage");
}

}  // extern "C"
