// Host-side HIP runtime helpers: CU-masked streams (the enforcement
// mechanism of cumask slices inside one process), device facts, graph-free
// synchronisation helpers.
//
// A cumask slice handed to a pod by the nos-amd device plugin is applied to a
// whole process with ROC_GLOBAL_CU_MASK; in-process tenants (bench.py, the
// gpuagent probes) get the same hardware mechanism per HW queue through
// hipExtStreamCreateWithCUMask.  Masks are arrays of 32-bit words, bit i =
// logical CU i as the HIP runtime numbers them (docs/cumask.md describes how
// probe_placement maps that numbering to XCDs).
#include "common.h"

#include <mutex>
#include <unordered_map>

namespace {
int g_cu_budget = 0;  // 0: no budget (one workgroup per item)
std::mutex g_occ_mu;
std::unordered_map<unsigned long long, int> g_occ;  // (kernel, lds) -> resident workgroups per CU
}  // namespace

// CUs this process may use (a CU-mask slice's popcount); 0 switches the cap off.
NOS_API int nos_set_cu_budget(int cus) {
  if (cus < 0) return (int)hipErrorInvalidValue;
  g_cu_budget = cus;
  return 0;
}

NOS_API int nos_get_cu_budget() { return g_cu_budget; }

int nos_effective_cus() {
  if (g_cu_budget > 0) return g_cu_budget;
  static int cached[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cached[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cached[dev] = n;
  }
  return cached[dev];
}

int nos_grid_for(const void* kernel, int block_threads, size_t lds_bytes, long long items) {
  if (g_cu_budget <= 0 || items <= 8) return (int)items;
  const unsigned long long key = (unsigned long long)(uintptr_t)kernel ^ ((unsigned long long)lds_bytes << 48);
  int occ = 0;
  {
    std::lock_guard<std::mutex> lk(g_occ_mu);
    auto it = g_occ.find(key);
    if (it != g_occ.end()) occ = it->second;
  }
  if (occ == 0) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kernel, block_threads, lds_bytes) != hipSuccess ||
        occ <= 0)
      occ = 1;
    std::lock_guard<std::mutex> lk(g_occ_mu);
    g_occ[key] = occ;
  }
  long long cap = (long long)occ * g_cu_budget;
  cap -= cap % 8;
  if (cap < 8) cap = 8;
  return (int)(items < cap ? items : cap);
}

NOS_API int nos_stream_create_cumask(const unsigned* mask_words, int nwords, void** out_stream) {
  hipStream_t s = nullptr;
  hipError_t e;
  if (nwords <= 0 || mask_words == nullptr)
    e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  else
    e = hipExtStreamCreateWithCUMask(&s, (uint32_t)nwords, mask_words);
  *out_stream = (void*)s;
  return (int)e;
}

NOS_API int nos_stream_get_cumask(void* stream, int nwords, unsigned* out_words) {
  return (int)hipExtStreamGetCUMask((hipStream_t)stream, (uint32_t)nwords, out_words);
}

NOS_API int nos_stream_destroy(void* stream) { return (int)hipStreamDestroy((hipStream_t)stream); }

NOS_API int nos_stream_sync(void* stream) { return (int)hipStreamSynchronize((hipStream_t)stream); }

// Device facts used by the gpuagent / bench: CU count, arch name, memory.
NOS_API int nos_device_info(int dev, int* num_cus, long long* total_mem, int* clock_khz,
                            char* arch, int arch_len) {
  hipDeviceProp_t p;
  HIP_CHECK_RET(hipGetDeviceProperties(&p, dev));
  *num_cus = p.multiProcessorCount;
  *total_mem = (long long)p.totalGlobalMem;
  *clock_khz = p.clockRate;
  int i = 0;
  for (; i < arch_len - 1 && p.gcnArchName[i]; ++i) arch[i] = p.gcnArchName[i];
  arch[i] = 0;
  return 0;
}

NOS_API int nos_runtime_version(int* v) { return (int)hipRuntimeGetVersion(v); }
