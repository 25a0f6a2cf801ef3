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
