// Dispatch head-of-line microbenchmark for CU-mask slices on MI355X.
//
// One process = one "pod": it runs with the device plugin's ROC_GLOBAL_CU_MASK
// and launches a chain of fixed-duration workgroups (each spins on the
// realtime counter for --spin-us) back to back on one stream.  Because every
// workgroup holds its slot for exactly the same time, the workgroups a pod
// completes per second divided by its slot capacity (masked CUs x workgroups
// per CU, set by the LDS each workgroup reserves) is the share of its slice
// the dispatcher actually kept busy.  A pod alone should read ~1.0; pods on
// disjoint masks should read ~1.0 each unless the command processor's pipes
// serialise them (head-of-line blocking of a dispatch whose masked CUs are
// full, or of a queue waiting on the previous kernel's barrier).
//
// holbench --seconds S --start-ns T --grid G --spin-us U --lds B --depth D
//   G = 0: one workgroup per resident slot of the mask ("fit"), G < 0:
//   -G x fit ("oversubscribed").  Prints one JSON line.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include <string>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                 \
    }                                                                          \
  } while (0)

__global__ __launch_bounds__(256) void spin_kernel(unsigned long long ticks, int* sink) {
  extern __shared__ int lds[];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long t = t0;
  while (t - t0 < ticks) t = __builtin_amdgcn_s_memrealtime();
  lds[threadIdx.x] = (int)t;
  __syncthreads();
  if (lds[(threadIdx.x + 1) & 255] == 0x7fffffff) sink[blockIdx.x] = 1;  // keep LDS live, never taken
}

static long long mono_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1000000000LL + ts.tv_nsec;
}

static int popcount_hex_mask(const char* s) {
  if (!s || !*s) return -1;
  if (s[0] == '0' && (s[1] == 'x' || s[1] == 'X')) s += 2;
  int n = 0;
  for (; *s; ++s) {
    char c = *s;
    int v = (c >= '0' && c <= '9') ? c - '0' : (c >= 'a' && c <= 'f') ? c - 'a' + 10
                                               : (c >= 'A' && c <= 'F') ? c - 'A' + 10 : 0;
    n += __builtin_popcount(v);
  }
  return n;
}

int main(int argc, char** argv) {
  double seconds = 3.0, spin_us = 50.0;
  long long start_ns = 0;
  int grid = 0, lds = 40960, depth = 16, null_stream = 0;
  const char* tag = "";
  for (int i = 1; i + 1 < argc; i += 2) {
    std::string k = argv[i];
    const char* v = argv[i + 1];
    if (k == "--seconds") seconds = atof(v);
    else if (k == "--start-ns") start_ns = atoll(v);
    else if (k == "--grid") grid = atoi(v);
    else if (k == "--spin-us") spin_us = atof(v);
    else if (k == "--lds") lds = atoi(v);
    else if (k == "--depth") depth = atoi(v);
    else if (k == "--null-stream") null_stream = atoi(v);
    else if (k == "--tag") tag = v;
    else {
      fprintf(stderr, "unknown option %s\n", k.c_str());
      return 2;
    }
  }
  if (lds < 1024 || lds > 65536 || depth < 1 || depth > 1024 || seconds <= 0 || seconds > 60) {
    fprintf(stderr, "bad arguments\n");
    return 2;
  }
  CK(hipSetDevice(0));
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  const char* mask = getenv("ROC_GLOBAL_CU_MASK");
  int cus = popcount_hex_mask(mask);
  if (cus <= 0 || cus > p.multiProcessorCount) cus = p.multiProcessorCount;
  // gfx950: 160 KB LDS per CU (one workgroup may allocate at most 64 KB);
  // 256-thread workgroups: at most 8 per CU by waves (32 waves / 4)
  const int wg_per_cu = (160 * 1024) / lds < 8 ? (160 * 1024) / lds : 8;
  const int fit = cus * wg_per_cu;
  const int g = grid > 0 ? grid : grid == 0 ? fit : -grid * fit;
  int* sink = nullptr;
  CK(hipMalloc(&sink, sizeof(int) * (size_t)g));
  hipStream_t st = nullptr;
  if (!null_stream) CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  // realtime counter: 100 MHz on MI300-class parts
  const unsigned long long ticks = (unsigned long long)(spin_us * 100.0);
  hipLaunchKernelGGL(spin_kernel, dim3(g), dim3(256), lds, st, ticks, sink);  // warm-up
  CK(hipGetLastError());
  CK(hipStreamSynchronize(st));
  while (start_ns && mono_ns() < start_ns) usleep(200);
  const long long t0 = mono_ns();
  const long long t_end = t0 + (long long)(seconds * 1e9);
  long long kernels = 0;
  std::vector<double> batch_ms;
  while (mono_ns() < t_end) {
    const long long b0 = mono_ns();
    for (int d = 0; d < depth; ++d) hipLaunchKernelGGL(spin_kernel, dim3(g), dim3(256), lds, st, ticks, sink);
    CK(hipStreamSynchronize(st));
    kernels += depth;
    batch_ms.push_back((mono_ns() - b0) / 1e6);
  }
  const double el = (mono_ns() - t0) / 1e9;
  const double wg_per_s = (double)kernels * g / el;
  const double eff = wg_per_s * spin_us * 1e-6 / fit;
  double mn = 1e30, mx = 0;
  for (double v : batch_ms) { mn = v < mn ? v : mn; mx = v > mx ? v : mx; }
  const double ideal_kernel_ms = spin_us * 1e-3 * ((g + fit - 1) / fit);
  printf("{\"tag\": \"%s\", \"pid\": %d, \"cus\": %d, \"mask\": \"%s\", \"wg_per_cu\": %d, \"fit\": %d, \"grid\": %d, "
         "\"spin_us\": %.1f, \"depth\": %d, \"null_stream\": %d, \"kernels\": %lld, \"elapsed_s\": %.4f, "
         "\"kernel_ms\": %.4f, \"ideal_kernel_ms\": %.4f, \"slot_efficiency\": %.4f, \"batch_ms_min\": %.3f, "
         "\"batch_ms_max\": %.3f, \"t0_ns\": %lld}\n",
         tag, (int)getpid(), cus, mask ? mask : "", wg_per_cu, fit, g, spin_us, depth, null_stream, kernels, el,
         el * 1e3 / (double)kernels, ideal_kernel_ms, eff, mn, mx, t0);
  fflush(stdout);
  CK(hipFree(sink));
  if (st) CK(hipStreamDestroy(st));
  return 0;
}
