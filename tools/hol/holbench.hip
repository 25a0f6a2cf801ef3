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
// holbench --seconds S --start-ns T --grid G --spin-us U --lds B --depth D [--phases P]
//   G = 0: one workgroup per resident slot of the mask ("fit"), G < 0:
//   -G x fit ("oversubscribed").  --phases P > 0: "megakernel" mode -- each
//   launch runs P spin phases separated by a grid-wide barrier (grid must be
//   "fit": every workgroup resident), so a pod keeps at most `depth` packets in
//   its queue for P phases of work.  The barrier gives up after 250 ms (flag
//   in the output) so a non-resident grid can never hang the GPU.
//   Prints one JSON line.
#include <hip/hip_ext.h>
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

// the work of one workgroup: spin on the realtime counter (iters == 0) or a
// fixed VALU chain (iters > 0: 8 independent FMA chains per lane, no memory
// traffic) -- the ALU form does not poll a shared counter, so thousands of
// co-running waves cannot slow each other down through it
__device__ __forceinline__ int work(unsigned long long ticks, int iters) {
  if (iters > 0) {
    float x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = (float)(threadIdx.x + j);
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = fmaf(x[j], 0.999f, 0.5f);
    }
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += x[j];
    return (int)s;
  }
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long t = t0;
  while (t - t0 < ticks) t = __builtin_amdgcn_s_memrealtime();
  return (int)t;
}

__global__ __launch_bounds__(256) void spin_kernel(unsigned long long ticks, int iters, int* sink) {
  extern __shared__ int lds[];
  lds[threadIdx.x] = work(ticks, iters);
  __syncthreads();
  if (lds[(threadIdx.x + 1) & 255] == 0x7fffffff) sink[blockIdx.x] = 1;  // keep LDS live, never taken
}

// grid-wide barrier over `nwg` co-resident workgroups (sense by generation);
// every wave leaves after `limit` realtime ticks even if the grid never meets
__device__ __forceinline__ bool grid_barrier(unsigned* count, unsigned* gen, unsigned nwg, int* abort_flag,
                                             unsigned long long limit) {
  __shared__ int ok;
  __syncthreads();
  if (threadIdx.x == 0) {
    ok = 1;
    const unsigned g = __hip_atomic_load(gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned arrived = __hip_atomic_fetch_add(count, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) + 1;
    if (arrived == nwg) {
      __hip_atomic_store(count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(gen, g + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      while (__hip_atomic_load(gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == g) {
        if (__hip_atomic_load(abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ||
            __builtin_amdgcn_s_memrealtime() - t0 > limit) {
          __hip_atomic_store(abort_flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ok = 0;
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
    }
  }
  __syncthreads();
  return ok != 0;
}

__global__ __launch_bounds__(256) void phases_kernel(unsigned long long ticks, int iters, int phases,
                                                     unsigned* bar, int* abort_flag, int* sink) {
  extern __shared__ int lds[];
  for (int p = 0; p < phases; ++p) {
    lds[threadIdx.x] = work(ticks, iters);
    if (!grid_barrier(bar, bar + 1, gridDim.x, abort_flag, 25000000ull)) return;  // 250 ms
  }
  if (lds[(threadIdx.x + 1) & 255] == 0x7fffffff) sink[blockIdx.x] = 1;
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
  int grid = 0, lds = 40960, depth = 16, null_stream = 0, phases = 0, iters = 0, streams = 1, per_xcd = 4;
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
    else if (k == "--phases") phases = atoi(v);
    else if (k == "--iters") iters = atoi(v);
    else if (k == "--streams") streams = atoi(v);
    else if (k == "--per-xcd") per_xcd = atoi(v);
    else if (k == "--tag") tag = v;
    else {
      fprintf(stderr, "unknown option %s\n", k.c_str());
      return 2;
    }
  }
  if (lds < 1024 || lds > 65536 || depth < 1 || depth > 1024 || seconds <= 0 || seconds > 60 || streams < 1 ||
      streams > 16 || per_xcd < 1 || streams * per_xcd > 32) {
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
  if (phases < 0 || phases > 4096 || (phases > 0 && g > fit)) {
    fprintf(stderr, "--phases needs a grid that fits the mask's slots\n");
    return 2;
  }
  int* sink = nullptr;
  CK(hipMalloc(&sink, sizeof(int) * (size_t)g));
  unsigned* bar = nullptr;
  int* abort_flag = nullptr;
  CK(hipMalloc(&bar, 2 * sizeof(unsigned)));
  CK(hipMalloc(&abort_flag, sizeof(int)));
  CK(hipMemset(bar, 0, 2 * sizeof(unsigned)));
  CK(hipMemset(abort_flag, 0, sizeof(int)));
  if (streams > 1) {
    // one process, `streams` streams each with its own XCD-symmetric CU mask
    // (hipExtStreamCreateWithCUMask: per-queue masks, the in-process analogue of
    // one pod per slice); kernels round-robin over the streams
    const int fit1 = 8 * per_xcd * wg_per_cu;
    std::vector<hipStream_t> ss(streams);
    for (int k = 0; k < streams; ++k) {
      uint32_t m[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (int x = 0; x < 8; ++x)
        for (int j = k * per_xcd; j < (k + 1) * per_xcd; ++j) {
          const int bit = j * 8 + x;
          m[bit / 32] |= 1u << (bit % 32);
        }
      CK(hipExtStreamCreateWithCUMask(&ss[k], 8, m));
    }
    const unsigned long long tk = (unsigned long long)(spin_us * 100.0);
    for (int k = 0; k < streams; ++k)
      hipLaunchKernelGGL(spin_kernel, dim3(fit1), dim3(256), lds, ss[k], tk, iters, sink);
    CK(hipDeviceSynchronize());
    while (start_ns && mono_ns() < start_ns) usleep(200);
    const long long t0 = mono_ns(), t_end = t0 + (long long)(seconds * 1e9);
    long long rounds = 0;
    while (mono_ns() < t_end) {
      for (int d = 0; d < depth; ++d)
        for (int k = 0; k < streams; ++k)
          hipLaunchKernelGGL(spin_kernel, dim3(fit1), dim3(256), lds, ss[k], tk, iters, sink);
      CK(hipDeviceSynchronize());
      rounds += depth;
    }
    const double el = (mono_ns() - t0) / 1e9;
    printf("{\"tag\": \"%s\", \"streams\": %d, \"per_xcd\": %d, \"fit\": %d, \"iters\": %d, \"kernels_per_stream\": %lld, "
           "\"elapsed_s\": %.4f, \"kernel_ms\": %.4f}\n", tag, streams, per_xcd, fit1, iters, rounds, el,
           el * 1e3 / (double)rounds);
    for (auto x : ss) CK(hipStreamDestroy(x));
    return 0;
  }
  hipStream_t st = nullptr;
  if (!null_stream) CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  // realtime counter: 100 MHz on MI300-class parts
  const unsigned long long ticks = (unsigned long long)(spin_us * 100.0);
  auto launch = [&]() {
    if (phases > 0)  // the barrier's own LDS word: keep the per-CU total at (160 KB / lds) workgroups
      hipLaunchKernelGGL(phases_kernel, dim3(g), dim3(256), lds - 1024, st, ticks, iters, phases, bar, abort_flag,
                         sink);
    else
      hipLaunchKernelGGL(spin_kernel, dim3(g), dim3(256), lds, st, ticks, iters, sink);
  };
  launch();  // warm-up
  CK(hipGetLastError());
  CK(hipStreamSynchronize(st));
  while (start_ns && mono_ns() < start_ns) usleep(200);
  const long long t0 = mono_ns();
  const long long t_end = t0 + (long long)(seconds * 1e9);
  long long kernels = 0;
  std::vector<double> batch_ms;
  while (mono_ns() < t_end) {
    const long long b0 = mono_ns();
    for (int d = 0; d < depth; ++d) launch();
    CK(hipStreamSynchronize(st));
    kernels += depth * (phases > 0 ? phases : 1);
    batch_ms.push_back((mono_ns() - b0) / 1e6);
  }
  const double el = (mono_ns() - t0) / 1e9;
  const double wg_per_s = (double)kernels * g / el;
  const double eff = wg_per_s * spin_us * 1e-6 / fit;
  double mn = 1e30, mx = 0;
  for (double v : batch_ms) { mn = v < mn ? v : mn; mx = v > mx ? v : mx; }
  const double ideal_kernel_ms = spin_us * 1e-3 * ((g + fit - 1) / fit);
  int aborted = 0;
  CK(hipMemcpy(&aborted, abort_flag, sizeof(int), hipMemcpyDeviceToHost));
  printf("{\"tag\": \"%s\", \"pid\": %d, \"cus\": %d, \"mask\": \"%s\", \"wg_per_cu\": %d, \"fit\": %d, \"grid\": %d, "
         "\"spin_us\": %.1f, \"depth\": %d, \"null_stream\": %d, \"kernels\": %lld, \"elapsed_s\": %.4f, "
         "\"kernel_ms\": %.4f, \"ideal_kernel_ms\": %.4f, \"slot_efficiency\": %.4f, \"batch_ms_min\": %.3f, "
         "\"batch_ms_max\": %.3f, \"t0_ns\": %lld, \"phases\": %d, \"barrier_aborted\": %d, \"iters\": %d}\n",
         tag, (int)getpid(), cus, mask ? mask : "", wg_per_cu, fit, g, spin_us, depth, null_stream, kernels, el,
         el * 1e3 / (double)kernels, ideal_kernel_ms, eff, mn, mx, t0, phases, aborted, iters);
  fflush(stdout);
  CK(hipFree(sink));
  CK(hipFree(bar));
  CK(hipFree(abort_flag));
  if (st) CK(hipStreamDestroy(st));
  return 0;
}
