// Shared helpers for the nos_amd gfx950 (CDNA4, MI355X) kernels.
//
// Every kernel in this directory is written for 64-lane wavefronts and the
// gfx950 MFMA fragment layouts (see docs/kernels.md).  Host entry points are
// plain `extern "C"` functions taking raw device pointers and a hipStream_t so
// the Python side can call them through ctypes and capture them into HIP graphs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define NOS_API extern "C" __attribute__((visibility("default")))

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4_t;
typedef __attribute__((ext_vector_type(8))) short s16x8_t;
typedef __attribute__((ext_vector_type(4))) short s16x4_t;
typedef __attribute__((ext_vector_type(16))) float f32x16_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(2))) float f32x2_t;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;

#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))

namespace nos {

__device__ __forceinline__ float bf16_to_f32(unsigned short u) {
  return __uint_as_float(((unsigned)u) << 16);
}

// Round-to-nearest-even f32 -> bf16 via the hardware cvt (keeps NaN a NaN).
__device__ __forceinline__ unsigned short f32_to_bf16(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(unsigned short, b);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// XCD-aware bijective remap of a linear workgroup id: blocks that the
// dispatcher deals to the same XCD (same id % 8) receive a contiguous range of
// work items, so neighbouring tiles share that XCD's L2.  Speed only.
__device__ __forceinline__ int xcd_remap(int id, int nwg) {
  const int nx = 8;
  if (nwg <= nx) return id;
  const int xcd = id % nx, idx = id / nx;
  const int q = nwg / nx, r = nwg % nx;
  const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + idx;
}

// Persistent, XCD-aware work split (slice-sized grids).  The dispatcher deals
// workgroup b to XCD b % 8; every XCD owns one contiguous chunk of the item
// range (neighbouring items share its L2) and its workgroups walk the chunk
// with a stride of the XCD's workgroup count.  With one workgroup per item
// this is exactly xcd_remap; with a smaller grid each workgroup runs several
// items.  Usage: for (int i = c.first; i < c.end; i += c.step) { ... }
struct XcdChunk {
  int first, end, step;
};
__device__ __forceinline__ XcdChunk xcd_chunk(int block, int grid, int n) {
  const int nx = 8, xcd = block % nx, j = block / nx;
  const int wgs_x = grid / nx + (xcd < grid % nx ? 1 : 0);
  const int lo = xcd * (n / nx) + min(xcd, n % nx);
  const int cnt = n / nx + (xcd < n % nx ? 1 : 0);
  return XcdChunk{lo + j, lo + cnt, wgs_x > 0 ? wgs_x : 1};
}

}  // namespace nos

// Grid cap for CU-slice tenants (runtime.hip): with a CU budget set
// (nos_set_cu_budget, the pod's ROC_GLOBAL_CU_MASK popcount) a launch of
// `items` workgroups is clamped to what the budgeted CUs hold at once
// (occupancy x CUs, a multiple of 8), so the dispatch completes at launch and
// never holds the command-processor pipe another pod's queue shares.
// Returns `items` when no budget is set.
int nos_grid_for(const void* kernel, int block_threads, size_t lds_bytes, long long items);

// CUs the tile/variant cost models plan for: the CU budget when one is set
// (a CU-mask slice), else the current device's CU count.
int nos_effective_cus();

#define HIP_CHECK_RET(expr)                       \
  do {                                            \
    hipError_t _e = (expr);                       \
    if (_e != hipSuccess) return (int)_e;         \
  } while (0)
