// Fused (residual-add +) LayerNorm, bf16 in/out, fp32 statistics.
//
//   s = x (+ res);  sum_out = s (optional);  y = (s - mean) / sqrt(var + eps) * gamma + beta
//
// Memory-bound: one wave per row, every lane moves 16 B (8 bf16) per access,
// statistics with 64-lane xor shuffles, two-pass variance from registers (the
// row is read once).  D must be a multiple of 8 and <= 4096.
#include "common.h"

namespace {

template <int V>  // 16-byte vectors per lane
__global__ __launch_bounds__(256) void layernorm_kernel(
    const unsigned short* __restrict__ x, const unsigned short* __restrict__ res,
    unsigned short* __restrict__ y, unsigned short* __restrict__ sum_out,
    const unsigned short* __restrict__ gamma, const unsigned short* __restrict__ beta, int rows,
    int D, int ldx, int ldy, int ldr, int lds, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nvec = D >> 3;
  float v[V][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int vi = lane + 64 * i;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[i][e] = 0.f;
    if (vi < nvec) {
      const s16x8_t xv = *reinterpret_cast<const s16x8_t*>(x + (long long)row * ldx + vi * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[i][e] = nos::bf16_to_f32((unsigned short)xv[e]);
      if (res) {
        const s16x8_t rv = *reinterpret_cast<const s16x8_t*>(res + (long long)row * ldr + vi * 8);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[i][e] += nos::bf16_to_f32((unsigned short)rv[e]);
      }
      if (sum_out) {
        s16x8_t sv;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          // keep the residual stream exactly what the next layer will read
          const unsigned short bb = nos::f32_to_bf16(v[i][e]);
          sv[e] = (short)bb;
          v[i][e] = nos::bf16_to_f32(bb);
        }
        *reinterpret_cast<s16x8_t*>(sum_out + (long long)row * lds + vi * 8) = sv;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) s += v[i][e];
    }
  }
  const float mean = nos::wave_sum(s) / (float)D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < V; ++i)
    if (lane + 64 * i < nvec)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float d = v[i][e] - mean;
        q += d * d;
      }
  const float rstd = rsqrtf(nos::wave_sum(q) / (float)D + eps);
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int vi = lane + 64 * i;
    if (vi < nvec) {
      const s16x8_t gv = *reinterpret_cast<const s16x8_t*>(gamma + vi * 8);
      const s16x8_t bv = *reinterpret_cast<const s16x8_t*>(beta + vi * 8);
      s16x8_t out;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float t = (v[i][e] - mean) * rstd * nos::bf16_to_f32((unsigned short)gv[e]) +
                        nos::bf16_to_f32((unsigned short)bv[e]);
        out[e] = (short)nos::f32_to_bf16(t);
      }
      *reinterpret_cast<s16x8_t*>(y + (long long)row * ldy + vi * 8) = out;
    }
  }
}

}  // namespace

NOS_API int nos_layernorm_bf16(const void* x, const void* res, void* y, void* sum_out,
                               const void* gamma, const void* beta, int rows, int D, int ldx,
                               int ldy, int ldr, int lds, float eps, hipStream_t stream) {
  // every row stride is the tensor's own (x, y, residual, sum_out); 16-byte vectors
  if (rows <= 0 || D <= 0 || (D % 8) != 0 || D > 4096) return (int)hipErrorInvalidValue;
  if ((ldx % 8) || (ldy % 8) || (ldr % 8) || (lds % 8) || ldx < D || ldy < D) return (int)hipErrorInvalidValue;
  if ((res && ldr < D) || (sum_out && lds < D)) return (int)hipErrorInvalidValue;
  const int nvec = D / 8;
  const dim3 grid((rows + 3) / 4), block(256);
  auto X = (const unsigned short*)x;
  auto Rs = (const unsigned short*)res;
  auto Y = (unsigned short*)y;
  auto S = (unsigned short*)sum_out;
  auto G = (const unsigned short*)gamma;
  auto Bt = (const unsigned short*)beta;
  if (nvec <= 64)
    hipLaunchKernelGGL(layernorm_kernel<1>, grid, block, 0, stream, X, Rs, Y, S, G, Bt, rows, D, ldx, ldy, ldr, lds, eps);
  else if (nvec <= 128)
    hipLaunchKernelGGL(layernorm_kernel<2>, grid, block, 0, stream, X, Rs, Y, S, G, Bt, rows, D, ldx, ldy, ldr, lds, eps);
  else if (nvec <= 256)
    hipLaunchKernelGGL(layernorm_kernel<4>, grid, block, 0, stream, X, Rs, Y, S, G, Bt, rows, D, ldx, ldy, ldr, lds, eps);
  else
    hipLaunchKernelGGL(layernorm_kernel<8>, grid, block, 0, stream, X, Rs, Y, S, G, Bt, rows, D, ldx, ldy, ldr, lds, eps);
  return (int)hipGetLastError();
}
