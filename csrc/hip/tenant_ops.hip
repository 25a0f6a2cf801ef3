// Row-wise and gather kernels of general pod-server tenant programs
// (nos_amd/podserver/program.py): embedding lookups, RMSNorm, softmax,
// rotary position embeddings, and the im2col pre-pass that turns a conv2d
// into an fp16x3 ("h3") GEMM (gemm_f32h.hip).  Decoder LLMs and conv nets
// lower onto these plus the h3 GEMM / attention kernels; the reference's MPS
// clients are arbitrary CUDA programs
// (/root/reference/docs/en/docs/dynamic-gpu-partitioning/partitioning-modes-comparison.md:29-34),
// the pod server's equivalent is this op set.
//
// CDNA4 notes: one 64-lane wave (or half-wave) per row, rows held in
// registers where they fit, wave-level reductions with DPP/permute
// shuffles, 16-byte global accesses; nothing here touches LDS except the
// im2col kernel's per-row scale.  dtype codes: 0 = fp32, 1 = bf16.
#include <float.h>
#include <math.h>

#include "common.h"
#include "split_f16.h"

namespace {

__device__ __forceinline__ float ld_as_f32(const void* p, long long i, int bf16) {
  return bf16 ? nos::bf16_to_f32(static_cast<const unsigned short*>(p)[i]) : static_cast<const float*>(p)[i];
}

__device__ __forceinline__ void st_from_f32(void* p, long long i, float v, int bf16) {
  if (bf16)
    static_cast<unsigned short*>(p)[i] = nos::f32_to_bf16(v);
  else
    static_cast<float*>(p)[i] = v;
}

// ------------------------------------------------------------------ embedding
// out[r, :] = table[ids[r], :]; an id outside [0, V) gives a zero row (the
// host validates ids before a replay; the kernel never reads out of bounds).
// One thread per 16-byte chunk of a row.
__global__ __launch_bounds__(256) void embedding_kernel(const int* __restrict__ ids, const uint4* __restrict__ table,
                                                        uint4* __restrict__ out, long long n16, int row16, int V) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n16) return;
  const long long r = i / row16;
  const int c = (int)(i - r * row16);
  const int id = ids[r];
  out[i] = (id >= 0 && id < V) ? table[(long long)id * row16 + c] : uint4{0u, 0u, 0u, 0u};
}

// ------------------------------------------------------------------ RMSNorm
// y = w * (x / sqrt(mean(x^2) + eps)), statistics in fp32 (a bf16 row is
// normalised in fp32 and rounded to bf16 before the weight, as HF's
// LlamaRMSNorm does).  One wave per row.
__global__ __launch_bounds__(256) void rmsnorm_kernel(const void* __restrict__ x, const void* __restrict__ w,
                                                      void* __restrict__ y, int rows, int D, int ldx, int ldy,
                                                      float eps, int bf16) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const long long xo = (long long)row * ldx, yo = (long long)row * ldy;
  float q = 0.f;
  for (int d = lane; d < D; d += 64) {
    const float v = ld_as_f32(x, xo + d, bf16);
    q = fmaf(v, v, q);
  }
  const float rs = rsqrtf(nos::wave_sum(q) / (float)D + eps);
  for (int d = lane; d < D; d += 64) {
    float v = ld_as_f32(x, xo + d, bf16) * rs;
    if (bf16) v = nos::bf16_to_f32(nos::f32_to_bf16(v));
    st_from_f32(y, yo + d, v * ld_as_f32(w, d, bf16), bf16);
  }
}

// ------------------------------------------------------------------ softmax
// softmax over the last dim: one wave per row, an online (max, sum) per lane
// merged across the wave, then one write pass.  Rows of -inf give NaN, as
// torch.softmax does.
__global__ __launch_bounds__(256) void softmax_kernel(const void* __restrict__ x, void* __restrict__ y, int rows, int L,
                                                      int ldx, int ldy, int bf16) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const long long xo = (long long)row * ldx, yo = (long long)row * ldy;
  float m = -INFINITY, s = 0.f;
  for (int d = lane; d < L; d += 64) {
    const float v = ld_as_f32(x, xo + d, bf16);
    if (v > m) {
      s = s * __expf(m - v) + 1.f;
      m = v;
    } else {
      s += __expf(v - m);
    }
  }
  const float M = nos::wave_max(m);
  s = (m == -INFINITY) ? 0.f : s * __expf(m - M);
  const float inv = 1.f / nos::wave_sum(s);
  for (int d = lane; d < L; d += 64) st_from_f32(y, yo + d, __expf(ld_as_f32(x, xo + d, bf16) - M) * inv, bf16);
}

// ------------------------------------------------------------------ rotary
// GPT-NeoX / Llama rotary embedding ("rotate_half"): for d < D/2
//   y[d]       = x[d] cos[s][d]       - x[d + D/2] sin[s][d]
//   y[d + D/2] = x[d + D/2] cos[s][d + D/2] + x[d] sin[s][d + D/2]
// x [B, S, H, D] (row stride ldx between tokens, batch stride bsx), cos /
// sin fp32 [S, D]; y [B, S, H, D] contiguous.  One thread per (b, s, h, d < D/2).
__global__ __launch_bounds__(256) void rotary_kernel(const void* __restrict__ x, const float* __restrict__ cs,
                                                     const float* __restrict__ sn, void* __restrict__ y, int B, int S,
                                                     int H, int D, int ldx, long long bsx, int bf16) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  const int hd = D / 2;
  const long long n = (long long)B * S * H * hd;
  if (i >= n) return;
  const int d = (int)(i % hd);
  long long r = i / hd;
  const int h = (int)(r % H);
  r /= H;
  const int s = (int)(r % S);
  const int b = (int)(r / S);
  const long long xo = b * bsx + (long long)s * ldx + h * D;
  const float x0 = ld_as_f32(x, xo + d, bf16), x1 = ld_as_f32(x, xo + d + hd, bf16);
  const float* c = cs + (long long)s * D;
  const float* sv = sn + (long long)s * D;
  const long long yo = (((long long)b * S + s) * H + h) * D;
  st_from_f32(y, yo + d, fmaf(x0, c[d], -x1 * sv[d]), bf16);
  st_from_f32(y, yo + d + hd, fmaf(x1, c[d + hd], x0 * sv[d + hd]), bf16);
}

// ------------------------------------------------------------------ cast + unary
// y = f(x) with the input and output dtypes independent (fp32 / bf16): a
// cast next to an activation (a bf16 head's fp32 sigmoid output) is one pass,
// f evaluated in fp32 and rounded once.  op: 0 identity, 1 relu, 2 sigmoid,
// 3 silu, 4 gelu (erf), 5 tanh, 6 exp, 7 neg.
// x rows of N at row stride ldx (ldx == N: flat) -> y [n / N, N] contiguous
__global__ __launch_bounds__(256) void unary_kernel(const void* __restrict__ x, int xbf, void* __restrict__ y, int ybf,
                                                    long long n, int op, int N, long long ldx) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const float v = ld_as_f32(x, ldx == N ? i : (i / N) * ldx + i % N, xbf);
  float r;
  switch (op) {
    case 1: r = fmaxf(v, 0.f); break;
    case 2: r = 1.f / (1.f + expf(-v)); break;
    case 3: r = v / (1.f + expf(-v)); break;
    case 4: r = 0.5f * v * (1.f + erff(v * 0.70710678118654752f)); break;
    case 5: r = tanhf(v); break;
    case 6: r = expf(v); break;
    case 7: r = -v; break;
    default: r = v;
  }
  st_from_f32(y, i, r, ybf);
}

// ------------------------------------------------------------------ gated unit
// y[m, n] = f(a[m, n]) * b[m, n] (SwiGLU's silu(gate) * up; the op codes of
// unary_kernel): a / b rows at their own strides (the two column halves of a
// merged gate-up GEMM), y [M, N] contiguous; one pass, f in fp32
__global__ __launch_bounds__(256) void glu_kernel(const void* __restrict__ a, int lda, const void* __restrict__ b,
                                                  int ldb, void* __restrict__ y, long long M, int N, int op, int bf) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= M * N) return;
  const long long m = i / N;
  const int n = (int)(i - m * N);
  const float v = ld_as_f32(a, m * lda + n, bf), u = ld_as_f32(b, m * ldb + n, bf);
  float r;
  switch (op) {
    case 1: r = fmaxf(v, 0.f); break;
    case 2: r = 1.f / (1.f + expf(-v)); break;
    case 3: r = v / (1.f + expf(-v)); break;
    case 4: r = 0.5f * v * (1.f + erff(v * 0.70710678118654752f)); break;
    default: r = v;
  }
  st_from_f32(y, i, r * u, bf);
}

// ------------------------------------------------------------------ conv2d im2col -> h3 planes
// The patches of one NCHW image as the B operand of the h3 GEMM
// out[n][oc][p] = sum_k W[oc][k] patch[n][p][k] (k = (c, kh, kw), torch's
// weight layout; p = (oh, ow)): patch rows [N*P][Kp] as hi / lo fp16 planes,
// each row on its own power-of-two scale (max |x| just under 2^14), columns
// K..Kp-1 zero (Kp = K rounded up to the GEMM's 32), rinv[row] = 1 / scale.
// A half-wave per patch row: pass 1 gathers the row's max, pass 2 gathers
// again (L1/L2 hits: neighbouring rows of the block overlap) and writes the
// pieces -- 32 lanes write 64 contiguous bytes of a plane row per step.
// The image is read through strides (unit stride along W): a cropped view
// (a ViT's input sliced to whole patches) needs no contiguous copy.  BF:
// plain bf16 rows instead (a bf16 tenant's patch GEMM operand; no scale,
// no max pass, rinv unused) -- the image's cast and patch relayout in one pass.
template <int KH, int KW, bool BF>
__global__ __launch_bounds__(256) void im2col_h3_kernel(const float* __restrict__ x, void* __restrict__ Pv,
                                                        long long pplane, float* __restrict__ rinv, int Nimg, int C,
                                                        int H, int W, long long sN, long long sC, long long sH, int OH,
                                                        int OW, int kh_rt, int kw_rt, int sh, int sw, int ph, int pw,
                                                        int dh, int dw, int K, int Kp) {
  const int kh_n = KH > 0 ? KH : kh_rt, kw_n = KW > 0 ? KW : kw_rt;
  const int khw = kh_n * kw_n;
  const long long P1 = (long long)OH * OW;
  const long long row = (long long)blockIdx.x * 8 + (threadIdx.x >> 5);
  const int lane = threadIdx.x & 31;
  if (row >= Nimg * P1) return;  // whole half-waves retire together
  const int n = (int)(row / P1);
  const int p = (int)(row - n * P1);
  const int oh = p / OW, ow = p - oh * OW;
  const int ih0 = oh * sh - ph, iw0 = ow * sw - pw;
  const float* xn = x + (long long)n * sN;
  auto gather = [&](int k) -> float {
    if (k >= K) return 0.f;
    const int c = k / khw;
    const int r = k - c * khw;
    const int i = r / kw_n, j = r - i * kw_n;
    const int ih = ih0 + i * dh, iw = iw0 + j * dw;
    return (ih >= 0 && ih < H && iw >= 0 && iw < W) ? xn[c * sC + ih * sH + iw] : 0.f;
  };
  if constexpr (BF) {
    unsigned short* pb = static_cast<unsigned short*>(Pv) + row * Kp;
    for (int k = lane; k < Kp; k += 32) pb[k] = nos::f32_to_bf16(gather(k));
    return;
  }
  float mx = 0.f;
  for (int k = lane; k < K; k += 32) mx = fmaxf(mx, fabsf(gather(k)));
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  const int e = nos::h3_scale_exp(mx);
  const float sc = nos::pow2i(e);
  _Float16* ph_ = static_cast<_Float16*>(Pv) + row * Kp;
  _Float16* pl_ = ph_ + pplane;
  for (int k = lane; k < Kp; k += 32) {
    const float v = gather(k) * sc;
    const _Float16 h0 = (_Float16)v;
    ph_[k] = h0;
    pl_[k] = (_Float16)(v - (float)h0);
  }
  if (lane == 0) rinv[row] = nos::pow2i(-e);
}

}  // namespace

NOS_API int nos_embedding(const int* ids, const void* table, void* out, long long n, int V, int row_bytes,
                          hipStream_t stream) {
  if (n <= 0 || V <= 0 || row_bytes <= 0 || (row_bytes % 16)) return (int)hipErrorInvalidValue;
  if ((((uintptr_t)table) | ((uintptr_t)out)) & 15) return (int)hipErrorInvalidValue;
  const int row16 = row_bytes / 16;
  const long long n16 = n * row16;
  hipLaunchKernelGGL(embedding_kernel, dim3((unsigned)((n16 + 255) / 256)), dim3(256), 0, stream, ids,
                     static_cast<const uint4*>(table), static_cast<uint4*>(out), n16, row16, V);
  return (int)hipGetLastError();
}

NOS_API int nos_rmsnorm(const void* x, const void* w, void* y, int rows, int D, int ldx, int ldy, float eps, int bf16,
                        hipStream_t stream) {
  if (rows <= 0 || D <= 0 || ldx < D || ldy < D || !(eps >= 0.f) || (bf16 != 0 && bf16 != 1))
    return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(rmsnorm_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, stream, x, w, y, rows, D, ldx,
                     ldy, eps, bf16);
  return (int)hipGetLastError();
}

NOS_API int nos_softmax(const void* x, void* y, int rows, int L, int ldx, int ldy, int bf16, hipStream_t stream) {
  if (rows <= 0 || L <= 0 || ldx < L || ldy < L || (bf16 != 0 && bf16 != 1)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(softmax_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, stream, x, y, rows, L, ldx, ldy,
                     bf16);
  return (int)hipGetLastError();
}

NOS_API int nos_rotary(const void* x, const float* cos_t, const float* sin_t, void* y, int B, int S, int H, int D,
                       int ldx, long long bsx, int bf16, hipStream_t stream) {
  if (B <= 0 || S <= 0 || H <= 0 || D <= 0 || (D % 2) || ldx < H * D || bsx < (long long)(S - 1) * ldx + H * D ||
      (bf16 != 0 && bf16 != 1))
    return (int)hipErrorInvalidValue;
  const long long n = (long long)B * S * H * (D / 2);
  hipLaunchKernelGGL(rotary_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, x, cos_t, sin_t, y, B, S,
                     H, D, ldx, bsx, bf16);
  return (int)hipGetLastError();
}

// Patches of x [N, C, H, W] (fp32; element strides sN / sC / sH, unit
// stride along W) for a KHxKW conv (stride, padding, dilation): rows
// [N * OH * OW][Kp], Kp >= C * KH * KW, columns past K zero.  bf16 == 0: h3
// planes, hi at P, lo at P + pplane elements, Kp % 32 == 0, rinv [N * OH *
// OW]; bf16 == 1: one bf16 matrix at P (pplane, rinv unused).
NOS_API int nos_im2col(const float* x, long long sN, long long sC, long long sH, void* P, long long pplane,
                       float* rinv, int N, int C, int H, int W, int KH, int KW, int sh, int sw, int ph, int pw, int dh,
                       int dw, int Kp, int bf16, hipStream_t stream) {
  if (N <= 0 || C <= 0 || H <= 0 || W <= 0 || KH <= 0 || KW <= 0 || sh <= 0 || sw <= 0 || ph < 0 || pw < 0 ||
      dh <= 0 || dw <= 0 || (bf16 != 0 && bf16 != 1) || sH < W || sC < (long long)(H - 1) * sH + W ||
      (N > 1 && sN < (long long)(C - 1) * sC + (long long)(H - 1) * sH + W))
    return (int)hipErrorInvalidValue;
  const int OH = (H + 2 * ph - dh * (KH - 1) - 1) / sh + 1, OW = (W + 2 * pw - dw * (KW - 1) - 1) / sw + 1;
  const long long K = (long long)C * KH * KW;
  const long long rows = (long long)N * OH * OW;
  if (OH <= 0 || OW <= 0 || K > INT_MAX || Kp < K || rows > (1LL << 31) ||
      (!bf16 && ((Kp % 32) || pplane < rows * Kp)))
    return (int)hipErrorInvalidValue;
  const dim3 grid((unsigned)((rows + 7) / 8)), blk(256);
#define NOS_IM2COL(kh, kw, bf)                                                                                        \
  hipLaunchKernelGGL((im2col_h3_kernel<kh, kw, bf>), grid, blk, 0, stream, x, P, pplane, rinv, N, C, H, W, sN, sC, sH, \
                     OH, OW, KH, KW, sh, sw, ph, pw, dh, dw, (int)K, Kp)
  // ViT patch embeddings (16x16, stride 16) and the common conv kernels get
  // compile-time sizes: the per-element (c, i, j) split is then multiplies
  if (bf16 && KH == 16 && KW == 16)
    NOS_IM2COL(16, 16, true);
  else if (bf16)
    NOS_IM2COL(0, 0, true);
  else if (KH == 16 && KW == 16)
    NOS_IM2COL(16, 16, false);
  else if (KH == 1 && KW == 1)
    NOS_IM2COL(1, 1, false);
  else if (KH == 3 && KW == 3)
    NOS_IM2COL(3, 3, false);
  else if (KH == 7 && KW == 7)
    NOS_IM2COL(7, 7, false);
  else
    NOS_IM2COL(0, 0, false);
#undef NOS_IM2COL
  return (int)hipGetLastError();
}

// the contiguous-image form (conv2d's im2col)
NOS_API int nos_im2col_h3(const float* x, void* P, long long pplane, float* rinv, int N, int C, int H, int W, int KH,
                          int KW, int sh, int sw, int ph, int pw, int dh, int dw, int Kp, hipStream_t stream) {
  return nos_im2col(x, (long long)C * H * W, (long long)H * W, W, P, pplane, rinv, N, C, H, W, KH, KW, sh, sw, ph, pw,
                    dh, dw, Kp, 0, stream);
}

NOS_API int nos_unary(const void* x, int xbf16, void* y, int ybf16, long long n, int op, hipStream_t stream) {
  if (n <= 0 || op < 0 || op > 7 || (xbf16 != 0 && xbf16 != 1) || (ybf16 != 0 && ybf16 != 1))
    return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(unary_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, x, xbf16, y, ybf16, n, op,
                     1, 1LL);
  return (int)hipGetLastError();
}

// the same over a row-strided x [M, N] (ldx >= N; e.g. a column slice of a merged
// GEMM's output) into a contiguous y [M, N] -- no contiguous copy of x first
NOS_API int nos_unary_rows(const void* x, long long ldx, int xbf16, void* y, int ybf16, long long M, int N, int op,
                           hipStream_t stream) {
  if (M <= 0 || N <= 0 || ldx < N || op < 0 || op > 7 || (xbf16 != 0 && xbf16 != 1) || (ybf16 != 0 && ybf16 != 1) ||
      !x || !y)
    return (int)hipErrorInvalidValue;
  const long long n = M * N;
  hipLaunchKernelGGL(unary_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, x, xbf16, y, ybf16, n, op,
                     N, ldx);
  return (int)hipGetLastError();
}

NOS_API int nos_glu(const void* a, int lda, const void* b, int ldb, void* y, long long M, int N, int op, int bf16,
                    hipStream_t stream) {
  if (!a || !b || !y || M <= 0 || N <= 0 || lda < N || ldb < N || op < 0 || op > 4 || (bf16 != 0 && bf16 != 1))
    return (int)hipErrorInvalidValue;
  const long long n = M * N;
  hipLaunchKernelGGL(glu_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, a, lda, b, ldb, y, M, N, op,
                     bf16);
  return (int)hipGetLastError();
}
