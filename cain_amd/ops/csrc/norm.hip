// RMSNorm and embedding gather (SURVEY §2.4 rows "Embedding gather", "RMSNorm").
//
// Memory-bound row ops: one workgroup per row, 16-byte vector loads/stores
// (cdna_hip_programming.md Guideline 13), fp32 accumulation, wave-shuffle then
// LDS reduction.  Gemma's (1 + w) gain is folded into the stored gain at load
// time (weights.py), so one kernel serves every model.
#include "common.h"

template <int THREADS>
__device__ __forceinline__ float block_sum(float v, float* sh) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) sh[w] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < THREADS / 64; ++i) t += sh[i];
  return t;
}

// y[m] = x[m] * rsqrt(mean(x[m]^2) + eps) * g       (d % 8 == 0)
template <int THREADS>
__global__ __launch_bounds__(THREADS) void rmsnorm_kernel(const __bf16* __restrict__ x, int ldx,
                                                          const __bf16* __restrict__ g, __bf16* __restrict__ y,
                                                          int ldy, int d, float eps) {
  __shared__ float sh[THREADS / 64];
  const int m = blockIdx.x;
  const bf16x8* xr = reinterpret_cast<const bf16x8*>(x + (size_t)m * ldx);
  const int nv = d >> 3;
  constexpr int MAXV = 4;  // up to 4*8*THREADS elements held in registers
  bf16x8 v[MAXV];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    int idx = threadIdx.x + i * THREADS;
    if (idx < nv) {
      v[i] = xr[idx];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float f = bf2f(v[i][j]);
        ss += f * f;
      }
    }
  }
  float tot = block_sum<THREADS>(ss, sh);
  float inv = rms_inv(tot, d, eps);
  const bf16x8* gr = reinterpret_cast<const bf16x8*>(g);
  bf16x8* yr = reinterpret_cast<bf16x8*>(y + (size_t)m * ldy);
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    int idx = threadIdx.x + i * THREADS;
    if (idx < nv) {
      bf16x8 gv = gr[idx], o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = f2bf(bf2f(f2bf(bf2f(v[i][j]) * inv)) * bf2f(gv[j]));
      yr[idx] = o;
    }
  }
}

// out[m] = E[tok[m]] * scale   (scale = sqrt(d) rounded to bf16 for Gemma, else 1)
__global__ __launch_bounds__(256) void embed_kernel(const int* __restrict__ tok, const __bf16* __restrict__ E,
                                                    __bf16* __restrict__ out, int ldo, int d, float scale) {
  const int m = blockIdx.x;
  const int id = tok[m];
  const bf16x8* src = reinterpret_cast<const bf16x8*>(E + (size_t)id * d);
  bf16x8* dst = reinterpret_cast<bf16x8*>(out + (size_t)m * ldo);
  for (int i = threadIdx.x; i < (d >> 3); i += 256) {
    bf16x8 v = src[i];
    if (scale != 1.0f) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = f2bf(bf2f(v[j]) * scale);
    }
    dst[i] = v;
  }
}

CAIN_API int cain_rmsnorm(const void* x, int ldx, const void* g, void* y, int ldy, int M, int d, float eps,
                          hipStream_t st) {
  if (d % 8 || d > 4 * 8 * 512) return -1;
  if (d <= 4 * 8 * 256)
    hipLaunchKernelGGL(rmsnorm_kernel<256>, dim3(M), dim3(256), 0, st, (const __bf16*)x, ldx, (const __bf16*)g,
                       (__bf16*)y, ldy, d, eps);
  else
    hipLaunchKernelGGL(rmsnorm_kernel<512>, dim3(M), dim3(512), 0, st, (const __bf16*)x, ldx, (const __bf16*)g,
                       (__bf16*)y, ldy, d, eps);
  return int(hipGetLastError());
}

CAIN_API int cain_embed(const int* tok, const void* E, void* out, int ldo, int M, int d, float scale, hipStream_t st) {
  if (d % 8) return -1;
  hipLaunchKernelGGL(embed_kernel, dim3(M), dim3(256), 0, st, tok, (const __bf16*)E, (__bf16*)out, ldo, d, scale);
  return int(hipGetLastError());
}
