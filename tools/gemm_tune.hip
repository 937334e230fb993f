// Tuning harness for the weight-streaming GEMM (not part of the library).
// Variants of the M<=16 main loop: NT row tiles per wave, WAVES per workgroup,
// U k-slices in flight, non-temporal vs default weight loads, and a
// register double-buffered (software-pipelined) loop.  Plain bf16 epilogue.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int NT, int WAVES, int U, bool NTL, bool PIPE>
__global__ __launch_bounds__(WAVES * 64) void tune_kernel(const bf16x8* __restrict__ Wp, const __bf16* __restrict__ X,
                                                          int K, int N, __bf16* __restrict__ Y) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int KS = K >> 5, tile0 = blockIdx.x * NT;
  const int s_beg = (wave * KS) / WAVES, s_end = ((wave + 1) * KS) / WAVES;
  f32x4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f32x4{0, 0, 0, 0};
  const bf16x8* wb[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) wb[t] = Wp + (size_t)(tile0 + t) * KS * 64 + lane;
  const __bf16* xb = X + (size_t)(lane & 15) * K + ((lane >> 4) << 3);
  auto ldw = [&](const bf16x8* p) -> bf16x8 {
    if constexpr (NTL) return __builtin_nontemporal_load(p);
    else return *p;
  };
  if constexpr (PIPE) {
    // two register sets: issue chunk i+1 before computing chunk i
    bf16x8 wa[U][NT], xa[U], wn[U][NT], xn[U];
    int s = s_beg;
    const int nfull = (s_end - s_beg) / U;
    if (nfull > 0) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
#pragma unroll
        for (int t = 0; t < NT; ++t) wa[u][t] = ldw(wb[t] + (size_t)(s + u) * 64);
        xa[u] = *reinterpret_cast<const bf16x8*>(xb + (s + u) * 32);
      }
      for (int c = 0; c < nfull; ++c) {
        const int sn = s + U;
        if (c + 1 < nfull) {
#pragma unroll
          for (int u = 0; u < U; ++u) {
#pragma unroll
            for (int t = 0; t < NT; ++t) wn[u][t] = ldw(wb[t] + (size_t)(sn + u) * 64);
            xn[u] = *reinterpret_cast<const bf16x8*>(xb + (sn + u) * 32);
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int t = 0; t < NT; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[u][t], xa[u], acc[t], 0, 0, 0);
#pragma unroll
        for (int u = 0; u < U; ++u) {
#pragma unroll
          for (int t = 0; t < NT; ++t) wa[u][t] = wn[u][t];
          xa[u] = xn[u];
        }
        s = sn;
      }
    }
    for (; s < s_end; ++s) {
      bf16x8 x = *reinterpret_cast<const bf16x8*>(xb + s * 32);
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ldw(wb[t] + (size_t)s * 64), x, acc[t], 0, 0, 0);
    }
  } else {
    int s = s_beg;
    for (; s + U <= s_end; s += U) {
      bf16x8 w[U][NT], x[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
#pragma unroll
        for (int t = 0; t < NT; ++t) w[u][t] = ldw(wb[t] + (size_t)(s + u) * 64);
        x[u] = *reinterpret_cast<const bf16x8*>(xb + (s + u) * 32);
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[u][t], x[u], acc[t], 0, 0, 0);
    }
    for (; s < s_end; ++s) {
      bf16x8 x = *reinterpret_cast<const bf16x8*>(xb + s * 32);
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ldw(wb[t] + (size_t)s * 64), x, acc[t], 0, 0, 0);
    }
  }
  __shared__ f32x4 red[WAVES][NT * 64];
#pragma unroll
  for (int t = 0; t < NT; ++t) red[wave][t * 64 + lane] = acc[t];
  __syncthreads();
  for (int u = threadIdx.x; u < NT * 64; u += WAVES * 64) {
    f32x4 v = red[0][u];
#pragma unroll
    for (int w = 1; w < WAVES; ++w) v += red[w][u];
    const int t = u >> 6, ln = u & 63;
    const int m = ln & 15, n = (tile0 + t) * 16 + (ln >> 4) * 4;
    bf16x4 o;
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = static_cast<__bf16>(v[i]);
    *reinterpret_cast<bf16x4*>(Y + (size_t)m * N + n) = o;
  }
}

#define V(NT, W, U, NTL, P)                                                                           \
  if (nt == NT && waves == W && u == U && ntl == NTL && pipe == P) {                                  \
    hipLaunchKernelGGL((tune_kernel<NT, W, U, NTL, P>), dim3(N / (16 * NT)), dim3(W * 64), 0, st, \
                       (const bf16x8*)Wp, (const __bf16*)X, K, N, (__bf16*)Y);                        \
    return int(hipGetLastError());                                                                    \
  }

extern "C" int tune_gemm(const void* Wp, const void* X, int K, int N, void* Y, int nt, int waves, int u, int ntl,
                         int pipe, hipStream_t st) {
  V(1, 4, 8, 1, 0) V(1, 8, 8, 1, 0) V(1, 16, 8, 1, 0)
  V(1, 4, 16, 1, 0) V(1, 8, 16, 1, 0) V(1, 16, 16, 1, 0)
  V(1, 8, 8, 0, 0) V(1, 16, 8, 0, 0) V(1, 8, 16, 0, 0)
  V(2, 4, 8, 1, 0) V(2, 8, 8, 1, 0) V(2, 16, 8, 1, 0) V(2, 8, 4, 1, 0) V(2, 16, 4, 1, 0)
  V(1, 8, 4, 1, 1) V(1, 8, 8, 1, 1) V(1, 16, 4, 1, 1) V(1, 16, 8, 1, 1) V(1, 4, 8, 1, 1)
  V(2, 8, 4, 1, 1) V(2, 16, 4, 1, 1)
  return -1;
}
