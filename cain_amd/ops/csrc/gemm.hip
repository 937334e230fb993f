// Weight-streaming skinny GEMM for decode / short prefill on gfx950 MFMA.
//
//   Y[m][n] = epilogue( sum_k X[m][k] * W[n][k] )      m < M <= 16*NB,  n < N
//
// W is stored MFMA-fragment-major (cain_amd/models/weights.py pack_mfma_a):
// Wp[(t*KS + s)*64 + lane] is the 16-byte A fragment of lane `lane` of
// v_mfma_f32_16x16x32_bf16 for rows 16t..16t+15 and k-slice 32s..32s+31, so every
// wave load instruction streams 1 KiB of contiguous HBM with a non-temporal hint
// (each weight byte is read once per decode step).  The B operand is the
// activation X[m][k] (row-major, 16 B per lane straight from L2: lane = (col m,
// k-group g) reads X[m][32s+8g .. +8]), so neither operand goes through LDS
// (cdna_hip_programming.md §5, 'GEMV / M <= 16' row: load straight to VGPRs,
// deep unroll, late vmcnt).
//
// Parallelism: a workgroup owns NT 16-row tiles; its WAVES waves split the
// K-slices, keep U slices of weight loads in flight each, and reduce their
// 16x16 accumulators through LDS once at the end (no cross-workgroup split-K,
// so no inter-workgroup hand-off).  The host picks WAVES so the grid carries
// >= ~2k waves (256 CUs x 8).
//
// Epilogues (fused, SURVEY §2.4 rows QKV/O/gate-up/down/LM-head):
//   EPI_BF16   y = bf16(acc + bias)            (QKV projection, Qwen2 bias)
//   EPI_RESID  y = bf16(acc + resid)           (o_proj / down_proj + residual, in-place OK)
//   EPI_F32    y = acc (fp32)                  (LM-head logits)
//   EPI_SILU / EPI_GELU: tile pairs (gate, up) -> y = bf16(act(gate) * up)
#include "common.h"

enum { EPI_BF16 = 0, EPI_RESID = 1, EPI_F32 = 2, EPI_SILU = 3, EPI_GELU = 4 };

template <int NT, int NB, int WAVES, int U, int EPI>
__global__ __launch_bounds__(WAVES * 64) void skinny_gemm_kernel(
    const bf16x8* __restrict__ Wp, const __bf16* __restrict__ X, int ldx, int K, int N, int M,
    void* __restrict__ Y, int ldy, const float* __restrict__ bias, const __bf16* __restrict__ resid, int ldr) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int KS = K >> 5;
  const int tile0 = blockIdx.x * NT;
  const int s_beg = (wave * KS) / WAVES;
  const int s_end = ((wave + 1) * KS) / WAVES;

  f32x4 acc[NT][NB];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int b = 0; b < NB; ++b) acc[t][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  const bf16x8* wbase[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) wbase[t] = Wp + (size_t)(tile0 + t) * KS * 64 + lane;
  // B fragment: column m = lane & 15 of column tile b, k group g = lane >> 4
  const __bf16* xbase[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) xbase[b] = X + (size_t)(b * 16 + (lane & 15)) * ldx + ((lane >> 4) << 3);

  int s = s_beg;
  for (; s + U <= s_end; s += U) {
    bf16x8 a[U][NT], xb[U][NB];
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int t = 0; t < NT; ++t) a[u][t] = __builtin_nontemporal_load(wbase[t] + (size_t)(s + u) * 64);
#pragma unroll
      for (int b = 0; b < NB; ++b) xb[u][b] = *reinterpret_cast<const bf16x8*>(xbase[b] + (s + u) * 32);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int b = 0; b < NB; ++b)
          acc[t][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[u][t], xb[u][b], acc[t][b], 0, 0, 0);
  }
  for (; s < s_end; ++s) {
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      bf16x8 a = __builtin_nontemporal_load(wbase[t] + (size_t)s * 64);
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        bf16x8 xb = *reinterpret_cast<const bf16x8*>(xbase[b] + s * 32);
        acc[t][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, xb, acc[t][b], 0, 0, 0);
      }
    }
  }

  // ---- cross-wave reduction through LDS: red[wave][unit][4], unit = (t*NB + b)*64 + lane
  constexpr int UNITS = NT * NB * 64;
  __shared__ __attribute__((aligned(16))) f32x4 red[WAVES][UNITS];
  if (WAVES > 1) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int b = 0; b < NB; ++b) red[wave][(t * NB + b) * 64 + lane] = acc[t][b];
    __syncthreads();
  }

  // each thread finalises 4 consecutive n of one (t, b, lane) unit
  constexpr int NUNITS = (EPI == EPI_SILU || EPI == EPI_GELU) ? (NT / 2) * NB * 64 : UNITS;
  for (int u = threadIdx.x; u < NUNITS; u += WAVES * 64) {
    const int ln = u & 63;
    const int tb = u >> 6;  // (t * NB + b) or ((t/2) * NB + b) for gate/up
    const int b = tb % NB;
    const int t = tb / NB;
    const int m = b * 16 + (ln & 15);
    const int nsub = (ln >> 4) * 4;
    if (m >= M) continue;
    if constexpr (EPI == EPI_SILU || EPI == EPI_GELU) {
      const int tg = 2 * t, tu = 2 * t + 1;
      f32x4 g = {0.f, 0.f, 0.f, 0.f}, up = {0.f, 0.f, 0.f, 0.f};
      if (WAVES > 1) {
#pragma unroll
        for (int w = 0; w < WAVES; ++w) {
          g += red[w][(tg * NB + b) * 64 + ln];
          up += red[w][(tu * NB + b) * 64 + ln];
        }
      } else {
        g = acc[tg][b];
        up = acc[tu][b];
      }
      const int n = ((tile0 >> 1) + t) * 16 + nsub;  // output feature index (gate/up pairs)
      bf16x4 o;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float a = (EPI == EPI_SILU) ? silu_f(g[i]) : gelu_tanh_f(g[i]);
        o[i] = f2bf(a * up[i]);
      }
      *reinterpret_cast<bf16x4*>(reinterpret_cast<__bf16*>(Y) + (size_t)m * ldy + n) = o;
    } else {
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (WAVES > 1) {
#pragma unroll
        for (int w = 0; w < WAVES; ++w) v += red[w][u];
      } else {
        v = acc[t][b];
      }
      const int n = (tile0 + t) * 16 + nsub;
      if constexpr (EPI == EPI_F32) {
        *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(Y) + (size_t)m * ldy + n) = v;
      } else {
        if constexpr (EPI == EPI_BF16) {
          if (bias) {
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] += bias[n + i];
          }
        } else {  // EPI_RESID
          bf16x4 r = *reinterpret_cast<const bf16x4*>(resid + (size_t)m * ldr + n);
#pragma unroll
          for (int i = 0; i < 4; ++i) v[i] += bf2f(r[i]);
        }
        bf16x4 o;
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = f2bf(v[i]);
        *reinterpret_cast<bf16x4*>(reinterpret_cast<__bf16*>(Y) + (size_t)m * ldy + n) = o;
      }
    }
  }
}

template <int NT, int NB, int WAVES, int EPI>
static hipError_t launch_t(const void* Wp, const void* X, int ldx, int K, int N, int M, void* Y, int ldy,
                           const float* bias, const void* resid, int ldr, hipStream_t st) {
  constexpr int U = (NB >= 4) ? 4 : 8;
  dim3 grid(N / (16 * NT)), block(WAVES * 64);
  hipLaunchKernelGGL((skinny_gemm_kernel<NT, NB, WAVES, U, EPI>), grid, block, 0, st,
                     reinterpret_cast<const bf16x8*>(Wp), reinterpret_cast<const __bf16*>(X), ldx, K, N, M, Y, ldy,
                     bias, reinterpret_cast<const __bf16*>(resid), ldr);
  return hipGetLastError();
}

template <int NT, int NB, int EPI>
static hipError_t launch_w(int waves, const void* Wp, const void* X, int ldx, int K, int N, int M, void* Y, int ldy,
                           const float* bias, const void* resid, int ldr, hipStream_t st) {
  switch (waves) {
    case 4: return launch_t<NT, NB, 4, EPI>(Wp, X, ldx, K, N, M, Y, ldy, bias, resid, ldr, st);
    case 8: return launch_t<NT, NB, 8, EPI>(Wp, X, ldx, K, N, M, Y, ldy, bias, resid, ldr, st);
    default: return launch_t<NT, NB, 16, EPI>(Wp, X, ldx, K, N, M, Y, ldy, bias, resid, ldr, st);
  }
}

template <int NT, int EPI>
static hipError_t launch_b(int nb, int waves, const void* Wp, const void* X, int ldx, int K, int N, int M, void* Y,
                           int ldy, const float* bias, const void* resid, int ldr, hipStream_t st) {
  switch (nb) {
    case 1: return launch_w<NT, 1, EPI>(waves, Wp, X, ldx, K, N, M, Y, ldy, bias, resid, ldr, st);
    case 2: return launch_w<NT, 2, EPI>(waves, Wp, X, ldx, K, N, M, Y, ldy, bias, resid, ldr, st);
    default: return launch_w<NT, 4, EPI>(waves, Wp, X, ldx, K, N, M, Y, ldy, bias, resid, ldr, st);
  }
}

// Pick the number of waves per workgroup so the grid carries enough waves to
// keep ~8 waves of weight streams per CU (256 CUs).
static int pick_waves(int n_wg, int ks) {
  int w = 4;
  while (w < 16 && n_wg * w < 2048 && ks / (w * 2) >= 4) w *= 2;
  return w;
}

// epi: 0 bf16(+bias) 1 resid 2 f32 3 silu-gateup 4 gelu-gateup.  M <= 64.
// Returns hipError_t; -1 on unsupported shape.
CAIN_API int cain_skinny_gemm(const void* Wp, const void* X, int ldx, int K, int N, int M, void* Y, int ldy,
                              const float* bias, const void* resid, int ldr, int epi, int waves, hipStream_t st) {
  if (K % 32 || N % 16 || M < 1 || M > 64) return -1;
  const bool pair = (epi == EPI_SILU || epi == EPI_GELU);
  int nt = pair ? 2 : ((N % 32 == 0 && N >= 32 * 256) ? 2 : 1);
  if (N % (16 * nt)) return -1;
  int nb = M <= 16 ? 1 : (M <= 32 ? 2 : 4);
  int n_wg = N / (16 * nt);
  if (waves <= 0) waves = pick_waves(n_wg, K / 32);
  hipError_t e;
  if (nt == 1) {
    switch (epi) {
      case EPI_BF16: e = launch_b<1, EPI_BF16>(nb, waves, Wp, X, ldx, K, N, M, Y, ldy, bias, resid, ldr, st); break;
      case EPI_RESID: e = launch_b<1, EPI_RESID>(nb, waves, Wp, X, ldx, K, N, M, Y, ldy, bias, resid, ldr, st); break;
      case EPI_F32: e = launch_b<1, EPI_F32>(nb, waves, Wp, X, ldx, K, N, M, Y, ldy, bias, resid, ldr, st); break;
      default: return -1;
    }
  } else {
    switch (epi) {
      case EPI_BF16: e = launch_b<2, EPI_BF16>(nb, waves, Wp, X, ldx, K, N, M, Y, ldy, bias, resid, ldr, st); break;
      case EPI_RESID: e = launch_b<2, EPI_RESID>(nb, waves, Wp, X, ldx, K, N, M, Y, ldy, bias, resid, ldr, st); break;
      case EPI_F32: e = launch_b<2, EPI_F32>(nb, waves, Wp, X, ldx, K, N, M, Y, ldy, bias, resid, ldr, st); break;
      case EPI_SILU: e = launch_b<2, EPI_SILU>(nb, waves, Wp, X, ldx, K, N, M, Y, ldy, bias, resid, ldr, st); break;
      case EPI_GELU: e = launch_b<2, EPI_GELU>(nb, waves, Wp, X, ldx, K, N, M, Y, ldy, bias, resid, ldr, st); break;
      default: return -1;
    }
  }
  return int(e);
}
