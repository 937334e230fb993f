// fp8 weight-only skinny GEMM (W8A16) for single-stream / small-batch decode, M <= 64.
//
// The reference's Ollama serves 4-bit GGUF weights [ext]; this is the MI355X-native low-precision
// option: weights stored as OCP e4m3 (gfx950 fp8) with one fp32 scale per output row, activations
// and accumulation unchanged (bf16 x bf16 MFMA, fp32 accumulators).  Decode at small M streams every
// weight byte once per step, so halving the bytes is what buys time.
//
// Layout (cain_amd/models/weights.py pack_mfma_a_fp8): Wq[(t*KP + p)*64 + lane] is 16 bytes: the e4m3
// A fragments of v_mfma_f32_16x16x32_bf16 for rows 16t..16t+15 and the two k-slices 64p..64p+31 (bytes
// 0-7) and 64p+32..64p+63 (bytes 8-15); lane = k-group * 16 + row, as in the bf16 packing.  One wave
// load instruction reads 1 KiB of contiguous HBM (non-temporal) = two k-slices of one 16-row tile.
// v_cvt_scalef32_pk_bf16_fp8 (scale 1) turns two e4m3 bytes into two bf16 values exactly, the MFMA
// accumulates q . x in fp32 and each wave multiplies its accumulators by the row scales before the
// cross-wave reduction; the epilogues (bias, RoPE + KV append, residual, SiLU/GeLU x up, fp32 logits)
// are the bf16 kernel's, unchanged (gemm_epi.h epi_load_at / epi_store).
//
// Structure: one workgroup per (16-row tile, 16-row M split); WAVES waves split the k-pairs and
// keep U pairs of loads in flight in two register sets (copy pipeline), then reduce through LDS;
// wave 0 runs the epilogue.  Fused RMSNorm as in gemm.hip (gain folded into W before quantisation).
#include <algorithm>

#include "common.h"
#include "gemm_epi.h"

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ bf16x8 w8_frag(const u32x4& w, int h) {
  const bf16x2v c0 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w[2 * h], 1.0f, false);
  const bf16x2v c1 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w[2 * h], 1.0f, true);
  const bf16x2v c2 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w[2 * h + 1], 1.0f, false);
  const bf16x2v c3 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w[2 * h + 1], 1.0f, true);
  return bf16x8{c0[0], c0[1], c1[0], c1[1], c2[0], c2[1], c3[0], c3[1]};
}

// XL (NB = 1, M <= 16, M * K * 2 <= 64 KiB): the workgroup's activation rows are staged once into LDS by
// LDS-DMA (global_load_lds_dwordx4) and every k pair reads its two fragments from LDS, so the vector-memory
// path carries one load instruction per KiB of weights instead of three.
typedef __attribute__((address_space(3))) void w8_lds_t;
typedef __attribute__((address_space(1))) const void w8_gbl_t;

template <int WAVES, int U, int NT, int NB, int EPI, bool NORM, bool XL0 = false>
__global__ __launch_bounds__(WAVES * 64) void skinny_w8_kernel(const GemmArgs a, const float* __restrict__ wscale) {
  constexpr bool XL = XL0 && NB == 1;
  extern __shared__ __attribute__((aligned(16))) char w8_xs[];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int KP = a.K >> 6;  // 64-wide k pairs
  // XCD-aware (tile, M split) mapping as in gemm.hip: the splits of one tile get ids 8 apart
  int tg, ms;
  {
    const int bid = blockIdx.x, msp = a.msplit;
    const int ntg = gridDim.x / msp;
    if (msp == 1) {
      tg = bid, ms = 0;
    } else if ((ntg & 7) == 0) {
      const int r = bid >> 3;
      ms = r % msp;
      tg = (r / msp) * 8 + (bid & 7);
    } else {
      tg = bid / msp, ms = bid - (bid / msp) * msp;
    }
  }
  const int mo = ms * 16 * NB;
  const int p_beg = (wave * KP) / WAVES, p_end = ((wave + 1) * KP) / WAVES;

  const int t0 = tg * NT;  // first 16-row tile of N of this workgroup
  EpiIn pre[NT][NB];
  if (wave == 0) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int b = 0; b < NB; ++b) pre[t][b] = epi_load_at<EPI>(a, t0 + t, mo + 16 * b + (lane & 15), lane);
  }

  const u32x4* wb = reinterpret_cast<const u32x4*>(a.Wp) + (size_t)t0 * KP * 64 + lane;
  const __bf16* xb[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b)
    xb[b] = a.X + (size_t)min(mo + 16 * b + (lane & 15), a.M - 1) * a.ldx + ((lane >> 4) << 3);
  f32x4 acc[NT][NB];
  float ssq[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    ssq[b] = 0.f;
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  // one k pair: 16-byte fp8 weight piece per tile + two bf16 activation fragments per row block
  // (each activation fragment feeds NT tiles: fewer load instructions per weight byte)
  struct Pair {
    u32x4 w[NT];
    bf16x8 x[XL ? 1 : NB][2];
    int p;
  };
  // XL: this lane's activation row in LDS (rows past M re-read row M-1) at its k-group
  const __bf16* xl_row =
      reinterpret_cast<const __bf16*>(w8_xs) + (size_t)min(lane & 15, a.M - 1) * a.K + ((lane >> 4) << 3);
  auto load = [&](Pair& q, int p) {
    q.p = p;
#pragma unroll
    for (int t = 0; t < NT; ++t) q.w[t] = __builtin_nontemporal_load(wb + ((size_t)t * KP + p) * 64);
    if constexpr (!XL) {
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        q.x[b][0] = *reinterpret_cast<const bf16x8*>(xb[b] + p * 64);
        q.x[b][1] = *reinterpret_cast<const bf16x8*>(xb[b] + p * 64 + 32);
      }
    }
  };
  auto xfrag = [&](const Pair& q, int b, int h) -> bf16x8 {
    if constexpr (XL) return *reinterpret_cast<const bf16x8*>(xl_row + q.p * 64 + h * 32);
    else return q.x[b][h];
  };
  auto step = [&](const Pair& q) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      bf16x8 xv[NB];
#pragma unroll
      for (int b = 0; b < NB; ++b) xv[b] = xfrag(q, b, h);
      if constexpr (NORM) {
#pragma unroll
        for (int b = 0; b < NB; ++b)
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float f = bf2f(xv[b][j]);
            ssq[b] += f * f;
          }
      }
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const bf16x8 wf = w8_frag(q.w[t], h);
#pragma unroll
        for (int b = 0; b < NB; ++b)
          acc[t][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, xv[b], acc[t][b], 0, 0, 0);
      }
    }
  };

  // copy pipeline: U pairs in flight while the previous U are multiplied
  int p = p_beg;
  const int nfull = (p_end - p_beg) / U;
  Pair cur[U];
  if (nfull > 0) {
#pragma unroll
    for (int u = 0; u < U; ++u) load(cur[u], p + u);
  }
  if constexpr (XL) {
    // stage rows [0, M) x K of X by LDS-DMA (the weight prologue above is already in flight): 16-byte chunk c of
    // the row-contiguous LDS copy <- row c / (K / 8), column chunk c % (K / 8); wave instruction j covers chunks
    // 64 j .. 64 j + 63 (lane l -> LDS byte 1024 j + 16 l)
    const int cpr = a.K >> 3, nch = a.M * cpr;
    for (int j = wave; j * 64 < nch; j += WAVES) {
      const int c = j * 64 + lane;
      if (c < nch) {
        const int r = c / cpr, col = c - r * cpr;
        __builtin_amdgcn_global_load_lds((w8_gbl_t*)(a.X + (size_t)r * a.ldx + col * 8), (w8_lds_t*)(w8_xs + j * 1024),
                                         16, 0, 0);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if (nfull > 0) {
    for (int c = 0; c < nfull; ++c) {
      Pair nxt[U];
      const int pn = p + U;
      const bool more = c + 1 < nfull;
      if (more) {
#pragma unroll
        for (int u = 0; u < U; ++u) load(nxt[u], pn + u);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) step(cur[u]);
      if (more) {
#pragma unroll
        for (int u = 0; u < U; ++u) cur[u] = nxt[u];
      }
      p = pn;
    }
  }
  for (; p < p_end; ++p) {
    Pair q;
    load(q, p);
    step(q);
  }

  // ---- cross-wave reduction through LDS, epilogue by wave 0
  __shared__ __attribute__((aligned(16))) f32x4 red[WAVES][NT][NB][64];
  __shared__ float red_ss[NORM ? WAVES : 1][NB][16];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    // accumulator i of this lane is output row 4*(lane>>4)+i of the tile
    const f32x4 sc = *reinterpret_cast<const f32x4*>(wscale + (t0 + t) * 16 + 4 * (lane >> 4));
#pragma unroll
    for (int b = 0; b < NB; ++b) red[wave][t][b][lane] = acc[t][b] * sc;
  }
  if constexpr (NORM) {
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      float v = ssq[b];
      v += __shfl_xor(v, 16, 64);  // the 4 k-groups of row m
      v += __shfl_xor(v, 32, 64);
      if (lane < 16) red_ss[wave][b][lane] = v;
    }
  }
  __syncthreads();
  if (wave != 0) return;
#pragma unroll
  for (int tb = 0; tb < NT * NB; ++tb) {
    const int t = tb / NB, b = tb % NB;
    auto unit_sum = [&](int l) -> f32x4 {
      f32x4 v = red[0][t][b][l];
#pragma unroll
      for (int w = 1; w < WAVES; ++w) v += red[w][t][b][l];
      if constexpr (NORM) {
        float ss = 0.f;
#pragma unroll
        for (int w = 0; w < WAVES; ++w) ss += red_ss[w][b][l & 15];
        v *= rms_inv(ss, a.K, a.eps);
      }
      return v;
    };
    if constexpr (EPI == EPI_F32) {  // the LM head: logits + chunk maxima
      const f32x4 v = unit_sum(lane);
      epi_store<EPI>(a, t0 + t, mo + 16 * b + (lane & 15), lane, pre[t][b], [&](int) { return v; });
      epi_cmax(a, t0 + t, mo + 16 * b + (lane & 15), lane, v);
    } else {
      epi_store<EPI>(a, t0 + t, mo + 16 * b + (lane & 15), lane, pre[t][b],
                     [&](int off) { return unit_sum(lane + off); });
    }
  }
}

template <int WAVES, int U, int NT, int NB, int EPI, bool NORM>
static hipError_t w8_launch(const GemmArgs& a, const float* wscale, bool xl, hipStream_t st) {
  if constexpr (NB == 1) {
    if (xl) {
      hipLaunchKernelGGL((skinny_w8_kernel<WAVES, U, NT, NB, EPI, NORM, true>), dim3(a.N / 16 / NT * a.msplit),
                         dim3(WAVES * 64), (size_t)a.M * a.K * 2, st, a, wscale);
      return hipGetLastError();
    }
  }
  hipLaunchKernelGGL((skinny_w8_kernel<WAVES, U, NT, NB, EPI, NORM>), dim3(a.N / 16 / NT * a.msplit),
                     dim3(WAVES * 64), 0, st, a, wscale);
  return hipGetLastError();
}

// kernel variants: (waves, pairs in flight, 16-row tiles of N, 16-row blocks of M) per workgroup
enum W8Var { W8_4_2_1_1, W8_8_2_1_1, W8_4_4_1_1, W8_8_4_1_1, W8_4_2_2_1, W8_8_2_2_1, W8_4_2_4_1, W8_4_2_1_2, W8_8_2_1_2,
              W8_4_4_2_1, W8_8_4_2_1 };

template <bool NORM>
static hipError_t w8_launch_e(int epi, int var, const GemmArgs& a, const float* wscale, bool xl, hipStream_t st) {
#define CAIN_W8_VAR(E)                                                       \
  switch (var) {                                                             \
    case W8_4_2_1_1: return w8_launch<4, 2, 1, 1, E, NORM>(a, wscale, xl, st);   \
    case W8_8_2_1_1: return w8_launch<8, 2, 1, 1, E, NORM>(a, wscale, xl, st);   \
    case W8_4_4_1_1: return w8_launch<4, 4, 1, 1, E, NORM>(a, wscale, xl, st);   \
    case W8_8_4_1_1: return w8_launch<8, 4, 1, 1, E, NORM>(a, wscale, xl, st);   \
    case W8_4_2_2_1: return w8_launch<4, 2, 2, 1, E, NORM>(a, wscale, xl, st);   \
    case W8_8_2_2_1: return w8_launch<8, 2, 2, 1, E, NORM>(a, wscale, xl, st);   \
    case W8_4_2_4_1: return w8_launch<4, 2, 4, 1, E, NORM>(a, wscale, xl, st);   \
    case W8_4_2_1_2: return w8_launch<4, 2, 1, 2, E, NORM>(a, wscale, xl, st);   \
    case W8_4_4_2_1: return w8_launch<4, 4, 2, 1, E, NORM>(a, wscale, xl, st);   \
    case W8_8_4_2_1: return w8_launch<8, 4, 2, 1, E, NORM>(a, wscale, xl, st);   \
    default: return w8_launch<8, 2, 1, 2, E, NORM>(a, wscale, xl, st);           \
  }
  switch (epi) {
    case EPI_BF16: CAIN_W8_VAR(EPI_BF16)
    case EPI_RESID: CAIN_W8_VAR(EPI_RESID)
    case EPI_F32: CAIN_W8_VAR(EPI_F32)
    case EPI_SILU: CAIN_W8_VAR(EPI_SILU)
    case EPI_GELU: CAIN_W8_VAR(EPI_GELU)
    case EPI_QKV_ROPE: CAIN_W8_VAR(EPI_QKV_ROPE)
    default: return hipErrorInvalidValue;
  }
#undef CAIN_W8_VAR
}

CAIN_API float* cain_gemm_cmax_claim(int N);  // gemm.hip

// Same arguments as cain_gemm (gemm.hip) plus the per-row weight scales; Wp is the fp8 packing.
CAIN_API int cain_gemm_w8(const void* Wp, const float* wscale, const void* X, int ldx, int K, int N, int M, void* Y,
                          int ldy, const float* bias, int norm, float eps, const int* slot, const int* pos,
                          const float* cos_t, const float* sin_t, void* kc, void* vtc, int H, int Hkv, int hd,
                          int T_max, int epi_flags, hipStream_t st) {
  const int epi = epi_flags & EPI_MASK;
  if (K % 64 || N % 16 || M < 1 || M > 64) return -1;
  if (epi == EPI_QKV_ROPE && (hd % 16 || (hd / 2) % 8)) return -1;
  GemmArgs a{};
  a.Wp = reinterpret_cast<const bf16x8*>(Wp);
  a.X = reinterpret_cast<const __bf16*>(X);
  a.ldx = ldx, a.K = K, a.N = N, a.M = M, a.Y = Y, a.ldy = ldy, a.bias = bias;
  a.eps = eps;
  a.slot = slot, a.pos = pos, a.cos_t = cos_t, a.sin_t = sin_t;
  a.kc = reinterpret_cast<__bf16*>(kc), a.vtc = reinterpret_cast<__bf16*>(vtc);
  a.H = H, a.Hkv = Hkv, a.hd = hd, a.T_max = T_max, a.kv8 = (epi_flags & EPI_KV_FP8) ? 1 : 0;
  if (epi == EPI_F32)  // the few-row LM head also writes the sampler's chunk maxima
    if (float* cm = cain_gemm_cmax_claim(N)) a.cmax = cm, a.ld_cm = N / 16;
  // (round 2-3's A/B overrides of waves / pairs in flight / tiles / row blocks are fixed at the measured rule)
  constexpr int f_w = 0, f_u = 0, f_nt = 0, f_nb = 0;
  const int nb = f_nb ? (f_nb >= 2 ? 2 : 1) : (M > 16 ? 2 : 1);
  // two tiles per workgroup only pay on LM-head-sized N (measured, profiles/w8_decode.md)
  int nt = nb == 2 ? 1 : (f_nt ? (f_nt >= 4 ? 4 : f_nt) : (N >= 65536 ? 2 : 1));
  if ((N / 16) % nt) nt = 1;
  a.msplit = (M + 16 * nb - 1) / (16 * nb);
  // activations staged in LDS (XL above): one row block, at most 64 KiB of rows.  Measured single stream (same box,
  // interleaved): llama3.1:8b 471.9 / 472.4 -> 478.5 / 479.9 tok/s, qwen2:1.5b 970.2 -> 982.1; gate/up 25.2 ->
  // 23.9 us, QKV 9.5 -> 9.2 (profiles/r3/README.md).
  const bool xl = nb == 1 && a.msplit == 1 && (long long)M * K * 2 <= 65536;
  // 8 waves when the grid is at most one workgroup per CU and there are enough k-pairs per wave, else 4.  (The
  // bound was 512 workgroups; with XL + U = 4, llama3.1:8b's 384-workgroup QKV runs 8.9 -> 8.2 us on 4 waves
  // while the 256-workgroup O / down stay faster on 8: 8.7 vs 9.9 us, profiles/r3/README.md.)
  const int n_cu = cain_cu_budget();
  int waves = (N / 16 / nt * a.msplit <= (xl ? n_cu : 511) && K / 64 >= 64) ? 8 : 4;
  if (f_w) waves = f_w >= 8 ? 8 : 4;
  // pairs in flight per wave: with the activations in LDS the registers of the deeper weight prologue are free
  // (U = 4: llama3.1:8b 480.7 -> 514.1 tok/s single stream); without, U = 4 measured no gain (w8_decode.md)
  // (U = 8 spilled 92-168 B per lane at 8 waves and was never selected: removed)
  int u = (nb == 1 && f_u >= 4) ? 4 : 2;
  if (!f_u && xl) u = 4;
  if (nt == 4) u = 2;
  int var;
  if (nb == 2)
    var = waves == 8 ? W8_8_2_1_2 : W8_4_2_1_2;
  else if (nt == 4)
    var = W8_4_2_4_1;
  else if (nt == 2)
    var = u == 4 ? (waves == 8 ? W8_8_4_2_1 : W8_4_4_2_1) : (waves == 8 ? W8_8_2_2_1 : W8_4_2_2_1);
  else
    var = u == 4 ? (waves == 8 ? W8_8_4_1_1 : W8_4_4_1_1) : (waves == 8 ? W8_8_2_1_1 : W8_4_2_1_1);
  const hipError_t e = norm ? w8_launch_e<true>(epi, var, a, wscale, xl, st)
                            : w8_launch_e<false>(epi, var, a, wscale, xl, st);
  return int(e);
}
