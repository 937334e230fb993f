// MXFP4 weight-only few-row GEMM (W4A16) for single-stream / small-batch decode, M <= 64.
//
// The reference's Ollama serves its seven models as 4-bit GGUF builds (/root/reference/README.md:29-30,
// the tags of experiment/RunnerConfig.py:80 without a quantisation suffix); this is the gfx950-native member of that
// precision class: OCP MXFP4 -- e2m1 elements, one e8m0 (power-of-two) scale per 32 consecutive k of a row.  Decode at
// one row streams every weight byte once per token, so the weight bytes (0.53 per parameter here, 1 for fp8, 2 for
// bf16) are the token's cost.
//
// Layout (cain_amd/models/weights.py pack_mxfp4): Wq[(t*KQ + p)*64 + lane] is 16 bytes = 32 e2m1 codes of ONE
// 32-element scale block: row 16t + r, k = 128p + 32g + 8s + 2b + h for lane = 16g + r, dword s, byte b, nibble h
// (h = 0 low).  One wave load instruction reads 1 KiB of contiguous HBM = a 16-row x 128-k tile.  The k order
// inside the MFMAs is permuted -- MFMA s of quad p multiplies lane group g's k = 128p + 32g + 8s .. +7 -- and the
// activation fragments are read in that same order, so the product is unchanged while every lane's 16 bytes share
// one scale: S[(t*KQ + p)*64 + lane] is the e8m0 byte of (row 16t + r, block 4p + g).
//
// Dequantisation is free-standing VALU work, four v_cvt_scalef32_pk_bf16_fp4 per MFMA (two codes -> two bf16,
// times the block scale, exact: e2m1 x 2^e is a bf16), feeding the bf16 v_mfma_f32_16x16x32_bf16 with fp32
// accumulation.  The fused RMSNorm, the epilogues and the activations-in-LDS (XL) staging are the fp8 kernel's
// (gemm_w8.hip, gemm_epi.h).
//
// Structure: one workgroup per (NT 16-row tiles, 16*NB-row M block); WAVES waves split the k quads, keep U quads of
// loads in flight (copy pipeline), reduce through LDS; wave 0 runs the epilogue.
#include "common.h"
#include "gemm_epi.h"

typedef uint32_t w4u32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 w4bf16x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void w4_lds_t;
typedef __attribute__((address_space(1))) const void w4_gbl_t;

// 8 e2m1 codes (one dword) -> the 8 bf16 of an MFMA A fragment, times the block scale
__device__ __forceinline__ bf16x8 w4_frag(uint32_t w, float sc) {
  const w4bf16x2 c0 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp4(w, sc, 0);
  const w4bf16x2 c1 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp4(w, sc, 1);
  const w4bf16x2 c2 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp4(w, sc, 2);
  const w4bf16x2 c3 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp4(w, sc, 3);
  return bf16x8{c0[0], c0[1], c1[0], c1[1], c2[0], c2[1], c3[0], c3[1]};
}

// e8m0 byte -> fp32 2^(e - 127) (the packer keeps e >= 1: never a zero / denormal scale)
__device__ __forceinline__ float e8m0_f32(uint32_t e) { return __builtin_bit_cast(float, (e & 0xffu) << 23); }

template <int WAVES, int U, int NT, int NB, int EPI, bool NORM, bool XL0>
__global__ __launch_bounds__(WAVES * 64) void skinny_w4_kernel(const GemmArgs a, const uint8_t* __restrict__ wsc) {
  constexpr bool XL = XL0 && NB == 1;
  extern __shared__ __attribute__((aligned(16))) char w4_xs[];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int KQ = a.K >> 7;  // 128-wide k quads
  // XCD-aware (tile, M block) mapping as gemm.hip: the M blocks of one tile get ids 8 apart (same L2)
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
  const int p_beg = (wave * KQ) / WAVES, p_end = ((wave + 1) * KQ) / WAVES;
  const int t0 = tg * NT;

  EpiIn pre[NT][NB];
  if (wave == 0) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int b = 0; b < NB; ++b) pre[t][b] = epi_load_at<EPI>(a, t0 + t, mo + 16 * b + (lane & 15), lane);
  }

  const w4u32x4* wb = reinterpret_cast<const w4u32x4*>(a.Wp) + (size_t)t0 * KQ * 64 + lane;
  const uint8_t* sb = wsc + (size_t)t0 * KQ * 64 + lane;
  // this lane's activation row and its k group: fragment s of quad p starts at element 128p + 32g + 8s
  const int kg = (lane >> 4) << 5;
  const __bf16* xb[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) xb[b] = a.X + (size_t)min(mo + 16 * b + (lane & 15), a.M - 1) * a.ldx + kg;
  const __bf16* xl_row = reinterpret_cast<const __bf16*>(w4_xs) + (size_t)min(lane & 15, a.M - 1) * a.K + kg;

  f32x4 acc[NT][NB];
  float ssq[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    ssq[b] = 0.f;
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  struct Quad {
    w4u32x4 w[NT];
    uint32_t s[NT];
    bf16x8 x[XL ? 1 : NB][4];
    int p;
  };
  auto load = [&](Quad& q, int p) {
    q.p = p;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      q.w[t] = __builtin_nontemporal_load(wb + ((size_t)t * KQ + p) * 64);
      q.s[t] = __builtin_nontemporal_load(sb + ((size_t)t * KQ + p) * 64);
    }
    if constexpr (!XL) {
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int s = 0; s < 4; ++s) q.x[b][s] = *reinterpret_cast<const bf16x8*>(xb[b] + p * 128 + s * 8);
    }
  };
  auto step = [&](const Quad& q) {
    float sc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) sc[t] = e8m0_f32(q.s[t]);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      bf16x8 xv[NB];
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        if constexpr (XL) xv[b] = *reinterpret_cast<const bf16x8*>(xl_row + q.p * 128 + s * 8);
        else xv[b] = q.x[b][s];
      }
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
        const bf16x8 wf = w4_frag(q.w[t][s], sc[t]);
#pragma unroll
        for (int b = 0; b < NB; ++b)
          acc[t][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, xv[b], acc[t][b], 0, 0, 0);
      }
    }
  };

  // copy pipeline: chunks of U quads, the next chunk's loads in flight while the current one is multiplied.  A
  // partial last chunk re-loads its last quad (clamped index, cache hit) instead of branching around loads, and
  // multiplies only its valid quads.
  const int nq = p_end - p_beg;
  const int nchunk = (nq + U - 1) / U;
  auto load_chunk = [&](Quad* q, int pc) {
#pragma unroll
    for (int u = 0; u < U; ++u) load(q[u], min(pc + u, p_end - 1));
  };
  Quad cur[U];
  if (nchunk > 0) load_chunk(cur, p_beg);
  if constexpr (XL) {
    // stage rows [0, M) x K of X by LDS-DMA under the weight prologue: 16-byte chunk c of the row-contiguous LDS copy
    // <- row c / (K / 8), column chunk c % (K / 8); wave instruction j covers chunks 64 j .. 64 j + 63
    const int cpr = a.K >> 3, nch = a.M * cpr;
    for (int j = wave; j * 64 < nch; j += WAVES) {
      const int c = j * 64 + lane;
      if (c < nch) {
        const int r = c / cpr, col = c - r * cpr;
        __builtin_amdgcn_global_load_lds((w4_gbl_t*)(a.X + (size_t)r * a.ldx + col * 8), (w4_lds_t*)(w4_xs + j * 1024),
                                         16, 0, 0);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  for (int c = 0; c < nchunk; ++c) {
    Quad nxt[U];
    const int pc = p_beg + c * U;
    const bool more = c + 1 < nchunk;
    if (more) load_chunk(nxt, pc + U);
    const int nv = p_end - pc;  // valid quads of this chunk (>= U except in the last one)
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (u < nv) step(cur[u]);
    if (more) {
#pragma unroll
      for (int u = 0; u < U; ++u) cur[u] = nxt[u];
    }
  }

  // ---- cross-wave reduction through LDS, epilogue by wave 0
  __shared__ __attribute__((aligned(16))) f32x4 red[WAVES][NT][NB][64];
  __shared__ float red_ss[NORM ? WAVES : 1][NB][16];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int b = 0; b < NB; ++b) red[wave][t][b][lane] = acc[t][b];
  if constexpr (NORM) {
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      float v = ssq[b];
      v += __shfl_xor(v, 16, 64);  // the 4 k groups of row m
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
    epi_store<EPI>(a, t0 + t, mo + 16 * b + (lane & 15), lane, pre[t][b],
                   [&](int off) { return unit_sum(lane + off); });
  }
}

template <int WAVES, int U, int NT, int NB, int EPI, bool NORM>
static hipError_t w4_launch(const GemmArgs& a, const uint8_t* wsc, bool xl, hipStream_t st) {
  const dim3 grid(a.N / 16 / NT * a.msplit), block(WAVES * 64);
  if constexpr (NB == 1) {
    if (xl) {
      hipLaunchKernelGGL((skinny_w4_kernel<WAVES, U, NT, NB, EPI, NORM, true>), grid, block, (size_t)a.M * a.K * 2, st,
                         a, wsc);
      return hipGetLastError();
    }
  }
  hipLaunchKernelGGL((skinny_w4_kernel<WAVES, U, NT, NB, EPI, NORM, false>), grid, block, 0, st, a, wsc);
  return hipGetLastError();
}

// kernel shapes: (waves, quads in flight, 16-row tiles of N, 16-row blocks of M) per workgroup
enum W4Var { W4_4_8_1_1, W4_8_4_1_1, W4_4_4_2_1, W4_8_2_2_1, W4_4_2_1_2, W4_8_2_1_2, W4_N_VARS };

template <bool NORM>
static hipError_t w4_launch_e(int epi, int var, const GemmArgs& a, const uint8_t* wsc, bool xl, hipStream_t st) {
#define CAIN_W4_VAR(E)                                                      \
  switch (var) {                                                            \
    case W4_4_8_1_1: return w4_launch<4, 8, 1, 1, E, NORM>(a, wsc, xl, st); \
    case W4_8_4_1_1: return w4_launch<8, 4, 1, 1, E, NORM>(a, wsc, xl, st); \
    case W4_4_4_2_1: return w4_launch<4, 4, 2, 1, E, NORM>(a, wsc, xl, st); \
    case W4_8_2_2_1: return w4_launch<8, 2, 2, 1, E, NORM>(a, wsc, xl, st); \
    case W4_4_2_1_2: return w4_launch<4, 2, 1, 2, E, NORM>(a, wsc, xl, st); \
    default: return w4_launch<8, 2, 1, 2, E, NORM>(a, wsc, xl, st);         \
  }
  switch (epi) {
    case EPI_BF16: CAIN_W4_VAR(EPI_BF16)
    case EPI_RESID: CAIN_W4_VAR(EPI_RESID)
    case EPI_F32: CAIN_W4_VAR(EPI_F32)
    case EPI_SILU: CAIN_W4_VAR(EPI_SILU)
    case EPI_GELU: CAIN_W4_VAR(EPI_GELU)
    case EPI_QKV_ROPE: CAIN_W4_VAR(EPI_QKV_ROPE)
    default: return hipErrorInvalidValue;
  }
#undef CAIN_W4_VAR
}

// Tuning override (tools / tests; -1: the rule below): the kernel shape index of W4Var
static int g_w4_var = -1;
CAIN_API void cain_gemm_w4_set_variant(int v) { g_w4_var = v < W4_N_VARS ? v : -1; }

// Few-row shape rule: the kernel variant for an (N, K, M) problem.
static int w4_variant(int N, int K, int M, int n_cu) {
  if (g_w4_var >= 0) return g_w4_var;
  if (M > 16) return (N / 16) * ((M + 31) / 32) <= n_cu ? W4_8_2_1_2 : W4_4_2_1_2;
  const int kq = K / 128;
  // two tiles per workgroup on LM-head-sized grids (fewer, longer workgroups); else one tile, its k quads
  // dealt to 8 waves when the grid is at most one workgroup per CU and each wave still gets >= 4 quads
  if (N >= 65536 && (N / 16) % 2 == 0) return kq >= 32 ? W4_8_2_2_1 : W4_4_4_2_1;
  return (N / 16 <= n_cu && kq >= 32) ? W4_8_4_1_1 : W4_4_8_1_1;
}

CAIN_API int cain_gemm_w4_variant(int N, int K, int M) {
  int dev = 0, n = 0;
  (void)hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) n = 256;
  return w4_variant(N, K, M, n);
}

// Same arguments as cain_gemm_w8 (gemm_w8.hip); Wp is the MXFP4 packing, wsc its e8m0 scale bytes.
CAIN_API int cain_gemm_w4(const void* Wp, const void* wsc, const void* X, int ldx, int K, int N, int M, void* Y, int ldy,
                          const float* bias, int norm, float eps, const int* slot, const int* pos, const float* cos_t,
                          const float* sin_t, void* kc, void* vtc, int H, int Hkv, int hd, int T_max, int epi_flags,
                          hipStream_t st) {
  const int epi = epi_flags & EPI_MASK;
  if (K % 128 || N % 16 || M < 1 || M > 64) return -1;
  if (epi == EPI_QKV_ROPE && (hd % 16 || (hd / 2) % 8)) return -1;
  GemmArgs a{};
  a.Wp = reinterpret_cast<const bf16x8*>(Wp);
  a.X = reinterpret_cast<const __bf16*>(X);
  a.ldx = ldx, a.K = K, a.N = N, a.M = M, a.Y = Y, a.ldy = ldy, a.bias = bias;
  a.eps = eps;
  a.slot = slot, a.pos = pos, a.cos_t = cos_t, a.sin_t = sin_t;
  a.kc = reinterpret_cast<__bf16*>(kc), a.vtc = reinterpret_cast<__bf16*>(vtc);
  a.H = H, a.Hkv = Hkv, a.hd = hd, a.T_max = T_max, a.kv8 = (epi_flags & EPI_KV_FP8) ? 1 : 0;
  static const int n_cu = [] {
    int dev = 0, n = 0;
    (void)hipGetDevice(&dev);
    return hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess ? n : 256;
  }();
  const int var = w4_variant(N, K, M, n_cu);
  const int nb = (var == W4_4_2_1_2 || var == W4_8_2_1_2) ? 2 : 1;
  const int nt = (var == W4_4_4_2_1 || var == W4_8_2_2_1) ? 2 : 1;
  if ((N / 16) % nt) return -1;
  a.msplit = (M + 16 * nb - 1) / (16 * nb);
  // activations in LDS: one row block, at most 64 KiB of rows
  const bool xl = nb == 1 && a.msplit == 1 && (long long)M * K * 2 <= 65536;
  const uint8_t* sc = reinterpret_cast<const uint8_t*>(wsc);
  const hipError_t e = norm ? w4_launch_e<true>(epi, var, a, sc, xl, st) : w4_launch_e<false>(epi, var, a, sc, xl, st);
  return int(e);
}
