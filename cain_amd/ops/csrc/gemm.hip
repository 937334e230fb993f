// Weight-streaming skinny GEMM for decode / short prefill on gfx950 MFMA,
// with the neighbouring elementwise ops fused into its prologue and epilogue.
//
//   Y[m][n] = epilogue( sum_k B(X)[m][k] * W[n][k] )      m < M <= 16*NB,  n < N
//
// W is stored MFMA-fragment-major (cain_amd/models/weights.py pack_mfma_a):
// Wp[(t*KS + s)*64 + lane] is the 16-byte A fragment of lane `lane` of
// v_mfma_f32_16x16x32_bf16 for rows 16t..16t+15 and k-slice 32s..32s+31, so every
// wave load instruction streams 1 KiB of contiguous HBM with a non-temporal hint
// (each weight byte is read once per decode step).  The B operand is the
// activation row m (16 B per lane straight from L2: lane = (col m, k-group g)
// reads X[m][32s+8g .. +8]); neither operand goes through LDS
// (cdna_hip_programming.md §5, 'GEMV / M <= 16' row).
//
// Fused RMSNorm (NORM): W.(x * inv * g) = inv * (W diag(g)).x with inv a per-row
// scalar; the gain g is folded into the weight columns at pack time
// (cain_amd/models/weights.py fold_gain), so the B fragment is x itself, every workgroup accumulates the
// row's sum of squares from the x fragments it streams anyway (its waves cover
// all of K), and the epilogue scales by rsqrt(mean(x^2) + eps): no separate
// normalisation kernel, no launch gap, no cross-kernel state.
//
// Parallelism: a workgroup owns NT 16-row tiles; its WAVES waves split the
// K-slices and run a register double-buffered loop (the next U slices' loads
// are in flight while the current U compute), then reduce their 16x16
// accumulators through LDS once at the end (no cross-workgroup split-K).
// Epilogue inputs (residual, bias, RoPE tables) are loaded before the loop.
//
// Epilogues (SURVEY §2.4 rows QKV / RoPE / KV-append / O / gate-up / down / LM head):
//   EPI_BF16      y = bf16(acc + bias)
//   EPI_RESID     y = bf16(acc + resid) (in place on the residual stream)
//   EPI_F32       y = acc (fp32 LM-head logits)
//   EPI_SILU/GELU gate/up rows interleaved by 8 inside each 16-row tile
//                 -> y = bf16(act(gate) * up)
//   EPI_QKV_ROPE  fused QKV epilogue: + bias, RoPE (rows pre-permuted so each
//                 16-row tile holds 8 rotation pairs), Q -> q buffer, K -> K cache
//                 at (slot[m], pos[m]), V -> transposed V cache.
#include <algorithm>
#include <cstdlib>

#include "common.h"

#include "gemm_epi.h"

// Split-K of the skinny kernel (SPLIT): a grid of N/16 tiles smaller than the chip (the O / down projections
// of qwen2:1.5b and gemma:2b at one row: 96-128 workgroups on 256 CUs, 2.7 TB/s) also splits K over ks
// workgroups.  Each publishes its fp32 16x16 partial (and the RMSNorm partial sums of squares) with
// write-through stores; the last arriver of the tile (ticket) adds the ks partials in fixed order and runs the
// fused epilogue -- the in-launch combine of cdna_hip_programming.md §5 item 2, as in bgemm_kernel.
struct SkArgs {
  int ks;              // workgroups per tile (k ranges)
  unsigned* counters;  // [ntiles], zero between launches (the reducer resets its own)
  float* part;         // [ntiles][ks][64 lanes] f32x4
  float* part_ss;      // [ntiles][ks][16]
};

// (Round 3 also kept the activations staged in LDS (XL) and a two-register-set ping-pong loop (PP) as A/B
// options of this kernel; both measured slower or level in the single-stream decode -- llama3.1:8b 340.8 -> 339.5
// tok/s with XL, profiles/r3/b1_xlds_ab.txt -- and were removed.  The MXFP4 kernel (gemm_w4.hip) stages its
// activations, where they replace four fragment loads per KiB of weights.)
template <int NT, int NB, int WAVES, int U, int EPI, bool NORM, bool SPLIT = false>
__global__ __launch_bounds__(WAVES * 64) void skinny_gemm_kernel(const GemmArgs a, const SkArgs sk) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int K = a.K;
  const int KS = K >> 5;
  // XCD-aware block -> (row tile, M split) mapping: blocks b and b + 8 share an XCD under the
  // round-robin dispatch, so the msplit workgroups of one weight tile are given ids that differ by
  // multiples of 8 and their repeated tile reads hit the same L2 (speed only: any placement is correct).
  // SPLIT (msplit = 1): the same mapping over the ks k-ranges, so a tile's partials and its reducer share an L2.
  int tg, ms, kc = 0;
  {
    const int bid = blockIdx.x, msp = SPLIT ? sk.ks : a.msplit;
    const int ntg = gridDim.x / msp;
    int sub;
    if (msp == 1) {
      tg = bid, sub = 0;
    } else if ((ntg & 7) == 0) {
      const int r = bid >> 3;
      sub = r % msp;
      tg = (r / msp) * 8 + (bid & 7);
    } else {
      tg = bid / msp, sub = bid - (bid / msp) * msp;
    }
    if constexpr (SPLIT) ms = 0, kc = sub;
    else ms = sub;
  }
  const int tile0 = tg * NT;
  const int mo = ms * 16 * NB;  // first row of this workgroup
  // k-slices of this workgroup (all of K unless SPLIT), dealt to its waves
  const int ksp = SPLIT ? (KS + sk.ks - 1) / sk.ks : KS;
  const int k_beg = min(KS, kc * ksp), k_n = min(KS, k_beg + ksp) - k_beg;
  const int s_beg = k_beg + (wave * k_n) / WAVES;
  const int s_end = k_beg + ((wave + 1) * k_n) / WAVES;
  constexpr int UNITS = NT * NB * 64;
  constexpr bool PRE = UNITS <= WAVES * 64;  // each wave finalises at most one 64-unit chunk

  EpiIn pre{};
  if constexpr (PRE) {
    if (wave * 64 < UNITS) pre = epi_load<NT, NB, EPI>(a, tile0, mo, wave * 64 + lane);
  }

  f32x4 acc[NT][NB];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int b = 0; b < NB; ++b) acc[t][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  const bf16x8* wbase[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) wbase[t] = a.Wp + (size_t)(tile0 + t) * KS * 64 + lane;
  const __bf16* xbase[NB];
  float ssq[NB];  // NORM: this lane's partial sum of x^2 of row m (its k-group of each slice)
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const int m = min(mo + b * 16 + (lane & 15), a.M - 1);  // rows past M re-read a valid row
    xbase[b] = a.X + (size_t)m * a.ldx + ((lane >> 4) << 3);
    ssq[b] = 0.f;
  }

  // raw fragment loads (issued early); normalisation happens at use, after the data landed
  // (always non-temporal: a runtime choice of the cache policy put a branch around every load, which
  // defeats the counted waits of the pipeline below; with msplit > 1 the tile-mates still hit L2/MALL)
  auto load_w = [&](int s, int t) -> bf16x8 { return __builtin_nontemporal_load(wbase[t] + (size_t)s * 64); };
  auto load_x = [&](int s, int b) -> bf16x8 { return *reinterpret_cast<const bf16x8*>(xbase[b] + s * 32); };
  // RMSNorm factorisation: (W diag(g)) (x * inv) = inv * ((W diag(g)) x); the per-row inv is applied in
  // the epilogue and the sum of squares is accumulated from the x fragments this WG streams anyway
  // (its waves cover all of K), so no separate norm kernel and no cross-kernel sum-of-squares buffer.
  auto norm_x = [&](bf16x8 v, int b, float wgt) -> bf16x8 {
    if constexpr (NORM) {
      float q = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float f = bf2f(v[j]);
        q += f * f;
      }
      ssq[b] += wgt * q;
    }
    return v;
  };
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  auto compute = [&](const bf16x8 (&w)[U][NT], const bf16x8 (&x)[U][NB], bool valid) {
    const uint32_t keep = valid ? 0xffffffffu : 0u;
    const float wgt = valid ? 1.f : 0.f;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      bf16x8 xb[NB];
#pragma unroll
      for (int b = 0; b < NB; ++b) xb[b] = norm_x(x[u][b], b, wgt);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const bf16x8 wm = __builtin_bit_cast(bf16x8, __builtin_bit_cast(u32x4, w[u][t]) & keep);
#pragma unroll
        for (int b = 0; b < NB; ++b)
          acc[t][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wm, xb[b], acc[t][b], 0, 0, 0);
      }
    }
  };

  // ---- copy pipeline: the next U slices' loads are issued before the current U compute (the compiler schedules
  // the loads and their counted waits itself)
  int s = s_beg;
  const int nfull = (s_end - s_beg) / U;
  if (nfull > 0) {
    bf16x8 wa[U][NT], xa[U][NB];
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int t = 0; t < NT; ++t) wa[u][t] = load_w(s + u, t);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int b = 0; b < NB; ++b) xa[u][b] = load_x(s + u, b);
    }
    for (int c = 0; c < nfull; ++c) {
      bf16x8 wn[U][NT], xn[U][NB];
      const int sn = s + U;
      const bool more = c + 1 < nfull;
      if (more) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
#pragma unroll
          for (int t = 0; t < NT; ++t) wn[u][t] = load_w(sn + u, t);
#pragma unroll
          for (int b = 0; b < NB; ++b) xn[u][b] = load_x(sn + u, b);
        }
      }
      compute(wa, xa, true);
      if (more) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
#pragma unroll
          for (int t = 0; t < NT; ++t) wa[u][t] = wn[u][t];
#pragma unroll
          for (int b = 0; b < NB; ++b) xa[u][b] = xn[u][b];
        }
      }
      s = sn;
    }
  }
  for (; s < s_end; ++s) {
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const bf16x8 w = load_w(s, t);
#pragma unroll
      for (int b = 0; b < NB; ++b)
        acc[t][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w, norm_x(load_x(s, b), b, 1.f), acc[t][b], 0, 0, 0);
    }
  }

  // ---- cross-wave reduction through LDS: red[wave][unit], unit = (t*NB + b)*64 + lane
  __shared__ __attribute__((aligned(16))) f32x4 red[WAVES][UNITS];
  __shared__ float red_ss[NORM ? WAVES : 1][NORM ? NB * 16 : 1];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int b = 0; b < NB; ++b) red[wave][(t * NB + b) * 64 + lane] = acc[t][b];
  if constexpr (NORM) {
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      float v = ssq[b];
      v += __shfl_xor(v, 16, 64);  // the 4 k-groups of row m
      v += __shfl_xor(v, 32, 64);
      if (lane < 16) red_ss[wave][b * 16 + lane] = v;
    }
  }
  __syncthreads();

  if constexpr (SPLIT) {
    // NT = NB = 1: one 64-lane unit per tile.  Wave 0 publishes this k-range's partial, takes the ticket; the
    // last of the tile's ks arrivals sums the partials (k-range order: deterministic) and finishes the tile.
    static_assert(NT == 1 && NB == 1, "split-K skinny body: one 16x16 unit per workgroup");
    __shared__ unsigned s_ticket;
    __shared__ float s_inv[16];
    if (wave == 0) {
      f32x4 v = red[0][lane];
#pragma unroll
      for (int w = 1; w < WAVES; ++w) v += red[w][lane];
      const size_t pi = (size_t)tg * sk.ks + kc;
      st_wt(slab_rsrc(sk.part), int((pi * 64 + lane) * 16), v);
      if constexpr (NORM) {
        if (lane < 16) {
          float ss = 0.f;
#pragma unroll
          for (int w = 0; w < WAVES; ++w) ss += red_ss[w][lane];
          st_wt_f32(slab_rsrc(sk.part_ss), int((pi * 16 + lane) * 4), ss);
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0)
        s_ticket = __hip_atomic_fetch_add(sk.counters + tg, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (s_ticket != unsigned(sk.ks - 1) || wave != 0) return;
    // reducer: every partial load issued before the first add (clamped index, surplus weighted 0)
    const __amdgpu_buffer_rsrc_t pr = slab_rsrc(sk.part), sr = slab_rsrc(sk.part_ss);
    f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
    float ss = 0.f;
    for (int k0 = 0; k0 < sk.ks; k0 += 4) {
      f32x4 l[4];
      float q[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const size_t pi = (size_t)tg * sk.ks + min(k0 + j, sk.ks - 1);
        l[j] = ld_wt(pr, int((pi * 64 + lane) * 16));
        q[j] = NORM ? ld_wt_f32(sr, int((pi * 16 + (lane & 15)) * 4)) : 0.f;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float wj = (k0 + j < sk.ks) ? 1.f : 0.f;
        v += wj * l[j];
        ss += wj * q[j];
      }
    }
    red[0][lane] = v;
    if constexpr (NORM) {
      if (lane < 16) s_inv[lane] = rms_inv(ss, a.K, a.eps);
    }
    if (lane == 0) sk.counters[tg] = 0u;  // ready for the next launch (launch-ordered)
    const int m = mo + (lane & 15);
    const EpiIn e = epi_load<NT, NB, EPI>(a, tile0, mo, lane);
    epi_store<EPI>(a, tile0, m, lane, e, [&](int off) {
      f32x4 r = red[0][lane + off];
      if constexpr (NORM) r *= s_inv[(lane + off) & 15];
      return r;
    });
    return;
  }

  auto unit_sum = [&](int u) -> f32x4 {
    f32x4 v = red[0][u];
#pragma unroll
    for (int w = 1; w < WAVES; ++w) v += red[w][u];
    if constexpr (NORM) {
      const int b = (u >> 6) % NB, m16 = b * 16 + (u & 15);
      float ss = 0.f;
#pragma unroll
      for (int w = 0; w < WAVES; ++w) ss += red_ss[w][m16];
      v *= rms_inv(ss, a.K, a.eps);
    }
    return v;
  };

  // whole waves walk the units (shuffles below need full waves)
  for (int ub = wave * 64; ub < UNITS; ub += WAVES * 64) {
    const int u = ub + lane;
    const int tb = u >> 6;
    const int b = tb % NB;
    const int t = tb / NB;
    const int m = mo + b * 16 + (lane & 15);
    const EpiIn e = (PRE && ub == wave * 64) ? pre : epi_load<NT, NB, EPI>(a, tile0, mo, u);
    epi_store<EPI>(a, tile0 + t, m, lane, e, [&](int off) { return unit_sum(u + off); });
    if constexpr (EPI == EPI_F32) {
      // the LM head's per-row maximum of this 16-column chunk (lanes c, c + 16, c + 32, c + 48 hold row c's 16)
      if (a.cmax) {
        const f32x4 v = unit_sum(u);
        float mx = fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3]));
        mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        if ((lane >> 4) == 0 && m < a.M) a.cmax[(size_t)m * a.ld_cm + tile0 + t] = mx;
      }
    }
  }
}

template <int NT, int NB, int WAVES, int EPI, bool NORM>
static hipError_t launch_t(const GemmArgs& a, const SkArgs& sk, hipStream_t st) {
  constexpr int U = (NB >= 2) ? 2 : 4;  // slices in flight per wave
  if (sk.ks > 1) {
    if constexpr (NT == 1 && NB == 1) {
      hipLaunchKernelGGL((skinny_gemm_kernel<NT, NB, WAVES, U, EPI, NORM, true>), dim3(a.N / 16 * sk.ks),
                         dim3(WAVES * 64), 0, st, a, sk);
      return hipGetLastError();
    }
    return hipErrorInvalidValue;
  }
  hipLaunchKernelGGL((skinny_gemm_kernel<NT, NB, WAVES, U, EPI, NORM>), dim3(a.N / (16 * NT) * a.msplit),
                     dim3(WAVES * 64), 0, st, a, sk);
  return hipGetLastError();
}

template <int NT, int NB, int EPI, bool NORM>
static hipError_t launch_w(int waves, const GemmArgs& a, const SkArgs& sk, hipStream_t st) {
  // the LDS reduction buffer is WAVES * NT * NB KiB: cap it at 64 KiB at compile time
  constexpr int WMAX = 64 / (NT * NB);
  if constexpr (WMAX >= 16) {
    if (waves >= 16) return launch_t<NT, NB, 16, EPI, NORM>(a, sk, st);
  }
  if constexpr (WMAX >= 8) {
    if (waves >= 8) return launch_t<NT, NB, 8, EPI, NORM>(a, sk, st);
  }
  return launch_t<NT, NB, 4, EPI, NORM>(a, sk, st);
}

template <bool NORM>
static hipError_t launch_e(int epi, int waves, const GemmArgs& a, const SkArgs& sk, hipStream_t st) {
  switch (epi) {
    case EPI_BF16: return launch_w<1, 1, EPI_BF16, NORM>(waves, a, sk, st);
    case EPI_RESID: return launch_w<1, 1, EPI_RESID, NORM>(waves, a, sk, st);
    case EPI_F32: return launch_w<1, 1, EPI_F32, NORM>(waves, a, sk, st);
    case EPI_SILU: return launch_w<1, 1, EPI_SILU, NORM>(waves, a, sk, st);
    case EPI_GELU: return launch_w<1, 1, EPI_GELU, NORM>(waves, a, sk, st);
    case EPI_QKV_ROPE: return launch_w<1, 1, EPI_QKV_ROPE, NORM>(waves, a, sk, st);
    default: return hipErrorInvalidValue;
  }
}

// Split rule of the skinny kernel (M <= 16 rows, one workgroup per 16-row tile): a grid under ~3/4 of the CUs
// whose tiles are long (K > 128 slices: the down projections of qwen2:1.5b / gemma:2b, 96-128 tiles of 280-512
// slices) takes ks ~ K / 80 slices k-ranges (at most 8 and ~512 workgroups), so ~4x the CUs stream.  Short tiles stay whole: there the split's combine round trip (measured +1 us on
// qwen2:1.5b's QKV) costs more than it spreads.  (Also measured and not kept: "one-shot" waves that load all of
// their <= 16 slices in one burst before any MFMA -- the 128 staging VGPRs halve the resident waves, and with
// them the bytes in flight: qwen2:1.5b gate/up 11.9 -> 12.5 us, split down 9.0 -> 10.4 us, gpurun_out/r3d.)
// cain_gemm_set_skinny_split(0) disables it (tests).  (Halving the k-range of grids between one and two tiles
// per CU -- llama3.1:8b QKV at one row -- measured slower, 338 -> 328 tok/s single stream, and was removed:
// profiles/r3/b1_skinny_split2_ab.txt.)
static int g_skinny_split = 1;
CAIN_API void cain_gemm_set_skinny_split(int mode) { g_skinny_split = mode; }
static int skinny_split(int N, int K, int M) {
  const int on = g_skinny_split;
  const int nt = N / 16, KS = K / 32;
  if (!on || M > 16 || nt >= 192 || nt < 1 || KS <= 128) return 1;
  // ~80 slices per workgroup, at most ~512 workgroups (qwen2:1.5b down: ks 4 = 9.0 us vs ks 3 = 10.4 us)
  return std::max(1, std::min(std::min(8, (KS + 79) / 80), 512 / nt));
}

// Waves per workgroup: 8 (the tuned choice on every llama3.1:8b decode shape, profiles/gemm_tune.md)
// unless the grid is small (then 16, to keep >= ~2k waves streaming) or K is too short to give each
// wave two pipelined chunks.
static int pick_waves(int n_wg, int ks, bool split = false) {
  // grids of (b, 2b] workgroups, b = the CU count, on 4 waves: llama3.1:8b's 384-workgroup QKV at one row 12.3 ->
  // 11.9 us, single stream 340.7 -> 341.8 tok/s (same box, interleaved; qwen2:7b 356.2 -> 356.9;
  // profiles/r3/b1_skinny_w4_ab.txt).  (A wider (b, 8b] range and 16-wave workgroups for grids of <= b measured
  // mixed / level and were removed.)
  const int w4 = cain_cu_budget();
  if (!split && w4 > 0 && n_wg > w4 && n_wg <= 2 * w4 && ks / 4 >= 8) return 4;  // unsplit grids (measured)
  int w = 8;
  if (n_wg * w < 1024 && ks / 16 >= 8) w = 16;
  while (w > 4 && ks / w < 8) w /= 2;
  return w;
}

static int gemm_dispatch(GemmArgs a, int epi, int norm, int waves, hipStream_t st, const SkArgs* split = nullptr) {
  if (a.K % 32 || a.N % 16 || a.M < 1 || a.M > 64) return -1;
  SkArgs sk{};
  sk.ks = 1;
  if (split && split->ks > 1 && a.M <= 16) sk = *split;
  const bool pair = (epi == EPI_SILU || epi == EPI_GELU);
  // Rows beyond 16 are split over workgroups (msplit) rather than widening a workgroup's
  // B operand: per k-step a wave then loads one weight and one activation fragment, and
  // the grid keeps N/16 * msplit workgroups (a wider NB would need NT > 1 to amortise the
  // activation loads, which halves the grid — measured 1.4-2.7 TB/s at M = 32-64).
  const int nb = 1;
  const int nt = 1;
  a.msplit = (a.M + 15) / 16;
  const int n_wg = a.N / 16 * a.msplit * sk.ks;
  if (waves <= 0) waves = pick_waves(n_wg, a.K / 32 / sk.ks, sk.ks > 1);
  while (waves > 4 && waves * nt * nb > 64) waves /= 2;  // LDS reduction buffer <= 64 KiB
  // 16-wave groups cap registers at 128/lane: the RoPE / norm-prologue / NB=4 bodies would spill
  if (waves > 8 && (epi == EPI_QKV_ROPE || norm || nb >= 4)) waves = 8;
  (void)pair;
  const hipError_t e = norm ? launch_e<true>(epi, waves, a, sk, st) : launch_e<false>(epi, waves, a, sk, st);
  return int(e);
}

// =====================================================================================================
// Batched weight-streaming GEMM, 16 < M <= 256 (batched decode, prefill chunks).
//
// The skinny kernel's waves split K and each wave reads its own activation fragments straight from L2:
// at M = 64 that is 4 B of activation traffic per weight byte and the CU's vector-memory path, not HBM,
// becomes the limit.  Here the waves of a workgroup split N instead (each owns NTW 16-row tiles) and
// walk the SAME k-range, so the activation chunk X[0..M)[k0..k0+256) is staged ONCE per workgroup into
// LDS (bf16, MFMA-B-fragment-major so both the staging write
// and every ds_read_b128 of a wave are 1 KiB contiguous, conflict-free) and double-buffered: chunk c+1
// streams in from L2 while chunk c feeds the MFMAs; one barrier per chunk.  Weights still stream from
// HBM as 1 KiB non-temporal fragment loads, prefetched one slice group ahead in registers.
//
// Parallelism: N/(16*NTW*8) row blocks x ksplit k-ranges.  With ksplit > 1 every workgroup publishes
// its fp32 16x16 blocks (and the RMSNorm partial sums of squares) with write-through stores and the
// LAST arriving workgroup of a row block adds them up and runs the fused epilogue (same ticket protocol
// as the attention combine).  Traffic per weight byte: M/(16*NTW*8) activation (L2) + 2M/k_range
// partials (MALL), against 4 for the skinny kernel at M = 64.
// =====================================================================================================
constexpr int BG_WAVES = 8;  // default waves per workgroup (template W: 4 or 8)
constexpr int BG_CK = 8;     // default 32-wide k-slices per LDS chunk (template CK: 8 or 16)

struct BgArgs {
  int ksplit;  // workgroups per row block
  int kspl;    // k-slices per workgroup (multiple of CK)
  float* part;       // [nblk][ksplit][W*NTW*NB][64] f32x4  (ksplit > 1)
  float* part_ss;    // [nblk][ksplit][NB*16]                   (ksplit > 1 && NORM)
  unsigned* counters;  // [nblk], zero between launches (the reducer resets its own)
};

// Split-K partial slabs: the write-through (sc1) helpers of common.h (slab_rsrc, st_wt, ld_wt).

// LB: minimum waves per SIMD the register allocation must allow (4 -> 128 VGPRs, 2 -> 256, 1 -> 512)
// AR: activation register ring (see the AR branch of the chunk loop)
// WM: wave groups along M.  The W waves form WN = W/WM columns (each owns NTW 16-row tiles of N) times WM
// rows (each owns NB/WM of the 16-row blocks of M): with WM = 2 and NTW = 2 a wave issues the same MFMAs per
// slice as WM = 1, NTW = 1 but reads half as many activation fragments from LDS (each feeds 2 tiles); the
// two wave rows of a tile column load the same weight fragments (the second from L2).
template <int NB, int NTW, int W, int CK, int U, int D, int XS, int LB, bool AR, int EPI, bool NORM, int WM = 1>
__global__ __launch_bounds__(W * 64, LB) void bgemm_kernel(const GemmArgs a, const BgArgs bg) {
  constexpr int BG_CK = CK;
  constexpr int FR = BG_CK * NB;        // B fragments per chunk
  constexpr int FPW = FR / W;           // staged per wave per chunk
  constexpr int NGRP = BG_CK / U;       // weight prefetch groups per chunk
  constexpr int WN = W / WM;            // wave columns (N)
  constexpr int NBW = NB / WM;          // row blocks of M per wave
  constexpr int UNITS = WN * NTW * NB;  // 64-lane output blocks per workgroup
  static_assert(FR % W == 0 && BG_CK % U == 0, "tiling");
  static_assert(W % WM == 0 && NB % WM == 0, "wave grid");
  static_assert(UNITS * 1024 <= XS * FR * 1024, "epilogue buffer must fit in the staging buffer");
  static_assert(XS == 2 || XS == 3, "activation stage depth");
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wn = wave % WN, b0 = (wave / WN) * NBW;  // wave column, first row block
  const int KS = a.K >> 5, ntiles = a.N >> 4;
  int blk, kc;
  {
    const int bid = blockIdx.x, ks = bg.ksplit, nblk = gridDim.x / ks;
    if (ks == 1) {
      blk = bid, kc = 0;
    } else if ((nblk & 7) == 0) {  // k-range partners share an XCD (ids differ by multiples of 8)
      const int r = bid >> 3;
      kc = r % ks;
      blk = (r / ks) * 8 + (bid & 7);
    } else {
      blk = bid / ks, kc = bid - (bid / ks) * ks;
    }
  }
  const int s_beg = kc * bg.kspl;
  const int nch = (min(KS, s_beg + bg.kspl) - s_beg) / BG_CK;

  // XS activation stages: chunk c is read from xs[c % XS]; with XS = 3 the loads of chunk c+2 are in
  // flight while c computes (two chunk-times to land instead of one)
  __shared__ __attribute__((aligned(16))) bf16x8 xs[XS][FR][64];
  __shared__ float s_ss[NORM ? NB * 16 : 1];  // NORM: per-row sum of squares of this k-range
  __shared__ float s_inv[NB * 16];
  __shared__ unsigned s_ticket;

  int gt[NTW];
  const bf16x8* wb[NTW];
#pragma unroll
  for (int t = 0; t < NTW; ++t) {
    gt[t] = (blk * WN + wn) * NTW + t;
    wb[t] = a.Wp + (size_t)min(gt[t], ntiles - 1) * KS * 64 + lane;  // idle tiles re-read a valid one
  }
  auto load_w = [&](int s, int t) -> bf16x8 { return __builtin_nontemporal_load(wb[t] + (size_t)s * 64); };

  // Activation staging in FULL 128-B lines: a chunk is rows [0, 16*NB) x CK slices = PPR 16-byte pieces per
  // row; wave instruction i of wave w covers rows RPI*(w + W*i) .. +RPI, lane l -> row RPI*(w + W*i) + l / PPR,
  // piece l % PPR (rows past M re-read row M-1).  A fragment-shaped load (16 rows x 64 B per instruction)
  // touches twice the cache lines per byte and made the vector-memory path, not HBM, the limit
  // (cdna_hip_programming.md §5, 'Projection GEMM at M = 256').  In LDS a row keeps its pieces in order
  // up to an XOR swizzle, piece p at p ^ (row & 15): the 8-lane groups of ds_write_b128 and the 16-lane
  // groups of the fragment reads (lane = row & 15 + 16 * k-group) are both bank-conflict free.
  constexpr int PPR = 4 * BG_CK;   // 16-byte pieces per row and chunk
  constexpr int RPI = 64 / PPR;    // rows per wave instruction
  constexpr int STAGE = FR * 1024;
  static_assert(BG_CK >= 4 && 16 * NB == RPI * FR, "full-line staging tiling");
  char* const xsb = reinterpret_cast<char*>(&xs[0][0][0]);
  const __bf16* xrow[FPW];
  int xoff[FPW];   // LDS byte offset of this lane's piece inside a stage
  float ssq[FPW];  // NORM: this lane's partial sum of x^2 of its row (its pieces)
#pragma unroll
  for (int i = 0; i < FPW; ++i) {
    const int r = RPI * (wave + W * i) + lane / PPR, pc = lane % PPR;
    xrow[i] = a.X + (size_t)min(r, a.M - 1) * a.ldx + pc * 8;
    xoff[i] = r * (PPR * 16) + ((pc ^ (r & 15)) << 4);
    ssq[i] = 0.f;
  }
  // fragment of slice sl (0..CK-1) and row block b: lane (m = lane & 15, k-group g = lane >> 4) reads piece
  // 4*sl + g of row 16b + m at (4*sl + g) ^ m = 4*((sl & ~3) | ((sl & 3) ^ (m >> 2))) + (g ^ (m & 3))
  int fo[4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
    fo[j] = (lane & 15) * (PPR * 16) + ((((j ^ ((lane & 15) >> 2)) << 2) | ((lane >> 4) ^ (lane & 3))) << 4);
  auto frag = [&](int buf, int sl, int b) -> bf16x8 {
    return *reinterpret_cast<const bf16x8*>(xsb + buf * STAGE + b * 16 * (PPR * 16) + (sl & ~3) * 64 + fo[sl & 3]);
  };
  auto stage_load = [&](int c, bf16x8 (&xr)[FPW]) {
    const int k0 = (s_beg + c * BG_CK) * 32;
#pragma unroll
    for (int i = 0; i < FPW; ++i) xr[i] = *reinterpret_cast<const bf16x8*>(xrow[i] + k0);
  };
  auto stage_store = [&](int buf, const bf16x8 (&xr)[FPW], float wgt) {
#pragma unroll
    for (int i = 0; i < FPW; ++i) {
      if constexpr (NORM) {  // the gain is folded into W: only the row's sum of squares is needed
        float q = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float f = bf2f(xr[i][j]);
          q += f * f;
        }
        ssq[i] += wgt * q;
      }
      *reinterpret_cast<bf16x8*>(xsb + buf * STAGE + xoff[i]) = xr[i];
    }
  };

  f32x4 acc[NTW][NBW];
#pragma unroll
  for (int t = 0; t < NTW; ++t)
#pragma unroll
    for (int b = 0; b < NBW; ++b) acc[t][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 wa[U][NTW];
  bf16x8 xa_[FPW], xb_[FPW];  // activation staging registers (see run_chunk)
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int t = 0; t < NTW; ++t) wa[u][t] = load_w(s_beg + u, t);
  if constexpr (NORM) {
    if (threadIdx.x < NB * 16) s_ss[threadIdx.x] = 0.f;  // ordered before the epilogue atomics by the barrier below
  }
  {
    bf16x8 xr[FPW];
    stage_load(0, xr);
    stage_store(0, xr, 1.f);
  }
  if constexpr (XS == 3) stage_load(min(1, nch - 1), xb_);  // chunk 1: stored at the end of chunk 0
  __syncthreads();

  // Steady state, branch-free and copy-free:
  //  * the next chunk's activation loads and the next group's weight loads are issued unconditionally
  //    (clamped to the last valid chunk / slice), so the compiler counts outstanding loads exactly;
  //  * two weight register sets ping-pong (group g computes from one while the loads of group g+1 land
  //    in the other), unrolled so neither is ever copied — a register copy of an in-flight load forces
  //    s_waitcnt vmcnt(0) and exposed the full HBM latency once per group.
  // With one group per chunk the chunk loop is unrolled by two; an odd chunk count runs one dummy
  // chunk whose weights are masked to zero (its activations are the last real chunk: finite).
  const int s_last = s_beg + nch * BG_CK - 1;
  bf16x8 wb_[U][NTW];
  // pf: prefetch distance in groups (1 for the ping-pong, D-1 for the register ring)
  auto run_group = [&](int c, int h, bool valid, bf16x8 (&cur)[U][NTW], bf16x8 (&nxt)[U][NTW], int pf) {
    const int buf = c % XS;
    const int sn = s_beg + c * BG_CK + (h + pf) * U;  // first slice of the group being prefetched
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int t = 0; t < NTW; ++t) nxt[u][t] = load_w(min(sn + u, s_last), t);
    __builtin_amdgcn_sched_barrier(0);  // issue the prefetch before this group's MFMAs, not after
    const uint32_t keep = valid ? 0xffffffffu : 0u;
    // LDS fragments double-buffered across slices: slice u+1's NB ds_reads are issued before slice u's
    // MFMAs, so every MFMA finds its operand landed.  Left to itself the scheduler minimised registers
    // and paired each MFMA with its own ds_read (2 reads in flight, an LDS round trip exposed every
    // second MFMA at one wave per SIMD).
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    if constexpr (NB >= 16) {
      // 256 rows: a P-deep ring over the group's (slice, row block) fragment sequence instead of a whole
      // second slice of fragments (2 x 16 fragments do not fit beside the 256-row accumulators)
      constexpr int NF = U * NBW, P = W == 16 ? 2 : 4;
      bf16x8 q[P];
#pragma unroll
      for (int i = 0; i < P; ++i) q[i] = frag(buf, h * U + i / NBW, b0 + i % NBW);
      bf16x8 w[NTW];
#pragma unroll
      for (int i = 0; i < NF; ++i) {
        const int u = i / NBW, b = i % NBW;
        if (b == 0) {
#pragma unroll
          for (int t = 0; t < NTW; ++t) w[t] = __builtin_bit_cast(bf16x8, __builtin_bit_cast(u32x4, cur[u][t]) & keep);
        }
        const bf16x8 x = q[i % P];
        if (i + P < NF) q[i % P] = frag(buf, h * U + (i + P) / NBW, b0 + (i + P) % NBW);
#pragma unroll
        for (int t = 0; t < NTW; ++t) acc[t][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[t], x, acc[t][b], 0, 0, 0);
      }
    } else {
      bf16x8 xf[2][NBW];
#pragma unroll
      for (int b = 0; b < NBW; ++b) xf[0][b] = frag(buf, h * U, b0 + b);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (u + 1 < U) {
#pragma unroll
          for (int b = 0; b < NBW; ++b) xf[(u + 1) & 1][b] = frag(buf, h * U + u + 1, b0 + b);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int t = 0; t < NTW; ++t) {
          const bf16x8 w = __builtin_bit_cast(bf16x8, __builtin_bit_cast(u32x4, cur[u][t]) & keep);
#pragma unroll
          for (int b = 0; b < NBW; ++b)
            acc[t][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w, xf[u & 1][b], acc[t][b], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };
  // xa_/xb_: activation staging registers.  XS = 2: chunk c loads chunk c+1 into xa_ and stores it at
  // its end.  XS = 3: chunk c loads chunk c+2 into one set and stores the other (chunk c+1, loaded one
  // chunk earlier); the sets alternate, so the chunk loop runs unrolled by 2 (or D) and never copies.
  auto run_chunk = [&](int c, bool valid, bf16x8 (&A)[U][NTW], bf16x8 (&B)[U][NTW], int pf, bf16x8 (&xl)[FPW],
                       bf16x8 (&xw)[FPW]) {
    stage_load(min(c + XS - 1, nch - 1), xl);
    // pin the activation loads ahead of the weight prefetch: issued later, they would be the youngest
    // loads at the staging write and force a vmcnt(0) that drains the weight prefetch too
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (NGRP == 1) {
      run_group(c, 0, valid, A, B, pf);
    } else {
#pragma unroll
      for (int h = 0; h < NGRP; h += 2) {
        run_group(c, h, valid, A, B, 1);
        run_group(c, h + 1, valid, B, A, 1);
      }
    }
    // stage chunk c+1 (XS = 2: just loaded into xl; XS = 3: loaded one chunk ago into xw); the final
    // (clamped, redundant) stages add nothing to the sum of squares
    if constexpr (XS == 2) stage_store((c + 1) % XS, xl, (valid && c + 1 < nch) ? 1.f : 0.f);
    else stage_store((c + 1) % XS, xw, (valid && c + 1 < nch) ? 1.f : 0.f);
    __syncthreads();
  };
  static_assert(NGRP == 1 || NGRP % 2 == 0, "weight prefetch groups per chunk");
  static_assert(D == 2 || NGRP == 1, "the deep register ring needs one group per chunk");
  static_assert(XS == 2 || NGRP == 1, "three activation stages need one group per chunk");
  if constexpr (NGRP % 2 == 0) {
    for (int c = 0; c < nch; ++c) run_chunk(c, true, wa, wb_, 1, xa_, xb_);
  } else if constexpr (AR) {
    // D-deep register rings for BOTH operands.  vmcnt retires loads in issue order, so with only the
    // weights ring-buffered the per-chunk wait for the next chunk's activations (issued one chunk ahead)
    // also drained every older weight prefetch and the effective prefetch depth fell back to ~1 chunk:
    // one HBM round trip per chunk.  Here chunk c issues chunk c+D-1's activations and then its weights,
    // computes chunk c and waits only for chunk c+1's activations, which are older than every weight
    // load still in flight; the LDS stage stays double-buffered (XS = 2).
    static_assert(XS == 2 && NGRP == 1, "activation ring: two LDS stages, one weight group per chunk");
    bf16x8 ring[D][U][NTW];
    bf16x8 xring[D][FPW];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int t = 0; t < NTW; ++t) ring[0][u][t] = wa[u][t];
#pragma unroll
    for (int j = 1; j < D - 1; ++j) {  // chunks 1 .. D-2, activations before weights (issue = wait order)
      stage_load(min(j, nch - 1), xring[j]);
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int t = 0; t < NTW; ++t) ring[j][u][t] = load_w(min(s_beg + j * U + u, s_last), t);
    }
    for (int c = 0; c < nch; c += D) {
#pragma unroll
      for (int j = 0; j < D; ++j) {
        const int cc = c + j;
        const bool valid = cc < nch;
        stage_load(min(cc + D - 1, nch - 1), xring[(j + D - 1) % D]);
        __builtin_amdgcn_sched_barrier(0);
        run_group(cc, 0, valid, ring[j], ring[(j + D - 1) % D], D - 1);
        stage_store((cc + 1) % XS, xring[(j + 1) % D], (valid && cc + 1 < nch) ? 1.f : 0.f);
        __syncthreads();
      }
    }
  } else if constexpr (D == 2) {
    for (int c = 0; c < nch; c += 2) {
      run_chunk(c, true, wa, wb_, 1, xa_, xb_);
      run_chunk(c + 1, c + 1 < nch, wb_, wa, 1, xb_, xa_);
    }
  } else {
    // D-deep register ring (narrow outputs: few waves per CU, so each wave keeps D-1 groups of weight
    // loads in flight): chunk c computes ring[c % D] and prefetches chunk c + D - 1 into the set that
    // chunk c - 1 just finished; the loop is unrolled by D so every ring index is static.
    static_assert(D % 2 == 0, "ring depth must keep the activation register sets alternating");
    bf16x8 ring[D][U][NTW];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int t = 0; t < NTW; ++t) ring[0][u][t] = wa[u][t];
#pragma unroll
    for (int j = 1; j < D - 1; ++j)
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int t = 0; t < NTW; ++t) ring[j][u][t] = load_w(min(s_beg + j * U + u, s_last), t);
    for (int c = 0; c < nch; c += D) {
#pragma unroll
      for (int j = 0; j < D; ++j) {
        if (j % 2 == 0) run_chunk(c + j, c + j < nch, ring[j], ring[(j + D - 1) % D], D - 1, xa_, xb_);
        else run_chunk(c + j, c + j < nch, ring[j], ring[(j + D - 1) % D], D - 1, xb_, xa_);
      }
    }
  }

  // ---- per-row sum of squares of this workgroup's k-range (NORM): the PPR lanes of a row, then LDS atomics
  if constexpr (NORM) {
#pragma unroll
    for (int i = 0; i < FPW; ++i) {
      float x = ssq[i];
#pragma unroll
      for (int o = 1; o < PPR; o <<= 1) x += __shfl_xor(x, o, 64);
      if (lane % PPR == 0) atomicAdd(&s_ss[RPI * (wave + W * i) + lane / PPR], x);
    }
  }
  // the staging buffer becomes the epilogue buffer: red[unit][lane], unit = (wn*NTW + t)*NB + b0 + b
  f32x4* red = reinterpret_cast<f32x4*>(&xs[0][0][0]);
  auto unit = [&](int t, int b) { return (wn * NTW + t) * NB + b0 + b; };
  if (bg.ksplit == 1) {
#pragma unroll
    for (int t = 0; t < NTW; ++t)
#pragma unroll
      for (int b = 0; b < NBW; ++b) red[unit(t, b) * 64 + lane] = acc[t][b];
    __syncthreads();
    if constexpr (NORM) {
      if (threadIdx.x < NB * 16) s_inv[threadIdx.x] = rms_inv(s_ss[threadIdx.x], a.K, a.eps);
      __syncthreads();
    }
  } else {
    const size_t pb = (size_t)blk * bg.ksplit;
    const __amdgpu_buffer_rsrc_t mine_r = slab_rsrc(bg.part + (pb + kc) * (size_t)UNITS * 256);
#pragma unroll
    for (int t = 0; t < NTW; ++t)
#pragma unroll
      for (int b = 0; b < NBW; ++b) st_wt(mine_r, (unit(t, b) * 64 + lane) * 16, acc[t][b]);
    if constexpr (NORM) {
      __syncthreads();  // s_ss complete
      if (threadIdx.x < NB * 16)
        __hip_atomic_store(bg.part_ss + (pb + kc) * (NB * 16) + threadIdx.x, s_ss[threadIdx.x], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
    // every storing wave drains, one lane takes a ticket; the last arriver of the row block reduces
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)
      s_ticket = __hip_atomic_fetch_add(bg.counters + blk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (s_ticket != unsigned(bg.ksplit - 1)) return;
    // sum the k-range partials, RB ranges x NTW*NB units of loads in flight per round trip (RB x NTW*NB
    // f32x4 registers: 2 ranges at 8 units keeps the 128-row variants inside 128 VGPRs)
    constexpr int RB = (NTW * NBW >= 16 || W == 16) ? 1 : (NTW * NBW >= 8 ? 2 : 4);
    const __amdgpu_buffer_rsrc_t base_r = slab_rsrc(bg.part + pb * (size_t)UNITS * 256);
    f32x4 sum[NTW][NBW];
#pragma unroll
    for (int t = 0; t < NTW; ++t)
#pragma unroll
      for (int b = 0; b < NBW; ++b) sum[t][b] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int k0 = 0; k0 < bg.ksplit; k0 += RB) {
      // every load issued unconditionally (a clamped range index; the surplus weighted 0): a select between a
      // load and a constant made hipcc branch around each load and wait for it alone
      f32x4 l[RB][NTW][NBW];
#pragma unroll
      for (int j = 0; j < RB; ++j)
#pragma unroll
        for (int t = 0; t < NTW; ++t)
#pragma unroll
          for (int b = 0; b < NBW; ++b)
            l[j][t][b] = ld_wt(base_r, min(k0 + j, bg.ksplit - 1) * (UNITS * 1024) + (unit(t, b) * 64 + lane) * 16);
#pragma unroll
      for (int j = 0; j < RB; ++j) {
        const float wj = (k0 + j < bg.ksplit) ? 1.f : 0.f;
#pragma unroll
        for (int t = 0; t < NTW; ++t)
#pragma unroll
          for (int b = 0; b < NBW; ++b) sum[t][b] += wj * l[j][t][b];
      }
    }
#pragma unroll
    for (int t = 0; t < NTW; ++t)
#pragma unroll
      for (int b = 0; b < NBW; ++b) red[unit(t, b) * 64 + lane] = sum[t][b];
    if constexpr (NORM) {
      if (threadIdx.x < NB * 16) {
        float x = 0.f;
        for (int k = 0; k < bg.ksplit; ++k)
          x += __hip_atomic_load(bg.part_ss + (pb + k) * (NB * 16) + threadIdx.x, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
        s_inv[threadIdx.x] = rms_inv(x, a.K, a.eps);
      }
    }
    if (threadIdx.x == 0) bg.counters[blk] = 0u;  // ready for the next launch (launch-ordered)
    __syncthreads();
  }

  // ---- fused epilogue: each wave finishes its own tiles
#pragma unroll
  for (int t = 0; t < NTW; ++t) {
    if (gt[t] >= ntiles) continue;
#pragma unroll
    for (int b = 0; b < NBW; ++b) {
      const int ub = unit(t, b) * 64;
      const int m = (b0 + b) * 16 + (lane & 15);
      const EpiIn e = epi_load_at<EPI>(a, gt[t], m, lane);
      epi_store<EPI>(a, gt[t], m, lane, e, [&](int off) {
        f32x4 v = red[ub + lane + off];
        if constexpr (NORM) v *= s_inv[(b0 + b) * 16 + ((lane + off) & 15)];
        return v;
      });
    }
  }
}

struct BgPlan {
  int nb, ntw, w, ck, nblk, ksplit, kspl;
  int wm;  // wave rows along M (1, or 2 with NTW = 2: half the LDS fragment reads per MFMA)
  int d;  // 128-row bodies: weight register-ring depth (0 = the default ping-pong / 4-deep ring)
  size_t part_floats, ss_floats;
};

// Launch shape (profiles/bgemm_sweep.md, llama3.1:8b decode shapes at M = 32 / 64):
//  * NTW = 2 tiles per wave when the grid has >= 512 row blocks anyway (LM head): halves the LDS
//    fragment reads per weight byte;
//  * no k-split once >= 128 row blocks exist (gate/up, LM head): the fp32 partials + combine cost more
//    than the idle CUs;
//  * otherwise ceil(target / row blocks) k-ranges, target 128 workgroups for K <= 4096 and 256 for longer
//    K (down projection), at most 8.
// (Round 1-2's A/B knobs of this plan -- workgroup target, waves, chunk, ring depth, wave rows -- are fixed at the
// measured defaults; the alternatives are in profiles/bgemm_sweep.md and profiles/bgemm_r1.md.)
static BgPlan bgemm_plan(int N, int K, int M, int ntw_req) {
  constexpr int ksmax = 8;
  BgPlan p{};
  p.wm = 1;
  p.nb = M <= 32 ? 2 : (M <= 64 ? 4 : (M <= 128 ? 8 : 16));
  const int rows1 = 16 * BG_WAVES;
  p.ntw = p.nb >= 8 ? 1 : (ntw_req > 0 ? ntw_req : ((N + rows1 - 1) / rows1 >= 512 ? 2 : 1));
  // the 4-wave and 16-slice-chunk variants exist for NTW = 1 only; 4-wave workgroups (64-row blocks)
  // measured faster on N <= 6144 (O / QKV / down projections at M = 64: 23.1 vs 25.6, 27.0 vs 30.0,
  // 41.1 vs 46.5 us; profiles/bgemm_sweep.md)
  const bool narrow = N <= 6144 && p.ntw == 1;
  p.w = narrow ? 4 : BG_WAVES;
  if (p.nb == 16) {
    // 256 rows: 8 waves x 1 tile, 4-slice chunks, 128 KiB of stages (4 waves x 2 tiles at one wave per SIMD
    // measured 10-20 % slower on every shape, profiles/bgemm_r1.md)
    p.w = 8;
    p.ck = 4;
  } else if (p.nb == 8) {
    // 128 rows: 4-slice chunks keep the double-buffered stage at 64 KiB (2 workgroups per CU); activation + weight
    // register rings, depth 4, on the 4-wave (narrow-output) bodies (depths 6 and 8, and the ring on the 8-wave
    // bodies, measured slower, profiles/bgemm_r1.md)
    p.ck = 4;
    p.d = p.w == 4 ? 4 : 0;
  } else {
    // 64 rows: the mid-width gate/up projection measured faster with 4-slice chunks too (43.8 vs 47.0 us)
    const int nblk8 = (N + 16 * BG_WAVES - 1) / (16 * BG_WAVES);
    const bool mid = p.nb == 4 && nblk8 >= 128 && nblk8 < 512;
    p.ck = p.w == 4 ? 4  // the 4-wave variants run the deep register ring: one prefetch group per chunk
           : (p.ntw == 1 && mid) ? 4 : BG_CK;
  }
  const int rows = 16 * (p.w / p.wm) * p.ntw;
  p.nblk = (N + rows - 1) / rows;
  const int nchunk = (K / 32) / p.ck;
  const int target = K > 4096 ? 256 : 128;
  int ks = p.nblk >= 128 ? 1 : std::max(1, std::min(std::min(nchunk, ksmax), (target + p.nblk - 1) / p.nblk));
  const int cpw = (nchunk + ks - 1) / ks;
  ks = (nchunk + cpw - 1) / cpw;
  p.ksplit = ks;
  p.kspl = cpw * p.ck;
  if (ks > 1) {
    p.part_floats = (size_t)p.nblk * ks * (p.w / p.wm) * p.ntw * p.nb * 64 * 4;
    p.ss_floats = (size_t)p.nblk * ks * p.nb * 16;
  }
  return p;
}

// GEMM workspace layout: [batched-path tickets, 64 KiB][wide-path counters, 16 KiB][split-K slabs ...].  Both
// counter regions must read zero at rest (each path resets its own); the slab area is shared scratch.
constexpr size_t BG_COUNTER_BYTES = 64 * 1024;
constexpr size_t WG_COUNTER_BYTES = 16 * 1024;
constexpr size_t GEMM_SLAB_OFFSET = BG_COUNTER_BYTES + WG_COUNTER_BYTES;

static size_t bgemm_ws_bytes(const BgPlan& p) {
  return GEMM_SLAB_OFFSET + (p.part_floats + p.ss_floats) * sizeof(float);
}

template <int NB, int NTW, int W, int CK, int EPI, bool NORM, int DD, int WM>
static hipError_t bg_launch(const GemmArgs& a, const BgArgs& b, int nblk, hipStream_t st) {
  // slices per weight prefetch group (2 on the 256-row fused-norm bodies: with 4 they spill; two groups
  // per chunk also let one activation staging register set serve every chunk)
  constexpr int U = (NB == 16 && (NORM || W == 16)) ? 2 : 4;
  // register sets of weight prefetch: 4-wave workgroups (narrow outputs, 2 waves per SIMD, 256-VGPR
  // budget) keep 3 groups in flight, the rest ping-pong between 2 (so do the fused-norm 4-wave bodies,
  // whose 8 staged fragments per wave leave no room for the deeper ring).  DD > 0 (128-row bodies): a
  // DD-deep ring with the register budget of one workgroup per CU (4 waves: 512 VGPRs, 8 waves: 256),
  // so DD-1 chunks of weights stay in flight per wave across the per-chunk barrier.
  constexpr int D = DD > 0 ? DD : ((W == 4 && CK == U && !NORM && NB < 16) ? 4 : 2);
  // three activation stages for the 4-wave bodies (one workgroup per CU on the narrow grids anyway)
  constexpr int XS = (W == 4 && CK == U && NB < 16) ? 3 : 2;  // 256-row stages are 64 KiB each
  // (the 128-row 8-wave body needs 256 VGPRs for its double-buffered LDS fragments: 1 workgroup per CU)
  constexpr int LB = W == 16 ? 4
                     : (DD > 0 || NB >= 16) ? (W == 4 ? 1 : 2)
                     : ((W == 8 && NTW == 1 && NB < 8 && CK * NB <= 32) ? 4 : 2);
  constexpr bool AR = DD > 0;  // explicit depth: the activation + weight register rings
  hipLaunchKernelGGL((bgemm_kernel<NB, NTW, W, CK, U, D, AR ? 2 : XS, LB, AR, EPI, NORM, WM>), dim3(nblk * b.ksplit),
                     dim3(W * 64), 0, st, a, b);
  return hipGetLastError();
}

template <int NB, int NTW, int W, int CK, bool NORM, int DD = 0, int WM = 1>
static hipError_t bg_launch_e(int epi, const GemmArgs& a, const BgArgs& b, int nblk, hipStream_t st) {
  switch (epi) {
    case EPI_BF16: return bg_launch<NB, NTW, W, CK, EPI_BF16, NORM, DD, WM>(a, b, nblk, st);
    case EPI_RESID: return bg_launch<NB, NTW, W, CK, EPI_RESID, NORM, DD, WM>(a, b, nblk, st);
    case EPI_F32: return bg_launch<NB, NTW, W, CK, EPI_F32, NORM, DD, WM>(a, b, nblk, st);
    case EPI_SILU: return bg_launch<NB, NTW, W, CK, EPI_SILU, NORM, DD, WM>(a, b, nblk, st);
    case EPI_GELU: return bg_launch<NB, NTW, W, CK, EPI_GELU, NORM, DD, WM>(a, b, nblk, st);
    case EPI_QKV_ROPE: return bg_launch<NB, NTW, W, CK, EPI_QKV_ROPE, NORM, DD, WM>(a, b, nblk, st);
    default: return hipErrorInvalidValue;
  }
}

template <int NB, bool NORM>
static hipError_t bg_launch_shape(int epi, const BgPlan& p, const GemmArgs& a, const BgArgs& b, hipStream_t st) {
  if constexpr (NB == 16) {
    return bg_launch_e<16, 1, 8, 4, NORM>(epi, a, b, p.nblk, st);
  } else if constexpr (NB == 8) {
    // register rings for activations AND weights (AR) of depth p.d; not for the fused-norm bodies, whose
    // staging sums of squares make the rings spill (profiles/bgemm_r1.md)
    if constexpr (!NORM) {
      if (p.d == 4) return bg_launch_e<8, 1, 4, 4, NORM, 4>(epi, a, b, p.nblk, st);
    }
    if (p.w == 4) return bg_launch_e<8, 1, 4, 4, NORM>(epi, a, b, p.nblk, st);
    return bg_launch_e<8, 1, 8, 4, NORM>(epi, a, b, p.nblk, st);
  } else {
    if (p.ntw == 2) return bg_launch_e<NB, 2, 8, 8, NORM>(epi, a, b, p.nblk, st);
    if (p.w == 4) return bg_launch_e<NB, 1, 4, 4, NORM>(epi, a, b, p.nblk, st);
    if (p.ck == 4) return bg_launch_e<NB, 1, 8, 4, NORM>(epi, a, b, p.nblk, st);
    return bg_launch_e<NB, 1, 8, 8, NORM>(epi, a, b, p.nblk, st);
  }
}

static int bgemm_dispatch(const GemmArgs& a, int epi, bool norm, const BgPlan& p, void* ws, hipStream_t st) {
  BgArgs b{};
  b.ksplit = p.ksplit;
  b.kspl = p.kspl;
  b.counters = reinterpret_cast<unsigned*>(ws);
  b.part = reinterpret_cast<float*>(reinterpret_cast<char*>(ws) + GEMM_SLAB_OFFSET);
  b.part_ss = b.part + p.part_floats;
  hipError_t e;
  if (p.nb == 2) e = norm ? bg_launch_shape<2, true>(epi, p, a, b, st) : bg_launch_shape<2, false>(epi, p, a, b, st);
  else if (p.nb == 4) e = norm ? bg_launch_shape<4, true>(epi, p, a, b, st) : bg_launch_shape<4, false>(epi, p, a, b, st);
  else if (p.nb == 8) e = norm ? bg_launch_shape<8, true>(epi, p, a, b, st) : bg_launch_shape<8, false>(epi, p, a, b, st);
  else e = norm ? bg_launch_shape<16, true>(epi, p, a, b, st) : bg_launch_shape<16, false>(epi, p, a, b, st);
  return int(e);
}

// Batched path is used for M > 16 when K is a multiple of 256.
static int bgemm_min_m() { return 16; }
static int bgemm_ntw() { return 0; }

// M <= 32 on narrow outputs with short K (N < 8192, K <= 4096: O / QKV projections) stays on the skinny
// kernel, which measured faster there (its whole grid streams from the first cycle; no staging, no combine).
static bool bgemm_eligible(int N, int K, int M) {
  return M > bgemm_min_m() && M <= 256 && K % (32 * BG_CK) == 0 && (M > 32 || N >= 8192 || K > 4096);
}

// wgemm.hip: the wide-batch (64 < M <= 256) kernel; its split-K slabs live after the batched path's counters
CAIN_API int cain_wgemm_eligible(int N, int K, int M);
CAIN_API long long cain_wgemm_ws_bytes(int N, int K, int M);
int wgemm_dispatch(const GemmArgs& a, int epi, bool norm, void* ws, long long ws_bytes, hipStream_t st);

// Skinny split-K slabs: [tiles][ks][64] f32x4 partials + [tiles][ks][16] row sums of squares, after the counters
static size_t skinny_split_ws_bytes(int N, int ks) {
  return GEMM_SLAB_OFFSET + (size_t)(N / 16) * ks * (256 + 16) * sizeof(float);
}

// Workspace the batched paths need for a GEMM of this shape (0 when the unsplit skinny kernel runs it).
CAIN_API long long cain_gemm_ws_bytes(int N, int K, int M) {
  if (cain_wgemm_eligible(N, K, M)) return (long long)BG_COUNTER_BYTES + cain_wgemm_ws_bytes(N, K, M);
  if (!bgemm_eligible(N, K, M)) {
    const int ks = (M <= 16) ? skinny_split(N, K, M) : 1;
    return ks > 1 ? (long long)skinny_split_ws_bytes(N, ks) : 0;
  }
  return (long long)bgemm_ws_bytes(bgemm_plan(N, K, M, bgemm_ntw()));
}

// Chunk maxima of the next few-row fp32-logits GEMM (the LM head at <= 16 rows): set by the runtime right before
// that call, consumed (and cleared) by it when it runs on the plain skinny kernel; cain_gemm_cmax_take() then
// reports that the buffer was written, so the runtime can hand it to the chunk-max sampler.
// (thread-local: engines of different models may run forwards on different threads of one process)
CAIN_API int cain_wgemm_plan(int N, int K, int M);
static thread_local float* g_next_cmax = nullptr;
static thread_local int g_cmax_used = 0;
CAIN_API void cain_gemm_set_cmax(float* cmax) { g_next_cmax = cmax, g_cmax_used = 0; }
CAIN_API int cain_gemm_cmax_take() {
  const int u = g_cmax_used;
  g_next_cmax = nullptr, g_cmax_used = 0;
  return u;
}
// The weight-format kernels' side (gemm_w8 / gemm_w4 / gemm_q4 at few rows): the pending buffer for an fp32-logits
// GEMM of N columns, now marked written (null: none pending or N not whole chunks).
CAIN_API float* cain_gemm_cmax_claim(int N) {
  if (!g_next_cmax || N % 16) return nullptr;
  float* p = g_next_cmax;
  g_next_cmax = nullptr, g_cmax_used = 1;
  return p;
}

// Entry used by the runtime and the bindings.  norm != 0 selects the fused RMSNorm (gain pre-folded into Wp).
CAIN_API int cain_skinny_gemm_ex(const void* Wp, const void* X, int ldx, int K, int N, int M, void* Y, int ldy,
                                 const float* bias, int norm, float eps, const int* slot, const int* pos,
                                 const float* cos_t, const float* sin_t, void* kc, void* vtc, int H, int Hkv, int hd,
                                 int T_max, int epi, int waves, hipStream_t st) {
  const int kv8 = (epi & EPI_KV_FP8) ? 1 : 0;
  epi &= EPI_MASK;
  GemmArgs a{};
  a.Wp = reinterpret_cast<const bf16x8*>(Wp);
  a.X = reinterpret_cast<const __bf16*>(X);
  a.ldx = ldx, a.K = K, a.N = N, a.M = M, a.Y = Y, a.ldy = ldy, a.bias = bias;
  a.eps = eps;
  a.slot = slot, a.pos = pos, a.cos_t = cos_t, a.sin_t = sin_t;
  a.kc = reinterpret_cast<__bf16*>(kc), a.vtc = reinterpret_cast<__bf16*>(vtc);
  a.H = H, a.Hkv = Hkv, a.hd = hd, a.T_max = T_max, a.kv8 = kv8;
  if (epi == EPI_QKV_ROPE && (hd % 16 || (hd / 2) % 8)) return -1;
  if (epi == EPI_F32 && g_next_cmax && M <= 16 && N % 16 == 0) {
    a.cmax = g_next_cmax, a.ld_cm = N / 16;
    g_next_cmax = nullptr, g_cmax_used = 1;
  }
  return gemm_dispatch(a, epi, norm != 0, waves, st);
}

// Full entry: the wide kernel (wgemm.hip) for 64 < M <= 256, the batched path for 16 < M <= 64, when a
// workspace of cain_gemm_ws_bytes() (zeroed once) is given; the skinny kernel otherwise.
CAIN_API int cain_gemm(const void* Wp, const void* X, int ldx, int K, int N, int M, void* Y, int ldy,
                       const float* bias, int norm, float eps, const int* slot, const int* pos,
                       const float* cos_t, const float* sin_t, void* kc, void* vtc, int H, int Hkv, int hd, int T_max,
                       void* ws, long long ws_bytes, int epi_flags, int waves, hipStream_t st) {
  const int epi = epi_flags & EPI_MASK, kv8 = (epi_flags & EPI_KV_FP8) ? 1 : 0;
  if (ws && cain_wgemm_eligible(N, K, M) && ws_bytes >= (long long)BG_COUNTER_BYTES) {
    if (epi == EPI_QKV_ROPE && (hd % 16 || (hd / 2) % 8)) return -1;
    GemmArgs a{};
    a.Wp = reinterpret_cast<const bf16x8*>(Wp);
    a.X = reinterpret_cast<const __bf16*>(X);
    a.ldx = ldx, a.K = K, a.N = N, a.M = M, a.Y = Y, a.ldy = ldy, a.bias = bias;
    a.eps = eps;
    a.slot = slot, a.pos = pos, a.cos_t = cos_t, a.sin_t = sin_t;
    a.kc = reinterpret_cast<__bf16*>(kc), a.vtc = reinterpret_cast<__bf16*>(vtc);
    a.H = H, a.Hkv = Hkv, a.hd = hd, a.T_max = T_max, a.kv8 = kv8;
    // the wide LM head writes the chunk maxima in its unsplit epilogue (the plan's split count is 1 there)
    const bool cm = epi == EPI_F32 && g_next_cmax && N % 16 == 0 && cain_wgemm_plan(N, K, M) / 64 == 1;
    if (cm) a.cmax = g_next_cmax, a.ld_cm = N / 16;
    // the batched path's counters (first BG_COUNTER_BYTES) must stay zero: the slabs go after them
    const int rc = wgemm_dispatch(a, epi, norm != 0, static_cast<char*>(ws) + BG_COUNTER_BYTES,
                                  ws_bytes - (long long)BG_COUNTER_BYTES, st);
    if (rc >= 0) {
      if (cm) g_next_cmax = nullptr, g_cmax_used = 1;
      return rc;
    }
  }
  if (ws && bgemm_eligible(N, K, M) && K % 32 == 0 && N % 16 == 0) {
    const BgPlan p = bgemm_plan(N, K, M, bgemm_ntw());
    if ((long long)bgemm_ws_bytes(p) <= ws_bytes && p.nblk * 4 <= (int)BG_COUNTER_BYTES) {
      GemmArgs a{};
      a.Wp = reinterpret_cast<const bf16x8*>(Wp);
      a.X = reinterpret_cast<const __bf16*>(X);
      a.ldx = ldx, a.K = K, a.N = N, a.M = M, a.Y = Y, a.ldy = ldy, a.bias = bias;
      a.eps = eps;
      a.slot = slot, a.pos = pos, a.cos_t = cos_t, a.sin_t = sin_t;
      a.kc = reinterpret_cast<__bf16*>(kc), a.vtc = reinterpret_cast<__bf16*>(vtc);
      a.H = H, a.Hkv = Hkv, a.hd = hd, a.T_max = T_max, a.kv8 = kv8;
      if (epi == EPI_QKV_ROPE && (hd % 16 || (hd / 2) % 8)) return -1;
      return bgemm_dispatch(a, epi, norm != 0, p, ws, st);
    }
  }
  if (ws && M <= 16 && K % 32 == 0 && N % 16 == 0) {
    const int ks = skinny_split(N, K, M);
    if (ks > 1 && (long long)skinny_split_ws_bytes(N, ks) <= ws_bytes && (N / 16) * 4 <= (int)BG_COUNTER_BYTES) {
      if (epi == EPI_QKV_ROPE && (hd % 16 || (hd / 2) % 8)) return -1;
      GemmArgs a{};
      a.Wp = reinterpret_cast<const bf16x8*>(Wp);
      a.X = reinterpret_cast<const __bf16*>(X);
      a.ldx = ldx, a.K = K, a.N = N, a.M = M, a.Y = Y, a.ldy = ldy, a.bias = bias;
      a.eps = eps;
      a.slot = slot, a.pos = pos, a.cos_t = cos_t, a.sin_t = sin_t;
      a.kc = reinterpret_cast<__bf16*>(kc), a.vtc = reinterpret_cast<__bf16*>(vtc);
      a.H = H, a.Hkv = Hkv, a.hd = hd, a.T_max = T_max, a.kv8 = kv8;
      SkArgs sk{};
      sk.ks = ks;
      sk.counters = reinterpret_cast<unsigned*>(ws);  // the batched path's tickets (both reset their own)
      sk.part = reinterpret_cast<float*>(static_cast<char*>(ws) + GEMM_SLAB_OFFSET);
      sk.part_ss = sk.part + (size_t)(N / 16) * ks * 256;
      return gemm_dispatch(a, epi, norm != 0, waves, st, &sk);
    }
  }
  return cain_skinny_gemm_ex(Wp, X, ldx, K, N, M, Y, ldy, bias, norm, eps, slot, pos, cos_t, sin_t, kc, vtc, H, Hkv,
                             hd, T_max, epi_flags, waves, st);
}

