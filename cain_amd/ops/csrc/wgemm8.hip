// W8A8 wide-batch GEMM (fp8 e4m3 weights x fp8 e4m3 activations, fp32 accumulate) for 16 < M <= 256 rows, gfx950.
//
//   Y[m][n] = epilogue( xs[m] * ws[n] * sum_k X8[m][k] * W8[n][k] )
//
// xs: per-row activation scale (amax / 448, times the RMSNorm factor rsqrt(mean(x^2) + eps) for the normed
// projections), written by quant_rows_kernel from the bf16 rows; ws: per-output-row weight scale
// (models/weights.py quantize_fp8_rows).  The reference runs its models 4-bit quantised inside Ollama
// (BASELINE.md); this is the MI355X 8-bit counterpart for the trial-batched decode step, reported
// as its own configuration (bf16 stays the headline).
//
// Same LDS-DMA ring, loader waves, split-K slabs and epilogues as the bf16 kernel (wgemm.hip), and the SAME
// LDS images: a ring stage is still one 128-B line per X row and 8 x 2 KiB of W, but it now spans 128 k, and
// its two 16-B fragment reads per operand (the bf16 kernel's two 32-k slices) are concatenated into the 32-B
// operands of one block-scaled v_mfma_scale_f32_16x16x128_f8f6f4 (unit e8m0 scales): per k twice the MFMA rate
// of bf16 and half the bytes through HBM, the per-CU load path and LDS.  A and B only need the same k order in
// their 32 bytes: lane (r, g) holds k = 64h + 16g + j (h = read 0/1, j < 16) of the stage in both -- W by its
// packing (pack_mfma_a_fp8_k128: [N/16][K/64][64 lanes][16 B]), X by the XOR-swizzled piece reads.
//
// FP4 = true is the W4A8 form for MXFP4 weights (the reference's 4-bit precision class at trial-batch widths):
// the SAME packed bytes as the few-row W4A16 kernel (models/weights.py pack_mxfp4: [N/16][K/128][64 lanes][16 B],
// lane (r, g) = row 16t + r, k = 128p + 32g + j at nibble j), which are exactly the fp4 A operand of the 16x16x128
// scaled MFMA (cbsz 4: 16 B per lane), and the block scales ([N/16][K/128][64] e8m0 bytes, one per lane = one
// 32-k block) go in as the MFMA's per-lane A scale.  A ring stage is 8 tiles x 1 KiB of W plus their 512 B of
// scales; X (fp8 rows) is read as pieces 2g, 2g + 1 of its 128-B line, the lane's 32 k.  Y = xs[m] * sum.
#include <algorithm>

#include "common.h"
#include "gemm_epi.h"
#include "wgemm_ring.h"

using namespace wg;

namespace {

constexpr int W8_BK = 128;  // k per ring stage (one 128-B X line per row, one scaled MFMA per tile pair)

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ i32x8 cat16(const i32x4& lo, const i32x4& hi) {
  return i32x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

}  // namespace

struct W8Scales {
  const float* xs;  // [M] per-row activation scale
  const float* ws;  // [N] per-output-row weight scale
};

// Scales of one lane's four outputs: rows n = 16 gt + 4 (lane >> 4) + i of W, activation row m (FP4: the weight
// scales were applied inside the MFMA).
template <bool FP4 = false>
__device__ __forceinline__ f32x4 w8_scaled(f32x4 v, const W8Scales& q, int gt, int m, int lane, int M) {
  const float x = q.xs[min(m, M - 1)];
  if constexpr (FP4) return v * x;
  const f32x4 w = *reinterpret_cast<const f32x4*>(q.ws + gt * 16 + (lane >> 4) * 4);
  return v * w * x;
}

// W bytes of one ring stage: fp8 8 tiles x 2 KiB; fp4 8 tiles x 1 KiB + 8 x 64 B of scales
template <int BM, bool FP4>
constexpr int w8_wbytes() { return FP4 ? WG_NT * 1024 + WG_NT * 64 : WgGeo<BM>::W_BYTES; }

template <int BM, int DX, int DW, int EPI, int NDMA, bool FP4 = false>
__global__ __launch_bounds__(64 * (8 + NDMA), (8 + NDMA) / 4) void wgemm8_kernel(const GemmArgs a, const WgArgs w,
                                                                                  const W8Scales q) {
  using G = WgGeo<BM>;
  constexpr int NX = DX + 1, NW = DW + 1;
  constexpr int NLOAD = NDMA ? NDMA : 8;
  constexpr int WPW = (FP4 ? WG_NT : 16) / NLOAD;  // W LDS-DMA pieces (1 KiB) per loader per stage
  // fp4: the stage's 512 scale bytes as two 256-B dword pieces, issued by loaders 0 and 1 (spw of them per wave)
  constexpr int XPW = (BM / 8) / NLOAD;
  constexpr int WB = w8_wbytes<BM, FP4>();
  static_assert(DW >= DX && DX >= 1, "W is issued no later than X of the same stage");
  static_assert(WPW * NLOAD == (FP4 ? WG_NT : 16) && XPW * NLOAD == BM / 8, "loader split");
  static_assert(!FP4 || NLOAD >= 2, "fp4 scale pieces: loaders 0 and 1");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool compute = wave < 8;
  const bool loader = NDMA ? !compute : true;
  const int lw = NDMA ? wave - 8 : wave;
  const int wm = wave % G::WM, wn = (wave / G::WM) % G::WN;
  const int KH = a.K >> 6, ntiles = a.N >> 4;  // 1-KiB W blocks (16 rows x 64 k) per tile
  const int nblk = (ntiles + WG_NT - 1) / WG_NT;

  int blk, kc;
  {
    wg_block_of(blockIdx.x, w.ks, nblk, w.xcd_blk, blk, kc);
  }
  const int tile0 = blk * WG_NT;
  const int st0 = kc * w.kst;
  const int nst = min(w.kst, (a.K >> 7) - st0);

  const char* wsrc[WPW];
#pragma unroll
  for (int j = 0; j < WPW; ++j) {
    if constexpr (FP4) {  // tile tn's 1-KiB block of 128 k per stage
      const int tn = lw * WPW + j;
      wsrc[j] = reinterpret_cast<const char*>(a.Wp) +
                ((size_t)min(tile0 + tn, ntiles - 1) * (KH >> 1) + (size_t)st0) * 1024 + lane * 16;
    } else {
      const int qq = lw * WPW + j, tn = qq >> 1, h = qq & 1;
      wsrc[j] = reinterpret_cast<const char*>(a.Wp) +
                ((size_t)min(tile0 + tn, ntiles - 1) * KH + (size_t)st0 * 2 + h) * 1024 + lane * 16;
    }
  }
  // fp4 scales: loader lw < 2 copies the 64 scale bytes of tiles 4 lw .. 4 lw + 3 (lane: tile 4 lw + lane / 16,
  // dword lane % 16)
  const char* ssrc = nullptr;
  const int spw = FP4 && loader && lw < 2 ? 1 : 0;
  if constexpr (FP4) {
    const int tn = 4 * max(min(lw, 1), 0) + (lane >> 4);
    ssrc = reinterpret_cast<const char*>(q.ws) + ((size_t)min(tile0 + tn, ntiles - 1) * (KH >> 1) + (size_t)st0) * 64 +
           (lane & 15) * 4;
  }
  const char* xsrc[XPW];
#pragma unroll
  for (int j = 0; j < XPW; ++j) {
    const int i = lw + NLOAD * j;
    const int r = 8 * i + (lane >> 3);
    const int p = (lane & 7) ^ ((r >> 1) & 7);
    xsrc[j] = reinterpret_cast<const char*>(a.X) + (size_t)min(r, a.M - 1) * a.ldx + (size_t)st0 * W8_BK + p * 16;
  }
  char* const xring = smem + NW * WB;
  auto issue_w = [&](int t) {
    char* base = smem + (t % NW) * WB;
#pragma unroll
    for (int j = 0; j < WPW; ++j) glds16(wsrc[j] + (size_t)t * (FP4 ? 1024 : 2048), base + (lw * WPW + j) * 1024, 1);
    if constexpr (FP4) {
      if (spw)
        __builtin_amdgcn_global_load_lds((gbl_void_t*)(ssrc + (size_t)t * 64),
                                         (lds_void_t*)(base + WG_NT * 1024 + lw * 256), 4, 0, 0);
    }
  };
  auto issue_x = [&](int t) {
    char* base = xring + (t % NX) * G::X_BYTES;
#pragma unroll
    for (int j = 0; j < XPW; ++j) glds16(xsrc[j] + (size_t)t * W8_BK, base + (lw + NLOAD * j) * 1024, 0);
  };
  auto younger_than = [&](int t) {
    int n = 0;
#pragma unroll
    for (int u = t - DX + 1; u < t; ++u) n += (WPW + spw) * (u + DW < nst) + XPW * (u + DX < nst);
    return n;
  };
  auto issue_step = [&](int t) {
    if (loader) {
      if (t + DW < nst) issue_w(t + DW);
      if (t + DX < nst) issue_x(t + DX);
    }
  };

  const int c = lane & 15, g = lane >> 4;
  int woff[G::TN];
#pragma unroll
  for (int tn = 0; tn < G::TN; ++tn) woff[tn] = (wn * G::TN + tn) * (FP4 ? 1024 : 2048) + lane * 16;
  // X pieces 4h + g: k = 64h + 16g + j, the fp8 B operand's own k order (measured, tools/w4a8_probe.py: byte 16h + j
  // of lane group g meets k 64h + 16g + j of A) -- the fp8 W packing uses the same order; the fp4 A operand holds
  // k = 32g + j at nibble j, which is pack_mxfp4's order
  int xoff[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) xoff[h] = c * 128 + (((4 * h + g) ^ (c >> 1)) << 4);
  const int xrow0 = wm * G::MB * 16 * 128;

  f32x4 acc[G::TN][G::MB];
#pragma unroll
  for (int tn = 0; tn < G::TN; ++tn)
#pragma unroll
    for (int mb = 0; mb < G::MB; ++mb) acc[tn][mb] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (loader) {
#pragma unroll
    for (int u = -DW; u < 0; ++u) {
      if (u + DW < nst) issue_w(u + DW);
      if (u + DX >= 0 && u + DX < nst) issue_x(u + DX);
    }
  }

  // one barrier per stage for every wave; after barrier t the loaders refill stage t - 1's slots (every wave's
  // reads of stage t - 1 completed before it: lgkmcnt(0) in ring_barrier)
  if (NDMA && !compute) {  // loader waves: their own loop, so the two roles' registers never overlap
    for (int t = 0; t < nst; ++t) {
      wait_vmcnt_rt(younger_than(t));
      ring_barrier();
      issue_step(t);
    }
  } else {
    for (int t = 0; t < nst; ++t) {
      if constexpr (!NDMA) wait_vmcnt_rt(younger_than(t));
      ring_barrier();
      if constexpr (!NDMA) issue_step(t);
      const char* wbase = smem + (t % NW) * WB;
      const char* xbase = xring + (t % NX) * G::X_BYTES + xrow0;
      i32x4 b0[G::MB], b1[G::MB], a0[G::TN], a1[G::TN];
      int sa[G::TN];
#pragma unroll
      for (int mb = 0; mb < G::MB; ++mb) {
        b0[mb] = *reinterpret_cast<const i32x4*>(xbase + mb * 2048 + xoff[0]);
        b1[mb] = *reinterpret_cast<const i32x4*>(xbase + mb * 2048 + xoff[1]);
      }
#pragma unroll
      for (int tn = 0; tn < G::TN; ++tn) {
        a0[tn] = *reinterpret_cast<const i32x4*>(wbase + woff[tn]);
        if constexpr (FP4)
          sa[tn] = *reinterpret_cast<const uint8_t*>(wbase + WG_NT * 1024 + (wn * G::TN + tn) * 64 + lane);
        else
          a1[tn] = *reinterpret_cast<const i32x4*>(wbase + 1024 + woff[tn]);
      }
#pragma unroll
      for (int tn = 0; tn < G::TN; ++tn) {
        if constexpr (FP4) {
          const i32x8 av = i32x8{a0[tn][0], a0[tn][1], a0[tn][2], a0[tn][3], 0, 0, 0, 0};  // 16 B of e2m1
#pragma unroll
          for (int mb = 0; mb < G::MB; ++mb)
            acc[tn][mb] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, cat16(b0[mb], b1[mb]), acc[tn][mb],
                                                                           4, 0, 0, sa[tn], 0, 127);
        } else {
          const i32x8 av = cat16(a0[tn], a1[tn]);
#pragma unroll
          for (int mb = 0; mb < G::MB; ++mb)
            acc[tn][mb] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, cat16(b0[mb], b1[mb]), acc[tn][mb],
                                                                           0, 0, 0, 127, 0, 127);
        }
      }
    }
  }
  ring_barrier();
  if (!compute) return;

  if (w.ks > 1) {
    // slabs in fp16 as the bf16 kernel's (wgemm.hip OPT 32), already scaled (the scales are linear, so the reduce
    // sums scaled partials): the raw e4m3 x e4m3 sums would overflow fp16
    const int n_units = nblk * WG_NT * G::RB;
#pragma unroll
    for (int tn = 0; tn < G::TN; ++tn)
#pragma unroll
      for (int mb = 0; mb < G::MB; ++mb) {
        const int gt = tile0 + wn * G::TN + tn;
        const int unit = gt * G::RB + wm * G::MB + mb;
        const int m = (wm * G::MB + mb) * 16 + c;
        const f32x4 v = gt < ntiles ? w8_scaled<FP4>(acc[tn][mb], q, gt, m, lane, a.M) : acc[tn][mb];
        f16x4 h;
#pragma unroll
        for (int i = 0; i < 4; ++i) h[i] = (_Float16)fminf(fmaxf(v[i], -65504.f), 65504.f);
        reinterpret_cast<f16x4*>(w.part)[((size_t)kc * n_units + unit) * 64 + lane] = h;
      }
    return;
  }
#pragma unroll
  for (int tn = 0; tn < G::TN; ++tn) {
    const int gt = tile0 + wn * G::TN + tn;
#pragma unroll
    for (int mb = 0; mb < G::MB; ++mb) {
      const int m = (wm * G::MB + mb) * 16 + c;
      f32x4 v = gt < ntiles ? w8_scaled<FP4>(acc[tn][mb], q, gt, m, lane, a.M) : acc[tn][mb];
      f32x4 pv;
#pragma unroll
      for (int i = 0; i < 4; ++i) pv[i] = __shfl_xor(v[i], 32, 64);
      if (gt < ntiles) {
        const EpiIn e = epi_load_at<EPI>(a, gt, m, lane);
        epi_store<EPI>(a, gt, m, lane, e, [&](int off) { return off ? pv : v; });
      }
    }
  }
}

// Split-K combine + fused epilogue: one wave per 16 x 16 output unit (the slabs hold scaled fp16 partials).  As
// wgemm.hip's reduce: the epilogue inputs and all KS slab pieces are issued before the first add (KS = 0: runtime
// count).
template <int BM, int EPI, int KS>
__global__ __launch_bounds__(256) void wgemm8_reduce_kernel(const GemmArgs a, const WgArgs w, const W8Scales q,
                                                            int n_units) {
  constexpr int RB = BM / 16;
  const int lane = threadIdx.x & 63;
  const int unit = wg_reduce_block(blockIdx.x, WG_NT * RB / 4, w.xcd_blk) * 4 + (threadIdx.x >> 6);
  if (unit >= n_units) return;
  const int gt = unit / RB, rb = unit - gt * RB;
  const int ntiles = a.N >> 4;
  const int m = rb * 16 + (lane & 15);
  const bool live = gt < ntiles;
  const EpiIn e = live ? epi_load_at<EPI>(a, gt, m, lane) : EpiIn{};
  const f16x4* src = reinterpret_cast<const f16x4*>(w.part) + (size_t)unit * 64 + lane;  // scaled fp16 partials
  auto widen = [](const f16x4& x) { return f32x4{(float)x[0], (float)x[1], (float)x[2], (float)x[3]}; };
  f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
  if constexpr (KS > 0) {
    f16x4 p[KS];
#pragma unroll
    for (int k = 0; k < KS; ++k) p[k] = src[(size_t)k * n_units * 64];
#pragma unroll
    for (int k = 0; k < KS; ++k) v += widen(p[k]);
  } else {
    for (int k = 0; k < w.ks; ++k) v += widen(src[(size_t)k * n_units * 64]);
  }
  f32x4 pv;
#pragma unroll
  for (int i = 0; i < 4; ++i) pv[i] = __shfl_xor(v[i], 32, 64);
  if (!live) return;
  epi_store<EPI>(a, gt, m, lane, e, [&](int off) { return off ? pv : v; });
}

// Per-row fp8 quantisation of bf16 activations: x8 = e4m3(x / s), s = amax / 448; xs = s * (norm ?
// rsqrt(mean(x^2) + eps) : 1) -- the RMSNorm of the bf16 rows folded into the row scale (gain in W).
// One 256-thread workgroup per row; the row stays in registers between the statistics and the store (one read
// of the row: a second pass over it cost a second L2 round trip in a launch this short).  K % 8 == 0,
// K <= QR_MAXK.
constexpr int QR_THREADS = 256, QR_CHUNKS = 12;  // 16-B chunks per thread
constexpr int QR_MAXK = QR_THREADS * QR_CHUNKS * 8;  // 24,576 = gemma:7b's ffn, the widest GEMM input
__global__ __launch_bounds__(QR_THREADS) void quant_rows_kernel(const __bf16* __restrict__ x, int ldx, int K,
                                                                uint8_t* __restrict__ x8, int ld8,
                                                                float* __restrict__ xs, int norm, float eps) {
  const int m = blockIdx.x;
  const __bf16* row = x + (size_t)m * ldx;
  bf16x8 v[QR_CHUNKS];
#pragma unroll
  for (int c = 0; c < QR_CHUNKS; ++c) {
    const int k = (c * QR_THREADS + threadIdx.x) * 8;
    if (k < K) v[c] = *reinterpret_cast<const bf16x8*>(row + k);
  }
  float amax = 0.f, ss = 0.f;
#pragma unroll
  for (int c = 0; c < QR_CHUNKS; ++c) {
    if ((c * QR_THREADS + threadIdx.x) * 8 < K) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float f = bf2f(v[c][j]);
        amax = fmaxf(amax, fabsf(f));
        ss += f * f;
      }
    }
  }
  amax = wave_max(amax);
  ss = wave_sum(ss);
  __shared__ float s_a[QR_THREADS / 64], s_s[QR_THREADS / 64];
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) s_a[wave] = amax, s_s[wave] = ss;
  __syncthreads();
  amax = fmaxf(fmaxf(s_a[0], s_a[1]), fmaxf(s_a[2], s_a[3]));
  ss = (s_s[0] + s_s[1]) + (s_s[2] + s_s[3]);
  const float scale = amax > 0.f ? amax / 448.f : 1.f;
  const float inv = 1.f / scale;
  uint8_t* orow = x8 + (size_t)m * ld8;
  typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
#pragma unroll
  for (int c = 0; c < QR_CHUNKS; ++c) {
    const int k = (c * QR_THREADS + threadIdx.x) * 8;
    if (k < K) {
      u32x2_t o;
      o[0] = fp8x4(bf2f(v[c][0]) * inv, bf2f(v[c][1]) * inv, bf2f(v[c][2]) * inv, bf2f(v[c][3]) * inv);
      o[1] = fp8x4(bf2f(v[c][4]) * inv, bf2f(v[c][5]) * inv, bf2f(v[c][6]) * inv, bf2f(v[c][7]) * inv);
      *reinterpret_cast<u32x2_t*>(orow + k) = o;
    }
  }
  if (threadIdx.x == 0) xs[m] = scale * (norm ? rms_inv(ss, K, eps) : 1.f);
}

namespace {

struct W8Plan {
  int bm, nblk, ks, kst;
  size_t part_floats;
};

W8Plan w8_plan(int N, int K, int M) {
  W8Plan p{};
  p.bm = M > 128 ? 256 : 128;
  p.nblk = ((N >> 4) + WG_NT - 1) / WG_NT;
  const int stages = K / W8_BK;
  int ks = p.nblk >= 128 ? 1 : std::max(1, std::min(8, (256 + p.nblk / 2) / p.nblk));
  ks = std::min(ks, std::max(1, stages / 4));
  p.kst = (stages + ks - 1) / ks;
  p.ks = (stages + p.kst - 1) / p.kst;
  if (p.ks > 1) p.part_floats = (size_t)p.ks * p.nblk * WG_NT * (p.bm / 16) * 256;
  return p;
}

template <int BM, int DX, int DW, int EPI, int NDMA, bool FP4 = false>
hipError_t w8_launch(const GemmArgs& a, const WgArgs& w, const W8Scales& q, const W8Plan& p, hipStream_t st) {
  using G = WgGeo<BM>;
  constexpr int lds = (DW + 1) * w8_wbytes<BM, FP4>() + (DX + 1) * G::X_BYTES;
  static_assert(lds <= 160 * 1024, "LDS");
  static bool attr = [] {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&wgemm8_kernel<BM, DX, DW, EPI, NDMA, FP4>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, lds) == hipSuccess;
  }();
  if (!attr) return hipErrorInvalidConfiguration;
  hipLaunchKernelGGL((wgemm8_kernel<BM, DX, DW, EPI, NDMA, FP4>), dim3(p.nblk * p.ks), dim3(64 * (8 + NDMA)), lds, st,
                     a, w, q);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || p.ks == 1) return e;
  const int n_units = p.nblk * WG_NT * G::RB;
  const dim3 grid((n_units + 3) / 4), blk(256);
  switch (w.ks) {
#define CAIN_W8_RED(K) \
  case K: hipLaunchKernelGGL((wgemm8_reduce_kernel<BM, EPI, K>), grid, blk, 0, st, a, w, q, n_units); break;
    CAIN_W8_RED(2) CAIN_W8_RED(3) CAIN_W8_RED(4) CAIN_W8_RED(5) CAIN_W8_RED(6) CAIN_W8_RED(7) CAIN_W8_RED(8)
#undef CAIN_W8_RED
    default: hipLaunchKernelGGL((wgemm8_reduce_kernel<BM, EPI, 0>), grid, blk, 0, st, a, w, q, n_units);
  }
  return hipGetLastError();
}

template <int BM, bool FP4 = false>
hipError_t w8_launch_e(int epi, const GemmArgs& a, const WgArgs& w, const W8Scales& q, const W8Plan& p,
                       hipStream_t st) {
  // 160 KiB rings, as the bf16 defaults; fp4's 8.5-KiB W stages: the same X ring, 6 W stages (147 / 115 KiB)
  constexpr int DX = BM == 256 ? 2 : 3, DW = FP4 ? 5 : (BM == 256 ? 3 : 5);
  switch (epi) {
    case EPI_BF16: return w8_launch<BM, DX, DW, EPI_BF16, 4, FP4>(a, w, q, p, st);
    case EPI_RESID: return w8_launch<BM, DX, DW, EPI_RESID, 4, FP4>(a, w, q, p, st);
    case EPI_F32: return w8_launch<BM, DX, DW, EPI_F32, 4, FP4>(a, w, q, p, st);
    case EPI_SILU: return w8_launch<BM, DX, DW, EPI_SILU, 4, FP4>(a, w, q, p, st);
    case EPI_GELU: return w8_launch<BM, DX, DW, EPI_GELU, 4, FP4>(a, w, q, p, st);
    case EPI_QKV_ROPE: return w8_launch<BM, DX, DW, EPI_QKV_ROPE, 4, FP4>(a, w, q, p, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

// Shapes the W8A8 kernel takes: 16 < M <= 256, whole 128-deep stages, >= 4 of them, 16-column tiles.
CAIN_API int cain_w8a8_eligible(int N, int K, int M) {
  return M > 16 && M <= 256 && K % W8_BK == 0 && K >= 4 * W8_BK && N % 16 == 0;
}

// The slabs go after the bf16 paths' counter regions (gemm.hip GEMM_SLAB_OFFSET), which must stay zero when
// the engine shares one workspace between both weight formats' launches.
constexpr long long W8_SLAB_OFFSET = 80 * 1024;

CAIN_API long long cain_w8a8_ws_bytes(int N, int K, int M) {
  if (!cain_w8a8_eligible(N, K, M)) return 0;
  return W8_SLAB_OFFSET + (long long)(w8_plan(N, K, M).part_floats * sizeof(float));
}

CAIN_API int cain_quant_rows(const void* x, int ldx, int K, int M, void* x8, int ld8, float* xs, int norm, float eps,
                             hipStream_t st) {
  if (K % 8 || K > QR_MAXK || ldx % 8 || ld8 % 8 || M < 1) return -1;
  hipLaunchKernelGGL(quant_rows_kernel, dim3(M), dim3(QR_THREADS), 0, st, (const __bf16*)x, ldx, K, (uint8_t*)x8, ld8, xs,
                     norm, eps);
  return int(hipGetLastError());
}

namespace {

int w8a8_run(bool fp4, const void* Wp8, const void* wscale, const void* X8, int ld8, const float* xs, int K, int N,
             int M, void* Y, int ldy, const float* bias, const int* slot, const int* pos, const float* cos_t,
             const float* sin_t, void* kc, void* vtc, int H, int Hkv, int hd, int T_max, void* ws, long long ws_bytes,
             int epi_flags, hipStream_t st) {
  const int epi = epi_flags & EPI_MASK;
  if (!cain_w8a8_eligible(N, K, M) || ld8 % 16) return -1;
  if (epi == EPI_QKV_ROPE && (hd % 16 || (hd / 2) % 8)) return -1;
  const W8Plan p = w8_plan(N, K, M);
  if (p.ks > 1 && (!ws || W8_SLAB_OFFSET + (long long)(p.part_floats * sizeof(float)) > ws_bytes)) return -1;
  GemmArgs a{};
  a.Wp = reinterpret_cast<const bf16x8*>(Wp8);
  a.X = reinterpret_cast<const __bf16*>(X8);
  a.ldx = ld8, a.K = K, a.N = N, a.M = M, a.Y = Y, a.ldy = ldy, a.bias = bias;
  a.slot = slot, a.pos = pos, a.cos_t = cos_t, a.sin_t = sin_t;
  a.kc = reinterpret_cast<__bf16*>(kc), a.vtc = reinterpret_cast<__bf16*>(vtc);
  a.H = H, a.Hkv = Hkv, a.hd = hd, a.T_max = T_max, a.kv8 = (epi_flags & EPI_KV_FP8) ? 1 : 0;
  WgArgs w{};
  w.ks = p.ks, w.kst = p.kst, w.part = ws ? reinterpret_cast<float*>(static_cast<char*>(ws) + W8_SLAB_OFFSET) : nullptr;
  w.xcd_blk = p.ks > 1 && p.nblk % 8 == 0;  // XCD-local split-K (wgemm_ring.h wg_block_of)
  const W8Scales q{xs, static_cast<const float*>(wscale)};
  hipError_t e;
  if (fp4) e = p.bm == 256 ? w8_launch_e<256, true>(epi, a, w, q, p, st) : w8_launch_e<128, true>(epi, a, w, q, p, st);
  else e = p.bm == 256 ? w8_launch_e<256>(epi, a, w, q, p, st) : w8_launch_e<128>(epi, a, w, q, p, st);
  return int(e);
}

}  // namespace

// Y = epi(xs[m] * ws[n] * X8 . W8^T).  Wp8: pack_mfma_a_fp8_k128; X8 [M][ld8] e4m3 rows (cain_quant_rows);
// ws: >= cain_w8a8_ws_bytes of scratch; the rest as cain_gemm (gemm.hip), including the EPI_KV_FP8 flag.
CAIN_API int cain_gemm_w8a8(const void* Wp8, const float* wscale, const void* X8, int ld8, const float* xs, int K,
                            int N, int M, void* Y, int ldy, const float* bias, const int* slot, const int* pos,
                            const float* cos_t, const float* sin_t, void* kc, void* vtc, int H, int Hkv, int hd,
                            int T_max, void* ws, long long ws_bytes, int epi_flags, hipStream_t st) {
  return w8a8_run(false, Wp8, wscale, X8, ld8, xs, K, N, M, Y, ldy, bias, slot, pos, cos_t, sin_t, kc, vtc, H, Hkv, hd,
                  T_max, ws, ws_bytes, epi_flags, st);
}

// W4A8: Y = epi(xs[m] * X8 . W^T) with MXFP4 weights in the few-row kernel's packing (pack_mxfp4: Wq
// [N/16][K/128][64][16] e2m1 bytes, wsc [N/16][K/128][64] e8m0 bytes); same shapes, workspace and epilogues as
// cain_gemm_w8a8 (cain_w8a8_eligible, cain_w8a8_ws_bytes).
CAIN_API int cain_gemm_w4a8(const void* Wq, const void* wsc, const void* X8, int ld8, const float* xs, int K, int N,
                            int M, void* Y, int ldy, const float* bias, const int* slot, const int* pos,
                            const float* cos_t, const float* sin_t, void* kc, void* vtc, int H, int Hkv, int hd,
                            int T_max, void* ws, long long ws_bytes, int epi_flags, hipStream_t st) {
  return w8a8_run(true, Wq, wsc, X8, ld8, xs, K, N, M, Y, ldy, bias, slot, pos, cos_t, sin_t, kc, vtc, H, Hkv, hd,
                  T_max, ws, ws_bytes, epi_flags, st);
}
