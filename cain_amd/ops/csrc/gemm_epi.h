// GEMM arguments and the fused epilogues shared by the bf16 kernels (gemm.hip) and the fp8-weight kernel
// (gemm_w8.hip): see gemm.hip's header for what each epilogue does.
#pragma once
#include "common.h"

enum { EPI_BF16 = 0, EPI_RESID = 1, EPI_F32 = 2, EPI_SILU = 3, EPI_GELU = 4, EPI_QKV_ROPE = 5 };
// flag or-ed into the epilogue id at the C entries: EPI_QKV_ROPE writes an fp8 (e4m3) KV cache
constexpr int EPI_KV_FP8 = 0x100;
constexpr int EPI_MASK = 0xff;

// fp8 e4m3 (OCP, gfx950) KV-cache elements: saturate to +-448, then v_cvt_pk_fp8_f32 (RNE)
__device__ __forceinline__ float fp8_sat(float v) { return fminf(fmaxf(v, -448.f), 448.f); }
__device__ __forceinline__ uint32_t fp8x4(float a, float b, float c, float d) {
  int p = __builtin_amdgcn_cvt_pk_fp8_f32(fp8_sat(a), fp8_sat(b), 0, false);
  p = __builtin_amdgcn_cvt_pk_fp8_f32(fp8_sat(c), fp8_sat(d), p, true);
  return uint32_t(p);
}

struct GemmArgs {
  const bf16x8* Wp;
  const __bf16* X;
  int ldx, K, N, M;
  int msplit;  // workgroups per row tile, each owning 16*NB of the M rows
  void* Y;
  int ldy;
  const float* bias;
  // NORM (fused RMSNorm, gain folded into W): acc *= rsqrt(mean(x^2) + eps)
  float eps;
  // QKV_ROPE
  const int* slot;
  const int* pos;
  const float* cos_t;
  const float* sin_t;
  __bf16* kc;   // bf16 caches; with kv8, the same element offsets in bytes (fp8 e4m3)
  __bf16* vtc;
  int H, Hkv, hd, T_max;
  int kv8;
  // EPI_F32 on the skinny kernel (the few-row LM head): also the max of every 16-column chunk of each row,
  // cmax[m * ld_cm + n / 16] (null: not written) -- the sampler's first stage (sample.hip sample_cm_kernel)
  float* cmax;
  int ld_cm;
};

// Epilogue inputs of one (tile, column-tile, lane) unit, loaded BEFORE the main loop
// so their latency hides under the weight stream (the residual row, bias, RoPE
// position / tables).
struct EpiIn {
  bf16x4 r;      // EPI_RESID: residual values
  f32x4 b1, b2;  // bias (QKV: rows n1.. and n2..)
  f32x4 c, sn;   // QKV: cos / sin of the 4 rotation pairs
  int p, sl;     // QKV: position, cache slot
};

// gt = global 16-row tile of N, m = output row of this lane
template <int EPI>
__device__ __forceinline__ EpiIn epi_load_at(const GemmArgs& a, int gt, int m, int lane) {
  EpiIn e{};
  const int nsub = (lane >> 4) * 4;
  if (m >= a.M) return e;
  if constexpr (EPI == EPI_RESID) {
    e.r = *reinterpret_cast<const bf16x4*>(reinterpret_cast<const __bf16*>(a.Y) + (size_t)m * a.ldy + gt * 16 + nsub);
  } else if constexpr (EPI == EPI_BF16) {
    if (a.bias) e.b1 = *reinterpret_cast<const f32x4*>(a.bias + gt * 16 + nsub);
  } else if constexpr (EPI == EPI_QKV_ROPE) {
    e.sl = a.slot[m];
    e.p = a.pos[m];
    if (a.bias) {
      e.b1 = *reinterpret_cast<const f32x4*>(a.bias + gt * 16 + nsub);
      e.b2 = *reinterpret_cast<const f32x4*>(a.bias + gt * 16 + ((nsub + 8) & 15));
    }
    const int tph = a.hd >> 4;
    if (gt < (a.H + a.Hkv) * tph && (lane >> 4) < 2 && e.sl >= 0) {
      const int half = a.hd >> 1;
      const int j0 = (gt - (gt / tph) * tph) * 8 + nsub;
      e.c = *reinterpret_cast<const f32x4*>(a.cos_t + (size_t)e.p * half + j0);
      e.sn = *reinterpret_cast<const f32x4*>(a.sin_t + (size_t)e.p * half + j0);
    }
  }
  return e;
}

template <int NT, int NB, int EPI>
__device__ __forceinline__ EpiIn epi_load(const GemmArgs& a, int tile0, int mo, int u) {
  const int lane = u & 63, tb = u >> 6, b = tb % NB, t = tb / NB;
  return epi_load_at<EPI>(a, tile0 + t, mo + b * 16 + (lane & 15), lane);
}

// One epilogue store; WT: write-through (relaxed agent-scope atomic store = global_store ... sc1), for outputs
// another workgroup of the same launch reads with sc1 loads (front.hip's in-launch hand-offs).
template <bool WT, class T>
__device__ __forceinline__ void st_epi(void* p, const T& v) {
  if constexpr (WT) {
    static_assert(sizeof(T) <= 8, "write-through epilogue stores are at most 8 bytes");
    using U = std::conditional_t<sizeof(T) == 8, uint64_t,
                                 std::conditional_t<sizeof(T) == 4, uint32_t,
                                                    std::conditional_t<sizeof(T) == 2, uint16_t, uint8_t>>>;
    __hip_atomic_store(reinterpret_cast<U*>(p), __builtin_bit_cast(U, v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    *reinterpret_cast<T*>(p) = v;
  }
}

// Finish and store one 64-unit chunk (one 16x16 output block: n in tile gt, 16 rows m).
// get(off) returns the final fp32 accumulator of the unit held by lane (lane + off) of the
// chunk; the pair epilogues read their partner rows (+8 of the tile) at off = 32.
template <int EPI, bool WT = false, class Get>
__device__ __forceinline__ void epi_store(const GemmArgs& a, int gt, int m, int lane, const EpiIn& e, Get get) {
  const int nsub = (lane >> 4) * 4;
  const bool mvalid = m < a.M;
  if constexpr (EPI == EPI_SILU || EPI == EPI_GELU) {
    // 8-row interleave: rows 0..7 of a tile are gate rows, rows 8..15 the matching up rows
    if ((lane >> 4) < 2) {
      const f32x4 g = get(0);
      const f32x4 up = get(32);
      const int n = gt * 8 + nsub;
      bf16x4 o;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float av = (EPI == EPI_SILU) ? silu_f(g[i]) : gelu_tanh_f(g[i]);
        o[i] = f2bf(av * up[i]);
      }
      if (mvalid) st_epi<WT>(reinterpret_cast<__bf16*>(a.Y) + (size_t)m * a.ldy + n, o);
    }
  } else if constexpr (EPI == EPI_QKV_ROPE) {
    const int tph = a.hd >> 4;  // tiles per head
    const int qt = a.H * tph, kt = a.Hkv * tph;
    const int sl = mvalid ? e.sl : -1;
    if (gt < qt + kt) {
      // rows 0..7 of the tile = pair elements j (first half), rows 8..15 = j + hd/2
      if ((lane >> 4) < 2 && sl >= 0) {
        const f32x4 x1 = get(0);
        const f32x4 x2 = get(32);  // partner rows +8 live in lane + 32
        const int head = gt / tph, it = gt - (gt / tph) * tph;
        const int half = a.hd >> 1;
        const int j0 = it * 8 + nsub;  // first pair element of this thread
        bf16x4 y1, y2;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          // round to bf16 first: the unfused path stores the projection in bf16 before RoPE
          const float v1 = bf2f(f2bf(x1[i] + e.b1[i]));
          const float v2 = bf2f(f2bf(x2[i] + e.b2[i]));
          y1[i] = f2bf(v1 * e.c[i] - v2 * e.sn[i]);
          y2[i] = f2bf(v2 * e.c[i] + v1 * e.sn[i]);
        }
        if (head < a.H) {
          __bf16* dst = reinterpret_cast<__bf16*>(a.Y) + (size_t)m * a.ldy + head * a.hd;
          st_epi<WT>(dst + j0, y1);
          st_epi<WT>(dst + j0 + half, y2);
        } else {
          // fragment-major K cache (attention.hip): 4 consecutive head dims of one position are contiguous
          const size_t base = ((size_t)sl * a.Hkv + (head - a.H)) * a.T_max * a.hd;
          if (a.kv8) {  // the bf16-rounded values, as e4m3: one dword per 4 head dims
            uint8_t* kb = reinterpret_cast<uint8_t*>(a.kc) + base;
            st_epi<WT>(kb + kfrag_off(e.p, j0, a.hd), fp8x4(bf2f(y1[0]), bf2f(y1[1]), bf2f(y1[2]), bf2f(y1[3])));
            st_epi<WT>(kb + kfrag_off(e.p, j0 + half, a.hd), fp8x4(bf2f(y2[0]), bf2f(y2[1]), bf2f(y2[2]), bf2f(y2[3])));
          } else {
            __bf16* kb = a.kc + base;
            st_epi<WT>(kb + kfrag_off(e.p, j0, a.hd), y1);
            st_epi<WT>(kb + kfrag_off(e.p, j0 + half, a.hd), y2);
          }
        }
      }
    } else if (sl >= 0) {
      const f32x4 v = get(0);
      const int vr = (gt - qt - kt) * 16 + nsub;  // row within the V block
      const int kh = vr / a.hd, d = vr - (vr / a.hd) * a.hd;
      // fragment-major V^T cache: head dims d..d+3 of position p sit in consecutive lanes (8 elements apart)
      const size_t off = ((size_t)sl * a.Hkv + kh) * a.hd * a.T_max + vfrag_off(e.p, d, a.hd);
      if (a.kv8) {
        uint8_t* dst = reinterpret_cast<uint8_t*>(a.vtc) + off;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int p8 = __builtin_amdgcn_cvt_pk_fp8_f32(fp8_sat(bf2f(f2bf(v[i] + e.b1[i]))), 0.f, 0, false);
          st_epi<WT>(dst + i * 8, uint8_t(p8 & 0xff));
        }
      } else {
        __bf16* dst = a.vtc + off;
#pragma unroll
        for (int i = 0; i < 4; ++i) st_epi<WT>(dst + i * 8, f2bf(v[i] + e.b1[i]));
      }
    }
  } else {
    const f32x4 v = get(0);
    const int n = gt * 16 + nsub;
    if constexpr (EPI == EPI_F32) {
      if (mvalid) *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(a.Y) + (size_t)m * a.ldy + n) = v;
    } else if constexpr (EPI == EPI_BF16) {
      bf16x4 o;
#pragma unroll
      for (int i = 0; i < 4; ++i) o[i] = f2bf(v[i] + e.b1[i]);
      if (mvalid) st_epi<WT>(reinterpret_cast<__bf16*>(a.Y) + (size_t)m * a.ldy + n, o);
    } else {  // EPI_RESID: in-place residual update
      if (mvalid) {
        bf16x4 o;
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = f2bf(v[i] + bf2f(e.r[i]));
        st_epi<WT>(reinterpret_cast<__bf16*>(a.Y) + (size_t)m * a.ldy + n, o);
      }
    }
  }
}

// The LM head's per-row maximum of the 16-column chunk gt (the chunk-maximum samplers' first stage, sample.hip):
// lanes c, c + 16, c + 32, c + 48 hold row c's 16 values v.  Called by whole waves (two xor shuffles); no-op without
// a cmax buffer (uniform).
__device__ __forceinline__ void epi_cmax(const GemmArgs& a, int gt, int m, int lane, const f32x4& v) {
  if (!a.cmax) return;
  float mx = fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3]));
  mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  if ((lane >> 4) == 0 && m < a.M) a.cmax[(size_t)m * a.ld_cm + gt] = mx;
}
