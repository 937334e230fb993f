// Decode / short-prefill attention over the KV cache, split over positions
// (flash-decoding) with both products on MFMA (SURVEY §2.4 row "Decode attention").
//
// One wave handles (row m, kv head kh, split sp).  The G = H/Hkv query heads of
// the group are the 16 MFMA columns (G <= 16 covers MHA, GQA 4/6/7/8 and MQA).
// Per 32-position block:
//   S^T[t][g] = K[t][:] . Q[g][:]     2 tiles of v_mfma_f32_16x16x32_bf16 x hd/32
//       A = K rows (lane: row t = l&15, 16 B of K[t][32i+8(l>>4)..]) straight from HBM,
//       B = Q^T (lane: col g) held in registers for the whole wave;
//   online softmax per column g in registers (exp2, scale*log2e folded);
//   O^T[d][g] += V^T[d][t] P^T[t][g]   hd/16 MFMAs, k = the block's 32 positions
//       B = P^T taken from the S accumulators WITHOUT moving data: lane (g, h)
//       holds t = 4h..4h+3 (tile 0) and 16+4h..16+4h+3 (tile 1), which defines a
//       permuted k order (cdna_hip_programming.md §3 'An accumulator tile as the
//       next MFMA's operand');
//       A = V^T rows in that same k order: two 8-byte loads from the transposed
//       V cache (rope_kv.hip) — so nothing is staged through LDS.
// Each split writes an unnormalised partial (O, m, l); attn_combine merges the
// splits (and normalises).  Split geometry is fixed at launch (hipGraph
// friendly) while the length comes from device memory each step.
#include "common.h"

constexpr float LOG2E = 1.4426950408889634f;

template <int HD>
__global__ __launch_bounds__(64) void attn_decode_kernel(
    const __bf16* __restrict__ q, const __bf16* __restrict__ kc, const __bf16* __restrict__ vtc,
    const int* __restrict__ slot, const int* __restrict__ pos, float* __restrict__ part_o,
    float* __restrict__ part_ml, int H, int Hkv, int T_max, int nsplit, float scale) {
  constexpr int NKS = HD / 32;  // MFMAs per S tile
  constexpr int NDT = HD / 16;  // O^T d-tiles
  const int lane = threadIdx.x;
  const int mk = blockIdx.x;
  const int m = mk / Hkv, kh = mk - (mk / Hkv) * Hkv;
  const int sp = blockIdx.y;
  const int G = H / Hkv;
  const int g = lane & 15, hq = lane >> 4;
  const int s = slot[m];
  const int L = (s >= 0) ? pos[m] + 1 : 0;
  const int nblk = (L + 31) >> 5;
  const int bps = (nblk + nsplit - 1) / nsplit;
  const int b0 = sp * bps;
  const int b1 = min(nblk, b0 + bps);

  // partial outputs: part_o[((m*H + h)*nsplit + sp)*HD + d], part_ml[((m*H + h)*nsplit + sp)*2 + {0,1}]
  float m_run = -INFINITY, l_run = 0.f;
  f32x4 o[NDT];
#pragma unroll
  for (int i = 0; i < NDT; ++i) o[i] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (b0 < b1) {
    // Q^T fragments (B operand): lane (g, hq) holds q[g][32i + 8hq .. +8]
    bf16x8 qf[NKS];
    const bool gvalid = g < G;
    const __bf16* qrow = q + ((size_t)m * H + kh * G + (gvalid ? g : 0)) * HD + hq * 8;
#pragma unroll
    for (int i = 0; i < NKS; ++i) {
      bf16x8 v = *reinterpret_cast<const bf16x8*>(qrow + i * 32);
      if (!gvalid) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = f2bf(0.f);
      }
      qf[i] = v;
    }
    const float sl2 = scale * LOG2E;
    const __bf16* kbase = kc + ((size_t)s * Hkv + kh) * T_max * HD;
    const __bf16* vbase = vtc + ((size_t)s * Hkv + kh) * HD * T_max;
    for (int blk = b0; blk < b1; ++blk) {
      const int t0 = blk * 32;
      // ---- S^T tiles
      f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f};
      const __bf16* k0 = kbase + (size_t)(t0 + g) * HD + hq * 8;  // A: row t = l&15
      const __bf16* k1 = k0 + 16 * HD;
      bf16x8 ka[NKS], kb[NKS];
#pragma unroll
      for (int i = 0; i < NKS; ++i) {
        ka[i] = *reinterpret_cast<const bf16x8*>(k0 + i * 32);
        kb[i] = *reinterpret_cast<const bf16x8*>(k1 + i * 32);
      }
      // V^T fragments for this block (issued early, consumed after softmax)
      u16x4 va[NDT], vb[NDT];
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        const __bf16* vr = vbase + (size_t)(dt * 16 + g) * T_max + t0 + hq * 4;
        va[dt] = *reinterpret_cast<const u16x4*>(vr);
        vb[dt] = *reinterpret_cast<const u16x4*>(vr + 16);
      }
#pragma unroll
      for (int i = 0; i < NKS; ++i) {
        s0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ka[i], qf[i], s0, 0, 0, 0);
        s1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kb[i], qf[i], s1, 0, 0, 0);
      }
      // ---- mask + online softmax (column g; this lane holds t = t0+4hq+r and t0+16+4hq+r)
      float bmax = -INFINITY;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ta = t0 + hq * 4 + r, tb = ta + 16;
        s0[r] = (ta < L) ? s0[r] * sl2 : -INFINITY;
        s1[r] = (tb < L) ? s1[r] * sl2 : -INFINITY;
        bmax = fmaxf(bmax, fmaxf(s0[r], s1[r]));
      }
      bmax = fmaxf(bmax, __shfl_xor(bmax, 16, 64));
      bmax = fmaxf(bmax, __shfl_xor(bmax, 32, 64));
      const float m_new = fmaxf(m_run, bmax);
      const float alpha = exp2f(m_run - m_new);
      m_run = m_new;
      bf16x8 pf;
      float psum = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float pa = exp2f(s0[r] - m_new), pb = exp2f(s1[r] - m_new);
        psum += pa + pb;
        pf[r] = f2bf(pa);
        pf[4 + r] = f2bf(pb);
      }
      l_run = l_run * alpha + psum;
      // ---- O^T += V^T . P^T
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        o[dt] *= alpha;
        u16x8 vv;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          vv[j] = va[dt][j];
          vv[4 + j] = vb[dt][j];
        }
        bf16x8 vf = __builtin_bit_cast(bf16x8, vv);
        o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf, o[dt], 0, 0, 0);
      }
    }
  }
  // l: sum the 4 lane-partials of column g
  l_run += __shfl_xor(l_run, 16, 64);
  l_run += __shfl_xor(l_run, 32, 64);
  if (g < G) {
    const int h = kh * G + g;
    const size_t base = ((size_t)m * H + h) * nsplit + sp;
    float* po = part_o + base * HD;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
      // lane (g, hq) holds d = dt*16 + 4hq + r
      *reinterpret_cast<f32x4*>(po + dt * 16 + hq * 4) = o[dt];
    }
    if (hq == 0) {
      part_ml[base * 2 + 0] = m_run;
      part_ml[base * 2 + 1] = l_run;
    }
  }
}

// out[m][h*HD + d] = sum_s O_s * 2^(m_s - M) / sum_s l_s * 2^(m_s - M)
template <int HD>
__global__ __launch_bounds__(HD) void attn_combine_kernel(const float* __restrict__ part_o,
                                                          const float* __restrict__ part_ml, __bf16* __restrict__ out,
                                                          int ldo, int H, int nsplit, const int* __restrict__ slot) {
  const int mh = blockIdx.x;
  const int m = mh / H, h = mh - (mh / H) * H;
  const int d = threadIdx.x;
  __bf16* dst = out + (size_t)m * ldo + h * HD + d;
  if (slot[m] < 0) {
    *dst = f2bf(0.f);
    return;
  }
  const size_t base = (size_t)mh * nsplit;
  float M = -INFINITY;
  for (int sp = 0; sp < nsplit; ++sp) M = fmaxf(M, part_ml[(base + sp) * 2]);
  float num = 0.f, den = 0.f;
  for (int sp = 0; sp < nsplit; ++sp) {
    float ms = part_ml[(base + sp) * 2];
    if (ms == -INFINITY) continue;
    float w = exp2f(ms - M);
    den += w * part_ml[(base + sp) * 2 + 1];
    num += w * part_o[(base + sp) * HD + d];
  }
  *dst = f2bf(den > 0.f ? num / den : 0.f);
}

template <int HD>
static hipError_t launch_attn(const void* q, const void* kc, const void* vtc, const int* slot, const int* pos,
                              float* part_o, float* part_ml, void* out, int ldo, int M, int H, int Hkv, int T_max,
                              int nsplit, float scale, hipStream_t st) {
  hipLaunchKernelGGL(attn_decode_kernel<HD>, dim3(M * Hkv, nsplit), dim3(64), 0, st, (const __bf16*)q,
                     (const __bf16*)kc, (const __bf16*)vtc, slot, pos, part_o, part_ml, H, Hkv, T_max, nsplit, scale);
  hipLaunchKernelGGL(attn_combine_kernel<HD>, dim3(M * H), dim3(HD), 0, st, part_o, part_ml, (__bf16*)out, ldo, H,
                     nsplit, slot);
  return hipGetLastError();
}

// Workspace: part_o  M*H*nsplit*hd floats, part_ml M*H*nsplit*2 floats.
CAIN_API int cain_attention(const void* q, const void* kc, const void* vtc, const int* slot, const int* pos,
                            float* part_o, float* part_ml, void* out, int ldo, int M, int H, int Hkv, int hd,
                            int T_max, int nsplit, float scale, hipStream_t st) {
  if (H % Hkv || H / Hkv > 16 || T_max % 32 || nsplit < 1) return -1;
  switch (hd) {
    case 64: return int(launch_attn<64>(q, kc, vtc, slot, pos, part_o, part_ml, out, ldo, M, H, Hkv, T_max, nsplit, scale, st));
    case 96: return int(launch_attn<96>(q, kc, vtc, slot, pos, part_o, part_ml, out, ldo, M, H, Hkv, T_max, nsplit, scale, st));
    case 128: return int(launch_attn<128>(q, kc, vtc, slot, pos, part_o, part_ml, out, ldo, M, H, Hkv, T_max, nsplit, scale, st));
    case 256: return int(launch_attn<256>(q, kc, vtc, slot, pos, part_o, part_ml, out, ldo, M, H, Hkv, T_max, nsplit, scale, st));
    default: return -1;
  }
}
