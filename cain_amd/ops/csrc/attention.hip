// Decode / short-prefill attention over the KV cache, split over positions
// (flash-decoding) with both products on MFMA (SURVEY §2.4 row "Decode attention").
//
// KV cache layout: fragment-major, written by the QKV GEMM epilogue (gemm.hip; element offsets
// kfrag_off / vfrag_off in common.h, torch mirrors in cain_amd/ops pack_kcache / pack_vcache).
// Per (slot, kv head):
//   K    [T/16][hd/32][64 lanes][8]: the A fragment of v_mfma_f32_16x16x32_bf16 for positions
//        16u..16u+15 x head dims 32s..32s+31 (lane = (t&15) + 16*((d&31)>>3), element d&7);
//   V^T  [T/32][hd/16][64 lanes][8]: the A fragment of the PV product for head dims 16c..16c+15 x
//        the 32 positions of block b in P's permuted k order below (lane = (d&15) + 16*((t&15)>>2),
//        element 4*((t>>4)&1) + (t&3)).
// A 32-position block of one (slot, kv head) is 2*hd*32 contiguous bytes of K and as many of V, and
// every load instruction of a wave reads one contiguous 1 KiB (full 128-B lines; a row-major cache
// made each K load touch 16 rows x 64 B and each V^T load 16 rows x 8 B).
//
// Workgroup = AW (4 or 8) waves = (row m, kv head kh, split sp).  The G = H/Hkv query
// heads of the group are the 16 MFMA columns (G <= 16 covers MHA, GQA 4/6/7/8
// and MQA).  The split's 32-position blocks are dealt to the AW waves.  Per block:
//   S^T[t][g] = K[t][:] . Q[g][:]     2 tiles of v_mfma_f32_16x16x32_bf16 x hd/32
//       A = K fragments straight from HBM, B = Q^T (lane: col g) held in registers
//       for the whole wave;
//   online softmax per column g in registers (exp2, scale*log2e folded);
//   O^T[d][g] += V^T[d][t] P^T[t][g]   hd/16 MFMAs, k = the block's 32 positions
//       B = P^T taken from the S accumulators WITHOUT moving data: lane (g, h)
//       holds t = 4h..4h+3 (tile 0) and 16+4h..16+4h+3 (tile 1), which defines a
//       permuted k order (cdna_hip_programming.md §3 'An accumulator tile as the
//       next MFMA's operand');
//       A = V^T fragments stored in that same k order — nothing is staged through LDS.
// fp8 KV cache (KV8): the same fragment-major layouts with e4m3 elements (the QKV epilogue writes them,
// gemm_epi.h EPI_KV_FP8), so a lane's fragment is 8 contiguous bytes and a block moves half the bytes; each
// fragment widens to bf16 in registers (v_cvt_scalef32_pk_bf16_fp8, 4 per fragment, the per-tensor scale
// folded in) and both products stay on the bf16 MFMA.
// The AW waves merge their (m, l, O) in LDS.  With one split the workgroup
// normalises and stores bf16 directly; otherwise each workgroup publishes an
// unnormalised partial with write-through (sc1) stores and the LAST arriving
// workgroup of (m, kh) merges all splits with sc1 loads (per-wave vmcnt drain ->
// barrier -> relaxed agent ticket; no release/acquire fences, counter reset by the
// reducer: cdna_hip_programming.md §5 'In-launch split-K reduction'), so there
// is no separate combine launch.
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "wgemm_ring.h"

constexpr float LOG2E = 1.4426950408889634f;
// AW: waves per workgroup (4; 8 for few (row, kv head) pairs: single-stream decode, where one workgroup per
// pair with more waves beats a position split and its in-kernel combine)
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// 8 e4m3 values (one lane's fragment) -> bf16x8, times `sc`
__device__ __forceinline__ bf16x8 fp8x8_to_bf16(u32x2 v, float sc) {
  bf16x8 r;
#pragma unroll
  for (int w = 0; w < 2; ++w) {
    const bf16x2 lo = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(int(v[w]), sc, false);
    const bf16x2 hi = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(int(v[w]), sc, true);
    r[4 * w + 0] = lo[0], r[4 * w + 1] = lo[1], r[4 * w + 2] = hi[0], r[4 * w + 3] = hi[1];
  }
  return r;
}

// ONESET: one register set of K / V fragments per wave instead of the two-set ping-pong, so more workgroups are
// resident (OCC: minimum waves per SIMD the register allocation must allow).  The two-set body needs ~220
// registers (2 waves per SIMD, 2 workgroups per CU: the 2,048-workgroup grid of 256 rows x 8 kv heads runs in 4
// rounds); the one-set body held to 128 registers (no spills) runs 4 workgroups per CU, 2 rounds, 16 waves each
// with one block in flight.  Measured (llama3.1:8b, 256 rows, tools/bench_kernels.py --attn-only, one box):
// 49.4 -> 33.2 us at 192 positions, 79.7 -> 58.1 at 350, 136.5 -> 113.4 at 700, 258.2 -> 220.9 at 1400 (6.6 TB/s);
// fp8 cache 65.3 -> 56.7 at 700; headline bench 25.1k -> 26.3k tok/s (profiles/r2/attn_occupancy.md).
template <int HD, int AW, bool KV8, bool NT_KV = true, bool ONESET = false, int OCC = 1>
__global__ __launch_bounds__(AW * 64, OCC) void attn_decode_kernel(
    const __bf16* __restrict__ q, const __bf16* __restrict__ kc, const __bf16* __restrict__ vtc,
    const int* __restrict__ slot, const int* __restrict__ pos, float* __restrict__ part_o,
    float* __restrict__ part_ml, unsigned* __restrict__ counters, __bf16* __restrict__ out, int ldo, int M, int H,
    int Hkv, int T_max, int nsplit, float scale, float kscale, float vscale) {
  constexpr int NKS = HD / 32;  // MFMAs per S tile
  constexpr int NDT = HD / 16;  // O^T d-tiles
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
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

  float m_run = -INFINITY, l_run = 0.f;
  f32x4 o[NDT];
#pragma unroll
  for (int i = 0; i < NDT; ++i) o[i] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (b0 + wave < b1) {
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
    // fragment-major caches (layout at the top of this file): a 32-position block of one (slot, kv head) is
    // 2*NKS contiguous 1-KiB K fragments and NDT contiguous 1-KiB V^T fragments; lane l's 16 B sit at 16*l
    // a fragment in registers: 16 B of bf16, or (KV8) 8 B of e4m3 widened right before its MFMA
    using frag_t = std::conditional_t<KV8, u32x2, bf16x8>;
    constexpr int ESZ = KV8 ? 1 : 2;  // bytes per cache element
    const char* kbase = reinterpret_cast<const char*>(kc) + (((size_t)s * Hkv + kh) * T_max * HD + lane * 8) * ESZ;
    const char* vbase = reinterpret_cast<const char*>(vtc) + (((size_t)s * Hkv + kh) * HD * T_max + lane * 8) * ESZ;
    // the caches stream once per step: non-temporal loads (MI355X_MICROARCH.md 'nt-weights': once-read bytes)
    auto ld = [](const char* p) -> frag_t {
      if constexpr (NT_KV) return __builtin_nontemporal_load(reinterpret_cast<const frag_t*>(p));
      else return *reinterpret_cast<const frag_t*>(p);
    };
    auto load_blk = [&](int blk, frag_t (&k_a)[NKS], frag_t (&k_b)[NKS], frag_t (&v)[NDT]) {
      const char* k0 = kbase + (size_t)blk * (2 * NKS * 512 * ESZ);
#pragma unroll
      for (int i = 0; i < NKS; ++i) {
        k_a[i] = ld(k0 + i * 512 * ESZ);
        k_b[i] = ld(k0 + (NKS + i) * 512 * ESZ);
      }
      const char* v0 = vbase + (size_t)blk * (NDT * 512 * ESZ);
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) v[dt] = ld(v0 + dt * 512 * ESZ);
    };
    auto widen = [&](const frag_t& f, float sc) -> bf16x8 {
      if constexpr (KV8) return fp8x8_to_bf16(f, sc);
      else return f;
    };
    auto process = [&](int blk, const frag_t (&ka)[NKS], const frag_t (&kb)[NKS], const frag_t (&va)[NDT]) {
      const int t0 = blk * 32;
      f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < NKS; ++i) {
        s0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(widen(ka[i], kscale), qf[i], s0, 0, 0, 0);
        s1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(widen(kb[i], kscale), qf[i], s1, 0, 0, 0);
      }
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
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        o[dt] *= alpha;
        o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(widen(va[dt], vscale), pf, o[dt], 0, 0, 0);
      }
    };

    const int first = b0 + wave;
    if constexpr (HD <= 128 && !ONESET) {
      frag_t ka[NKS], kb[NKS], va[NDT];
      load_blk(first, ka, kb, va);
      // two register sets ping-pong, the next block's loads issued before the current block computes;
      // no register copy of an in-flight load (that forces vmcnt(0)) and no load under a branch: a
      // prefetch past the wave's last block is clamped to it (a cache hit, never used)
      const int last = first + ((b1 - 1 - first) / AW) * AW;
      frag_t kc2[NKS], kd2[NKS], vb2[NDT];
      for (int blk = first; blk < b1; blk += 2 * AW) {
        load_blk(min(blk + AW, last), kc2, kd2, vb2);
        __builtin_amdgcn_sched_barrier(0);
        process(blk, ka, kb, va);
        load_blk(min(blk + 2 * AW, last), ka, kb, va);
        __builtin_amdgcn_sched_barrier(0);
        if (blk + AW < b1) process(blk + AW, kc2, kd2, vb2);
      }
    } else {  // hd 256: one register set (two would spill); ONESET: 3 waves per SIMD instead of 2
      frag_t ka[NKS], kb[NKS], va[NDT];
      load_blk(first, ka, kb, va);
      for (int blk = first; blk < b1; blk += AW) {
        process(blk, ka, kb, va);
        if (blk + AW < b1) load_blk(blk + AW, ka, kb, va);
      }
    }
  }
  l_run += __shfl_xor(l_run, 16, 64);
  l_run += __shfl_xor(l_run, 32, 64);

  // ---- merge the 4 waves in LDS: ml[w][g] = (m, l); ob[w][d][g]
  __shared__ float s_m[AW][16], s_l[AW][16];
  __shared__ float s_o[AW][HD][16];
  __shared__ unsigned s_ticket;
  if (hq == 0) {
    s_m[wave][g] = m_run;
    s_l[wave][g] = l_run;
  }
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
    for (int r = 0; r < 4; ++r) s_o[wave][dt * 16 + hq * 4 + r][g] = o[dt][r];
  __syncthreads();

  // each thread finalises (g, d) pairs of this workgroup
  const int nout = G * HD;
  const size_t pbase = (size_t)(m * H + kh * G) * nsplit;  // partial (head kh*G+gg, split j) = pbase + gg*nsplit + j
  // part_ml regions of different (m, kh) never share a 128-B line (ML_STRIDE), so a
  // reducer's L2 never holds another group's line that is still being written
  const int mls = ((G * nsplit * 2 + 31) / 32) * 32;
  float* pml = part_ml + (size_t)mk * mls;
  // 3 to 8 outputs per thread (gemma:2b's 8 query heads x 256 dims on 4 waves): publish and merge 4 consecutive dims
  // per thread with 16-byte write-through stores and sc1 loads, and request every split's partials and (m, l) in one
  // round trip -- the per-element path below issued 8 x 8 dependent-free but 4-byte loads per thread
  // (compiled for head_dim 256 only: the hd <= 128 bodies keep their code unchanged)
  const bool vec = HD >= 256 && nsplit > 1 && nsplit <= 16 && nout > 2 * AW * 64 && nout <= 8 * AW * 64;
  if (vec) {
    const __amdgpu_buffer_rsrc_t po_r = slab_rsrc(part_o);
    for (int qd = threadIdx.x; qd < nout / 4; qd += AW * 64) {
      const int e0 = qd * 4, gg = e0 / HD, d0 = e0 - (e0 / HD) * HD;
      float Mx = -INFINITY;
#pragma unroll
      for (int w = 0; w < AW; ++w) Mx = fmaxf(Mx, s_m[w][gg]);
      float lsum = 0.f;
      f32x4 osum = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int w = 0; w < AW; ++w) {
        const float mw = s_m[w][gg];
        if (mw == -INFINITY) continue;
        const float f = exp2f(mw - Mx);
        lsum += f * s_l[w][gg];
#pragma unroll
        for (int i = 0; i < 4; ++i) osum[i] += f * s_o[w][d0 + i][gg];
      }
      const size_t pi = pbase + (size_t)gg * nsplit + sp;
      st_wt(po_r, (int)((pi * HD + d0) * 4), osum);
      if (d0 == 0) {
        const int li = gg * nsplit + sp;
        __hip_atomic_store(pml + li * 2 + 0, Mx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(pml + li * 2 + 1, lsum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  for (int e = threadIdx.x; e < (vec ? 0 : nout); e += AW * 64) {
    const int gg = e / HD, d = e - (e / HD) * HD;
    float Mx = -INFINITY;
#pragma unroll
    for (int w = 0; w < AW; ++w) Mx = fmaxf(Mx, s_m[w][gg]);
    float lsum = 0.f, osum = 0.f;
#pragma unroll
    for (int w = 0; w < AW; ++w) {
      const float mw = s_m[w][gg];
      if (mw == -INFINITY) continue;
      const float f = exp2f(mw - Mx);
      lsum += f * s_l[w][gg];
      osum += f * s_o[w][d][gg];
    }
    if (nsplit == 1) {
      out[(size_t)m * ldo + (kh * G + gg) * HD + d] = f2bf(lsum > 0.f ? osum * fast_rcp(lsum) : 0.f);
    } else {
      // publish write-through (sc1) so the reducer needs no release/acquire fences
      // (MI355X_MICROARCH.md 'Valid forms', first table row; cdna_hip_programming.md Guideline 16)
      const size_t pi = pbase + (size_t)gg * nsplit + sp;
      __hip_atomic_store(part_o + pi * HD + d, osum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (d == 0) {
        const int li = gg * nsplit + sp;
        __hip_atomic_store(pml + li * 2 + 0, Mx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(pml + li * 2 + 1, lsum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  if (nsplit == 1) return;

  // ---- every storing wave drains, one lane takes a ticket; the last arriver reduces
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    s_ticket = __hip_atomic_fetch_add(counters + mk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  if (s_ticket != unsigned(nsplit - 1)) return;
  if (vec) {
    if (threadIdx.x == 0) counters[mk] = 0u;  // ready for the next launch (launch-ordered)
    const __amdgpu_buffer_rsrc_t po_r = slab_rsrc(part_o);
    auto merge = [&](auto ns_c) {  // NS >= nsplit loads per output, clamped (every load unconditional, masked after)
      constexpr int NS = decltype(ns_c)::value;
      for (int qd = threadIdx.x; qd < nout / 4; qd += AW * 64) {
        const int e0 = qd * 4, gg = e0 / HD, d0 = e0 - (e0 / HD) * HD;
        float mj[NS], lj[NS];
        f32x4 oj[NS];
#pragma unroll
        for (int j = 0; j < NS; ++j) {
          const int jj = min(j, nsplit - 1);
          const int li = gg * nsplit + jj;
          const f32x2 ml = __builtin_bit_cast(
              f32x2, __hip_atomic_load(reinterpret_cast<const uint64_t*>(pml + li * 2), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT));
          mj[j] = ml[0], lj[j] = ml[1];
          oj[j] = ld_wt(po_r, (int)(((pbase + (size_t)gg * nsplit + jj) * HD + d0) * 4));
        }
        float Mx = -INFINITY;
#pragma unroll
        for (int j = 0; j < NS; ++j) Mx = j < nsplit ? fmaxf(Mx, mj[j]) : Mx;
        float den = 0.f;
        f32x4 num = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < NS; ++j) {
          const float f = (j < nsplit && mj[j] != -INFINITY) ? exp2f(mj[j] - Mx) : 0.f;
          den += f * lj[j];
          num += f * oj[j];
        }
        const float r = den > 0.f ? fast_rcp(den) : 0.f;
        bf16x4 o4;
#pragma unroll
        for (int i = 0; i < 4; ++i) o4[i] = f2bf(num[i] * r);
        *reinterpret_cast<bf16x4*>(out + (size_t)m * ldo + (kh * G + gg) * HD + d0) = o4;
      }
    };
    if (nsplit <= 8)
      merge(std::integral_constant<int, 8>{});
    else
      merge(std::integral_constant<int, 16>{});
    return;
  }
  if (nsplit <= 16 && nout <= 2 * AW * 64) {
    // up to 16 splits and 2 outputs per thread (the few-row decode of every study model but gemma:2b's 8 x 256 query
    // dims): each thread loads its outputs' partials and every split's (m, l) at once -- one round trip of sc1 loads,
    // no LDS pass, instead of the (m, l) pass, a barrier and then the partials.  Measured one box, interleaved
    // (profiles/r6/attn_combine/): batch-1 MXFP4 llama3.1:8b +0.9 %, qwen2:1.5b +1.2 %; an LDS variant for 4 outputs
    // per thread lost on llama / qwen and gemma:2b takes the 16-byte path above.
    if (threadIdx.x == 0) counters[mk] = 0u;  // ready for the next launch (launch-ordered)
    auto merge = [&](auto ns_c) {  // NS >= nsplit loads per output, clamped (every load unconditional, masked after)
      constexpr int NS = decltype(ns_c)::value;
      for (int e = threadIdx.x; e < nout; e += AW * 64) {
        const int gg = e / HD, d = e - (e / HD) * HD;
        float mj[NS], lj[NS], oj[NS];
#pragma unroll
        for (int j = 0; j < NS; ++j) {
          const int jj = min(j, nsplit - 1);
          const int li = gg * nsplit + jj;
          mj[j] = __hip_atomic_load(pml + li * 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          lj[j] = __hip_atomic_load(pml + li * 2 + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          oj[j] = __hip_atomic_load(part_o + (pbase + (size_t)gg * nsplit + jj) * HD + d, __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_AGENT);
        }
        float Mx = -INFINITY;
#pragma unroll
        for (int j = 0; j < NS; ++j) Mx = j < nsplit ? fmaxf(Mx, mj[j]) : Mx;
        float num = 0.f, den = 0.f;
#pragma unroll
        for (int j = 0; j < NS; ++j) {
          const float f = (j < nsplit && mj[j] != -INFINITY) ? exp2f(mj[j] - Mx) : 0.f;
          num += f * oj[j];
          den += f * lj[j];
        }
        out[(size_t)m * ldo + (kh * G + gg) * HD + d] = f2bf(den > 0.f ? num * fast_rcp(den) : 0.f);
      }
    };
    if (nsplit <= 8)
      merge(std::integral_constant<int, 8>{});
    else
      merge(std::integral_constant<int, 16>{});
    return;
  }
  // split weights into LDS once (sc1 loads: never served from this CU's stale L1)
  __shared__ float s_w[16 * 64];   // [gg][j] merge weight 2^(m_j - M) / den
  const int nw = G * nsplit;      // <= 16 * 64
  for (int e = threadIdx.x; e < nw; e += AW * 64) {
    const int gg = e / nsplit, j = e - (e / nsplit) * nsplit;
    s_w[gg * 64 + j] = __hip_atomic_load(pml + e * 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_o[1][j][gg] = __hip_atomic_load(pml + e * 2 + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (threadIdx.x < G) {
    const int gg = threadIdx.x;
    float Mx = -INFINITY;
    for (int j = 0; j < nsplit; ++j) Mx = fmaxf(Mx, s_w[gg * 64 + j]);
    float den = 0.f;
    for (int j = 0; j < nsplit; ++j) {
      const float mj = s_w[gg * 64 + j];
      const float f = (mj == -INFINITY) ? 0.f : exp2f(mj - Mx);
      s_w[gg * 64 + j] = f;
      den += f * s_o[1][j][gg];
    }
    s_l[0][gg] = den > 0.f ? 1.f / den : 0.f;
  }
  if (threadIdx.x == 0) counters[mk] = 0u;  // ready for the next launch (launch-ordered)
  __syncthreads();
  for (int e = threadIdx.x; e < nout; e += AW * 64) {
    const int gg = e / HD, d = e - (e / HD) * HD;
    const float* po = part_o + (pbase + (size_t)gg * nsplit) * HD + d;
    float num = 0.f;
#pragma unroll 8
    for (int j = 0; j < nsplit; ++j)
      num += s_w[gg * 64 + j] * __hip_atomic_load(po + (size_t)j * HD, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    out[(size_t)m * ldo + (kh * G + gg) * HD + d] = f2bf(num * s_l[0][gg]);
  }
}

// Cache loads are non-temporal (default-policy loads measured slower); the hd <= 128 body holds one register set to
// 128 registers (4 waves per SIMD; the two-set and 3-wave bodies of rounds 1-2 measured slower,
// profiles/r2/attn_occupancy.md).  cain_attention_set_body selects them for A/B runs: 2 = default, 1 = one set at
// 3 waves per SIMD, 0 = two register sets.
static int g_attn_body = 2;
CAIN_API void cain_attention_set_body(int v) { g_attn_body = v; }
static bool attn_nt() { return true; }
static int attn_variant() { return g_attn_body; }

template <int HD, int AW, bool KV8, bool NT>
static void launch_attn_t(const void* q, const void* kc, const void* vtc, const int* slot, const int* pos,
                          float* part_o, float* part_ml, unsigned* counters, void* out, int ldo, int M, int H, int Hkv,
                          int T_max, int nsplit, float scale, float kscale, float vscale, hipStream_t st) {
  // (a four-set prefetch for the half-size fp8 blocks measured slower: 90 vs 68 us at 256 rows x 700 positions)
  const int var = HD <= 128 ? attn_variant() : 0;
  // (hd 256 keeps 1 wave per SIMD: held to 256 registers, 2 waves per SIMD, gemma:7b's 256-row attention
  // measured 144.5 vs 139.6 us at 192 positions and 454 vs 438 at 700 -- it already streams 6.7 TB/s)
  if (var == 1)
    hipLaunchKernelGGL((attn_decode_kernel<HD, AW, KV8, NT, true>), dim3(M * Hkv, nsplit), dim3(AW * 64), 0, st,
                       (const __bf16*)q, (const __bf16*)kc, (const __bf16*)vtc, slot, pos, part_o, part_ml, counters,
                       (__bf16*)out, ldo, M, H, Hkv, T_max, nsplit, scale, kscale, vscale);
  else if (var == 2)
    hipLaunchKernelGGL((attn_decode_kernel<HD, AW, KV8, NT, true, 4>), dim3(M * Hkv, nsplit), dim3(AW * 64), 0,
                       st, (const __bf16*)q, (const __bf16*)kc, (const __bf16*)vtc, slot, pos, part_o, part_ml,
                       counters, (__bf16*)out, ldo, M, H, Hkv, T_max, nsplit, scale, kscale, vscale);
  else
    hipLaunchKernelGGL((attn_decode_kernel<HD, AW, KV8, NT>), dim3(M * Hkv, nsplit), dim3(AW * 64), 0, st,
                       (const __bf16*)q, (const __bf16*)kc, (const __bf16*)vtc, slot, pos, part_o, part_ml, counters,
                       (__bf16*)out, ldo, M, H, Hkv, T_max, nsplit, scale, kscale, vscale);
}

template <int HD, int AW>
static hipError_t launch_attn(const void* q, const void* kc, const void* vtc, const int* slot, const int* pos,
                              float* part_o, float* part_ml, unsigned* counters, void* out, int ldo, int M, int H,
                              int Hkv, int T_max, int nsplit, float scale, int kv8, float kscale, float vscale,
                              hipStream_t st) {
  const bool nt = attn_nt();
  if (kv8 && nt)
    launch_attn_t<HD, AW, true, true>(q, kc, vtc, slot, pos, part_o, part_ml, counters, out, ldo, M, H, Hkv, T_max,
                                      nsplit, scale, kscale, vscale, st);
  else if (kv8)
    launch_attn_t<HD, AW, true, false>(q, kc, vtc, slot, pos, part_o, part_ml, counters, out, ldo, M, H, Hkv, T_max,
                                       nsplit, scale, kscale, vscale, st);
  else if (nt)
    launch_attn_t<HD, AW, false, true>(q, kc, vtc, slot, pos, part_o, part_ml, counters, out, ldo, M, H, Hkv, T_max,
                                       nsplit, scale, 1.f, 1.f, st);
  else
    launch_attn_t<HD, AW, false, false>(q, kc, vtc, slot, pos, part_o, part_ml, counters, out, ldo, M, H, Hkv, T_max,
                                        nsplit, scale, 1.f, 1.f, st);
  return hipGetLastError();
}


// =====================================================================================================
// Wide decode attention on an LDS-DMA ring (LDS-staged KV tiles; the default wide body).
//
// One workgroup per CU, persistent over the (row, kv head) pairs: 4 compute waves, each owning whole pairs (pair
// blockIdx.x + (c + 4 i) * gridDim.x for compute wave c), so no cross-wave merge; and 4 loader waves, loader c
// streaming compute wave c's next 32-position block (K 2*hd/32 + V hd/16 fragments of 1 KiB = 16 KiB at hd 128,
// the fragment-major cache layout, so every piece is one lane-linear `global_load_lds_dwordx4 ... nt` and every
// fragment read a conflict-free `ds_read_b128`) into that wave's R-slot sub-ring.  One barrier per ring step for
// all 8 waves; the loader keeps R - 1 blocks per compute wave in flight across it (counted vmcnt), and a slot is
// refilled only after the barrier that follows its reads.  Both roles walk the same per-wave block schedule.
// Compute per block is the register kernel's (QK^T and PV on v_mfma_f32_16x16x32_bf16, online softmax).
// Why it might pay: the per-CU DMA stream reaches ~7 TB/s chip-wide with ~32-64 KiB in flight
// (tools/ingest_bench.hip), against ~6.0-6.5 TB/s for the register kernel's 16 waves of loads.
// =====================================================================================================
namespace ring {
constexpr int NC = 4;  // compute waves (= loader waves); the schedule's lane layout needs a power of two
constexpr int R = 2;   // ring slots per compute wave
constexpr int LMAX = 64 / NC;  // pairs per compute wave the lane-held schedule covers

// The workgroup's schedule, one list entry per lane, the same in every wave: lane l describes pair i = l / NC of
// compute wave w = l % NC, i.e. pair blockIdx.x + (w + NC i) * gridDim.x -- its cache slot, length (positions) and
// 32-position blocks.  Built by one parallel load of slot / pos per lane at the start; afterwards the cursors
// read it by lane index (readlane), so no global load sits in the loops.
struct Sched {
  int s, L, nb;
};
struct Cursor {
  int i;  // pair index within the wave's list (LMAX: done)
  int b;  // block within the pair
};
}  // namespace ring

template <int HD>
__global__ __launch_bounds__(64 * 2 * ring::NC, 1) void attn_ring_kernel(
    const __bf16* __restrict__ q, const __bf16* __restrict__ kc, const __bf16* __restrict__ vtc,
    const int* __restrict__ slot, const int* __restrict__ pos, __bf16* __restrict__ out, int ldo, int M, int H,
    int Hkv, int T_max, float scale) {
  using namespace ring;
  constexpr int NKS = HD / 32, NDT = HD / 16;
  constexpr int PIECES = 2 * NKS + NDT;
  constexpr int BLK = PIECES * 1024;  // bytes of one 32-position block (K then V fragments)
  extern __shared__ __attribute__((aligned(16))) char smem[];  // [NC][R][BLK]
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool loader = wave >= NC;
  const int c = loader ? wave - NC : wave;  // the compute wave this wave is, or feeds
  const int P = M * Hkv;
  const int G = H / Hkv;
  char* sub = smem + c * R * BLK;

  // ---- the lane-held schedule (host check: P <= 64 * gridDim.x, so LMAX entries per wave cover every pair)
  Sched me{-1, 0, 0};
  {
    const int pl = blockIdx.x + ((lane % NC) + NC * (lane / NC)) * gridDim.x;
    if (pl < P) {
      const int m = pl / Hkv;
      me.s = slot[m];
      me.L = pos[m] + 1;
      me.nb = me.s >= 0 ? (me.L + 31) >> 5 : 0;
    }
  }
  // steps = the longest of the NC compute waves' block totals
  int tot = me.nb;
#pragma unroll
  for (int o = NC; o < 64; o <<= 1) tot += __shfl_xor(tot, o, 64);
#pragma unroll
  for (int o = 1; o < NC; o <<= 1) tot = max(tot, __shfl_xor(tot, o, 64));
  const int steps = __builtin_amdgcn_readfirstlane(tot);
  auto pair_id = [&](int i) { return blockIdx.x + (c + NC * i) * gridDim.x; };
  auto entry_nb = [&](int i) { return __builtin_amdgcn_readlane(me.nb, c + NC * i); };
  auto live = [&](int i) { return i < LMAX && pair_id(i) < P; };
  // first pair with blocks at or after list index i (pairs with none get zero outputs from the compute wave)
  auto seek = [&](Cursor& k) {
    while (live(k.i) && entry_nb(k.i) == 0) ++k.i;
    if (!live(k.i)) k.i = LMAX;
    k.b = 0;
  };
  auto advance = [&](Cursor& k) {
    if (++k.b == entry_nb(k.i)) {
      ++k.i;
      seek(k);
    }
  };
  Cursor cur{0, 0};
  seek(cur);

  if (loader) {
    auto issue = [&](const Cursor& k, int n) {  // the block under cursor k into slot n % R
      const int p = pair_id(k.i), m = p / Hkv, kh = p - m * Hkv;
      const int s = __builtin_amdgcn_readlane(me.s, c + NC * k.i);
      const char* kb = reinterpret_cast<const char*>(kc) + ((size_t)s * Hkv + kh) * T_max * HD * 2 +
                       (size_t)k.b * (2 * NKS * 1024) + lane * 16;
      const char* vb = reinterpret_cast<const char*>(vtc) + ((size_t)s * Hkv + kh) * HD * T_max * 2 +
                       (size_t)k.b * (NDT * 1024) + lane * 16;
      char* dst = sub + (n % R) * BLK;
#pragma unroll
      for (int j = 0; j < 2 * NKS; ++j) wg::glds16(kb + j * 1024, dst + j * 1024, 1);
#pragma unroll
      for (int j = 0; j < NDT; ++j) wg::glds16(vb + j * 1024, dst + (2 * NKS + j) * 1024, 1);
    };
    Cursor ahead = cur;
    auto issue_next = [&](int n) {
      if (ahead.i < LMAX) {
        issue(ahead, n);
        advance(ahead);
      }
    };
    issue_next(0);
    for (int st = 0; st < steps; ++st) {
      wg::wait_vmcnt<0>();  // R = 2: block st is the only one outstanding
      wg::ring_barrier();
      issue_next(st + 1);
    }
    return;
  }

  // ---- compute wave c
  const int g = lane & 15, hq = lane >> 4;
  const float sl2 = scale * LOG2E;
  bf16x8 qf[NKS];
  float m_run = -INFINITY, l_run = 0.f;
  f32x4 o[NDT];
  int written = 0;  // pairs of this wave's list with their output written (empty ones as zeros)
  auto zero_pairs_before = [&](int upto) {
    for (; written < upto && live(written); ++written) {
      const int p = pair_id(written), m = p / Hkv, kh = p - m * Hkv;
      for (int e = lane; e < G * HD; e += 64) out[(size_t)m * ldo + kh * G * HD + e] = f2bf(0.f);
    }
  };
  // q of the wave's next pair, requested a block ahead (a pair's start no longer waits for a global load while the
  // other waves wait at the next barrier); lanes of columns g >= G are zeroed when it is taken
  const bool gvalid = g < G;
  bf16x8 qn[NKS];
  auto load_q = [&](int i) {
    const int p = pair_id(i), m = p / Hkv, kh = p - m * Hkv;
    const __bf16* qrow = q + ((size_t)m * H + kh * G + (gvalid ? g : 0)) * HD + hq * 8;
#pragma unroll
    for (int k = 0; k < NKS; ++k) qn[k] = *reinterpret_cast<const bf16x8*>(qrow + k * 32);
  };
  if (cur.i < LMAX) load_q(cur.i);
  for (int st = 0; st < steps; ++st) {
    wg::ring_barrier();
    if (cur.i >= LMAX) continue;
    const int p = pair_id(cur.i), m = p / Hkv, kh = p - m * Hkv;
    const int L = __builtin_amdgcn_readlane(me.L, c + NC * cur.i);
    const int nb = entry_nb(cur.i);
    if (cur.b == 0) {
      zero_pairs_before(cur.i);
#pragma unroll
      for (int i = 0; i < NKS; ++i) {
        bf16x8 v = qn[i];
        if (!gvalid) {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = f2bf(0.f);
        }
        qf[i] = v;
      }
      m_run = -INFINITY, l_run = 0.f;
#pragma unroll
      for (int i = 0; i < NDT; ++i) o[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    if (cur.b == max(nb - 2, 0)) {
      Cursor nx = cur;
      nx.b = nb - 1;
      advance(nx);
      if (nx.i < LMAX) load_q(nx.i);
    }
    const char* blk = sub + (st % R) * BLK + lane * 16;
    bf16x8 ka[NKS], kb[NKS];
#pragma unroll
    for (int i = 0; i < NKS; ++i) {
      ka[i] = *reinterpret_cast<const bf16x8*>(blk + i * 1024);
      kb[i] = *reinterpret_cast<const bf16x8*>(blk + (NKS + i) * 1024);
    }
    f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < NKS; ++i) {
      s0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ka[i], qf[i], s0, 0, 0, 0);
      s1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kb[i], qf[i], s1, 0, 0, 0);
    }
    bf16x8 va[NDT];
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) va[dt] = *reinterpret_cast<const bf16x8*>(blk + (2 * NKS + dt) * 1024);
    const int t0 = cur.b * 32;
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
      const float pa = exp2f(s0[r] - m_new), pb = exp2f(s1[r] - m_new);
      psum += pa + pb;
      pf[r] = f2bf(pa);
      pf[4 + r] = f2bf(pb);
    }
    l_run = l_run * alpha + psum;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
      o[dt] *= alpha;
      o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va[dt], pf, o[dt], 0, 0, 0);
    }
    if (cur.b == nb - 1) {  // pair done: normalise and store O (lane (g, hq) holds d = 16 dt + 4 hq + r)
      float l = l_run + __shfl_xor(l_run, 16, 64);
      l += __shfl_xor(l, 32, 64);
      const float inv = l > 0.f ? fast_rcp(l) : 0.f;
      if (g < G) {
        __bf16* dst = out + (size_t)m * ldo + (kh * G + g) * HD + hq * 4;
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) {
          bf16x4 v;
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = f2bf(o[dt][r] * inv);
          *reinterpret_cast<bf16x4*>(dst + dt * 16) = v;
        }
      }
      written = cur.i + 1;
    }
    advance(cur);
  }
  zero_pairs_before(LMAX);
}

static int g_attn_ring = -1;
CAIN_API void cain_attention_set_ring(int on) { g_attn_ring = on; }


// Workspace: part_o M*H*nsplit*hd floats, part_ml M*Hkv*align32(G*nsplit*2) floats, counters M*Hkv uints
// (zeroed once; the reducer resets them).  kv8: the caches hold e4m3 elements (value = element * k/vscale).
CAIN_API int cain_attention_ex(const void* q, const void* kc, const void* vtc, const int* slot, const int* pos,
                               float* part_o, float* part_ml, unsigned* counters, void* out, int ldo, int M, int H,
                               int Hkv, int hd, int T_max, int nsplit, float scale, int kv8, float kscale,
                               float vscale, hipStream_t st) {
  if (H % Hkv || H / Hkv > 16 || T_max % 32 || nsplit < 1 || nsplit > 64 || M > 256) return -1;
  // LDS-DMA ring body (default for hd 128, bf16 cache, no position split, >= 2 pairs per CU;
  // cain_attention_set_ring(0) selects the register kernel).  Measured (profiles/r3/README.md, same box): 113.3 vs
  // 113.7 us at 256 rows x 700 positions, 217.8 vs 221.5 at 1400 (6.74 TB/s), 60.3 vs 58.6 at 350; in the
  // graph-replayed headline 27.44k vs 27.21-27.23k tok/s.  The 2 x 4 and 3 x 3 ring shapes measured slower and
  // were removed (profiles/r3/attn_ring_isolated.log).
  if (g_attn_ring < 0) g_attn_ring = 1;
  const int n_cu = cain_cu_budget();
  if (g_attn_ring && hd == 128 && !kv8 && nsplit == 1 && n_cu > 0 && M * Hkv >= 2 * n_cu &&
      M * Hkv <= ring::LMAX * ring::NC * n_cu) {
    constexpr int lds = ring::NC * ring::R * 16 * 1024;
    static const bool attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&attn_ring_kernel<128>),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, lds) == hipSuccess;
    if (!attr) return int(hipErrorInvalidConfiguration);
    hipLaunchKernelGGL((attn_ring_kernel<128>), dim3(n_cu), dim3(64 * 2 * ring::NC), lds, st, (const __bf16*)q,
                       (const __bf16*)kc, (const __bf16*)vtc, slot, pos, (__bf16*)out, ldo, M, H, Hkv, T_max, scale);
    return int(hipGetLastError());
  }
  // 8-wave workgroups for few (row, kv head) pairs (hd <= 128: the hd-256 body needs one wave per SIMD)
  const bool wide = M * Hkv <= 64;
#define CAIN_ATTN_CASE(HDV)                                                                                        \
  case HDV:                                                                                                      \
    return wide ? int(launch_attn<HDV, 8>(q, kc, vtc, slot, pos, part_o, part_ml, counters, out, ldo, M, H, Hkv,  \
                                          T_max, nsplit, scale, kv8, kscale, vscale, st))                        \
                : int(launch_attn<HDV, 4>(q, kc, vtc, slot, pos, part_o, part_ml, counters, out, ldo, M, H, Hkv,  \
                                          T_max, nsplit, scale, kv8, kscale, vscale, st));
  switch (hd) {
    CAIN_ATTN_CASE(64)
    CAIN_ATTN_CASE(96)
    CAIN_ATTN_CASE(128)
    case 256:
      return int(launch_attn<256, 4>(q, kc, vtc, slot, pos, part_o, part_ml, counters, out, ldo, M, H, Hkv, T_max,
                                     nsplit, scale, kv8, kscale, vscale, st));
    default: return -1;
  }
#undef CAIN_ATTN_CASE
}

CAIN_API int cain_attention(const void* q, const void* kc, const void* vtc, const int* slot, const int* pos,
                            float* part_o, float* part_ml, unsigned* counters, void* out, int ldo, int M, int H,
                            int Hkv, int hd, int T_max, int nsplit, float scale, hipStream_t st) {
  return cain_attention_ex(q, kc, vtc, slot, pos, part_o, part_ml, counters, out, ldo, M, H, Hkv, hd, T_max, nsplit,
                           scale, 0, 1.f, 1.f, st);
}
