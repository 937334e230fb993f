// Layer front for few-row decode (M <= 4 rows: the single-stream protocol of the reference study and small
// continuous batches): QKV projection -> attention -> O projection of one layer in ONE launch.
//
// At one row the three ops are latency-bound, not bandwidth-bound: qwen2:1.5b's QKV moves 6.3 MB in ~5 us, its
// attention 0.7 MB in ~8 us, its O projection 4.7 MB in ~4.7 us, each behind a ~1.5 us kernel boundary, and each
// starts by waiting for its first HBM round trip (profiles/r3/prof_b1_*).  The bytes of the later ops do not
// depend on the earlier ones -- the KV cache of the positions already decoded and the O weights are known before
// the step starts -- so here the workgroups of all three ops are resident together and the later ones PREFETCH
// their bytes into registers while the earlier ones compute; only the small data-dependent pieces (q, the new
// position's K/V, the attention output) wait:
//
//   role QKV  (blocks [0, n_qkv)):            one 16-row tile of W_qkv per workgroup, 8 waves split K; fused
//                                             RMSNorm, bias, RoPE, K/V append (gemm_epi.h EPI_QKV_ROPE) with
//                                             write-through stores; then sets its own tile flag
//   role ATT  ([n_qkv, n_qkv + n_att)):       one (row, kv head, position split) per workgroup, one 32-position
//                                             block per wave: blocks of past positions are loaded BEFORE waiting
//                                             for the flags of the q / K / V tiles of its kv head; then q and the
//                                             block holding the new position (sc1
//                                             loads), both products on MFMA, in-register online softmax, LDS merge
//                                             of the waves, last-arriver merge of the splits (attention.hip's
//                                             scheme); the output row goes out write-through, then flags[1]
//   role O    ([n_qkv + n_att, ...)):         one 16-row tile of W_o per workgroup: all of its weight fragments are
//                                             loaded BEFORE waiting for flags[1]; then the attention output (sc1
//                                             loads), MFMA, LDS reduce, residual epilogue into x; the last O
//                                             workgroup resets the flags for the next launch
//
// Hand-offs follow MI355X_MICROARCH.md's first 'Valid forms' row: every byte another workgroup of this launch
// reads is stored write-through (sc1) and loaded with sc1 loads; each producer drains its stores (vmcnt(0)) and
// one lane then adds to the counter; consumers poll it with relaxed agent loads.  Only workgroups of the two
// consumer roles ever wait, and they never wait on their own role; the producer role (QKV) comes first in block
// order and never waits, so as long as the consumers (<= 64 + d/16 workgroups) fit beside one resident QKV
// workgroup the launch makes progress; every spin is bounded all the same.  Replaces the QKV / attention / O
// launches of runtime.hip for M <= 4 on bf16 weights and bf16 caches with head_dim <= 128 (SURVEY §2.4 rows QKV,
// RoPE, KV append, decode attention, O projection; reference workload: experiment/RunnerConfig.py:128-131).
#include "common.h"
#include "gemm_epi.h"

namespace front {

constexpr int W = 8;          // waves per workgroup (every role)
constexpr int NTHR = W * 64;
constexpr int U = 4;          // slices per load group (QKV role pipeline)
constexpr int OPF = 16;       // O role: weight fragments per wave prefetched (K <= 16 * 8 * 32 = 4096)
constexpr int NSPLIT_MAX = 8; // attention splits per (row, kv head)
constexpr float LOG2E = 1.4426950408889634f;
constexpr int SPIN_MAX = 1 << 22;  // bounded waits (a few hundred ms): never a hang
constexpr int FL_ATT = 0, FL_O = 1, FL_TILE = 64;
constexpr int MAX_TILES = 4096 - FL_TILE;  // flags buffer: 4096 words

struct Args {
  GemmArgs qkv;   // EPI_QKV_ROPE (+NORM), X = residual x, Y = q buffer, caches in kc / vtc
  GemmArgs o;     // EPI_RESID, X = attention output, Y = x (residual, in place)
  float* part_o;  // attention split partials (attention.hip layout)
  float* part_ml;
  unsigned* att_ctr;  // [M * Hkv] split tickets, zero at rest
  __bf16* attn;       // [M][H * hd] attention output (the O role's X)
  int nsplit;
  float scale;
  int n_qkv, n_att, n_o;
  // [FL_ATT] (row, kv head) groups done, [FL_O] O workgroups done, [FL_TILE + t] QKV tile t done; zero at rest
  unsigned* flags;
  unsigned long long* trace;  // optional [grid][4] timestamps (s_memrealtime, 100 MHz): start, wait begin, wait end, end
};

__device__ __forceinline__ void stamp(const Args& A, int i) {
  if (A.trace && threadIdx.x == 0) A.trace[blockIdx.x * 4 + i] = __builtin_amdgcn_s_memrealtime();
}

__device__ __forceinline__ void spin_until(const unsigned* f, unsigned target) {
  for (int it = 0; it < SPIN_MAX; ++it) {
    if (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) return;
    __builtin_amdgcn_s_sleep(2);
  }
}

// every storing wave drains, then one lane arrives (the producer side of the hand-off)
__device__ __forceinline__ void arrive(unsigned* f) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(f, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// 16-byte write-through-coherent load (sc1: served from the memory side, never a stale cache line)
__device__ __forceinline__ bf16x8 ld_sc1_16(const void* base, int byte_off) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
  return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 16));
}

// ---- cross-wave reduction of a 16x16 accumulator unit through LDS and the fused epilogue (wave 0)
template <int EPI, bool NORM, bool WT>
__device__ void gemv_finish(const GemmArgs& a, int tile, const f32x4& acc, float ssq, float* lds, const EpiIn& e) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  f32x4* red = reinterpret_cast<f32x4*>(lds);           // [W][64]
  float* red_ss = lds + W * 64 * 4;                     // [W][16]
  red[wave * 64 + lane] = acc;
  if constexpr (NORM) {
    float v = ssq;
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    if (lane < 16) red_ss[wave * 16 + lane] = v;
  }
  __syncthreads();
  if (wave == 0) {
    epi_store<EPI, WT>(a, tile, lane & 15, lane, e, [&](int off) {
      const int u = lane + off;
      f32x4 v = red[u];
#pragma unroll
      for (int w = 1; w < W; ++w) v += red[w * 64 + u];
      if constexpr (NORM) {
        float ss = 0.f;
#pragma unroll
        for (int w = 0; w < W; ++w) ss += red_ss[w * 16 + (u & 15)];
        v *= rms_inv(ss, a.K, a.eps);
      }
      return v;
    });
  }
}

// ---- role QKV: one tile, 8 waves split K, pipelined groups of U slices (two register sets)
template <bool NORM>
__device__ void role_qkv(const Args& A, int tile, float* lds) {
  const GemmArgs& a = A.qkv;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int KS = a.K >> 5;
  const int s_beg = (wave * KS) / W, s_end = ((wave + 1) * KS) / W;
  const bf16x8* wb = a.Wp + (size_t)tile * KS * 64 + lane;
  const __bf16* xb = a.X + (size_t)min(lane & 15, a.M - 1) * a.ldx + ((lane >> 4) << 3);
  // epilogue inputs (bias, RoPE tables, slot / position) in flight under the weight stream
  const EpiIn e = wave == 0 ? epi_load_at<EPI_QKV_ROPE>(a, tile, lane & 15, lane) : EpiIn{};
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  float ssq = 0.f;
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  auto mac = [&](const bf16x8& w, const bf16x8& x, bool valid) {
    if constexpr (NORM) {
      float q = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) q += bf2f(x[j]) * bf2f(x[j]);
      ssq += valid ? q : 0.f;
    }
    const bf16x8 wm = __builtin_bit_cast(bf16x8, __builtin_bit_cast(u32x4, w) & (valid ? 0xffffffffu : 0u));
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wm, x, acc, 0, 0, 0);
  };
  const int n = s_end - s_beg;
  if (n > 0) {
    bf16x8 wa[U], xa[U], wc[U], xc[U];
    auto load = [&](int g, bf16x8 (&w)[U], bf16x8 (&x)[U]) {
#pragma unroll
      for (int u = 0; u < U; ++u) {  // clamped (unconditional) loads; the surplus is masked in mac
        const int s = s_beg + min(g * U + u, n - 1);
        w[u] = __builtin_nontemporal_load(wb + (size_t)s * 64);
        x[u] = *reinterpret_cast<const bf16x8*>(xb + s * 32);
      }
    };
    const int ng = (n + U - 1) / U;
    load(0, wa, xa);
    for (int g = 0; g < ng; g += 2) {
      load(min(g + 1, ng - 1), wc, xc);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < U; ++u) mac(wa[u], xa[u], g * U + u < n);
      load(min(g + 2, ng - 1), wa, xa);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < U; ++u) mac(wc[u], xc[u], g + 1 < ng && (g + 1) * U + u < n);
    }
  }
  stamp(A, 1);
  stamp(A, 2);
  gemv_finish<EPI_QKV_ROPE, NORM, true>(a, tile, acc, ssq, lds, e);
  // every storing wave drains its write-through stores, then one lane sets this tile's flag (sc1 store)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(A.flags + FL_TILE + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---- role O: all of the wave's weight fragments prefetched before the wait, then the attention output
__device__ void role_o(const Args& A, int tile, float* lds, unsigned att_groups) {
  const GemmArgs& a = A.o;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int KS = a.K >> 5;
  const int s_beg = (wave * KS) / W, s_end = ((wave + 1) * KS) / W;
  const int n = s_end - s_beg;  // <= OPF (host-checked)
  const bf16x8* wb = a.Wp + (size_t)tile * KS * 64 + lane;
  bf16x8 wp[OPF];
#pragma unroll
  for (int u = 0; u < OPF; ++u) wp[u] = __builtin_nontemporal_load(wb + (size_t)(s_beg + min(u, max(n - 1, 0))) * 64);
  // the residual rows (not written by this launch before this epilogue)
  const EpiIn e = wave == 0 ? epi_load_at<EPI_RESID>(a, tile, lane & 15, lane) : EpiIn{};
  stamp(A, 1);
  if (threadIdx.x == 0) spin_until(A.flags + FL_ATT, att_groups);
  __syncthreads();
  stamp(A, 2);
  const int xoff = (min(lane & 15, a.M - 1) * a.ldx + ((lane >> 4) << 3)) * 2;  // bytes
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
  for (int g = 0; g < OPF; g += U) {
    bf16x8 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] = ld_sc1_16(a.X, xoff + (s_beg + min(g + u, max(n - 1, 0))) * 64);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool valid = g + u < n;
      const bf16x8 wm = __builtin_bit_cast(bf16x8, __builtin_bit_cast(u32x4, wp[g + u]) & (valid ? 0xffffffffu : 0u));
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wm, x[u], acc, 0, 0, 0);
    }
  }
  gemv_finish<EPI_RESID, false, false>(a, tile, acc, 0.f, lds, e);
  // the last O workgroup resets the flags: every consumer has passed its wait by then (each attention workgroup
  // polled its tile flags before its group could arrive, all groups arrived before any O workgroup got past its
  // wait, and every O workgroup takes this ticket after its own wait)
  __syncthreads();
  unsigned* s_last = reinterpret_cast<unsigned*>(lds);
  if (threadIdx.x == 0)
    *s_last = __hip_atomic_fetch_add(A.flags + FL_O, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
              unsigned(A.n_o - 1);
  __syncthreads();
  if (*s_last) {
    for (int i = threadIdx.x; i < FL_TILE + A.n_qkv; i += NTHR)
      __hip_atomic_store(A.flags + i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ---- role ATT: (row m, kv head kh, split sp); one block of 32 positions per wave per round
template <int HD>
__device__ void role_att(const Args& A, int unit, float* lds) {
  constexpr int NKS = HD / 32, NDT = HD / 16;
  const GemmArgs& a = A.qkv;  // H, Hkv, T_max, slot, pos, caches
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int Hkv = a.Hkv, H = a.H, G = H / Hkv, nsplit = A.nsplit;
  const int mk = unit / nsplit, sp = unit - (unit / nsplit) * nsplit;
  const int m = mk / Hkv, kh = mk - (mk / Hkv) * Hkv;
  const int g = lane & 15, hq = lane >> 4;
  const int s = a.slot[m];
  const int T = a.pos[m];              // the new position (its K / V are written by the QKV role)
  const int L = (s >= 0) ? T + 1 : 0;
  const int nblk = (L + 31) >> 5;
  const int bps = (nblk + nsplit - 1) / nsplit;
  const int b0 = sp * bps, b1 = min(nblk, b0 + bps);
  // blocks that may hold a position written by this launch: this row's own, and (prefill rows of one sequence)
  // up to M - 1 earlier ones; only blocks below them are prefetched before the wait
  const int fresh_lo = max(T - (a.M - 1), 0) >> 5;
  const char* kbase = reinterpret_cast<const char*>(a.kc) + (((size_t)max(s, 0) * Hkv + kh) * a.T_max * HD) * 2;
  const char* vbase = reinterpret_cast<const char*>(a.vtc) + (((size_t)max(s, 0) * Hkv + kh) * HD * a.T_max) * 2;
  auto blk_k = [&](int blk, int i) { return (blk * (2 * NKS) + i) * 1024 + lane * 16; };
  auto blk_v = [&](int blk, int dt) { return (blk * NDT + dt) * 1024 + lane * 16; };

  // prefetch the wave's first block if it holds past positions only (it does not depend on this step)
  int blk = b0 + wave;
  bf16x8 ka[NKS], kb[NKS], va[NDT];
  const bool pre = blk < b1 && blk < fresh_lo;
  if (pre) {
#pragma unroll
    for (int i = 0; i < NKS; ++i) {
      ka[i] = __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(kbase + blk_k(blk, i)));
      kb[i] = __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(kbase + blk_k(blk, NKS + i)));
    }
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) va[dt] = __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(vbase + blk_v(blk, dt)));
  }
  stamp(A, 1);
  // the last wave polls the flags of the q tiles of heads kh*G.. and of the K / V tiles of head kh (the last wave:
  // the one least likely to hold a prefetch, which its first poll would wait for -- loads retire in order)
  if (wave == W - 1) {
    const int tph = HD / 16, nt = (G + 2) * tph;
    for (int it = 0; it < SPIN_MAX; ++it) {
      bool ok = true;
      for (int i = lane; i < nt; i += 64) {
        const int t = i < G * tph ? kh * G * tph + i
                                  : (i < (G + 1) * tph ? (H + kh) * tph + i - G * tph : (H + Hkv + kh) * tph + i - (G + 1) * tph);
        ok &= __hip_atomic_load(A.flags + FL_TILE + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
      }
      if (__all(ok)) break;
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  stamp(A, 2);

  float m_run = -INFINITY, l_run = 0.f;
  f32x4 o[NDT];
#pragma unroll
  for (int i = 0; i < NDT; ++i) o[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (blk < b1) {
    bf16x8 qf[NKS];
    const bool gvalid = g < G;
    const int qoff = (((m * H + kh * G + (gvalid ? g : 0)) * HD) + hq * 8) * 2;
#pragma unroll
    for (int i = 0; i < NKS; ++i) {
      bf16x8 v = ld_sc1_16(A.qkv.Y, qoff + i * 64);
      if (!gvalid) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = f2bf(0.f);
      }
      qf[i] = v;
    }
    const float sl2 = A.scale * LOG2E;
    for (bool first = true; blk < b1; blk += W, first = false) {
      if (!(first && pre)) {  // the new position's block (written this launch) or a later round: sc1 loads
#pragma unroll
        for (int i = 0; i < NKS; ++i) {
          ka[i] = ld_sc1_16(kbase, blk_k(blk, i));
          kb[i] = ld_sc1_16(kbase, blk_k(blk, NKS + i));
        }
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) va[dt] = ld_sc1_16(vbase, blk_v(blk, dt));
      }
      const int t0 = blk * 32;
      f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < NKS; ++i) {
        s0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ka[i], qf[i], s0, 0, 0, 0);
        s1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kb[i], qf[i], s1, 0, 0, 0);
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
    }
  }
  l_run += __shfl_xor(l_run, 16, 64);
  l_run += __shfl_xor(l_run, 32, 64);

  // ---- merge the waves in LDS: s_m / s_l [W][16], s_o [W][HD][16]
  float* s_m = lds;
  float* s_l = s_m + W * 16;
  float* s_o = s_l + W * 16;
  unsigned* s_ticket = reinterpret_cast<unsigned*>(s_o + W * HD * 16);
  if (hq == 0) {
    s_m[wave * 16 + g] = m_run;
    s_l[wave * 16 + g] = l_run;
  }
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
    for (int r = 0; r < 4; ++r) s_o[(wave * HD + dt * 16 + hq * 4 + r) * 16 + g] = o[dt][r];
  __syncthreads();
  const int nout4 = G * HD / 4;
  const int ldo = H * HD;
  const size_t pbase = (size_t)(m * H + kh * G) * nsplit;
  const int mls = ((G * nsplit * 2 + 31) / 32) * 32;
  float* pml = A.part_ml + (size_t)mk * mls;
  const __amdgpu_buffer_rsrc_t rpo = slab_rsrc(A.part_o);
  for (int e = threadIdx.x; e < nout4; e += NTHR) {
    const int gg = (e * 4) / HD, d0 = e * 4 - gg * HD;
    float Mx = -INFINITY;
#pragma unroll
    for (int w = 0; w < W; ++w) Mx = fmaxf(Mx, s_m[w * 16 + gg]);
    float lsum = 0.f;
    f32x4 osum = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int w = 0; w < W; ++w) {
      const float mw = s_m[w * 16 + gg];
      if (mw == -INFINITY) continue;
      const float f = exp2f(mw - Mx);
      lsum += f * s_l[w * 16 + gg];
#pragma unroll
      for (int i = 0; i < 4; ++i) osum[i] += f * s_o[(w * HD + d0 + i) * 16 + gg];
    }
    if (nsplit == 1) {
      const float inv = lsum > 0.f ? 1.f / lsum : 0.f;
      bf16x4 ov;
#pragma unroll
      for (int i = 0; i < 4; ++i) ov[i] = f2bf(osum[i] * inv);
      st_epi<true>(A.attn + (size_t)m * ldo + (kh * G + gg) * HD + d0, ov);
    } else {
      const size_t pi = pbase + (size_t)gg * nsplit + sp;
      st_wt(rpo, int((pi * HD + d0) * 4), osum);
      if (d0 == 0) {
        const int li = gg * nsplit + sp;
        __hip_atomic_store(pml + li * 2 + 0, Mx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(pml + li * 2 + 1, lsum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  if (nsplit == 1) {
    arrive(A.flags + FL_ATT);
    return;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    *s_ticket = __hip_atomic_fetch_add(A.att_ctr + mk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  if (*s_ticket != unsigned(nsplit - 1)) return;
  // last arriver of (m, kh): merge the splits, write the output rows write-through, arrive.  The partial rows and
  // the (max, sum) pairs are requested together (sc1 loads, one round trip): <= NSPLIT_MAX partials per thread in
  // registers while the merge weights are formed in LDS
  float* s_w = s_o;  // [16][64] merge weights, reusing the wave merge area
  float* s_den = s_o + 16 * 64;
  const int nw = G * nsplit;
  const int e4 = threadIdx.x < nout4 ? threadIdx.x : 0;  // nout4 <= 16 * 128 / 4 = 512 = NTHR
  const int gg4 = (e4 * 4) / HD, d04 = e4 * 4 - gg4 * HD;
  const int po0 = int(((pbase + (size_t)gg4 * nsplit) * HD + d04) * 4);  // bytes
  f32x4 pv[NSPLIT_MAX];
#pragma unroll
  for (int j = 0; j < NSPLIT_MAX; ++j) pv[j] = ld_wt(rpo, po0 + min(j, nsplit - 1) * HD * 4);
  for (int e = threadIdx.x; e < nw; e += NTHR) {
    const int gg = e / nsplit, j = e - (e / nsplit) * nsplit;
    s_w[gg * 64 + j] = __hip_atomic_load(pml + e * 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_den[gg * 64 + j] = __hip_atomic_load(pml + e * 2 + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
      den += f * s_den[gg * 64 + j];
    }
    s_l[gg] = den > 0.f ? 1.f / den : 0.f;
  }
  if (threadIdx.x == 0) A.att_ctr[mk] = 0u;  // ready for the next launch (launch-ordered)
  __syncthreads();
  if (threadIdx.x < nout4) {
    f32x4 num = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < NSPLIT_MAX; ++j)
      if (j < nsplit) num += s_w[gg4 * 64 + j] * pv[j];
    bf16x4 ov;
#pragma unroll
    for (int i = 0; i < 4; ++i) ov[i] = f2bf(num[i] * s_l[gg4]);
    st_epi<true>(A.attn + (size_t)m * ldo + (kh * G + gg4) * HD + d04, ov);
  }
  arrive(A.flags + FL_ATT);
}

// LDS: the attention role's wave merge is the largest user (W x HD x 16 floats + W x 32 + a ticket)
template <int HD>
constexpr int lds_floats() {
  return W * 16 * 2 + W * HD * 16 + 4;
}

template <int HD, bool NORM>
__global__ __launch_bounds__(NTHR, 2) void front_kernel(const Args A) {
  __shared__ __attribute__((aligned(16))) float lds[lds_floats<HD>()];
  const int b = blockIdx.x;
  stamp(A, 0);
  if (b < A.n_qkv) {
    role_qkv<NORM>(A, b, lds);
  } else if (b < A.n_qkv + A.n_att) {
    role_att<HD>(A, b - A.n_qkv, lds);
  } else {
    role_o(A, b - A.n_qkv - A.n_att, lds, unsigned(A.qkv.M * A.qkv.Hkv));
  }
  stamp(A, 3);
}

}  // namespace front

// Eligible shapes: <= 4 rows, bf16 weights and caches, head_dim 64 / 96 / 128, the O projection's whole K covered
// by the 8 waves' register prefetch (q_dim <= 4096), <= 8 attention splits and <= 64 attention workgroups.
CAIN_API int cain_front_eligible(int M, int d, int q_dim, int hd, int H, int Hkv, int nsplit, int kv8) {
  if (M < 1 || M > 4 || kv8) return 0;
  if (hd != 64 && hd != 96 && hd != 128) return 0;
  if (d % 32 || q_dim % 32) return 0;
  if (q_dim / 32 > front::OPF * front::W) return 0;
  if (Hkv < 1 || H % Hkv || H / Hkv > 16 || nsplit < 1 || nsplit > front::NSPLIT_MAX || M * Hkv * nsplit > 64)
    return 0;
  if ((H + 2 * Hkv) * hd / 16 > front::MAX_TILES) return 0;
  return 1;
}

// One launch for QKV (+RMSNorm, bias, RoPE, KV append) -> attention -> O (+residual) of a layer.  Same operands
// as the three launches it replaces (runtime.hip forward): wqkv / wo packed bf16 (gemm.hip layout), x the residual
// stream [M][d] (read by QKV, updated in place by O), q [M][q_dim], attn [M][q_dim], part_o / part_ml / att_ctr
// the attention split workspace (att_ctr zero at rest), flags 4096 zeroed words (zero again when the launch ends).
CAIN_API int cain_front(const void* wqkv, const float* bqkv, const void* wo, void* x, void* q, void* attn,
                        void* kc, void* vtc, const int* slot, const int* pos, const float* cos_t, const float* sin_t,
                        int M, int d, int H, int Hkv, int hd, int T_max, float eps, int norm, float* part_o,
                        float* part_ml, unsigned* att_ctr, int nsplit, float scale, unsigned* flags,
                        unsigned long long* trace, hipStream_t st) {
  const int q_dim = H * hd, qkv_dim = (H + 2 * Hkv) * hd;
  if (!cain_front_eligible(M, d, q_dim, hd, H, Hkv, nsplit, 0) || T_max % 32) return -1;
  front::Args A{};
  GemmArgs& g = A.qkv;
  g.Wp = static_cast<const bf16x8*>(wqkv), g.X = static_cast<const __bf16*>(x), g.ldx = d, g.K = d;
  g.N = qkv_dim, g.M = M, g.msplit = 1, g.Y = q, g.ldy = q_dim, g.bias = bqkv, g.eps = eps;
  g.slot = slot, g.pos = pos, g.cos_t = cos_t, g.sin_t = sin_t;
  g.kc = static_cast<__bf16*>(kc), g.vtc = static_cast<__bf16*>(vtc);
  g.H = H, g.Hkv = Hkv, g.hd = hd, g.T_max = T_max, g.kv8 = 0;
  GemmArgs& o = A.o;
  o.Wp = static_cast<const bf16x8*>(wo), o.X = static_cast<const __bf16*>(attn), o.ldx = q_dim, o.K = q_dim;
  o.N = d, o.M = M, o.msplit = 1, o.Y = x, o.ldy = d;
  o.H = H, o.Hkv = Hkv, o.hd = hd, o.T_max = T_max;
  A.part_o = part_o, A.part_ml = part_ml, A.att_ctr = att_ctr;
  A.attn = static_cast<__bf16*>(attn);
  A.nsplit = nsplit, A.scale = scale, A.flags = flags, A.trace = trace;
  A.n_qkv = qkv_dim / 16;
  A.n_att = M * Hkv * nsplit;
  A.n_o = d / 16;
  const dim3 grid(A.n_qkv + A.n_att + A.n_o), blk(front::NTHR);
#define CAIN_FRONT_CASE(HDV)                                                                 \
  case HDV:                                                                                  \
    if (norm) hipLaunchKernelGGL((front::front_kernel<HDV, true>), grid, blk, 0, st, A);    \
    else hipLaunchKernelGGL((front::front_kernel<HDV, false>), grid, blk, 0, st, A);        \
    break;
  switch (hd) {
    CAIN_FRONT_CASE(64)
    CAIN_FRONT_CASE(96)
    CAIN_FRONT_CASE(128)
    default: return -1;
  }
#undef CAIN_FRONT_CASE
  return int(hipGetLastError());
}
