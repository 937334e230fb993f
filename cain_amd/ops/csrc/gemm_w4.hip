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
// Two kernels.  The single-stream one (w4_stream_kernel, rows <= 16 whose activations fit the LDS copy) is a
// persistent stream: a grid of G <= (CUs x workgroups per CU) workgroups; workgroup b takes the
// (16-row tile, 16*NB-row M block) pairs b, b + G, b + 2G, ...  Its WAVES waves deal every tile's k quads among
// themselves (wave w: quads w, w + WAVES, ...) and walk ONE flattened sequence of (pair, quad) items with U items
// of weight loads in flight in a register ring, across tile boundaries: while a tile's last quads are multiplied
// the next tile's weights are already streaming, so a workgroup never drains its loads at a tile edge (a one-tile
// workgroup did: the few-row fp4 tiles are only 32 KiB at K = 4096).  At each tile edge the waves drop their
// 16x16 partials into a double-buffered LDS slab, one raw barrier, and wave 0 runs the fused epilogue while the
// others go on.  The activation rows (XL: M x K <= 32 KiB) are staged into LDS once per workgroup by plain loads
// issued ahead of the weight prologue (the compiler counts both load streams, so nothing drains early); the
// RMSNorm sums of squares are taken once per workgroup from that LDS copy, one wave per row in a fixed order (8
// VALU ops per MFMA when taken from every activation fragment: +2-4 us per GEMM, profiles/r4/).
// Wider problems (w4_tile_kernel: up to 64 rows, or activation rows beyond the LDS copy) run one workgroup per
// (tile, 16*NB-row block) with the activation fragments loaded beside each weight quad.
#include <algorithm>

#include "common.h"
#include "gemm_epi.h"

typedef uint32_t w4u32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 w4bf16x2 __attribute__((ext_vector_type(2)));

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

__device__ __forceinline__ void w4_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// pair j -> (16-row tile, M block): the M blocks of one tile get ids 8 apart (the same XCD's L2 under round-robin
// dispatch when the grid is a multiple of 8; any placement is correct)
__device__ __forceinline__ void w4_pair_tile(int j, int msp, int ntg, int& t, int& ms) {
  if (msp == 1) {
    t = j, ms = 0;
  } else if ((ntg & 7) == 0) {
    const int r = j >> 3;
    ms = r % msp;
    t = (r / msp) * 8 + (j & 7);
  } else {
    t = j / msp, ms = j - (j / msp) * msp;
  }
}

// ================================================================ single stream: persistent, activations in LDS
// LDS copy of the activation rows: 48 KiB for 8-wave workgroups (2 per CU), 28 KiB for 4-wave ones (4 per CU) --
// every real model's down projection (K <= 24576) fits at one row
template <int WAVES>
constexpr int w4_xl_bytes() { return WAVES == 8 ? 49152 : 28672; }

// Split-K of the stream kernel for narrow outputs (fewer 16-row tiles than CUs: the small models' O and down
// projections, 96-128 tiles, left half the chip idle): pair j = (tile j / ks, k range j % ks).  Wave 0 of each pair
// publishes its 16x16 partial write-through (sc1) and, after its stores drain, takes the tile's ticket with one
// agent-scope atomic add; the LAST arriving pair sums the ks partials with sc1 loads, applies the RMSNorm factor and
// runs the tile's epilogue, and resets the ticket (cdna_hip_programming.md 'In-launch split-K reduction'; the
// attention kernel's merge).  No workgroup ever waits for another.
struct W4Split {
  int ks;          // k ranges per tile (1: no split)
  float* part;     // [tiles * ks][64 lanes][4] fp32 partial blocks
  unsigned* ctr;   // [tiles] tickets, zero at rest
};
// The engine's GEMM workspace is shared by every weight format: [0, 64 KiB) holds the bf16 batched path's tickets and
// [64, 80 KiB) the wide path's counters, both zero at rest (gemm.hip GEMM_SLAB_OFFSET).  The W4 tickets (4,096 tiles)
// live in [0, 16 KiB) -- they too are zero at rest -- and the partials, which are not, start at 80 KiB as the other
// formats' slabs do (wgemm8.hip W8_SLAB_OFFSET), so a mixed-format forward never reads a partial as a ticket.
constexpr long long W4_CTR_BYTES = 16 * 1024;
constexpr long long W4_PART_OFFSET = 80 * 1024;

// 4 waves per SIMD (<= 128 VGPRs): the grid below assumes 16 resident waves per CU.
// SPLIT is a template parameter, not a runtime branch: with the split path compiled into every instance (round 5),
// hipcc lost the loop's counted waits -- 15-20 vmcnt(0) per kernel instead of 0-5, the steady-state ring drained at
// every item -- and MXFP4 batch-1 decode fell 5-13 % on all seven models (tests/test_isa_guard.py now
// checks the built code object).  Unsplit launches run the SPLIT = false instance, which compiles as before.
template <int WAVES, int U, int EPI, bool NORM, bool SPLIT>
__global__ __launch_bounds__(WAVES * 64) __attribute__((amdgpu_waves_per_eu(4, 4))) void w4_stream_kernel(
    const GemmArgs a, const uint8_t* __restrict__ wsc, int npairs, const W4Split sp) {
  constexpr int XLB = w4_xl_bytes<WAVES>();
  constexpr int XCH = XLB / (WAVES * 64 * 16);  // 16-byte activation chunks staged per thread
  __shared__ __attribute__((aligned(16))) char w4_xs[XLB];
  __shared__ __attribute__((aligned(16))) f32x4 red[2][WAVES][64];
  __shared__ float row_ss[16];  // NORM: the sum of squares of each activation row
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int KS = SPLIT ? sp.ks : 1;
  const int KQT = a.K >> 7;                   // 128-wide k quads per tile
  const int KQ = KQT / KS;                    // k quads per pair (the host keeps KQT % KS == 0)
  const int qmax = (KQ + WAVES - 1) / WAVES;  // items per pair (every wave walks the same sequence length)
  const int G = gridDim.x;
  const int my_tiles = (npairs - (int)blockIdx.x + G - 1) / G;
  const int n_items = my_tiles * qmax;
  constexpr int R = U + 1;                      // ring slots: U items in flight + the one being multiplied
  const int n_pad = (n_items + R - 1) / R * R;  // whole ring rounds; the padding items load clamped, compute nothing

  // ---- this thread's activation chunks first (row-contiguous copy of rows [0, M) x K), then the weight prologue:
  // the compiler counts both streams of plain loads, so staging X waits for X alone
  bf16x8 xst[XCH];
  const int cpr = a.K >> 3, nch = a.M * cpr;
#pragma unroll
  for (int i = 0; i < XCH; ++i) {
    const int c = min((int)threadIdx.x + i * WAVES * 64, nch - 1);
    const int r = c / cpr, col = c - r * cpr;
    xst[i] = *reinterpret_cast<const bf16x8*>(a.X + (size_t)r * a.ldx + col * 8);
  }

  struct Quad {
    w4u32x4 w;
    uint32_t s;
  };
  const w4u32x4* wbase = reinterpret_cast<const w4u32x4*>(a.Wp) + lane;
  const uint8_t* sbase = wsc + lane;
  int ld_t = blockIdx.x, ld_e = 0, ld_i = 0;
  const int last_t = (int)blockIdx.x + (my_tiles - 1) * G;
  auto load_next = [&](Quad& q) {
    // past the end of the sequence: re-load this wave's last item (a cache hit).  Not a branch around the load:
    // hipcc then loses its counted waits and drains the ring (vmcnt(0)) at every item
    const bool in = ld_i < n_items;
    const int p = min(wave + (in ? ld_e : qmax - 1) * WAVES, KQ - 1);
    const int j = in ? ld_t : last_t, jt = j / KS;  // pair -> (tile, k range)
    const size_t off = ((size_t)jt * KQT + (j - jt * KS) * KQ + p) * 64;
    q.w = __builtin_nontemporal_load(wbase + off);
    q.s = __builtin_nontemporal_load(sbase + off);
    ++ld_i;
    if (++ld_e == qmax) ld_e = 0, ld_t += G;
  };
  Quad ring[R];
#pragma unroll
  for (int u = 0; u < U; ++u) load_next(ring[u]);

  int cp_t = blockIdx.x;
  EpiIn pre{};
  if (wave == 0 && my_tiles > 0) pre = epi_load_at<EPI>(a, cp_t / KS, lane & 15, lane);
#pragma unroll
  for (int i = 0; i < XCH; ++i) {
    const int c = (int)threadIdx.x + i * WAVES * 64;
    if (c < nch) *reinterpret_cast<bf16x8*>(w4_xs + (size_t)c * 16) = xst[i];
  }
  w4_barrier();
  if constexpr (NORM) {
    // RMSNorm sums of squares once per workgroup from the staged copy (not per weight fragment, where they cost 8
    // VALU ops per MFMA, +2-4 us per GEMM), in a fixed order so identical seeded runs agree bit for bit (ADVICE r4:
    // LDS float atomics summed in arrival order): wave w owns rows w, w + WAVES, ...; each lane sums its chunks in
    // k order, then the wave reduces by xor shuffles.  The first tile_end barrier orders these stores before the
    // epilogue reads them.
    for (int r = wave; r < a.M; r += WAVES) {
      const char* xr = w4_xs + (size_t)r * cpr * 16;
      float v = 0.f;
      for (int c = lane; c < cpr; c += 64) {
        const bf16x8 x8 = *reinterpret_cast<const bf16x8*>(xr + (size_t)c * 16);
#pragma unroll
        for (int j = 0; j < 8; ++j) v += bf2f(x8[j]) * bf2f(x8[j]);
      }
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
      if (lane == 0) row_ss[r] = v;
    }
  }
  // this lane's activation row in LDS and its k group: fragment s of quad p starts at 128p + 32g + 8s.  Lanes of
  // output columns >= M (padding rows) read nothing and multiply zeros: at one row 1/16 of the LDS traffic.
  const bool xrow = (lane & 15) < a.M;
  const __bf16* xl_row = reinterpret_cast<const __bf16*>(w4_xs) + (size_t)min(lane & 15, a.M - 1) * a.K + ((lane >> 4) << 5);

  f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
  int cp_e = 0, cp_n = 0, buf = 0;

  auto step = [&](const Quad& q, int p) {
    const float sc = e8m0_f32(q.s);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const bf16x8 wf = w4_frag(q.w[s], sc);
      bf16x8 xv = {};
      if (xrow) xv = *reinterpret_cast<const bf16x8*>(xl_row + p * 128 + s * 8);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, xv, acc, 0, 0, 0);
    }
  };

  // end of a tile: partials -> LDS slab `buf`, one barrier, wave 0 finishes the 16x16 block
  auto tile_end = [&]() {
    red[buf][wave][lane] = acc;
    acc = f32x4{0.f, 0.f, 0.f, 0.f};
    w4_barrier();
    if (wave == 0) {
      const int tile = cp_t / KS;
      if (cp_n > 0) pre = epi_load_at<EPI>(a, tile, lane & 15, lane);  // later tiles (none for fp32 / act epis)
      if constexpr (SPLIT) {
        // split-K: publish this pair's partial, take the tile's ticket; the last arriver finishes the tile
        f32x4 v = red[buf][0][lane];
#pragma unroll
        for (int w = 1; w < WAVES; ++w) v += red[buf][w][lane];
        uint64_t* pp = reinterpret_cast<uint64_t*>(sp.part + ((size_t)cp_t * 64 + lane) * 4);
        __hip_atomic_store(pp, __builtin_bit_cast(uint64_t, f32x2{v[0], v[1]}), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(pp + 1, __builtin_bit_cast(uint64_t, f32x2{v[2], v[3]}), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        unsigned t = 0;
        if (lane == 0) t = __hip_atomic_fetch_add(sp.ctr + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        t = __shfl(t, 0, 64);
        if (t == unsigned(KS - 1)) {
          f32x4 sum = f32x4{0.f, 0.f, 0.f, 0.f};
          for (int k = 0; k < KS; ++k) {  // every pair's partial, this one's included, in k order
            const uint64_t* q = reinterpret_cast<const uint64_t*>(sp.part + (((size_t)tile * KS + k) * 64 + lane) * 4);
            const f32x2 lo = __builtin_bit_cast(f32x2, __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            const f32x2 hi = __builtin_bit_cast(f32x2, __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            sum += f32x4{lo[0], lo[1], hi[0], hi[1]};
          }
          if constexpr (NORM) sum *= rms_inv(row_ss[min(lane & 15, a.M - 1)], a.K, a.eps);
          if (lane == 0) sp.ctr[tile] = 0u;  // ready for the next launch (launch-ordered)
          red[buf][0][lane] = sum;  // one wave: its LDS operations complete in order
          epi_store<EPI>(a, tile, lane & 15, lane, pre, [&](int off) { return red[buf][0][lane + off]; });
          if constexpr (EPI == EPI_F32) epi_cmax(a, tile, lane & 15, lane, sum);
        }
        buf ^= 1;
        return;
      }
      auto unit_sum = [&](int l) -> f32x4 {
        f32x4 v = red[buf][0][l];
#pragma unroll
        for (int w = 1; w < WAVES; ++w) v += red[buf][w][l];
        if constexpr (NORM) v *= rms_inv(row_ss[min(l & 15, a.M - 1)], a.K, a.eps);
        return v;
      };
      if constexpr (EPI == EPI_F32) {  // the LM head: logits + chunk maxima
        const f32x4 v = unit_sum(lane);
        epi_store<EPI>(a, tile, lane & 15, lane, pre, [&](int) { return v; });
        epi_cmax(a, tile, lane & 15, lane, v);
      } else {
        epi_store<EPI>(a, tile, lane & 15, lane, pre, [&](int off) { return unit_sum(lane + off); });
      }
    }
    buf ^= 1;
  };

  for (int i0 = 0; i0 < n_pad; i0 += R) {
#pragma unroll
    for (int u = 0; u < R; ++u) {
      const int p = wave + cp_e * WAVES;  // k quad within the pair's range
      const bool live = i0 + u < n_items;
      // item i0 + u + U goes into the spare slot (the one consumed by the previous item) BEFORE this item's math: a
      // ring of U + 1 slots walked in whole rounds keeps every slot index a constant (a register copy of an
      // in-flight load would force the compiler to drain the ring: vmcnt(0) at every round)
      load_next(ring[(u + U) % (U + 1)]);
      if (live && p < KQ) step(ring[u], (cp_t - (cp_t / KS) * KS) * KQ + p);
      if (live && cp_e == qmax - 1) tile_end();
      if (++cp_e == qmax) cp_e = 0, ++cp_n, cp_t += G;
    }
  }
}

// ================================================================ wide / fallback: one workgroup per (tile, M block)
template <int WAVES, int U, int NB, int EPI, bool NORM>
__global__ __launch_bounds__(WAVES * 64) void w4_tile_kernel(const GemmArgs a, const uint8_t* __restrict__ wsc) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int KQ = a.K >> 7;  // 128-wide k quads
  int tg, ms;
  w4_pair_tile(blockIdx.x, a.msplit, gridDim.x / a.msplit, tg, ms);
  const int mo = ms * 16 * NB;
  const int p_beg = (wave * KQ) / WAVES, p_end = ((wave + 1) * KQ) / WAVES;

  EpiIn pre[NB];
  if (wave == 0) {
#pragma unroll
    for (int b = 0; b < NB; ++b) pre[b] = epi_load_at<EPI>(a, tg, mo + 16 * b + (lane & 15), lane);
  }
  const w4u32x4* wb = reinterpret_cast<const w4u32x4*>(a.Wp) + (size_t)tg * KQ * 64 + lane;
  const uint8_t* sb = wsc + (size_t)tg * KQ * 64 + lane;
  // this lane's activation row and its k group: fragment s of quad p starts at element 128p + 32g + 8s
  const int kg = (lane >> 4) << 5;
  const __bf16* xb[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) xb[b] = a.X + (size_t)min(mo + 16 * b + (lane & 15), a.M - 1) * a.ldx + kg;

  f32x4 acc[NB];
  float ssq[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) acc[b] = f32x4{0.f, 0.f, 0.f, 0.f}, ssq[b] = 0.f;

  struct Quad {
    w4u32x4 w;
    uint32_t s;
    bf16x8 x[NB][4];
  };
  auto load = [&](Quad& q, int p) {
    q.w = __builtin_nontemporal_load(wb + (size_t)p * 64);
    q.s = __builtin_nontemporal_load(sb + (size_t)p * 64);
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int s = 0; s < 4; ++s) q.x[b][s] = *reinterpret_cast<const bf16x8*>(xb[b] + p * 128 + s * 8);
  };
  auto step = [&](const Quad& q) {
    const float sc = e8m0_f32(q.s);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const bf16x8 wf = w4_frag(q.w[s], sc);
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        if constexpr (NORM) {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float f = bf2f(q.x[b][s][j]);
            ssq[b] += f * f;
          }
        }
        acc[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, q.x[b][s], acc[b], 0, 0, 0);
      }
    }
  };

  // copy pipeline: chunks of U quads, the next chunk's loads in flight while the current one is multiplied; a
  // partial last chunk re-loads its last quad (clamped, a cache hit) and multiplies only its valid quads
  const int nq = p_end - p_beg;
  const int nchunk = (nq + U - 1) / U;
  auto load_chunk = [&](Quad* q, int pc) {
#pragma unroll
    for (int u = 0; u < U; ++u) load(q[u], min(pc + u, p_end - 1));
  };
  Quad cur[U];
  if (nchunk > 0) load_chunk(cur, p_beg);
  for (int c = 0; c < nchunk; ++c) {
    Quad nxt[U];
    const int pc = p_beg + c * U;
    const bool more = c + 1 < nchunk;
    if (more) load_chunk(nxt, pc + U);
    const int nv = p_end - pc;
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (u < nv) step(cur[u]);
    if (more) {
#pragma unroll
      for (int u = 0; u < U; ++u) cur[u] = nxt[u];
    }
  }

  // ---- cross-wave reduction through LDS, epilogue by wave 0
  __shared__ __attribute__((aligned(16))) f32x4 red[WAVES][NB][64];
  __shared__ float red_ss[NORM ? WAVES : 1][NB][16];
#pragma unroll
  for (int b = 0; b < NB; ++b) red[wave][b][lane] = acc[b];
  if constexpr (NORM) {
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      float v = ssq[b];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (lane < 16) red_ss[wave][b][lane] = v;
    }
  }
  __syncthreads();
  if (wave != 0) return;
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    auto unit_sum = [&](int l) -> f32x4 {
      f32x4 v = red[0][b][l];
#pragma unroll
      for (int w = 1; w < WAVES; ++w) v += red[w][b][l];
      if constexpr (NORM) {
        float ss = 0.f;
#pragma unroll
        for (int w = 0; w < WAVES; ++w) ss += red_ss[w][b][l & 15];
        v *= rms_inv(ss, a.K, a.eps);
      }
      return v;
    };
    epi_store<EPI>(a, tg, mo + 16 * b + (lane & 15), lane, pre[b], [&](int off) { return unit_sum(lane + off); });
  }
}

// ================================================================ launch
// kernel shapes (W4Var): stream kernels (waves, items in flight) and tile kernels (waves, quads in flight, row blocks)
enum W4Var { W4S_8_4, W4S_4_4, W4T_8_2_1, W4T_4_4_1, W4T_8_2_2, W4T_4_2_2, W4_N_VARS };
static const int W4_WAVES[W4_N_VARS] = {8, 4, 8, 4, 8, 4};
static const int W4_NB[W4_N_VARS] = {1, 1, 1, 1, 2, 2};
static bool w4_is_stream(int v) { return v <= W4S_4_4; }

template <bool NORM, int EPI>
static hipError_t w4_launch_var(int var, const GemmArgs& a, const uint8_t* wsc, int grid, int npairs,
                                const W4Split& sp, hipStream_t st) {
  const dim3 g(grid), b8(512), b4(256);
  switch (var) {
    case W4S_8_4:
      // the fused QKV epilogue runs on 4 waves only (at 8 its partner-unit sums spill; w4_variant never picks it)
      if constexpr (EPI == EPI_QKV_ROPE)
        hipLaunchKernelGGL((w4_stream_kernel<4, 4, EPI, NORM, false>), g, b4, 0, st, a, wsc, npairs, sp);
      else if (sp.ks > 1)
        hipLaunchKernelGGL((w4_stream_kernel<8, 4, EPI, NORM, true>), g, b8, 0, st, a, wsc, npairs, sp);
      else
        hipLaunchKernelGGL((w4_stream_kernel<8, 4, EPI, NORM, false>), g, b8, 0, st, a, wsc, npairs, sp);
      break;
    case W4S_4_4:
      if constexpr (EPI != EPI_QKV_ROPE) {
        if (sp.ks > 1) {
          hipLaunchKernelGGL((w4_stream_kernel<4, 4, EPI, NORM, true>), g, b4, 0, st, a, wsc, npairs, sp);
          break;
        }
      }
        hipLaunchKernelGGL((w4_stream_kernel<4, 4, EPI, NORM, false>), g, b4, 0, st, a, wsc, npairs, sp);
      break;
    case W4T_8_2_1: hipLaunchKernelGGL((w4_tile_kernel<8, 2, 1, EPI, NORM>), g, b8, 0, st, a, wsc); break;
    case W4T_4_4_1: hipLaunchKernelGGL((w4_tile_kernel<4, 4, 1, EPI, NORM>), g, b4, 0, st, a, wsc); break;
    case W4T_8_2_2: hipLaunchKernelGGL((w4_tile_kernel<8, 2, 2, EPI, NORM>), g, b8, 0, st, a, wsc); break;
    default: hipLaunchKernelGGL((w4_tile_kernel<4, 2, 2, EPI, NORM>), g, b4, 0, st, a, wsc); break;
  }
  return hipGetLastError();
}

template <bool NORM>
static hipError_t w4_launch(int epi, int var, const GemmArgs& a, const uint8_t* wsc, int grid, int npairs,
                            const W4Split& sp, hipStream_t st) {
  switch (epi) {
    case EPI_BF16: return w4_launch_var<NORM, EPI_BF16>(var, a, wsc, grid, npairs, sp, st);
    case EPI_RESID: return w4_launch_var<NORM, EPI_RESID>(var, a, wsc, grid, npairs, sp, st);
    case EPI_F32: return w4_launch_var<NORM, EPI_F32>(var, a, wsc, grid, npairs, sp, st);
    case EPI_SILU: return w4_launch_var<NORM, EPI_SILU>(var, a, wsc, grid, npairs, sp, st);
    case EPI_GELU: return w4_launch_var<NORM, EPI_GELU>(var, a, wsc, grid, npairs, sp, st);
    case EPI_QKV_ROPE: return w4_launch_var<NORM, EPI_QKV_ROPE>(var, a, wsc, grid, npairs, sp, st);
    default: return hipErrorInvalidValue;
  }
}

// Tuning / test overrides (-1 / 0: the rules below): the kernel shape (W4Var) and the stream grid's workgroups per CU
static int g_w4_var = -1, g_w4_wgs_per_cu = 0, g_w4_split = 0, g_w4_split_cap = 1, g_w4_split_min_q = 32;
CAIN_API void cain_gemm_w4_set_variant(int v) { g_w4_var = v < W4_N_VARS ? v : -1; }
// split-K of the stream kernel: 0 = the rule (w4_split), 1 = off, k > 1 = k ranges wherever the shape allows it
CAIN_API void cain_gemm_w4_set_split(int ks) { g_w4_split = ks > 0 ? ks : 0; }
// A/B of the rule's pair budget: tiles x ks <= cap x CUs (1: the rule)
CAIN_API void cain_gemm_w4_set_split_cap(int cap) { g_w4_split_cap = cap > 0 ? cap : 1; }
// A/B of the rule's shortest k range in quads (32: the rule)
CAIN_API void cain_gemm_w4_set_split_min_quads(int q) { g_w4_split_min_q = q > 0 ? q : 32; }
CAIN_API void cain_gemm_w4_set_occupancy(int wgs_per_cu) { g_w4_wgs_per_cu = wgs_per_cu > 0 ? wgs_per_cu : 0; }

static int w4_n_cu() {
  const int n = cain_cu_budget();
  return n;
}

static bool w4_stream_fits(int waves, int K, int M) {
  return M <= 16 && (long long)M * K * 2 <= (waves == 8 ? w4_xl_bytes<8>() : w4_xl_bytes<4>());
}

// Shape rule (tools/w4_bench.py, in-graph, llama3.1:8b shapes at one row: profiles/r4/README.md).  Up to 16 rows
// whose activations fit the LDS copy: the stream kernel, 4 items in flight per wave (8 lost 1-4 us on every shape:
// deeper queues, no faster stream), 8 waves (gate/up 14.9 vs 16.3 us on 4, LM head 46.6 vs 53.8, O 5.2 vs 5.8),
// except the fused QKV epilogue, whose registers at 8 waves spill (9.1 vs 10.2 us on 4).  Otherwise the tile
// kernel, two 16-row blocks per workgroup above 16 rows.
static int w4_variant(int N, int K, int M, int epi, int n_cu) {
  (void)N, (void)n_cu;
  const int kq = K / 128;
  if (g_w4_var >= 0) {
    const int v = g_w4_var == W4S_8_4 && epi == EPI_QKV_ROPE ? W4S_4_4 : g_w4_var;  // no 8-wave QKV kernel
    if (!w4_is_stream(v) || w4_stream_fits(W4_WAVES[v], K, M)) return v;  // a stream shape needs its LDS copy
  }
  // 4 waves as well when K is short: below 3 quads per wave of the 8-wave shape its waves idle on the padding
  // items (qwen2:1.5b, K = 1536: gate/up 7.4 vs 8.6 us, O 3.9 vs 4.1; profiles/r4/ab/w4_short_k.jsonl)
  const bool w4 = (epi == EPI_QKV_ROPE || kq < 24) && w4_stream_fits(4, K, M);
  if (w4) return W4S_4_4;
  // (not the fused QKV epilogue: it has no 8-wave instance, and the 4-wave one stages only 28 KiB of activations --
  // rows x K beyond that take the tile kernel)
  if (epi != EPI_QKV_ROPE && w4_stream_fits(8, K, M)) return W4S_8_4;
  if (M > 16) return kq >= 32 ? W4T_8_2_2 : W4T_4_2_2;
  return kq >= 32 ? W4T_8_2_1 : W4T_4_4_1;
}

CAIN_API int cain_gemm_w4_variant(int N, int K, int M, int epi) { return w4_variant(N, K, M, epi & EPI_MASK, w4_n_cu()); }

static long long w4_split_bytes(int N, int ks) { return W4_PART_OFFSET + (long long)(N / 16) * ks * 64 * 16; }

// k ranges per tile of a stream-kernel GEMM: the most (up to 4) that keep tiles x ks <= CUs (one pair per CU: the
// ticket's last arriver adds a memory round trip, so pairs beyond the CU count buy nothing), every range >= 32 k
// quads (4,096 k), every wave >= one quad per range, and the workspace large enough.  Wider outputs (>= one tile per
// CU) are not split.  Measured in the graph-replayed batch-1 decode (tools/w4_split_ab.py, profiles/r5/w4split/):
// splitting every narrow output in two, gemma:2b (down K = 16,384, O K = 2,048) 1,087 -> 1,099-1,106 tok/s and
// qwen2:1.5b (down K = 8,960, O K = 1,536) 981 -> 921 -- ranges of 35 and 6 quads save less stream time than the
// ticket's round trip; with this rule (gemma:2b's down alone) 1,084 -> 1,127 tok/s, qwen2:1.5b unchanged.  A budget
// of 2 x CUs (gemma:7b / qwen2:7b down, 192 / 224 tiles, in two) measured slower: 559 -> 548, 628 -> 615.  Ranges
// down to 32 quads (qwen2:1.5b's down alone, 35): 985 / 978 -> 991 / 993 tok/s; its O (6 quads) stays unsplit.
static int w4_split(int var, int N, int K, int epi, int n_cu, long long ws_bytes) {
  // the fused QKV epilogue has no split instance (its outputs are never narrow enough to pay: 128+ tiles of <= 16
  // quads on the study's models)
  if (!w4_is_stream(var) || g_w4_split == 1 || epi == EPI_QKV_ROPE) return 1;
  const int tiles = N / 16, kq = K / 128, waves = W4_WAVES[var];
  auto ok = [&](int k) {
    return k > 1 && kq % k == 0 && kq / k >= waves && tiles <= 4096 && w4_split_bytes(N, k) <= ws_bytes;
  };
  if (g_w4_split > 1) return ok(g_w4_split) ? g_w4_split : 1;
  int best = 1;
  for (int k = 2; k <= 4; ++k)
    if (tiles * k <= g_w4_split_cap * n_cu && kq / k >= g_w4_split_min_q && ok(k)) best = k;
  return best;
}

CAIN_API int cain_gemm_w4_split(int N, int K, int M, int epi, long long ws_bytes) {
  const int n_cu = w4_n_cu();
  return w4_split(w4_variant(N, K, M, epi & EPI_MASK, n_cu), N, K, epi & EPI_MASK, n_cu, ws_bytes);
}

// Workspace a W4 GEMM of this shape may use (split-K tickets + partials; 0: none)
CAIN_API long long cain_gemm_w4_ws_bytes(int N, int K, int M) {
  (void)K, (void)M;
  return N % 16 ? 0 : w4_split_bytes(N, 4);
}

CAIN_API int cain_gemm_w4_ex(const void* Wp, const void* wsc, const void* X, int ldx, int K, int N, int M, void* Y,
                             int ldy, const float* bias, int norm, float eps, const int* slot, const int* pos,
                             const float* cos_t, const float* sin_t, void* kc, void* vtc, int H, int Hkv, int hd,
                             int T_max, void* ws, long long ws_bytes, int epi_flags, hipStream_t st);
CAIN_API float* cain_gemm_cmax_claim(int N);  // gemm.hip

// Same arguments as cain_gemm_w8 (gemm_w8.hip); Wp is the MXFP4 packing, wsc its e8m0 scale bytes.  No workspace:
// never split (cain_gemm_w4_ex is the engine's entry).
CAIN_API int cain_gemm_w4(const void* Wp, const void* wsc, const void* X, int ldx, int K, int N, int M, void* Y, int ldy,
                          const float* bias, int norm, float eps, const int* slot, const int* pos, const float* cos_t,
                          const float* sin_t, void* kc, void* vtc, int H, int Hkv, int hd, int T_max, int epi_flags,
                          hipStream_t st) {
  return cain_gemm_w4_ex(Wp, wsc, X, ldx, K, N, M, Y, ldy, bias, norm, eps, slot, pos, cos_t, sin_t, kc, vtc, H, Hkv,
                         hd, T_max, nullptr, 0, epi_flags, st);
}

// ws: zeroed at allocation; its first W4_CTR_BYTES are tickets that every split launch leaves zero
CAIN_API int cain_gemm_w4_ex(const void* Wp, const void* wsc, const void* X, int ldx, int K, int N, int M, void* Y,
                             int ldy, const float* bias, int norm, float eps, const int* slot, const int* pos,
                             const float* cos_t, const float* sin_t, void* kc, void* vtc, int H, int Hkv, int hd,
                             int T_max, void* ws, long long ws_bytes, int epi_flags, hipStream_t st) {
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
  const int n_cu = w4_n_cu();
  const int var = w4_variant(N, K, M, epi, n_cu);
  const int nb = W4_NB[var], waves = W4_WAVES[var];
  if (epi == EPI_F32 && w4_is_stream(var))  // the few-row LM head also writes the sampler's chunk maxima
    if (float* cm = cain_gemm_cmax_claim(N)) a.cmax = cm, a.ld_cm = N / 16;
  a.msplit = (M + 16 * nb - 1) / (16 * nb);
  const int npairs = N / 16 * a.msplit;
  int grid = npairs;
  W4Split sp{1, nullptr, nullptr};
  int np = npairs;
  if (w4_is_stream(var)) {  // persistent: at most the resident workgroups (2 of 8 waves / 4 of 4 waves per CU)
    a.msplit = 1;
    sp.ks = ws ? w4_split(var, N, K, epi, n_cu, ws_bytes) : 1;
    if (sp.ks > 1) {
      sp.ctr = static_cast<unsigned*>(ws);
      sp.part = reinterpret_cast<float*>(static_cast<char*>(ws) + W4_PART_OFFSET);
      np = npairs * sp.ks;
    }
    grid = std::min(np, n_cu * (g_w4_wgs_per_cu ? g_w4_wgs_per_cu : (waves == 8 ? 2 : 4)));
  }
  const uint8_t* sc = reinterpret_cast<const uint8_t*>(wsc);
  const hipError_t e = norm ? w4_launch<true>(epi, var, a, sc, grid, np, sp, st)
                            : w4_launch<false>(epi, var, a, sc, grid, np, sp, st);
  return int(e);
}
