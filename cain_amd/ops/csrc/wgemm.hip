// Wide-batch projection GEMM for 64 < M <= 256 rows (the batched decode step and prefill chunks), gfx950.
//
//   Y[m][n] = epilogue( inv[m] * sum_k X[m][k] * W[n][k] )
//
// Replaces, at the trial-batched decode shapes, the per-token GEMVs llama.cpp runs inside Ollama for the
// reference's workload (reference experiment/RunnerConfig.py:128-131; SURVEY §2.4 rows QKV / O / gate-up / down /
// LM head).  The M <= 64 shapes stay on the weight-streaming kernels of gemm.hip.
//
// Why a different kernel at these widths: at M = 256 every weight byte feeds 256 MFMA rows, so the GEMM is no
// longer a pure weight stream -- per CU it has to ingest its weight slice AND the activation panel it multiplies,
// and the per-CU load path (~60-70 GB/s per CU, MI355X_MICROARCH.md rows 'ldsdma-fill' / 'ring-gemm') becomes the
// limit long before HBM.  A workgroup therefore owns the largest output tile the LDS ring allows, BM = all rows x
// BN = 128 columns, so per weight byte it ingests (BM + BN) / BN = 3 bytes, and both operands move by LDS-DMA
// (global_load_lds_dwordx4: no VGPR staging, no ds_write pass; cdna_hip_programming.md §5 'glds vs register
// staging', rows 'M = 256 projection GEMM'):
//
//   * W tiles come straight from the engine's MFMA-fragment-major packing (models/weights.py pack_mfma_a): a
//     16-row x 32-k fragment block is 1 KiB contiguous in HBM, so one LDS-DMA instruction moves one block and
//     the LDS image is fragment-major too -- every A-fragment read is lane-linear ds_read_b128, conflict-free.
//     Streamed once: non-temporal (aux = nt).
//   * X (activations, [M][ldx] bf16 row-major, L2-resident) is staged in full 128-B lines: a stage holds BK = 64
//     k, i.e. one line per row, and one LDS-DMA instruction covers 8 rows.  The lane-linear LDS image is
//     XOR-swizzled by permuting the per-lane SOURCE piece (rule 21): LDS slot q of row r holds global piece
//     q ^ ((r >> 1) & 7), which makes the 16-lane groups of the B-fragment ds_read_b128 conflict-free.
//   * Two LDS rings, X (DX + 1 slots of 32 KiB at BM = 256) and W (DW + 1 slots of 16 KiB), the deeper one for
//     the HBM stream; one raw s_barrier per 64-deep k-step; counted `s_waitcnt vmcnt` keeps the younger stages
//     in flight across it (§5 'Pipelining across barriers').
//   * Warp-specialised: 4 loader waves (one per SIMD) issue every LDS-DMA piece and wait for it; 8 MFMA waves
//     only read fragments and compute.  Measured on the 256-row gate/up shape, DMA alone took 55-63 us and the
//     MFMA body alone 60 us, but 85-92 us when the MFMA waves issued the DMA themselves; split roles: 68 us.
//   * 8 waves as WM (M) x WN (N): each wave owns MB 16-row blocks x TN 16-column tiles (4 x 4 at BM = 256), so
//     per 32-deep slice it reads TN + MB fragments for TN * MB v_mfma_f32_16x16x32_bf16 (LDS ~50 % busy at full
//     MFMA rate).
//   * Fused RMSNorm: the norm gain is folded into W (models/weights.py fold_gain), so only the per-row sum of
//     squares of X is needed; it comes from the MFMA unit itself -- mfma(xfrag, xfrag) accumulates X X^T whose
//     diagonal is the row's sum of squares (exact fp32 accumulation of bf16 products), one extra MFMA per
//     fragment, split between the WN waves that read the same rows.
//
// Split-K: narrow outputs (QKV, O, down: 32-48 column tiles) split K over ks workgroups so ~256 workgroups
// stream; each writes its tile to a workspace slab (plain stores, fp16: OPT bit 32 below; the sums stay fp32) and
// `wgemm_reduce_kernel` -- the next launch on the stream, so the kernel boundary orders the hand-off -- sums the
// slabs in fp32 and runs the fused epilogue.  With ks = 1 (gate/up, LM head) the GEMM kernel runs the epilogue itself.  The epilogues are
// gemm_epi.h's (residual, bias, SiLU/GeLU x up, RoPE + KV-cache append, fp32 logits).
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "gemm_epi.h"
#include "wgemm_ring.h"

using namespace wg;

constexpr int WG_CTR_BYTES = 16 * 1024;  // the workspace region before the slabs (gemm.hip WG_COUNTER_BYTES)

// DX / DW: prefetch distance (stages in flight) of the X and the W ring; the rings have DX + 1 and DW + 1 slots.
// W streams from HBM (latency ~2-3 us under load) and gets the deeper ring; X comes from L2.
//
// NDMA: waves dedicated to the LDS-DMA (0: the 8 MFMA waves issue their own shares).  Measured on the 256-row
// gate/up shape (tools/wgemm_bench.py ablations): DMA alone 63 us, fragment reads + MFMAs alone 60 us, both in
// the same waves 85-92 us -- a wave cannot issue MFMAs while it issues ~60-cycle DMA pieces, and the per-stage
// barrier keeps the two waves of a SIMD in the same phase.  With NDMA = 4 one loader wave per SIMD issues every
// piece and waits for it; the MFMA waves only compute.  Both roles pass the same one barrier per stage.
//
// Loop (compute waves): the barrier of stage t + 1 sits between stage t's two slices, so the next slice's
// fragment reads are always in flight under 16 MFMAs and no wave restarts the matrix pipe behind a barrier.
//
// ABL (diagnostics only): 1 = DMA without the fragment reads and MFMAs, 2 = fragment reads and MFMAs without the
// DMA.  Results are garbage in both.  3 = the full kernel plus timestamps (tools/wgemm_trace.py): lane 0 of wave 0
// (compute) and of the first loader wave store s_memrealtime / s_memtime at fixed points to w.stamps.
//
// H16: split-K slabs in fp16 instead of fp32 (wgemm_reduce_kernel H16 = true reads them): half the slab bytes
// stored, written back at the kernel boundary (MI355X_MICROARCH.md 'boundary': + dirty bytes / 6 TB/s) and read by
// the reduce.  Each lane's partials (one activation row) are stored scaled -- NORM: by rsqrt of the row's split sum
// of squares, else by a power of two -- so rows of outliers keep fp16's relative precision (the reduce sums in
// fp32); tests/test_wgemm_gpu.py compares them with fp32 slabs on such rows.  (Round 3's loader alternatives -- loader-wave sums of squares, W-only / X-only
// loader roles, rotated k start, non-temporal X, stage-ordered prologue -- and the in-launch split-K combine all
// measured within box-to-box noise or slower, profiles/r3/README.md, and were removed.)
template <int BM, int EPI, bool NORM, bool H16, bool COH>
__device__ __forceinline__ void wg_reduce_unit(const GemmArgs& a, const WgArgs& w, int unit, int n_units, int lane,
                                               int ks);

template <int BM, int EPI, bool NORM, bool H16>
__device__ void wg_inline_combine(const GemmArgs& a, const WgArgs& w, int blk, int kc, int n_units, int nthr,
                                  unsigned* flags);

// INL: the split-K combine inside this launch (wg_inline_combine below) instead of wgemm_reduce_kernel
template <int BM, int DX, int DW, int EPI, bool NORM, int NDMA, int ABL = 0, bool H16 = false, bool INL = false>
__global__ __launch_bounds__(64 * (8 + NDMA), (8 + NDMA) / 4) void wgemm_kernel(const GemmArgs a, const WgArgs w) {
  using G = WgGeo<BM>;
  constexpr bool MSQ = NORM;                        // MFMA X X^T sums of squares
  constexpr int NX = DX + 1, NW = DW + 1;
  constexpr int NLOAD = NDMA ? NDMA : 8;            // waves issuing LDS-DMA
  constexpr int NWL = NLOAD;                        // waves issuing W pieces
  constexpr int NXL = NLOAD;                        // waves issuing X pieces
  constexpr int WPW = 16 / NWL;                     // W blocks (1 KiB) per W-loader wave per stage
  constexpr int XPW = (BM / 8) / NXL;               // X row octets per X-loader wave per stage
  constexpr int NTHR = 64 * (8 + NDMA);
  static_assert(DW >= DX && DX >= 1, "W is issued no later than X of the same stage");
  static_assert(WPW * NWL == 16 && XPW * NXL == BM / 8, "loader split");
  extern __shared__ __attribute__((aligned(16))) char smem[];  // the one LDS array: [NW W slots][NX X slots]
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool compute = wave < 8;
  const bool loader = NDMA ? !compute : true;
  const int lw = NDMA ? wave - 8 : wave;  // loader index
  const bool wload = loader, xload = loader;
  const int xl = lw;  // X-loader index
  const int wm = wave % G::WM, wn = (wave / G::WM) % G::WN;
  const int KS = a.K >> 5, ntiles = a.N >> 4;
  const int nblk = (ntiles + WG_NT - 1) / WG_NT;
  // ABL 3: slots 0/1 start (realtime / memtime), 2 stage 0 ready, 3 stage nst/2 ready, 4 loop end, 5 slab stores
  // drained, 6/7 end (realtime / memtime)
  auto stamp = [&](int sl, bool cyc) {
    if constexpr (ABL == 3) {
      const unsigned long long v = cyc ? __builtin_amdgcn_s_memtime() : __builtin_amdgcn_s_memrealtime();
      if (lane == 0 && (wave == 0 || wave == 8)) w.stamps[((size_t)blockIdx.x * 2 + (wave == 8)) * 8 + sl] = v;
    }
  };
  stamp(0, false);
  stamp(1, true);

  // block -> (column block, k-split); the k-split partners of one column block read disjoint X panels, the
  // column blocks of one k-split read the SAME X panel: split-major placement keeps those on one XCD (blocks b
  // and b + 8 share an XCD under round-robin dispatch); the default xcd_blk placement keeps a column block's
  // split partners together instead, for the reduce (wgemm_dispatch).  Speed only, any placement is correct.
  int blk, kc;
  {
    wg_block_of(blockIdx.x, w.ks, nblk, w.xcd_blk, blk, kc);
  }
  const int tile0 = blk * WG_NT;
  const int st0 = kc * w.kst;                    // first stage (64-deep k-step) of this split
  const int nst = min(w.kst, (a.K >> 6) - st0);  // stages of this split
  auto kstage = [&](int t) { return t; };  // ring stage t -> stage of this split's k range

  // ---- LDS-DMA sources of this loader (per stage: WPW W blocks + XPW X row-octets)
  // W block j of loader lw: tile (lw * WPW + j) / 2, slice (lw * WPW + j) & 1 (a tile's two slices are 2 KiB
  // contiguous in the packing); LDS W image: block (tile * 2 + slice) at 1 KiB each
  const char* wsrc[WPW];
#pragma unroll
  for (int j = 0; j < WPW; ++j) {
    const int q = lw * WPW + j, tn = q >> 1, sl = q & 1;
    wsrc[j] = reinterpret_cast<const char*>(a.Wp) +
              ((size_t)min(tile0 + tn, ntiles - 1) * KS + (size_t)st0 * 2 + sl) * 1024 + lane * 16;
  }
  // X: octet i covers rows 8i .. 8i + 7; lane -> row 8i + (lane >> 3), LDS slot lane & 7 holding global piece
  // (lane & 7) ^ ((r >> 1) & 7) (the read side's XOR swizzle)
  const char* xsrc[XPW];
#pragma unroll
  for (int j = 0; j < XPW; ++j) {
    const int i = xl + NXL * j;
    const int r = 8 * i + (lane >> 3);
    const int p = (lane & 7) ^ ((r >> 1) & 7);
    xsrc[j] = reinterpret_cast<const char*>(a.X) + ((size_t)min(r, a.M - 1) * a.ldx + (size_t)st0 * WG_BK + p * 8) * 2;
  }
  char* const xring = smem + NW * G::W_BYTES;
  auto issue_w = [&](int t) {  // W stage t (relative to st0) into W slot t % NW
    if constexpr (ABL == 2) return;
    if (!wload) return;
    char* base = smem + (t % NW) * G::W_BYTES;
    const size_t off = (size_t)kstage(t) * 2048;
#pragma unroll
    for (int j = 0; j < WPW; ++j) glds16(wsrc[j] + off, base + (lw * WPW + j) * 1024, 1);
  };
  auto issue_x = [&](int t) {  // X stage t into X slot t % NX
    if constexpr (ABL == 2) return;
    if (!xload) return;
    char* base = xring + (t % NX) * G::X_BYTES;
    const size_t off = (size_t)kstage(t) * (WG_BK * 2);
#pragma unroll
    for (int j = 0; j < XPW; ++j) glds16(xsrc[j] + off, base + (xl + NXL * j) * 1024, 0);
  };
  // issue order: step u (u < 0: prologue) issues W(u + DW), then X(u + DX); so W(t) is always older than X(t) and
  // waiting for X(t) covers both (vmcnt retires in issue order).  Loads younger than X(t): steps t-DX+1 .. t-1.
  auto younger_than = [&](int t) {
    int n = 0;
#pragma unroll
    for (int u = t - DX + 1; u < t; ++u) n += WPW * (u + DW < nst) + XPW * (u + DX < nst);
    return n;
  };
  auto land = [&](int t) {  // this loader's pieces of stage t have landed (a loader's own counted wait)
    if constexpr (ABL != 2) {
      if (loader) wait_vmcnt_rt(younger_than(t));
    }
  };
  auto issue_step = [&](int t) {
    if (loader) {
      if (t + DW < nst) issue_w(t + DW);
      if (t + DX < nst) issue_x(t + DX);
    }
  };

  // ---- fragment read offsets inside a stage (compute waves)
  const int c = lane & 15, g = lane >> 4;
  int woff[G::TN];
#pragma unroll
  for (int tn = 0; tn < G::TN; ++tn) woff[tn] = (wn * G::TN + tn) * 2048 + lane * 16;
  int xoff[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) xoff[s] = c * 128 + (((4 * s + g) ^ (c >> 1)) << 4);
  const int xrow0 = wm * G::MB * 16 * 128;  // byte offset of this wave's first row block in the X image

  f32x4 acc[G::TN][G::MB];
#pragma unroll
  for (int tn = 0; tn < G::TN; ++tn)
#pragma unroll
    for (int mb = 0; mb < G::MB; ++mb) acc[tn][mb] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 ssq[G::MB];  // NORM: X X^T diagonal blocks of this wave's rows (slice wn of every stage)
#pragma unroll
  for (int mb = 0; mb < G::MB; ++mb) ssq[mb] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto read_slice = [&](int t, int s, bf16x8 (&af)[G::TN], bf16x8 (&bfr)[G::MB]) {
    const char* wbase = smem + (t % NW) * G::W_BYTES + s * 1024;
    const char* xbase = xring + (t % NX) * G::X_BYTES + xrow0 + xoff[s];
#pragma unroll
    for (int tn = 0; tn < G::TN; ++tn) af[tn] = *reinterpret_cast<const bf16x8*>(wbase + woff[tn]);
#pragma unroll
    for (int mb = 0; mb < G::MB; ++mb) bfr[mb] = *reinterpret_cast<const bf16x8*>(xbase + mb * 2048);
  };
  // MFMAs of one slice; `mid` runs after the first one (the next slice's reads go there, so only the first MFMA
  // waits for this slice's reads and the reads in flight never hold an MFMA back)
  auto mfma_slice = [&](int s, const bf16x8 (&af)[G::TN], const bf16x8 (&bfr)[G::MB], auto mid) {
#pragma unroll
    for (int tn = 0; tn < G::TN; ++tn)
#pragma unroll
      for (int mb = 0; mb < G::MB; ++mb) {
        acc[tn][mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[tn], bfr[mb], acc[tn][mb], 0, 0, 0);
        if (tn == 0 && mb == 0) {
          __builtin_amdgcn_sched_barrier(0);
          mid();
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    if constexpr (MSQ) {
      if (wn == s) {
#pragma unroll
        for (int mb = 0; mb < G::MB; ++mb)
          ssq[mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[mb], bfr[mb], ssq[mb], 0, 0, 0);
      }
    }
  };
  // ---- prologue: steps -DW .. -1
  if (loader) {
#pragma unroll
    for (int u = -DW; u < 0; ++u) {
      if (u + DW < nst) issue_w(u + DW);
      if (u + DX >= 0 && u + DX < nst) issue_x(u + DX);
    }
  }

  // ---- main loop: nst barriers for every wave; the barrier of stage t + 1 retires stage t's slots, which take
  // the loads of step t + 1 (every wave's reads of stage t completed: lgkmcnt(0) in ring_barrier)
  if (NDMA && !compute) {
    for (int t = 0; t < nst; ++t) {
      land(t);
      ring_barrier();
      if (t == 0) stamp(2, false);
      if (t == nst / 2) stamp(3, false);
      issue_step(t);
    }
  } else if constexpr (ABL == 1) {
    for (int t = 0; t < nst; ++t) {
      land(t);
      ring_barrier();
      issue_step(t);
    }
  } else {
    bf16x8 a0[G::TN], b0[G::MB], a1[G::TN], b1[G::MB];
    land(0);
    ring_barrier();
    stamp(2, false);
    if constexpr (!NDMA) issue_step(0);
    read_slice(0, 0, a0, b0);
    for (int t = 0; t < nst; ++t) {
      __builtin_amdgcn_sched_barrier(0);
      mfma_slice(0, a0, b0, [&] { read_slice(t, 1, a1, b1); });
      __builtin_amdgcn_sched_barrier(0);
      const bool more = t + 1 < nst;
      if (more) {
        land(t + 1);
        ring_barrier();
        if (t + 1 == nst / 2) stamp(3, false);
        if constexpr (!NDMA) issue_step(t + 1);
      }
      __builtin_amdgcn_sched_barrier(0);
      // the next stage's slice-0 reads go in after slice 1's first MFMA: issued before it, they made the
      // compiler wait for them (lgkmcnt(0)) ahead of slice 1 as well
      mfma_slice(1, a1, b1, [&] {
        if (more) read_slice(t + 1, 0, a0, b0);
      });
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  ring_barrier();  // every wave is done with the ring: its LDS becomes epilogue scratch
  stamp(4, false);

  // ---- per-row sums of squares: the diagonal of each X X^T block (lane (c, g) holds C[4g + i][c], so the
  // diagonal element of row c sits in lane c + 16 * (c >> 2), register c & 3)
  float* s_ss = reinterpret_cast<float*>(smem);  // [2][BM]
  if constexpr (MSQ) {
    if (compute && wn < 2 && (c >> 2) == g) {
#pragma unroll
      for (int mb = 0; mb < G::MB; ++mb) s_ss[wn * BM + (wm * G::MB + mb) * 16 + c] = ssq[mb][c & 3];
    }
    __syncthreads();
  }

  if (w.ks > 1) {
    // fp32 slab of this split (unit (gt, rb) = 16 x 16 outputs, lane-major f32x4: the reducer's layout) and this
    // split's per-row sums of squares.
    const int n_units = nblk * WG_NT * G::RB;
    // wgemm_reduce_kernel, the next launch on the stream, combines them
    if (compute) {
      float rs[G::MB];  // NORM: 1 / sqrt(the lane's row sum of squares over this split)
#pragma unroll
      for (int mb = 0; mb < G::MB; ++mb) {
        const int m = (wm * G::MB + mb) * 16 + c;
        rs[mb] = MSQ ? __builtin_amdgcn_rsqf(s_ss[m] + s_ss[BM + m] + 1e-30f) : 1.f;
      }
#pragma unroll
      for (int tn = 0; tn < G::TN; ++tn)
#pragma unroll
        for (int mb = 0; mb < G::MB; ++mb) {
          const int unit = (tile0 + wn * G::TN + tn) * G::RB + wm * G::MB + mb;
          const size_t e = ((size_t)kc * n_units + unit) * 64 + lane;
          if constexpr (H16) {
            // fp16 partials scaled per activation row (each lane holds one row m of the unit): NORM shapes by
            // rsqrt of the row's split sum of squares (|partial| <= sqrt(ss) * |W row|, so a row of residual-stream
            // outliers stores weight-sized values), the others by a power of two keeping the lane's largest
            // partial < 2^14 (exponent byte per lane in part_ex); the reducer multiplies back -- no cross-lane work
            // (tests/test_wgemm_gpu.py test_fp16_slabs_scale_outlier_rows; costs, profiles/r4/README.md)
            const f32x4 v = acc[tn][mb];
            f32x4 sv;
            if constexpr (MSQ) {
              sv = v * rs[mb];
            } else {
              const float mx = fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3])));
              const int ex = max(__builtin_amdgcn_frexp_expf(mx) - 14, 0);  // mx < 2^(ex + 14)
#pragma unroll
              for (int i = 0; i < 4; ++i) sv[i] = __builtin_amdgcn_ldexpf(v[i], -ex);
              if constexpr (INL) __hip_atomic_store(w.part_ex + e, (uint8_t)ex, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              else w.part_ex[e] = (uint8_t)ex;
            }
            f16x4 h;  // (the clamp only bites on non-finite partials)
#pragma unroll
            for (int i = 0; i < 4; ++i) h[i] = (_Float16)fminf(fmaxf(sv[i], -65504.f), 65504.f);
            if constexpr (INL)  // write-through: read by the partners' combine in this launch
              __hip_atomic_store(reinterpret_cast<uint64_t*>(w.part) + e, __builtin_bit_cast(uint64_t, h),
                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else
              reinterpret_cast<f16x4*>(w.part)[e] = h;
          } else if constexpr (INL) {
            const f32x4 v = acc[tn][mb];
            uint64_t* d = reinterpret_cast<uint64_t*>(reinterpret_cast<f32x4*>(w.part) + e);
            __hip_atomic_store(d, __builtin_bit_cast(uint64_t, f32x2{v[0], v[1]}), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(d + 1, __builtin_bit_cast(uint64_t, f32x2{v[2], v[3]}), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
          } else {
            reinterpret_cast<f32x4*>(w.part)[e] = acc[tn][mb];
          }
        }
    }
    if constexpr (NORM) {
      for (int r = threadIdx.x; r < BM; r += NTHR) {
        float* d = w.part_ss + ((size_t)blk * w.ks + kc) * BM + r;
        if constexpr (INL) __hip_atomic_store(d, s_ss[r] + s_ss[BM + r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else *d = s_ss[r] + s_ss[BM + r];
      }
    }
    if constexpr (INL) {
      // two words of the (drained) ring past the row sums: the kernel's LDS is all dynamic, sized to 160 KiB, so
      // a static __shared__ here would not fit
      wg_inline_combine<BM, EPI, NORM, H16>(a, w, blk, kc, nblk * WG_NT * G::RB, NTHR,
                                            reinterpret_cast<unsigned*>(smem + 2 * BM * sizeof(float)));
      return;
    }
    if constexpr (ABL == 3) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      stamp(5, false);
      stamp(6, false);
      stamp(7, true);
    }
    return;
  }
  if (!compute) return;

  // ---- fused epilogue (ks = 1); the RMSNorm scale once per row block
  float rn[G::MB];
#pragma unroll
  for (int mb = 0; mb < G::MB; ++mb) {
    const int m = (wm * G::MB + mb) * 16 + c;
    rn[mb] = NORM ? rms_inv(s_ss[m] + s_ss[BM + m], a.K, a.eps) : 1.f;
  }
#pragma unroll
  for (int tn = 0; tn < G::TN; ++tn) {
    const int gt = tile0 + wn * G::TN + tn;
#pragma unroll
    for (int mb = 0; mb < G::MB; ++mb) {
      const int rb = wm * G::MB + mb;
      const int m = rb * 16 + c;
      f32x4 v = acc[tn][mb];
      if constexpr (NORM) v *= rn[mb];
      // the pair epilogues read the partner rows (+8 of the tile) from lane + 32: exchanged by every lane
      f32x4 pv;
#pragma unroll
      for (int i = 0; i < 4; ++i) pv[i] = __shfl_xor(v[i], 32, 64);
      if (gt < ntiles) {
        const EpiIn e = epi_load_at<EPI>(a, gt, m, lane);
        epi_store<EPI>(a, gt, m, lane, e, [&](int off) { return off ? pv : v; });
      }
      if constexpr (EPI == EPI_F32) {
        // LM head: this 16-column chunk's maximum of row m (lanes c, c + 16, c + 32, c + 48), as gemm.hip's skinny
        // kernel writes it for the chunk-maximum sampler
        if (a.cmax) {
          float mx = fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3]));
          mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
          mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
          if ((lane >> 4) == 0 && gt < ntiles && m < a.M) a.cmax[(size_t)m * a.ld_cm + gt] = mx;
        }
      }
    }
  }
  if constexpr (ABL == 3) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    stamp(5, false);
    stamp(6, false);
    stamp(7, true);
  }
}

// Split-K combine + fused epilogue: one wave per 16 x 16 output unit.  The kernel is a few dependent memory
// round trips long, so every load goes out before the first add: the epilogue inputs (residual row, RoPE position
// and then its cos / sin) first, then all KS slab pieces and row sums (KS a compile-time split count; KS = 0 is
// the runtime-count fallback).  Issued after the sum, as before, the epilogue loads were one more round trip
// (two for QKV: position, then the tables).
template <int BM, int EPI, bool NORM, int KS, bool H16 = false>
__global__ __launch_bounds__(256) void wgemm_reduce_kernel(const GemmArgs a, const WgArgs w, int n_units) {
  const int lane = threadIdx.x & 63;
  // this workgroup's 4 units on the XCD that wrote their column block's slabs (wg_block_of; w.bnt tiles per block)
  const int unit = wg_reduce_block(blockIdx.x, w.bnt * (BM / 16) / 4, w.xcd_blk) * 4 + (threadIdx.x >> 6);
  if (unit >= n_units) return;
  wg_reduce_unit<BM, EPI, NORM, H16, false>(a, w, unit, n_units, lane, KS ? KS : w.ks);
}

// One unit's combine: the ks slab pieces (+ row sums / exponents), the epilogue.  COH: the slabs were published
// write-through by partners still running in this launch -- read them with agent-scope loads (past this CU's L1),
// as the W4 split-K and the attention merge do.  Up to WG_INL_KS pieces are loaded before the first add.
constexpr int WG_INL_KS = 8;
template <int BM, int EPI, bool NORM, bool H16, bool COH>
__device__ __forceinline__ void wg_reduce_unit(const GemmArgs& a, const WgArgs& w, int unit, int n_units, int lane,
                                               int ks) {
  constexpr int RB = BM / 16;
  const int gt = unit / RB, rb = unit - gt * RB;
  const int ntiles = a.N >> 4;
  const int m = rb * 16 + (lane & 15);
  const bool live = gt < ntiles;
  const EpiIn e = live ? epi_load_at<EPI>(a, gt, m, lane) : EpiIn{};
  using slab_t = std::conditional_t<H16, f16x4, f32x4>;
  const slab_t* src = reinterpret_cast<const slab_t*>(w.part) + (size_t)unit * 64 + lane;
  auto ld_slab = [&](int k) -> f32x4 {
    const slab_t* q = src + (size_t)k * n_units * 64;
    if constexpr (COH && H16) {
      const f16x4 h = __builtin_bit_cast(f16x4, __hip_atomic_load(reinterpret_cast<const uint64_t*>(q),
                                                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
      return f32x4{(float)h[0], (float)h[1], (float)h[2], (float)h[3]};
    } else if constexpr (COH) {
      const uint64_t* d = reinterpret_cast<const uint64_t*>(q);
      const f32x2 lo = __builtin_bit_cast(f32x2, __hip_atomic_load(d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
      const f32x2 hi = __builtin_bit_cast(f32x2, __hip_atomic_load(d + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
      return f32x4{lo[0], lo[1], hi[0], hi[1]};
    } else if constexpr (H16) {
      const f16x4 h = *q;
      return f32x4{(float)h[0], (float)h[1], (float)h[2], (float)h[3]};
    } else {
      return *q;
    }
  };
  const uint8_t* exsrc = w.part_ex + (size_t)unit * 64 + lane;  // H16 without NORM: the lane's exponent per split
  auto ld_ex = [&](int k) -> int {
    const uint8_t* q = exsrc + (size_t)k * n_units * 64;
    if constexpr (COH) return __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else return *q;
  };
  const float* ssrc = w.part_ss + (size_t)(gt / w.bnt) * ks * BM + m;
  auto ld_ss = [&](int k) -> float {
    if constexpr (COH) return __hip_atomic_load(ssrc + k * BM, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else return ssrc[k * BM];
  };
  auto unscale = [](f32x4 x, int ex) {
#pragma unroll
    for (int i = 0; i < 4; ++i) x[i] = __builtin_amdgcn_ldexpf(x[i], ex);
    return x;
  };
  f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
  float ss = 0.f;
  f32x4 p[WG_INL_KS];
  float q[WG_INL_KS];
  int ex[WG_INL_KS];
  // every piece's loads before the first add (up to WG_INL_KS; more pieces in a second pass).  No branch around a
  // load: past the last piece a lane re-loads the last one (a cache hit) and adds it times 0 -- a conditional load
  // made hipcc wait for each one (vmcnt(0) per piece: one memory round trip per piece)
  for (int k0 = 0; k0 < ks; k0 += WG_INL_KS) {
#pragma unroll
    for (int k = 0; k < WG_INL_KS; ++k) p[k] = ld_slab(min(k0 + k, ks - 1));
    if constexpr (H16 && !NORM) {
#pragma unroll
      for (int k = 0; k < WG_INL_KS; ++k) ex[k] = ld_ex(min(k0 + k, ks - 1));
    }
    if constexpr (NORM) {
#pragma unroll
      for (int k = 0; k < WG_INL_KS; ++k) q[k] = ld_ss(min(k0 + k, ks - 1));
    }
#pragma unroll
    for (int k = 0; k < WG_INL_KS; ++k) {
      const float on = k0 + k < ks ? 1.f : 0.f;
      if constexpr (H16 && NORM) v += p[k] * (__builtin_sqrtf(q[k] + 1e-30f) * on);
      else if constexpr (H16) v += unscale(p[k], ex[k]) * on;
      else v += p[k] * on;
      if constexpr (NORM) ss += q[k] * on;
    }
  }
  if constexpr (NORM) v *= rms_inv(ss, a.K, a.eps);
  f32x4 pv;
#pragma unroll
  for (int i = 0; i < 4; ++i) pv[i] = __shfl_xor(v[i], 32, 64);
  if (!live) return;
  epi_store<EPI>(a, gt, m, lane, e, [&](int off) { return off ? pv : v; });
}

// In-launch split-K combine (the three wgemm_reduce_kernel launches per layer were 0.62 ms of the
// 8.98 ms headline step).  The ks partners of a column block are one workgroup per CU, all resident together (the
// host takes this path only when the grid fits the CU budget), so after publishing its slab write-through each
// partner arrives on the block's ticket and WAITS for the others -- bounded: past WG_INL_SPIN the wait gives up --
// then claims its own 1/ks of the block's units (one bit of the block's claim word) and combines them.  The LAST
// arriver never waits: it combines its own piece, then claims every piece still unclaimed (a partner that gave up
// waiting, or has not claimed yet) and combines those too, so the block completes whatever the residency; the
// claim bit decides who combines a piece, exactly once.  The workgroup that leaves the block last resets its three
// words (arrivals, claims, exits) for the next launch.  Counters: w.counters[3 * blk + {0, 1, 2}], zero at rest.
constexpr long long WG_INL_SPIN = 20000;  // s_memrealtime ticks (100 MHz): 200 us
template <int BM, int EPI, bool NORM, bool H16>
__device__ void wg_inline_combine(const GemmArgs& a, const WgArgs& w, int blk, int kc, int n_units, int nthr,
                                  unsigned* flags) {
  unsigned& s_go = flags[0];
  unsigned& s_claim = flags[1];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nwaves = nthr >> 6;
  unsigned* ctr = w.counters + 3 * blk;
  const int ks = w.ks;
  const unsigned all = ks >= 32 ? 0xffffffffu : (1u << ks) - 1u;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this thread's slab stores are done
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned go = t + 1 == unsigned(ks) ? 2u : 0u;  // 2: last arriver
    if (!go) {
      const long long t0 = __builtin_amdgcn_s_memrealtime();
      while (true) {
        if (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= unsigned(ks)) {
          go = 1u;
          break;
        }
        if (__builtin_amdgcn_s_memrealtime() - t0 > w.spin) break;
        __builtin_amdgcn_s_sleep(2);
      }
    }
    s_go = go;
    s_claim = go ? (__hip_atomic_fetch_or(ctr + 1, 1u << kc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> kc) & 1u
                 : 1u;  // 1: not mine to combine
  }
  __syncthreads();
  const int upb = WG_NT * (BM / 16);  // units per column block
  const int u0 = blk * upb;
  auto combine = [&](int piece) {  // units [piece * upb / ks, (piece + 1) * upb / ks) of the block
    const int b = piece * upb / ks, e = (piece + 1) * upb / ks;
    for (int u = b + wave; u < e; u += nwaves) wg_reduce_unit<BM, EPI, NORM, H16, true>(a, w, u0 + u, n_units, lane, ks);
  };
  if (!s_claim) combine(kc);
  if (s_go == 2u) {
    __syncthreads();
    if (threadIdx.x == 0)
      s_claim = __hip_atomic_fetch_or(ctr + 1, all, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const unsigned left = ~s_claim & all;
    for (int pc = 0; pc < ks; ++pc)
      if ((left >> pc) & 1u) combine(pc);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    if (__hip_atomic_fetch_add(ctr + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1 == unsigned(ks)) {
      // every partner is past its last use of the block's words: ready for the next launch (launch-ordered)
      __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ctr + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ctr + 2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

template <int BM, int EPI, bool NORM, bool H16 = false>
void wg_reduce_launch(const GemmArgs& a, const WgArgs& w, int n_units, hipStream_t st) {
  const dim3 grid((n_units + 3) / 4), blk(256);
  switch (w.ks) {
#define CAIN_WG_RED(K) \
  case K: hipLaunchKernelGGL((wgemm_reduce_kernel<BM, EPI, NORM, K, H16>), grid, blk, 0, st, a, w, n_units); return;
    CAIN_WG_RED(2) CAIN_WG_RED(3) CAIN_WG_RED(4) CAIN_WG_RED(5) CAIN_WG_RED(6) CAIN_WG_RED(7) CAIN_WG_RED(8)
    CAIN_WG_RED(10) CAIN_WG_RED(12) CAIN_WG_RED(16)
#undef CAIN_WG_RED
    default: hipLaunchKernelGGL((wgemm_reduce_kernel<BM, EPI, NORM, 0, H16>), grid, blk, 0, st, a, w, n_units);
  }
}

namespace {

struct WgPlan {
  int bm, nblk, ks, kst;
  size_t part_floats, ss_floats, sc_floats;
  int variant = 0;  // ring variant (wg_launch_v)
  int bnt = WG_NT;  // 16-column tiles per column block
};

// Split count: ~256 streaming workgroups (one per CU: the ring takes 128-144 KiB of LDS), at most 8 splits and
// at least 4 stages per split.  Column-block counts >= 128 (gate/up, LM head) run unsplit.
int g_wg_target = -1, g_wg_ksmax = -1;

// Per-shape plan overrides (split count, ring variant) keyed by (N, K, row tile): set before any graph is captured
// (engine CAIN_WGEMM_PLANS, tools/wgemm_bench.py) for in-graph A/B runs of split plans.
// The default split rule is a heuristic; measured on one box at 256 rows, the O projection (N = K = 4096) ran
// 24.7 us at 6 splits against 29.4 at 8 and 29.5 at 4, and the best split and ring differ per shape.
struct WgShape {
  int N, K, bm, ks, variant;
};
constexpr int WG_MAX_SHAPES = 64;
WgShape g_wg_shapes[WG_MAX_SHAPES];
int g_wg_nshapes = 0;

const WgShape* wg_shape(int N, int K, int bm) {
  for (int i = 0; i < g_wg_nshapes; ++i) {
    const WgShape& s = g_wg_shapes[i];
    if (s.N == N && s.K == K && s.bm == bm) return &s;
  }
  return nullptr;
}

int g_wgemm_variant = 0;
// (round 5's 256-column kernel, variants 5-7 / 10 / 11, measured slower on every headline shape -- 24.1k against
// 28.4k tok/s, profiles/r5/README.md -- and left the shipped library in round 6: tools/attic/wgemm256.hip)

WgPlan wg_plan(int N, int K, int M) {
  const int target = g_wg_target > 0 ? g_wg_target : 256, ksmax = g_wg_ksmax > 0 ? g_wg_ksmax : 8;
  WgPlan p{};
  p.bm = M > 128 ? 256 : 128;
  {
    const WgShape* o = wg_shape(N, K, p.bm);
    p.variant = o && o->variant >= 0 ? o->variant : g_wgemm_variant;
  }
  p.nblk = ((N >> 4) + WG_NT - 1) / WG_NT;
  const int stages = K / WG_BK;
  int ks = p.nblk >= 128 ? 1 : std::max(1, std::min(ksmax, (target + p.nblk / 2) / p.nblk));
  // 256-row tiles with short splits (< 16 stages): ~3/4 of the workgroups, longer splits and fewer slabs.  In the
  // graph-replayed headline (llama3.1:8b, gpurun_out/r20-r21, same box, interleaved): O 8 -> 6 splits and QKV
  // 5 -> 4 took 26.5k -> 26.7k tok/s (each alone +1 %); down (28 stages per split at 8) lost at 6.
  if (p.bm == 256 && ks > 1 && stages / ks < 16) ks = std::max(1, std::min(ks, (target * 3 / 4 + p.nblk / 2) / p.nblk));
  if (const WgShape* o = wg_shape(N, K, p.bm)) {
    if (o->ks > 0) ks = o->ks;
  }
  ks = std::min(ks, std::max(1, stages / 4));
  p.kst = (stages + ks - 1) / ks;
  p.ks = (stages + p.kst - 1) / p.kst;
  if (p.ks > 1) {
    p.part_floats = (size_t)p.ks * p.nblk * WG_NT * (p.bm / 16) * 256;
    p.ss_floats = (size_t)p.nblk * p.ks * p.bm;
    p.sc_floats = (size_t)p.ks * p.nblk * WG_NT * (p.bm / 16) * 16;  // one exponent byte per lane per unit
  }
  return p;
}

// In-launch split-K combine (wg_inline_combine): cain_wgemm_set_inline(1) (CAIN_WGEMM_INLINE=1); 0 (default) the separate
// wgemm_reduce_kernel launch (A/B, tests).  Taken only where every partner can be resident at once -- one
// workgroup per CU (the ring's LDS), so grid <= the CU budget -- and the block's words fit the counter region.
int g_wg_inline = 0;
inline bool wg_use_inline(const WgPlan& p) {
  return g_wg_inline && p.ks > 1 && p.ks <= 32 && p.nblk * p.ks <= cain_cu_budget() &&
         3 * p.nblk * (int)sizeof(unsigned) <= WG_CTR_BYTES;
}

template <int BM, int DX, int DW, int EPI, bool NORM, int NDMA, int ABL = 0, bool H16 = true>
hipError_t wg_launch(const GemmArgs& a, const WgArgs& w, const WgPlan& p, hipStream_t st) {
  using G = WgGeo<BM>;
  constexpr int lds = (DW + 1) * G::W_BYTES + (DX + 1) * G::X_BYTES;
  static_assert(lds <= 160 * 1024, "LDS");
  auto set_lds = [](const void* k) {
    return hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, lds) == hipSuccess;
  };
  if constexpr (ABL == 0) {
    if (wg_use_inline(p)) {
      static bool attr_inl = set_lds(reinterpret_cast<const void*>(&wgemm_kernel<BM, DX, DW, EPI, NORM, NDMA, 0, H16, true>));
      if (!attr_inl) return hipErrorInvalidConfiguration;
      hipLaunchKernelGGL((wgemm_kernel<BM, DX, DW, EPI, NORM, NDMA, 0, H16, true>), dim3(p.nblk * p.ks),
                         dim3(64 * (8 + NDMA)), lds, st, a, w);
      return hipGetLastError();
    }
  }
  static bool attr = set_lds(reinterpret_cast<const void*>(&wgemm_kernel<BM, DX, DW, EPI, NORM, NDMA, ABL, H16>));
  if (!attr) return hipErrorInvalidConfiguration;
  hipLaunchKernelGGL((wgemm_kernel<BM, DX, DW, EPI, NORM, NDMA, ABL, H16>), dim3(p.nblk * p.ks), dim3(64 * (8 + NDMA)),
                     lds, st, a, w);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || p.ks == 1) return e;
  wg_reduce_launch<BM, EPI, NORM, H16>(a, w, p.nblk * WG_NT * G::RB, st);
  return hipGetLastError();
}

// variants: 0 = default (fp16 split-K slabs: in the graph-replayed headline 26.33 / 26.17k -> 27.34 / 27.17k tok/s
// against fp32 slabs, same box, interleaved, profiles/r3/README.md); 4 = fp32 slabs (tests, A/B); diagnostics of
// tools/wgemm_trace.py / wgemm_bench.py: 7 = default + timestamps, 8 = DMA only, 9 = fragment reads + MFMAs only
// (results garbage).  Set with cain_wgemm_set_variant / cain_wgemm_set_shape.

template <int BM, int EPI, bool NORM>
hipError_t wg_launch_v(const GemmArgs& a, const WgArgs& w, const WgPlan& p, hipStream_t st) {
  const int variant = p.variant;
  if constexpr (BM == 256) {  // X stage 32 KiB, W stage 16 KiB: 160 KiB of ring
    switch (variant) {
      case 4: return wg_launch<BM, 2, 3, EPI, NORM, 4, 0, false>(a, w, p, st);
      case 7: return wg_launch<BM, 2, 3, EPI, NORM, 4, 3>(a, w, p, st);
      case 8: return wg_launch<BM, 2, 3, EPI, NORM, 4, 1>(a, w, p, st);
      case 9: return wg_launch<BM, 2, 3, EPI, NORM, 4, 2>(a, w, p, st);
      default: return wg_launch<BM, 2, 3, EPI, NORM, 4>(a, w, p, st);
    }
  } else {  // X stage 16 KiB, W stage 16 KiB: 160 KiB of ring
    switch (variant) {
      case 4: return wg_launch<BM, 3, 5, EPI, NORM, 4, 0, false>(a, w, p, st);
      default: return wg_launch<BM, 3, 5, EPI, NORM, 4>(a, w, p, st);
    }
  }
}

template <int BM, bool NORM>
hipError_t wg_launch_e(int epi, const GemmArgs& a, const WgArgs& w, const WgPlan& p, hipStream_t st) {
  switch (epi) {
    case EPI_BF16: return wg_launch_v<BM, EPI_BF16, NORM>(a, w, p, st);
    case EPI_RESID: return wg_launch_v<BM, EPI_RESID, NORM>(a, w, p, st);
    case EPI_F32: return wg_launch_v<BM, EPI_F32, NORM>(a, w, p, st);
    case EPI_SILU: return wg_launch_v<BM, EPI_SILU, NORM>(a, w, p, st);
    case EPI_GELU: return wg_launch_v<BM, EPI_GELU, NORM>(a, w, p, st);
    case EPI_QKV_ROPE: return wg_launch_v<BM, EPI_QKV_ROPE, NORM>(a, w, p, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

// Rows from which the wide kernel takes a GEMM (default 64: M in (64, 256]; 0 disables; cain_wgemm_set_min_m).
static int g_wgemm_min_m = 64;
CAIN_API int cain_wgemm_min_m() { return g_wgemm_min_m; }
// A/B switches for tests and tuning tools (take effect for launches and graph captures after the call).
CAIN_API void cain_wgemm_set_min_m(int m) { g_wgemm_min_m = m; }
CAIN_API void cain_wgemm_set_variant(int v) { g_wgemm_variant = v; }
// 0: separate reduce launch; 1: in-launch combine (default); 2: in-launch combine whose partners never wait, so the
// last arriver combines every piece (the give-up path, for tests)
CAIN_API void cain_wgemm_set_inline(int mode) { g_wg_inline = mode < 0 ? 0 : mode > 2 ? 2 : mode; }
CAIN_API int cain_wgemm_get_inline() { return g_wg_inline; }

CAIN_API void cain_wgemm_set_split(int target, int ksmax) { g_wg_target = target, g_wg_ksmax = ksmax; }
// Per-shape plan: split count (<= 0: the default rule) and ring variant (< 0: the global one) for GEMMs of N
// columns over K with the bm-row tile (128 or 256).  Returns 0, or -1 when the table is full.
CAIN_API int cain_wgemm_set_shape(int N, int K, int bm, int ks, int variant) {
  for (int i = 0; i < g_wg_nshapes; ++i) {
    WgShape& s = g_wg_shapes[i];
    if (s.N == N && s.K == K && s.bm == bm) {
      s.ks = ks, s.variant = variant;
      return 0;
    }
  }
  if (g_wg_nshapes == WG_MAX_SHAPES) return -1;
  g_wg_shapes[g_wg_nshapes++] = WgShape{N, K, bm, ks, variant};
  return 0;
}
CAIN_API void cain_wgemm_clear_shapes() { g_wg_nshapes = 0; }
// Timestamp buffer of the diagnostic variant 7 (>= grid * 16 uint64; tools/wgemm_trace.py).
static unsigned long long* g_wg_stamps = nullptr;
CAIN_API void cain_wgemm_set_stamps(void* p) { g_wg_stamps = static_cast<unsigned long long*>(p); }
CAIN_API int cain_wgemm_eligible(int N, int K, int M);
// The plan the next launch of this shape would use: ks * 64 + variant (tests, tools).
CAIN_API int cain_wgemm_plan(int N, int K, int M) {
  if (!cain_wgemm_eligible(N, K, M)) return -1;
  const WgPlan p = wg_plan(N, K, M);
  return p.ks * 64 + p.variant;
}

CAIN_API int cain_wgemm_eligible(int N, int K, int M) {
  const int mm = cain_wgemm_min_m();
  return mm > 0 && M > mm && M <= 256 && K % WG_BK == 0 && N % 16 == 0 && K >= 4 * WG_BK;
}

CAIN_API int cain_wgemm_inline(int N, int K, int M) {  // 1: this shape's next launch combines in-launch
  return cain_wgemm_eligible(N, K, M) && wg_use_inline(wg_plan(N, K, M));
}

CAIN_API long long cain_wgemm_ws_bytes(int N, int K, int M) {
  if (!cain_wgemm_eligible(N, K, M)) return 0;
  const WgPlan p = wg_plan(N, K, M);
  return (long long)(WG_CTR_BYTES + (p.part_floats + p.ss_floats + p.sc_floats) * sizeof(float));
}


// a: the GEMM (gemm_epi.h); ws: >= cain_wgemm_ws_bytes of scratch (no zeroing needed).
int wgemm_dispatch(const GemmArgs& a, int epi, bool norm, void* ws, long long ws_bytes, hipStream_t st) {
  if (!cain_wgemm_eligible(a.N, a.K, a.M)) return -1;
  const WgPlan p = wg_plan(a.N, a.K, a.M);
  if ((long long)(WG_CTR_BYTES + (p.part_floats + p.ss_floats + p.sc_floats) * sizeof(float)) > ws_bytes) return -1;
  WgArgs w{};
  w.ks = p.ks;
  w.kst = p.kst;
  // XCD-local split-K: the split partners of a column block, and the reduce workgroups of its units, run on one
  // XCD (blocks b and b + 8 share one under round-robin dispatch), so the reduce reads the slabs from the L2
  // that holds them instead of across the fabric.  Measured on the headline (rocprof, gpurun_out/r15): O / down
  // reduce 8.7 -> 6.9 us, QKV 22.5 + 11.2 -> 20.1 + 10.9 us, O / down main +1.1 us (their X panels are now
  // fetched per XCD); 25.8k -> 26.3k tok/s.
  w.xcd_blk = p.ks > 1 && p.nblk % 8 == 0;
  w.bnt = p.bnt;
  // [counter region: 3 words per column block for the in-launch combine, zero at rest][slabs][sums]
  w.counters = static_cast<unsigned*>(ws);
  w.stamps = g_wg_stamps;
  w.spin = g_wg_inline == 2 ? 0 : WG_INL_SPIN;
  w.part = reinterpret_cast<float*>(static_cast<char*>(ws) + WG_CTR_BYTES);
  w.part_ss = w.part + p.part_floats;
  w.part_ex = reinterpret_cast<uint8_t*>(w.part_ss + p.ss_floats);
  hipError_t e;
  if (p.bm == 256) e = norm ? wg_launch_e<256, true>(epi, a, w, p, st) : wg_launch_e<256, false>(epi, a, w, p, st);
  else e = norm ? wg_launch_e<128, true>(epi, a, w, p, st) : wg_launch_e<128, false>(epi, a, w, p, st);
  return int(e);
}
