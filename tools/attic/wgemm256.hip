// Wide-batch projection GEMM with 256-column workgroup tiles (BM = 256 rows x BN = 256 columns), gfx950.
//
//   Y[m][n] = epilogue( inv[m] * sum_k X[m][k] * W[n][k] )        (M in (128, 256]: the trial-batched decode step)
//
// Replaces, like wgemm.hip, the per-token GEMVs llama.cpp runs inside Ollama for the reference's workload (reference
// experiment/RunnerConfig.py:128-131; SURVEY §2.4 rows QKV / O / gate-up / down / LM head), at the headline's 256 rows.
//
// Why a second wide kernel.  At 256 rows a workgroup has to ingest its weight slice AND the activation panel it
// multiplies through the CU's load path, which sustains ~30 B/clk per CU (profiles/r3: the down projection's loop
// ran 1,590 clk per 48 KiB stage at 1.59 GHz); wgemm.hip's 256 x 128 tile ingests (BM + BN) / BN = 3 bytes per
// weight byte and is bound there, at ~half of its MFMA rate.  A 256 x 256 tile ingests 2 bytes per weight byte and
// does twice the MACs per ingested byte, so the same load path feeds the matrix cores ~1.5x faster (VERDICT r4
// item 1: "256-column tiles").  What that takes:
//
//   * accumulators: 256 x 256 fp32 = 128 registers per lane over 8 waves, so 2 waves per SIMD and NO loader waves
//     (a 3rd wave per SIMD would cap every wave at 168 registers): every wave issues its own LDS-DMA, 2 W + 2 X
//     pieces (1 KiB each) per 32-deep stage, spread over its MFMAs so the other wave of the SIMD keeps the matrix
//     pipe busy while it issues (MI355X_MICROARCH.md: an LDS-DMA piece costs ~60 issue cycles among MFMAs);
//   * v_mfma_f32_32x32x16_bf16: each wave owns a 128-row x 64-column block = 4 x 2 MFMA blocks of 32 x 32; per
//     16-deep k step it reads 4 X + 2 W fragments (6 ds_read_b128) for 8 MFMAs (256 matrix cycles), and a 32x32
//     fragment is half the registers of the 16x16x32 form for the same k, so both k steps' fragments fit
//     double-buffered (48 VGPRs) beside the 128 accumulators;
//   * W tiles come straight from the engine's 16x16x32 fragment-major packing (models/weights.py pack_mfma_a: a
//     16-row x 32-k block is 1 KiB contiguous): one DMA piece per tile per stage, and a 32x32x16 A fragment is
//     the k-group pair (2s, 2s + 1) of two adjacent tiles -- lanes 0-15 / 16-31 read tile 2b / 2b + 1, 256 B
//     apart per 16-lane group: conflict-free ds_read_b128;
//   * X (activations, [M][ldx] bf16, L2-resident) is staged 64 B per row per stage, 16 rows per DMA piece, XOR-
//     swizzled by permuting the per-lane SOURCE piece: LDS slot q of row r holds global piece q ^ ((r >> 2) & 3),
//     which makes every 16-lane group of the B-fragment ds_read_b128 hit 16 distinct bank quads;
//   * ring: 5 W + 5 X slots of 16 KiB = 160 KiB, prefetch distance 4 stages; one raw s_barrier per stage, placed
//     between the stage's two k steps so the next step's fragments are already in registers and no wave restarts
//     the matrix pipe behind a barrier (as wgemm.hip);
//   * fused RMSNorm (gain folded into W): the row sums of squares come from the MFMA unit, mfma(x, x) accumulating
//     X X^T over all k for one 32-row X block per wave (8 waves = 8 blocks; the wave's X blocks are held rotated
//     so that one is register block 0), whose diagonal is each row's sum of squares: one extra MFMA per 8, and 16
//     registers.
//
// Split-K (the narrow QKV / O / down shapes; gate/up runs 2 splits so 224 workgroups stream): each split stores its
// 16x16 units as fp16 slabs in wgemm.hip's layout (scaled per activation row: NORM by rsqrt of the row's split sum
// of squares, else by a power of two per lane) and wgemm.hip's wgemm_reduce_kernel sums them and runs the fused
// epilogue.  Unsplit (the LM head), each wave stages its 32x32 blocks through LDS into the 16x16 unit layout of
// gemm_epi.h and runs the epilogue itself (fp32 logits + the sampler's 16-column chunk maxima).
#include <algorithm>

#include "common.h"
#include "gemm_epi.h"
#include "wgemm_ring.h"

using namespace wg;

typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace w256 {
constexpr int NT = 16;                         // 16-column tiles per workgroup (BN = 256)
constexpr int BM = 256;                        // rows per workgroup
constexpr int BK = 32;                         // k per W stage (an X stage is 2 W stages: 64 k)
constexpr int NSW = 6, NSX = 2;                // ring slots: W (32-deep stages), X (64-deep stages)
constexpr int DW = NSW - 1;                    // W prefetch distance (W stages in flight)
constexpr int W_BYTES = NT * 1024;             // one W stage: 16 tiles x one 32-k slice of 1 KiB
constexpr int X_BYTES = BM * 2 * BK * 2;       // one X stage: 256 rows x 128 B
constexpr int LDS = NSW * W_BYTES + NSX * X_BYTES;  // 96 + 64 = 160 KiB
constexpr int SCR = 32 * 36;                   // floats of one wave's 32x32 epilogue staging block (rows padded)
}  // namespace w256

// Epilogue of the 256-column kernels, by the 8 compute waves (wave = 2 wn + wm): split-K slabs (ks > 1) or the
// fused epilogue (ks = 1).  s_ss: the row sums of squares (NORM) in LDS; the ring is free (scratch).
// ROT: register block xb holds X row block (xb + wn) & 3 (wg256_kernel), else xb (wg256l_kernel).
template <int EPI, bool NORM, bool ROT = true>
__device__ __forceinline__ void wg256_epilogue(const GemmArgs& a, const WgArgs& w, f32x16 (&acc)[2][4],
                                               const float* s_ss, char* smem, int wave, int lane, int wm, int wn,
                                               int tile0, int blk, int kc) {
  using namespace w256;
  const int ntiles = a.N >> 4;
  const int c32 = lane & 31, h = lane >> 5;
  auto xr = [&](int xb) { return ROT ? (xb + wn) & 3 : xb; };
  if (w.ks > 1) {
    // fp16 slabs in wgemm.hip's unit layout (wgemm_reduce_kernel): unit (gt, rb) = 16 x 16 outputs, lane
    // l' = 16 g' + c' holding row c' and columns 4 g' .. 4 g' + 3.  This lane holds, for MFMA block (wb, xb), row
    // m = 128 wm + 32 xr(xb) + c32 and columns 8 q + 4 h + i of the block (q = 2 a + s: 16-column tile a, g' = 2 s + h)
    const int n_units = ntiles * (BM / 16);
    float rs[4];
#pragma unroll
    for (int xb = 0; xb < 4; ++xb) {
      const int m = 128 * wm + 32 * xr(xb) + c32;
      rs[xb] = NORM ? __builtin_amdgcn_rsqf(s_ss[m] + 1e-30f) : 1.f;
    }
#pragma unroll
    for (int wb = 0; wb < 2; ++wb)
#pragma unroll
      for (int xb = 0; xb < 4; ++xb) {
        const int rb = 2 * (4 * wm + xr(xb)) + ((lane >> 4) & 1);
#pragma unroll
        for (int ta = 0; ta < 2; ++ta) {
          const int gt = tile0 + 4 * wn + 2 * wb + ta;
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            const int q = 2 * ta + s;
            const size_t e = ((size_t)kc * n_units + (size_t)gt * (BM / 16) + rb) * 64 + 16 * (2 * s + h) + (lane & 15);
            f32x4 v{acc[wb][xb][4 * q], acc[wb][xb][4 * q + 1], acc[wb][xb][4 * q + 2], acc[wb][xb][4 * q + 3]};
            f32x4 sv;
            if constexpr (NORM) {
              sv = v * rs[xb];  // |partial| <= sqrt(ss) |W row|: weight-sized after the scale
            } else {
              const float mx = fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3])));
              const int ex = max(__builtin_amdgcn_frexp_expf(mx) - 14, 0);  // mx < 2^(ex + 14)
#pragma unroll
              for (int i = 0; i < 4; ++i) sv[i] = __builtin_amdgcn_ldexpf(v[i], -ex);
              w.part_ex[e] = (uint8_t)ex;
            }
            f16x4 hv;
#pragma unroll
            for (int i = 0; i < 4; ++i) hv[i] = (_Float16)fminf(fmaxf(sv[i], -65504.f), 65504.f);
            reinterpret_cast<f16x4*>(w.part)[e] = hv;
          }
        }
      }
    if constexpr (NORM) {
      for (int r = lane + 64 * wave; r < BM; r += 512) w.part_ss[((size_t)blk * w.ks + kc) * BM + r] = s_ss[r];
    }
    return;
  }

  // ---- unsplit: fused epilogue.  Each wave stages one 32x32 block at a time through its own LDS scratch into the
  // unit layout (row-major [m][n], rows padded to 36 floats), then runs gemm_epi.h's epilogue per 16x16 unit.
  // Wave-local: LDS operations of one wave execute in order, so no barrier is needed between the writes and reads.
  float* scr = reinterpret_cast<float*>(smem + 4096) + wave * SCR;
  float rn[4];
#pragma unroll
  for (int xb = 0; xb < 4; ++xb) {
    const int m = 128 * wm + 32 * xr(xb) + c32;
    rn[xb] = NORM ? rms_inv(s_ss[m], a.K, a.eps) : 1.f;
  }
  const int cp = lane & 15, gp = lane >> 4;
#pragma unroll
  for (int wb = 0; wb < 2; ++wb)
#pragma unroll
    for (int xb = 0; xb < 4; ++xb) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x4 v{acc[wb][xb][4 * q], acc[wb][xb][4 * q + 1], acc[wb][xb][4 * q + 2], acc[wb][xb][4 * q + 3]};
        *reinterpret_cast<f32x4*>(scr + c32 * 36 + 8 * q + 4 * h) = v * rn[xb];
      }
#pragma unroll
      for (int ta = 0; ta < 2; ++ta) {
        const int gt = tile0 + 4 * wn + 2 * wb + ta;
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          const int m = 128 * wm + 32 * xr(xb) + 16 * b + cp;
          const float* row = scr + (16 * b + cp) * 36 + 16 * ta;
          const f32x4 v0 = *reinterpret_cast<const f32x4*>(row + 4 * gp);
          const f32x4 v32 = *reinterpret_cast<const f32x4*>(row + 4 * (gp ^ 2));  // partner rows +8: lane + 32
          if (gt < ntiles) {
            const EpiIn e = epi_load_at<EPI>(a, gt, m, lane);
            epi_store<EPI>(a, gt, m, lane, e, [&](int off) { return off ? v32 : v0; });
          }
          if constexpr (EPI == EPI_F32) {
            // LM head: this 16-column chunk's maximum of row m (lanes cp, cp + 16, cp + 32, cp + 48), as the
            // skinny kernel writes it for the chunk-maximum sampler
            if (a.cmax) {
              float mx = fmaxf(fmaxf(v0[0], v0[1]), fmaxf(v0[2], v0[3]));
              mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
              mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
              if (gp == 0 && gt < ntiles && m < a.M) a.cmax[(size_t)m * a.ld_cm + gt] = mx;
            }
          }
        }
      }
    }
}

// ABL (diagnostics only, results garbage): 1 = the LDS-DMA stream without fragment reads and MFMAs, 2 = fragment
// reads and MFMAs without the DMA (tools/wgemm_bench.py variants 6 / 7)
// LW: waves that issue the LDS-DMA (8: all; 4: waves 0-3, one per SIMD -- the SIMD's other wave only computes)
template <int EPI, bool NORM, int ABL = 0, int LW = 8>
__global__ __launch_bounds__(512, 2) void wg256_kernel(const GemmArgs a, const WgArgs w) {
  using namespace w256;
  constexpr int WP = 16 / LW, XP = 32 / LW;  // LDS-DMA pieces per loading wave: per W stage, per X stage
  extern __shared__ __attribute__((aligned(16))) char smem[];  // [NSX X slots][NSW W slots]
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool ld = wave < LW;                // this wave issues LDS-DMA pieces
  const int lw = ld ? wave : 0;
  const int wm = wave & 1, wn = wave >> 1;  // rows 128 wm .. +127, columns 64 wn .. +63 of the tile
  const int KS = a.K >> 5;                  // 32-k slices per W tile
  const int ntiles = a.N >> 4;
  const int nblk = ntiles / NT;
  int blk, kc;
  wg_block_of(blockIdx.x, w.ks, nblk, w.xcd_blk, blk, kc);
  const int tile0 = blk * NT;
  const int st0 = kc * w.kst;                // first stage of this split
  const int nst = min(w.kst, KS - st0);      // stages of this split (>= 1: wg_plan256)

  const int nsx = nst >> 1;                  // X stages (64-deep; nst is even: wg_plan256)

  // ---- LDS-DMA sources of this wave: W tiles 2 wave + j (one 1 KiB slice per 32-deep W stage); X row octets
  // 4 wave + j (8 rows x 128 B per piece and 64-deep X stage: whole 128-B lines -- staged as 16 rows x 64 B, the
  // X stream issued twice the L2 requests per byte and the whole kernel's DMA ran 1.5x slower per byte)
  const char* wsrc[WP];
#pragma unroll
  for (int j = 0; j < WP; ++j)
    wsrc[j] = reinterpret_cast<const char*>(a.Wp) + ((size_t)(tile0 + lw * WP + j) * KS + st0) * 1024 + lane * 16;
  const char* xsrc[XP];
#pragma unroll
  for (int j = 0; j < XP; ++j) {
    const int r = 8 * (lw * XP + j) + (lane >> 3);
    const int p = (lane & 7) ^ ((r >> 1) & 7);  // LDS slot lane & 7 of row r holds global piece p
    xsrc[j] = reinterpret_cast<const char*>(a.X) + ((size_t)min(r, a.M - 1) * a.ldx + (size_t)st0 * BK + p * 8) * 2;
  }
  char* const xring = smem;
  char* const wring = smem + NSX * X_BYTES;
  auto issue_w = [&](int t) {  // W stage t into W slot t % NSW
    if (ABL == 2 || !ld) return;
    char* base = wring + (t % NSW) * W_BYTES + lw * WP * 1024;
#pragma unroll
    for (int j = 0; j < WP; ++j) glds16(wsrc[j] + (size_t)t * 1024, base + j * 1024, 1);  // streamed once: nt
  };
  auto issue_x = [&](int u) {  // X stage u into X slot u % NSX
    if (ABL == 2 || !ld) return;
    char* base = xring + (u % NSX) * X_BYTES + lw * XP * 1024;
#pragma unroll
    for (int j = 0; j < XP; ++j) glds16(xsrc[j] + (size_t)u * (2 * BK * 2), base + j * 1024, 0);
  };
  auto issue_w1 = [&](int t, int j) {  // piece j of W stage t
    if (ABL == 2 || !ld) return;
    glds16(wsrc[j] + (size_t)t * 1024, wring + (t % NSW) * W_BYTES + (lw * WP + j) * 1024, 1);
  };
  auto issue_x1 = [&](int u, int j) {  // piece j of X stage u
    if (ABL == 2 || !ld) return;
    glds16(xsrc[j] + (size_t)u * (2 * BK * 2), xring + (u % NSX) * X_BYTES + (lw * XP + j) * 1024, 0);
  };
  // Issue order: step v issues W stage v + DW, then for even v >= 0 X stage v/2 + 1 (inside the first k step of W
  // stage v, after barrier v: its slot held X stage v/2 - 1, whose last reads finished before barrier v).  The
  // prologue is steps -DW .. -1 (W stages 0 .. DW - 1), preceded by X stage 0.  Barrier s certifies W stage s and,
  // for even s, X stage s/2.  vmcnt retires in issue order, so land(s) -- called in step s - 1 -- lets the pieces
  // issued after the youngest needed one stay outstanding: for even s >= 2 X stage s/2 (step s - 2; W stage s is
  // older), so step s - 1's pieces; for s = 0 W stage 0 (after X stage 0), so steps -DW + 1 .. -1; for odd s W
  // stage s (step s - DW), so steps s - DW + 1 .. s - 1.
  auto w_at = [&](int v) { return (v >= -DW && v + DW < nst) ? WP : 0; };            // W pieces of step v
  auto x_at = [&](int v) { return (v >= 0 && !(v & 1) && v / 2 + 1 < nsx) ? XP : 0; };  // X pieces of step v
  auto land = [&](int s) {
    if (ABL != 2 && ld) {
      const int from = (s & 1) ? s - DW + 1 : (s == 0 ? -DW + 1 : s - 1);
      int n = 0;
      for (int v = from; v < s; ++v) n += w_at(v) + x_at(v);
      wait_vmcnt_rt(n);
    }
  };

  // ---- fragment read offsets inside a stage
  const int c32 = lane & 31, h = lane >> 5;
  // A (W) block wb of this wave: tile 4 wn + 2 wb + (c32 >> 4), row c32 & 15, k group 2 s + h (s = k step)
  int woff[2];
#pragma unroll
  for (int wb = 0; wb < 2; ++wb) woff[wb] = (4 * wn + 2 * wb + (c32 >> 4)) * 1024 + (16 * h + (c32 & 15)) * 16;
  // B (X) row n = 128 wm + 32 xr(xb) + c32, 16-B piece p = 4 (t & 1) + 2 s + h of the 128-B row of X stage t / 2,
  // in LDS slot p ^ ((n >> 1) & 7) = p ^ ((c32 >> 1) & 7).  The wave's X blocks are held rotated, register block
  // xb = row block xr(xb) = (xb + wn) & 3, so register block 0 is the one whose X X^T this wave accumulates (NORM):
  // a fixed operand, no wave-uniform branch (a branch there made hipcc copy the accumulator through a phi: s_nop
  // + 16 moves per k step)
  int xoff[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) xoff[q] = wm * 128 * 128 + c32 * 128 + (((2 * q + h) ^ ((c32 >> 1) & 7)) << 4);
  auto xr = [&](int xb) { return (xb + wn) & 3; };

  f32x16 acc[2][4];
#pragma unroll
  for (int wb = 0; wb < 2; ++wb)
#pragma unroll
    for (int xb = 0; xb < 4; ++xb) acc[wb][xb] = f32x16{};
  f32x16 ssq = f32x16{};  // NORM: X X^T of X block wn of this wave's rows

  auto read_step = [&](int t, int s, bf16x8 (&af)[2], bf16x8 (&bfr)[4]) {
    if constexpr (ABL == 1) return;
    const char* wbase = wring + (t % NSW) * W_BYTES + s * 512;
    const char* xbase = xring + ((t >> 1) % NSX) * X_BYTES + xoff[2 * (t & 1) + s];
#pragma unroll
    for (int wb = 0; wb < 2; ++wb) af[wb] = *reinterpret_cast<const bf16x8*>(wbase + woff[wb]);
#pragma unroll
    for (int xb = 0; xb < 4; ++xb) bfr[xb] = *reinterpret_cast<const bf16x8*>(xbase + xr(xb) * 32 * 128);
  };
  // the MFMAs of one k step; hook(i) runs after MFMA i (the next step's fragment reads after the first, this wave's
  // DMA pieces one at a time after later ones: issued in a burst, the 8 waves' pieces queued at the CU's address
  // unit and held every wave's next MFMA back -- 92.6 us against 57 us for the DMA alone and 61 us for the MFMAs
  // alone on llama3.1:8b's gate/up, profiles/r5)
  auto mfma_step = [&](const bf16x8 (&af)[2], const bf16x8 (&bfr)[4], auto hook) {
    if constexpr (ABL == 1) {
#pragma unroll
      for (int i = 0; i < 8; ++i) hook(i);
      return;
    }
#pragma unroll
    for (int wb = 0; wb < 2; ++wb)
#pragma unroll
      for (int xb = 0; xb < 4; ++xb) {
        acc[wb][xb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[wb], bfr[xb], acc[wb][xb], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        hook(4 * wb + xb);
        __builtin_amdgcn_sched_barrier(0);
      }
    if constexpr (NORM) ssq = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bfr[0], bfr[0], ssq, 0, 0, 0);
  };

  // ---- prologue: X stage 0 and W stages 0 .. DW - 1, then barrier 0 and step 0's W pieces (its X pieces go in the
  // first k step of W stage 0)
  issue_x(0);
#pragma unroll
  for (int v = 0; v < DW; ++v) {
    if (v < nst) issue_w(v);
  }
  land(0);
  ring_barrier();
  if (DW < nst) issue_w(DW);

  // ---- main loop over W stages: barrier t + 1 sits between W stage t's two k steps; it retires stage t's slots
  // (every wave has read both of its k steps into registers: lgkmcnt(0) in ring_barrier), which then take W stage
  // t + 1 + DW (and, after an even barrier, X stage (t + 1)/2 + 1 in the X slot of the stage that just ended)
  bf16x8 a0[2] = {}, b0[4] = {}, a1[2] = {}, b1[4] = {};
  read_step(0, 0, a0, b0);
  for (int t = 0; t < nst; ++t) {
    __builtin_amdgcn_sched_barrier(0);
    const bool xs = x_at(t) != 0;  // this step issues X stage t/2 + 1: its pieces spread over MFMAs 1 .. 7
    mfma_step(a0, b0, [&](int i) {
      if (i == 0) read_step(t, 1, a1, b1);
      else if (xs) {
        if constexpr (XP == 4) {
          if (i & 1) issue_x1(t / 2 + 1, i >> 1);
        } else {
          issue_x1(t / 2 + 1, i - 1);
          if (i == 7) issue_x1(t / 2 + 1, 7);
        }
      }
    });
    __builtin_amdgcn_sched_barrier(0);
    const bool more = t + 1 < nst;
    if (more) {
      land(t + 1);
      ring_barrier();
    }
    const bool ws = t + 1 + DW < nst;  // W stage t + 1 + DW: its pieces spread over the k step's MFMAs
    __builtin_amdgcn_sched_barrier(0);
    mfma_step(a1, b1, [&](int i) {
      if (i == 0) {
        if (more) read_step(t + 1, 0, a0, b0);
      } else if (ws) {
        if constexpr (WP == 2) {
          if (i == 2) issue_w1(t + 1 + DW, 0);
          else if (i == 5) issue_w1(t + 1 + DW, 1);
        } else {
          if (i & 1) issue_w1(t + 1 + DW, i >> 1);
        }
      }
    });
    __builtin_amdgcn_sched_barrier(0);
  }
  ring_barrier();  // every wave is done with the ring: its LDS becomes epilogue scratch

  // ---- per-row sums of squares: the diagonal of this wave's X X^T block.  Lane (c32, h) holds C[i][c32] for
  // i = 8 (r >> 2) + 4 h + (r & 3), so row c32's diagonal element sits in the lanes with ((c32 >> 2) & 1) == h,
  // register 4 (c32 >> 3) + (c32 & 3)
  float* s_ss = reinterpret_cast<float*>(smem);  // [BM]
  if constexpr (NORM) {
    if (((c32 >> 2) & 1) == h) {
      const int ri = 4 * (c32 >> 3) + (c32 & 3);
      float v = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) v = (r == ri) ? ssq[r] : v;
      s_ss[128 * wm + 32 * wn + c32] = v;
    }
    __syncthreads();
  }

  wg256_epilogue<EPI, NORM>(a, w, acc, s_ss, smem, wave, lane, wm, wn, tile0, blk, kc);
}

// The same 256 x 256 tile with 4 dedicated loader waves (one per SIMD, waves 8-11) beside the 8 compute waves, as
// wgemm.hip does at 256 x 128: 3 waves per SIMD cap every wave at 168 registers, so the compute waves keep only
// their 128 accumulators, the W fragments double-buffered and the X fragments single-buffered (each reloaded for
// the next k step right after its last MFMA), and the RMSNorm sums of squares move to the loader waves, which read
// back the X pieces they staged once each has landed (8 rows x 128 B per piece: every element exactly once).
template <int EPI, bool NORM>
__global__ __launch_bounds__(768, 3) void wg256l_kernel(const GemmArgs a, const WgArgs w) {
  using namespace w256;
  constexpr int WP = 4, XP = 8;  // pieces per loader wave: per W stage (16 / 4), per X stage (32 / 4)
  extern __shared__ __attribute__((aligned(16))) char smem[];  // [NSX X slots][NSW W slots]
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool loader = wave >= 8;
  const int lw = loader ? wave - 8 : 0;
  const int wm = wave & 1, wn = (wave >> 1) & 3;
  const int KS = a.K >> 5;
  const int ntiles = a.N >> 4;
  const int nblk = ntiles / NT;
  int blk, kc;
  wg_block_of(blockIdx.x, w.ks, nblk, w.xcd_blk, blk, kc);
  const int tile0 = blk * NT;
  const int st0 = kc * w.kst;
  const int nst = min(w.kst, KS - st0);
  const int nsx = nst >> 1;
  char* const xring = smem;
  char* const wring = smem + NSX * X_BYTES;
  float* s_ss = reinterpret_cast<float*>(smem);  // [BM], after the loop

  if (loader) {
    const char* wsrc[WP];
#pragma unroll
    for (int j = 0; j < WP; ++j)
      wsrc[j] = reinterpret_cast<const char*>(a.Wp) + ((size_t)(tile0 + lw * WP + j) * KS + st0) * 1024 + lane * 16;
    const char* xsrc[XP];
#pragma unroll
    for (int j = 0; j < XP; ++j) {
      const int r = 8 * (lw * XP + j) + (lane >> 3);
      const int p = (lane & 7) ^ ((r >> 1) & 7);
      xsrc[j] = reinterpret_cast<const char*>(a.X) + ((size_t)min(r, a.M - 1) * a.ldx + (size_t)st0 * BK + p * 8) * 2;
    }
    auto issue_w = [&](int t) {
      char* base = wring + (t % NSW) * W_BYTES + lw * WP * 1024;
#pragma unroll
      for (int j = 0; j < WP; ++j) glds16(wsrc[j] + (size_t)t * 1024, base + j * 1024, 1);
    };
    auto issue_x = [&](int u) {
      char* base = xring + (u % NSX) * X_BYTES + lw * XP * 1024;
#pragma unroll
      for (int j = 0; j < XP; ++j) glds16(xsrc[j] + (size_t)u * (2 * BK * 2), base + j * 1024, 0);
    };
    // issue order and waits as wg256_kernel: step v = W stage v + DW, then (even v) X stage v/2 + 1
    auto w_at = [&](int v) { return (v >= -DW && v + DW < nst) ? WP : 0; };
    auto x_at = [&](int v) { return (v >= 0 && !(v & 1) && v / 2 + 1 < nsx) ? XP : 0; };
    auto land = [&](int s) {
      const int from = (s & 1) ? s - DW + 1 : (s == 0 ? -DW + 1 : s - 1);
      int n = 0;
      for (int v = from; v < s; ++v) n += w_at(v) + x_at(v);
      wait_vmcnt_rt(n);
    };
    float ss[XP];
#pragma unroll
    for (int j = 0; j < XP; ++j) ss[j] = 0.f;
    issue_x(0);
    for (int v = 0; v < DW && v < nst; ++v) issue_w(v);
    land(0);
    ring_barrier();
    for (int t = 0; t < nst; ++t) {
      if (t + DW < nst) issue_w(t + DW);
      if (x_at(t)) issue_x(t / 2 + 1);
      if constexpr (NORM) {
        if (!(t & 1)) {  // X stage t/2 landed (barrier t): its rows' squares, from this wave's own pieces
          const char* base = xring + ((t >> 1) % NSX) * X_BYTES + lw * XP * 1024 + lane * 16;
#pragma unroll
          for (int j = 0; j < XP; ++j) {
            const bf16x8 v = *reinterpret_cast<const bf16x8*>(base + j * 1024);
#pragma unroll
            for (int e = 0; e < 8; ++e) ss[j] += bf2f(v[e]) * bf2f(v[e]);
          }
        }
      }
      if (t + 1 < nst) {
        land(t + 1);
        ring_barrier();
      }
    }
    ring_barrier();  // the compute waves are done with the ring
    if constexpr (NORM) {
      // piece i = 4 lw + j holds rows 8i .. 8i + 7, lane l row 8i + (l >> 3): sum the 8 lanes of each row
#pragma unroll
      for (int j = 0; j < XP; ++j) {
        float v = ss[j];
        v += __shfl_xor(v, 1, 64);
        v += __shfl_xor(v, 2, 64);
        v += __shfl_xor(v, 4, 64);
        if ((lane & 7) == 0) s_ss[8 * (lw * XP + j) + (lane >> 3)] = v;
      }
      __syncthreads();
    }
    return;
  }

  // ---- compute waves.  Fragment registers: one W pair and one X quad (each reloaded for the next k step right
  // after its last MFMA: the W pair after MFMAs 4 / 8, X block xb after MFMA 5 + xb -- 3-4 MFMAs of this wave, and
  // the SIMD's other compute wave's, cover the LDS latency); with the 128 accumulators that stays within the 168
  // registers of 3 waves per SIMD (double-buffered fragments spilled).
  const int c32 = lane & 31, h = lane >> 5;
  // W fragment wb, k step s of W slot j: wring + j W_BYTES + s 512 + wlane + wb 2048
  const int wlane = (4 * wn + (c32 >> 4)) * 1024 + (16 * h + (c32 & 15)) * 16;
  // X fragment xb, k step q4 (of 4) of X slot u: xring + u X_BYTES + xb 4096 + xlane + (((2 q4) ^ xph) << 4)
  const int xlane = wm * 128 * 128 + c32 * 128;
  const int xph = h ^ ((c32 >> 1) & 7);  // piece 2 q4 + h in slot (2 q4 + h) ^ ((row >> 1) & 7) = (2 q4) ^ xph
  f32x16 acc[2][4];
#pragma unroll
  for (int wb = 0; wb < 2; ++wb)
#pragma unroll
    for (int xb = 0; xb < 4; ++xb) acc[wb][xb] = f32x16{};
  // k step q = 2 t + s: W slot t % NSW, X slot (t / 2) % NSX, X k step 2 (t & 1) + s
  auto w_ptr = [&](int q, int wb) {
    return reinterpret_cast<const bf16x8*>(wring + ((q >> 1) % NSW) * W_BYTES + (q & 1) * 512 + wlane + wb * 2048);
  };
  auto x_ptr = [&](int q, int xb) {
    const int t = q >> 1, q4 = 2 * (t & 1) + (q & 1);
    return reinterpret_cast<const bf16x8*>(xring + ((t >> 1) % NSX) * X_BYTES + xb * 4096 + xlane +
                                           (((2 * q4) ^ xph) << 4));
  };
  bf16x8 af[2], bfr[4];
  auto mfmas = [&](int q, bool next) {
#pragma unroll
    for (int wb = 0; wb < 2; ++wb) {
#pragma unroll
      for (int xb = 0; xb < 4; ++xb) {
        acc[wb][xb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[wb], bfr[xb], acc[wb][xb], 0, 0, 0);
        if (next) {
          __builtin_amdgcn_sched_barrier(0);
          if (wb == 1) bfr[xb] = *x_ptr(q + 1, xb);
          if (xb == 3) af[wb] = *w_ptr(q + 1, wb);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
  };
  ring_barrier();  // barrier 0: W stage 0 and X stage 0 landed
#pragma unroll
  for (int wb = 0; wb < 2; ++wb) af[wb] = *w_ptr(0, wb);
#pragma unroll
  for (int xb = 0; xb < 4; ++xb) bfr[xb] = *x_ptr(0, xb);
  for (int t = 0; t < nst; ++t) {
    const bool more = t + 1 < nst;
    // k step 0 of W stage t; the barrier before k step 1 must not pass before every wave read k step 1's
    // fragments of this stage's slots -- they are read inside k step 0, so the barrier retires W stage t's slots
    __builtin_amdgcn_sched_barrier(0);
    mfmas(2 * t, true);
    __builtin_amdgcn_sched_barrier(0);
    if (more) ring_barrier();  // barrier t + 1: W stage t + 1 (and X stage (t + 1) / 2) landed
    __builtin_amdgcn_sched_barrier(0);
    mfmas(2 * t + 1, more);
    __builtin_amdgcn_sched_barrier(0);
  }
  ring_barrier();  // every wave is done with the ring
  if constexpr (NORM) __syncthreads();  // the loaders' row sums of squares are in s_ss
  wg256_epilogue<EPI, NORM, false>(a, w, acc, s_ss, smem, wave, lane, wm, wn, tile0, blk, kc);
}

template <int EPI, bool NORM>
static hipError_t wg256l_launch(const GemmArgs& a, const WgArgs& w, int nblk, hipStream_t st) {
  static bool attr = [] {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&wg256l_kernel<EPI, NORM>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, w256::LDS) == hipSuccess;
  }();
  if (!attr) return hipErrorInvalidConfiguration;
  hipLaunchKernelGGL((wg256l_kernel<EPI, NORM>), dim3(nblk * w.ks), dim3(768), w256::LDS, st, a, w);
  return hipGetLastError();
}

template <int EPI, bool NORM, int ABL, int LW>
static hipError_t wg256_launch1(const GemmArgs& a, const WgArgs& w, int nblk, hipStream_t st) {
  static bool attr = [] {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&wg256_kernel<EPI, NORM, ABL, LW>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, w256::LDS) == hipSuccess;
  }();
  if (!attr) return hipErrorInvalidConfiguration;
  hipLaunchKernelGGL((wg256_kernel<EPI, NORM, ABL, LW>), dim3(nblk * w.ks), dim3(512), w256::LDS, st, a, w);
  return hipGetLastError();
}

// abl: 0 the kernel, 1 DMA only, 2 MFMAs only (diagnostics); 3: the kernel with 4 loading waves (LW = 4); 4: the
// loader-wave kernel (wg256l_kernel)
template <int EPI, bool NORM>
static hipError_t wg256_launch(const GemmArgs& a, const WgArgs& w, int nblk, int abl, hipStream_t st) {
  if (abl == 4) return wg256l_launch<EPI, NORM>(a, w, nblk, st);
  if (abl == 1) return wg256_launch1<EPI, NORM, 1, 8>(a, w, nblk, st);
  if (abl == 2) return wg256_launch1<EPI, NORM, 2, 8>(a, w, nblk, st);
  if (abl == 3) return wg256_launch1<EPI, NORM, 0, 4>(a, w, nblk, st);
  return wg256_launch1<EPI, NORM, 0, 8>(a, w, nblk, st);
}

// The main kernel of a 256-column plan (wgemm.hip wgemm_dispatch launches the split-K reduce after it); abl: the
// diagnostic builds (1 DMA only, 2 MFMAs only).
hipError_t wg256_main(int epi, bool norm, const GemmArgs& a, const WgArgs& w, int nblk, int abl, hipStream_t st) {
#define CAIN_W256(E)                                                                   \
  case E:                                                                              \
    return norm ? wg256_launch<E, true>(a, w, nblk, abl, st) : wg256_launch<E, false>(a, w, nblk, abl, st);
  switch (epi) {
    CAIN_W256(EPI_BF16) CAIN_W256(EPI_RESID) CAIN_W256(EPI_F32) CAIN_W256(EPI_SILU) CAIN_W256(EPI_GELU)
    CAIN_W256(EPI_QKV_ROPE)
    default: return hipErrorInvalidValue;
  }
#undef CAIN_W256
}
