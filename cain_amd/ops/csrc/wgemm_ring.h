// LDS-DMA ring helpers shared by the wide-batch GEMMs: bf16 (wgemm.hip) and fp8 W8A8 (wgemm8.hip).
#pragma once
#include <cstdlib>

#include "common.h"
namespace wg {

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void gbl_void_t;

constexpr int WG_NT = 8;    // output columns per workgroup: 8 tiles of 16
constexpr int WG_BK = 64;   // k per ring stage (2 slices of 32)

template <int BM>
struct WgGeo {
  static constexpr int WM = BM == 256 ? 4 : 2;  // waves along M
  static constexpr int WN = 8 / WM;             // waves along N
  static constexpr int MB = BM / 16 / WM;       // 16-row blocks per wave
  static constexpr int TN = WG_NT / WN;         // 16-column tiles per wave
  static constexpr int W_BYTES = WG_NT * 2 * 1024;  // one W stage: 8 tiles x 2 slices of 1 KiB
  static constexpr int X_BYTES = BM * WG_BK * 2;    // one X stage: BM rows x 128 B
  static constexpr int XPW = BM / 8 / 8;        // X LDS-DMA instructions per wave per stage (8 rows each)
  static constexpr int RB = BM / 16;            // row blocks per tile (split-K slab units)
};

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// wave-uniform runtime count (the pipeline tail issues fewer stages): one uniform branch per value
template <int N = 0>
__device__ __forceinline__ void wait_vmcnt_rt(int n) {
  if constexpr (N >= 30) {
    wait_vmcnt<N>();
  } else {
    if (n <= N) wait_vmcnt<N>();
    else wait_vmcnt_rt<N + 1>(n);
  }
}

// every wave's LDS-DMA of the stage being consumed has landed (its own counted wait before this), and every
// wave has finished reading the slot about to be refilled
__device__ __forceinline__ void ring_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

__device__ __forceinline__ void glds16(const void* src, char* lds_wave_base, int aux_nt) {
  if (aux_nt)
    __builtin_amdgcn_global_load_lds((gbl_void_t*)src, (lds_void_t*)lds_wave_base, 16, 0, 2);
  else
    __builtin_amdgcn_global_load_lds((gbl_void_t*)src, (lds_void_t*)lds_wave_base, 16, 0, 0);
}

// Workgroup -> (column block, k-split) of the wide GEMMs.  xcd_blk (nblk % 8 == 0): XCD x = bid % 8 (round-robin
// dispatch) owns column blocks x, x + 8, ... with all their splits, so the split-K reduce can read the slabs from
// that XCD's L2 (wg_reduce_block); otherwise split-major: the column blocks of one split (which read the same X
// panel) share an XCD.  Speed only, any placement is correct.
__device__ __forceinline__ void wg_block_of(int bid, int ks, int nblk, int xcd_blk, int& blk, int& kc) {
  if (ks == 1) blk = bid, kc = 0;
  else if (xcd_blk) {
    const int j = bid >> 3;
    blk = (bid & 7) + 8 * (j / ks), kc = j % ks;
  } else if ((8 % ks) == 0) kc = bid % ks, blk = bid / ks;
  else kc = bid / nblk, blk = bid - kc * nblk;
}
// Reduce workgroup index (units of per_blk consecutive workgroups per column block) on the XCD of its block.
__device__ __forceinline__ int wg_reduce_block(int bid, int per_blk, int xcd_blk) {
  if (!xcd_blk) return bid;
  const int j = bid >> 3;
  return ((bid & 7) + 8 * (j / per_blk)) * per_blk + j % per_blk;
}

}  // namespace wg

struct WgArgs {
  int ks;           // k-splits (workgroups per column block)
  int kst;          // ring stages (64-deep k-steps) per split
  float* part;      // [ks][n_units][64 lanes] f32x4 (ks > 1)
  float* part_ss;   // [nblk][ks][BM] per-row partial sums of squares (ks > 1 && NORM)
  uint8_t* part_ex; // [ks][n_units][64 lanes] power-of-two exponent of each non-NORM fp16 slab lane (value = half * 2^ex)
  int xcd_blk;      // 1: a column block's split partners and its reducers share one XCD (wgemm.hip)
  int bnt;          // 16-column tiles per column block of the main kernel (wgemm.hip: WG_NT = 8, wgemm256.hip: 16)
  unsigned* counters;  // workspace head (WG_CTR_BYTES, zero at rest): the in-launch combine's words (wgemm.hip)
  unsigned long long* stamps;  // diagnostic build only (wgemm.hip ABL 3): [grid][2 waves][8] timestamps
  long long spin;   // in-launch combine: how long a partner waits for the others (s_memrealtime ticks; 0: never)
};

