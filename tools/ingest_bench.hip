// Per-CU ingest ceiling of the wide-GEMM operand paths (profiles/r3/README.md, 'Wide GEMM').
//
// One workgroup per CU (256), each moving the bytes a 256-row gate/up workgroup moves: its own 1 MiB slice of a
// 512 MiB "weight" buffer (HBM, streamed once) plus the whole 2 MiB "activation" panel (L2-resident, re-read by
// every workgroup), in 48 KiB stages (16 KiB W + 32 KiB X).  Modes:
//   0  LDS-DMA (global_load_lds_dwordx4) into a 3-slot LDS ring, NL loader waves, counted vmcnt per stage (the
//      wgemm.hip loader without compute waves)
//   1  plain global_load_dwordx4 into VGPRs, NL waves, DEPTH stages in flight per wave, xor-folded (no LDS)
//   2  mode 1 + ds_write_b128 of every piece into an LDS ring (register staging)
//   3  X only by LDS-DMA (L2 path alone)
//   4  W only by LDS-DMA (HBM path alone)
//   5  LDS-DMA with split roles: waves 0 .. NL/2-1 issue only W (DW stages in flight), the others only X (2 in
//      flight), so no X piece waits behind an HBM-bound W piece in a wave's in-order vmcnt
// Prints GB/s per CU and bytes per shader clock (s_memtime / s_memrealtime over the kernel).
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/ingest tools/ingest_bench.hip && /tmp/ingest
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void gbl_void_t;
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));  \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

constexpr int STAGES = 64;              // 64 stages x 48 KiB = 3 MiB per workgroup
constexpr int W_STAGE = 16 * 1024, X_STAGE = 32 * 1024;

__device__ __forceinline__ void glds(const char* src, char* lds, int nt) {
  if (nt)
    __builtin_amdgcn_global_load_lds((gbl_void_t*)src, (lds_void_t*)lds, 16, 0, 2);
  else
    __builtin_amdgcn_global_load_lds((gbl_void_t*)src, (lds_void_t*)lds, 16, 0, 0);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// MODE 0/3/4: LDS-DMA ring of 3 stages, NL loader waves, 2 stages in flight
template <int NL, int MODE>
__global__ __launch_bounds__(64 * NL) void dma_kernel(const char* W, const char* X, unsigned long long* clk,
                                                       unsigned* sink) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const char* wb = W + (size_t)blockIdx.x * STAGES * W_STAGE;
  constexpr int WP = (MODE == 3) ? 0 : W_STAGE / 1024 / NL;  // pieces per wave per stage
  constexpr int XP = (MODE == 4) ? 0 : X_STAGE / 1024 / NL;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  auto issue = [&](int t) {
    char* slot = smem + (t % 3) * (W_STAGE + X_STAGE);
#pragma unroll
    for (int j = 0; j < WP; ++j)
      glds(wb + (size_t)t * W_STAGE + (wave * WP + j) * 1024 + lane * 16, slot + (wave * WP + j) * 1024, 1);
#pragma unroll
    for (int j = 0; j < XP; ++j)
      glds(X + (size_t)t * X_STAGE + (wave * XP + j) * 1024 + lane * 16, slot + W_STAGE + (wave * XP + j) * 1024, 0);
  };
  issue(0);
  issue(1);
  for (int t = 0; t < STAGES; ++t) {
    if (t + 1 < STAGES) wait_vm<WP + XP>();
    else wait_vm<0>();
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (t + 2 < STAGES) issue(t + 2);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (threadIdx.x == 0) {
    clk[blockIdx.x * 2] = __builtin_amdgcn_s_memtime() - t0;
    clk[blockIdx.x * 2 + 1] = __builtin_amdgcn_s_memrealtime() - r0;
    sink[blockIdx.x] = *reinterpret_cast<const unsigned*>(smem);
  }
}

// MODE 1/2: register loads, DEPTH stages in flight per wave; MODE 2 writes every piece to an LDS ring
template <int NL, int DEPTH, int MODE>
__global__ __launch_bounds__(64 * NL) void reg_kernel(const char* W, const char* X, unsigned long long* clk,
                                                       unsigned* sink) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const char* wb = W + (size_t)blockIdx.x * STAGES * W_STAGE;
  constexpr int WP = W_STAGE / 1024 / NL, XP = X_STAGE / 1024 / NL, P = WP + XP;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  u32x4 buf[DEPTH][P];
  u32x4 acc = {0, 0, 0, 0};
  auto issue = [&](int t, u32x4 (&b)[P]) {
#pragma unroll
    for (int j = 0; j < WP; ++j)
      b[j] = __builtin_nontemporal_load(
          reinterpret_cast<const u32x4*>(wb + (size_t)t * W_STAGE + (wave * WP + j) * 1024 + lane * 16));
#pragma unroll
    for (int j = 0; j < XP; ++j)
      b[WP + j] = *reinterpret_cast<const u32x4*>(X + (size_t)t * X_STAGE + (wave * XP + j) * 1024 + lane * 16);
  };
  auto consume = [&](int t, u32x4 (&b)[P]) {
    if constexpr (MODE == 2) {
      char* slot = smem + (t % 2) * (W_STAGE + X_STAGE);
#pragma unroll
      for (int j = 0; j < WP; ++j) *reinterpret_cast<u32x4*>(slot + (wave * WP + j) * 1024 + lane * 16) = b[j];
#pragma unroll
      for (int j = 0; j < XP; ++j)
        *reinterpret_cast<u32x4*>(slot + W_STAGE + (wave * XP + j) * 1024 + lane * 16) = b[WP + j];
    } else {
#pragma unroll
      for (int j = 0; j < P; ++j) acc ^= b[j];
    }
  };
#pragma unroll
  for (int d = 0; d < DEPTH; ++d) issue(d, buf[d]);
  for (int t = 0; t < STAGES; t += DEPTH) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      consume(t + d, buf[d]);
      if (t + d + DEPTH < STAGES) issue(t + d + DEPTH, buf[d]);
      if constexpr (MODE == 2) {
        if (d % 2 == 1) __syncthreads();
      }
    }
  }
  if (threadIdx.x == 0) {
    clk[blockIdx.x * 2] = __builtin_amdgcn_s_memtime() - t0;
    clk[blockIdx.x * 2 + 1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
  sink[blockIdx.x * 64 * NL + threadIdx.x] = acc[0] ^ acc[1] ^ acc[2] ^ acc[3] ^ (MODE == 2 ? smem[threadIdx.x] : 0);
}

// MODE 5: split roles, W ring of DW + 1 slots, X ring of 3 slots
template <int NL, int DW, int NXS>
__global__ __launch_bounds__(64 * NL) void split_kernel(const char* W, const char* X, unsigned long long* clk,
                                                         unsigned* sink) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const bool wl = wave < NL / 2;
  const int lw = wl ? wave : wave - NL / 2;
  const char* wb = W + (size_t)blockIdx.x * STAGES * W_STAGE;
  constexpr int WP = W_STAGE / 1024 / (NL / 2), XP = X_STAGE / 1024 / (NL / 2);
  char* xring = smem + (DW + 1) * W_STAGE;  // X ring of NXS slots, NXS - 1 stages in flight
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  auto issue_w = [&](int t) {
#pragma unroll
    for (int j = 0; j < WP; ++j)
      glds(wb + (size_t)t * W_STAGE + (lw * WP + j) * 1024 + lane * 16, smem + (t % (DW + 1)) * W_STAGE + (lw * WP + j) * 1024, 1);
  };
  auto issue_x = [&](int t) {
#pragma unroll
    for (int j = 0; j < XP; ++j)
      glds(X + (size_t)t * X_STAGE + (lw * XP + j) * 1024 + lane * 16, xring + (t % NXS) * X_STAGE + (lw * XP + j) * 1024, 0);
  };
  if (wl) {
    for (int t = 0; t < DW; ++t) issue_w(t);
  } else {
    for (int t = 0; t < NXS - 1; ++t) issue_x(t);
  }
  for (int t = 0; t < STAGES; ++t) {
    if (wl) {
      if (t + DW - 1 < STAGES) wait_vm<WP * (DW - 1)>();
      else wait_vm<0>();
    } else {
      if (t + NXS - 2 < STAGES) wait_vm<XP * (NXS - 2)>();
      else wait_vm<0>();
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (wl) {
      if (t + DW < STAGES) issue_w(t + DW);
    } else {
      if (t + NXS - 1 < STAGES) issue_x(t + NXS - 1);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (threadIdx.x == 0) {
    clk[blockIdx.x * 2] = __builtin_amdgcn_s_memtime() - t0;
    clk[blockIdx.x * 2 + 1] = __builtin_amdgcn_s_memrealtime() - r0;
    sink[blockIdx.x] = *reinterpret_cast<const unsigned*>(smem);
  }
}

template <class K>
void run(const char* name, K kern, int threads, int lds, const char* const* Ws, const char* X, unsigned long long* clk,
         unsigned* sink, size_t bytes_per_wg) {
  CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  const int grid = 256;
  // launches alternate two 256 MiB weight buffers: 512 MiB per pair, past the 256 MiB Infinity Cache
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(kern, dim3(grid), dim3(threads), lds, 0, Ws[i & 1], X, clk, sink);
  CHECK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  const int iters = 20;
  CHECK(hipEventRecord(a));
  for (int i = 0; i < iters; ++i) hipLaunchKernelGGL(kern, dim3(grid), dim3(threads), lds, 0, Ws[i & 1], X, clk, sink);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  std::vector<unsigned long long> h(grid * 2);
  CHECK(hipMemcpy(h.data(), clk, grid * 2 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  double cyc = 0, rt = 0;
  for (int i = 0; i < grid; ++i) cyc += h[2 * i], rt += h[2 * i + 1];
  cyc /= grid, rt /= grid;  // mean per workgroup (last launch)
  const double us = ms * 1e3 / iters;
  printf("%-34s %8.2f us/launch  %6.1f GB/s per CU  WG: %7.0f cycles %6.2f us  %5.1f B/clk  clock %.2f GHz\n", name,
         us, bytes_per_wg / (us * 1e-6) / 1e9, cyc, rt * 0.01, bytes_per_wg / cyc, cyc / (rt * 10.0));
}

int main() {
  const size_t wbytes = (size_t)256 * STAGES * W_STAGE;  // 256 MiB of W slices: rotate 2 buffers = 512 MiB
  char *W0, *W1, *X;
  CHECK(hipMalloc(&W0, wbytes));
  CHECK(hipMalloc(&W1, wbytes));
  CHECK(hipMalloc(&X, (size_t)STAGES * X_STAGE));
  CHECK(hipMemset(W0, 1, wbytes));
  CHECK(hipMemset(W1, 2, wbytes));
  CHECK(hipMemset(X, 3, (size_t)STAGES * X_STAGE));
  unsigned long long* clk;
  unsigned* sink;
  CHECK(hipMalloc(&clk, 256 * 2 * sizeof(unsigned long long)));
  CHECK(hipMalloc(&sink, 256 * 1024 * sizeof(unsigned)));
  const size_t full = (size_t)STAGES * (W_STAGE + X_STAGE), xo = (size_t)STAGES * X_STAGE, wo = (size_t)STAGES * W_STAGE;
  const int ring = 3 * (W_STAGE + X_STAGE);
  const char* W[2] = {W0, W1};
  for (int rep = 0; rep < 2; ++rep) {
    printf("-- rep %d\n", rep);
    run("lds-dma 4 waves (wgemm loader)", dma_kernel<4, 0>, 256, ring, W, X, clk, sink, full);
    run("lds-dma 8 waves", dma_kernel<8, 0>, 512, ring, W, X, clk, sink, full);
    run("lds-dma 16 waves", dma_kernel<16, 0>, 1024, ring, W, X, clk, sink, full);
    run("lds-dma 4 waves, X only (L2)", dma_kernel<4, 3>, 256, ring, W, X, clk, sink, xo);
    run("lds-dma 4 waves, W only (HBM)", dma_kernel<4, 4>, 256, ring, W, X, clk, sink, wo);
    run("lds-dma 8 waves, X only (L2)", dma_kernel<8, 3>, 512, ring, W, X, clk, sink, xo);
    run("split 4 waves, W 3 / X 2 ahead", split_kernel<4, 3, 3>, 256, 4 * W_STAGE + 3 * X_STAGE, W, X, clk, sink, full);
    run("split 4 waves, W 5 / X 1 ahead", split_kernel<4, 5, 2>, 256, 6 * W_STAGE + 2 * X_STAGE, W, X, clk, sink, full);
    run("split 8 waves, W 3 / X 2 ahead", split_kernel<8, 3, 3>, 512, 4 * W_STAGE + 3 * X_STAGE, W, X, clk, sink, full);
    run("split 8 waves, W 4 / X 1 ahead", split_kernel<8, 4, 2>, 512, 5 * W_STAGE + 2 * X_STAGE, W, X, clk, sink, full);
    run("regs 4 waves depth 2", reg_kernel<4, 2, 1>, 256, 0, W, X, clk, sink, full);
    run("regs 16 waves depth 2", reg_kernel<16, 2, 1>, 1024, 0, W, X, clk, sink, full);
    run("regs+ds_write 8 waves depth 2", reg_kernel<8, 2, 2>, 512, 2 * (W_STAGE + X_STAGE), W, X, clk, sink, full);
    run("regs+ds_write 16 waves depth 2", reg_kernel<16, 2, 2>, 1024, 2 * (W_STAGE + X_STAGE), W, X, clk, sink, full);
  }
  return 0;
}
