// OPT-IN A/B build (``python -m cain_amd.build --blas`` -> cain_amd/ops/libcain_blas.so): the default kernel
// library has no hipBLASLt dependency and the headline runs hand-written kernels only.  Loading this library
// (cain_amd.ops.enable_lt) registers these entries with the runtime (runtime.hip cain_set_lt_api), which then
// sends O and gate/up of forwards with >= CAIN_LT_MIN_ROWS rows here -- for A/B runs against the hand kernels.
//
// Library-GEMM path for the wide decode batches (M >= 128 rows): hipBLASLt for the plain GEMM, one
// hand-written row kernel for what the fused MFMA bodies did in their epilogue.
//
// At 256 rows the hand-written batched GEMM (gemm.hip) is latency-bound on its one-group weight prefetch
// (profiles/bgemm_r1.md, PMC: MFMA 27 % busy), while hipBLASLt's tuned gfx950 kernels stream the same
// weights at up to 3.6 TB/s: O projection 23 vs 39 us, gate/up 66 vs 103 us (llama3.1:8b shapes,
// profiles/lt_gemm.md).  The runtime therefore sends exactly those two projections to the library once a
// forward has enough rows, and keeps the fused kernels (QKV + RoPE + KV append, down + residual, LM head +
// sampler) everywhere they win:
//
//   * O projection:   x += attn . Wo^T        hipBLASLt, beta = 1 with C = D = x (in-place residual)
//   * gate/up:        gu  = x . Wgu^T         hipBLASLt on the UN-normalised x, then
//                     act = f(s*g) * (s*u)    rownorm_act_kernel, s = rsqrt(mean(x^2) + eps)
//
// The RMSNorm commutes with the GEMM (its gain is folded into Wgu's columns, models/weights.py fold_gain),
// so the per-row scale is applied in the activation kernel: no normalised copy of x is ever written.
// Wgu keeps the engine's 8-row gate/up interleave, so gate i of block b sits at column 16b+i and its up
// partner at 16b+8+i: one 16-byte load of each per thread.
#include <hipblaslt/hipblaslt.h>

#include <map>
#include <mutex>
#include <tuple>

#include "../csrc/common.h"

namespace {

struct LtPlan {
  hipblasLtMatmulDesc_t md = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr;
  hipblasLtMatmulAlgo_t algo{};
  size_t ws = 0;
  bool ok = false;
};

std::mutex g_mu;
hipblasLtHandle_t g_handle = nullptr;
std::map<std::tuple<int, int, int, int, int, int, long long, int, int>, LtPlan> g_plans;

// Y[M, N] (+)= X[M, K] . W[N, K]^T, all row-major = column-major D[N x M] = op_T(W[K x N]) . X[K x M]; X and W
// bf16, Y bf16 or (f32out: the LM head's logits) fp32.
const LtPlan* lt_plan(int N, int K, int M, int ldx, int ldy, bool accumulate, long long ws_bytes, int dev,
                      bool f32out = false) {
  std::lock_guard<std::mutex> lk(g_mu);
  auto key = std::make_tuple(N, K, M, ldx, ldy, int(accumulate), ws_bytes, dev, int(f32out));
  auto it = g_plans.find(key);
  if (it != g_plans.end()) return it->second.ok ? &it->second : nullptr;
  LtPlan p;
  // every failure path releases what it created and caches nothing, so a later call retries
  auto fail = [&p]() -> const LtPlan* {
    if (p.lc) hipblasLtMatrixLayoutDestroy(p.lc);
    if (p.lb) hipblasLtMatrixLayoutDestroy(p.lb);
    if (p.la) hipblasLtMatrixLayoutDestroy(p.la);
    if (p.md) hipblasLtMatmulDescDestroy(p.md);
    return nullptr;
  };
  if (!g_handle && hipblasLtCreate(&g_handle) != HIPBLAS_STATUS_SUCCESS) {
    g_handle = nullptr;
    return nullptr;
  }
  if (hipblasLtMatmulDescCreate(&p.md, HIPBLAS_COMPUTE_32F, HIP_R_32F) != HIPBLAS_STATUS_SUCCESS) {
    p.md = nullptr;
    return fail();
  }
  const hipblasOperation_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
  hipblasLtMatmulDescSetAttribute(p.md, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta));
  hipblasLtMatmulDescSetAttribute(p.md, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb));
  if (hipblasLtMatrixLayoutCreate(&p.la, HIP_R_16BF, K, N, K) != HIPBLAS_STATUS_SUCCESS) { p.la = nullptr; return fail(); }
  if (hipblasLtMatrixLayoutCreate(&p.lb, HIP_R_16BF, K, M, ldx) != HIPBLAS_STATUS_SUCCESS) { p.lb = nullptr; return fail(); }
  if (hipblasLtMatrixLayoutCreate(&p.lc, f32out ? HIP_R_32F : HIP_R_16BF, N, M, ldy) != HIPBLAS_STATUS_SUCCESS) {
    p.lc = nullptr;
    return fail();
  }
  hipblasLtMatmulPreference_t pref = nullptr;
  if (hipblasLtMatmulPreferenceCreate(&pref) != HIPBLAS_STATUS_SUCCESS) return fail();
  uint64_t wsb = (uint64_t)ws_bytes;
  hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb, sizeof(wsb));
  hipblasLtMatmulHeuristicResult_t res[1];
  int n = 0;
  hipblasStatus_t s = hipblasLtMatmulAlgoGetHeuristic(g_handle, p.md, p.la, p.lb, p.lc, p.lc, pref, 1, res, &n);
  hipblasLtMatmulPreferenceDestroy(pref);
  (void)accumulate;
  if (s != HIPBLAS_STATUS_SUCCESS || n < 1) return fail();
  p.algo = res[0].algo;
  p.ws = res[0].workspaceSize;
  p.ok = true;
  return &(g_plans[key] = p);
}

constexpr int ACT_THREADS = 256;

// One workgroup per row: the row's sum of squares of x (the RMSNorm scale), then the gated activation of
// the scaled gate/up GEMM output, 8 outputs (one 16-byte load of gate, one of up) per thread and pass.
template <int KIND>
__global__ __launch_bounds__(ACT_THREADS) void rownorm_act_kernel(const __bf16* __restrict__ x, int ldx, int d,
                                                                  float eps, int norm, const __bf16* __restrict__ gu,
                                                                  int ldgu, __bf16* __restrict__ act, int ldact,
                                                                  int ffn) {
  const int m = blockIdx.x, tid = threadIdx.x;
  float s = 1.0f;
  if (norm) {
    __shared__ float red[ACT_THREADS / 64];
    const __bf16* xr = x + (size_t)m * ldx;
    float ss = 0.f;
    for (int i = tid * 8; i < d; i += ACT_THREADS * 8) {
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(xr + i);
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += bf2f(v[j]) * bf2f(v[j]);
    }
    ss = wave_sum(ss);
    if ((tid & 63) == 0) red[tid >> 6] = ss;
    __syncthreads();
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < ACT_THREADS / 64; ++w) t += red[w];
    s = rsqrtf(t / d + eps);
  }
  const __bf16* g = gu + (size_t)m * ldgu;
  __bf16* o = act + (size_t)m * ldact;
  for (int b = blockIdx.y * ACT_THREADS + tid; b < ffn / 8; b += gridDim.y * ACT_THREADS) {
    const bf16x8 gv = *reinterpret_cast<const bf16x8*>(g + 16 * (size_t)b);
    const bf16x8 uv = *reinterpret_cast<const bf16x8*>(g + 16 * (size_t)b + 8);
    bf16x8 r;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float gg = s * bf2f(gv[j]), uu = s * bf2f(uv[j]);
      r[j] = f2bf((KIND == 1 ? gelu_tanh_f(gg) : silu_f(gg)) * uu);
    }
    *reinterpret_cast<bf16x8*>(o + 8 * (size_t)b) = r;
  }
}

// xn[m, :] = x[m, :] * rsqrt(mean(x[m]^2) + eps): the final RMSNorm ahead of the library LM head (its gain is
// folded into the LM head's columns, as for every fused-norm GEMM).  One workgroup per row.
__global__ __launch_bounds__(ACT_THREADS) void rownorm_kernel(const __bf16* __restrict__ x, int ldx, int d, float eps,
                                                              __bf16* __restrict__ xn, int ldxn) {
  __shared__ float red[ACT_THREADS / 64];
  const int m = blockIdx.x, tid = threadIdx.x;
  const __bf16* xr = x + (size_t)m * ldx;
  float ss = 0.f;
  for (int i = tid * 8; i < d; i += ACT_THREADS * 8) {
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(xr + i);
#pragma unroll
    for (int j = 0; j < 8; ++j) ss += bf2f(v[j]) * bf2f(v[j]);
  }
  ss = wave_sum(ss);
  if ((tid & 63) == 0) red[tid >> 6] = ss;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int w = 0; w < ACT_THREADS / 64; ++w) t += red[w];
  const float s = rsqrtf(t / d + eps);
  __bf16* o = xn + (size_t)m * ldxn;
  for (int i = tid * 8; i < d; i += ACT_THREADS * 8) {
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(xr + i);
    bf16x8 r;
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = f2bf(s * bf2f(v[j]));
    *reinterpret_cast<bf16x8*>(o + i) = r;
  }
}

}  // namespace

// Y = X . W^T (+ Y when accumulate): W plain row-major [N, K] bf16, X [M, ldx], Y [M, ldy].  The heuristic
// runs once per shape (outside any stream capture: call it once eagerly, as cain_plan_capture does).
CAIN_API int cain_lt_gemm(const void* W, const void* X, int ldx, int K, int N, int M, void* Y, int ldy, int accumulate,
                          void* ws, long long ws_bytes, hipStream_t st) {
  if (M < 1 || N < 1 || K < 1 || ldx < K || ldy < N || (ldx % 8) || (ldy % 8) || (K % 8)) return -1;
  int dev = 0;
  (void)hipGetDevice(&dev);
  const LtPlan* p = lt_plan(N, K, M, ldx, ldy, accumulate != 0, ws ? ws_bytes : 0, dev);
  if (!p) return -2;
  if (p->ws > (size_t)(ws ? ws_bytes : 0)) return -3;
  const float alpha = 1.0f, beta = accumulate ? 1.0f : 0.0f;
  hipblasStatus_t s = hipblasLtMatmul(g_handle, p->md, &alpha, W, p->la, X, p->lb, &beta, Y, p->lc, Y, p->lc,
                                      &p->algo, ws, p->ws, st);
  return s == HIPBLAS_STATUS_SUCCESS ? 0 : 1000 + int(s);
}

// Build (and cache) the plan of one shape outside any stream capture; 0 when hipBLASLt has an algorithm.
CAIN_API int cain_lt_prepare(int N, int K, int M, int ldx, int ldy, int accumulate, long long ws_bytes) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  const LtPlan* p = lt_plan(N, K, M, ldx, ldy, accumulate != 0, ws_bytes, dev);
  return !p ? -2 : (p->ws > (size_t)ws_bytes ? -3 : 0);
}

// fp32 Y[M, N] = X . W^T (LM head logits; W plain row-major [N, K] bf16).
CAIN_API int cain_lt_gemm_f32(const void* W, const void* X, int ldx, int K, int N, int M, float* Y, int ldy, void* ws,
                              long long ws_bytes, hipStream_t st) {
  if (M < 1 || N < 1 || K < 1 || ldx < K || ldy < N || (ldx % 8) || (ldy % 4) || (K % 8)) return -1;
  int dev = 0;
  (void)hipGetDevice(&dev);
  const LtPlan* p = lt_plan(N, K, M, ldx, ldy, false, ws ? ws_bytes : 0, dev, true);
  if (!p) return -2;
  if (p->ws > (size_t)(ws ? ws_bytes : 0)) return -3;
  const float alpha = 1.0f, beta = 0.0f;
  hipblasStatus_t s = hipblasLtMatmul(g_handle, p->md, &alpha, W, p->la, X, p->lb, &beta, Y, p->lc, Y, p->lc,
                                      &p->algo, ws, p->ws, st);
  return s == HIPBLAS_STATUS_SUCCESS ? 0 : 1000 + int(s);
}

CAIN_API int cain_lt_prepare_f32(int N, int K, int M, int ldx, int ldy, long long ws_bytes) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  const LtPlan* p = lt_plan(N, K, M, ldx, ldy, false, ws_bytes, dev, true);
  return !p ? -2 : (p->ws > (size_t)ws_bytes ? -3 : 0);
}

// xn[m, :d] = x[m, :d] * rsqrt(mean(x[m]^2) + eps), M rows.
CAIN_API int cain_rownorm(const void* x, int ldx, int d, float eps, void* xn, int ldxn, int M, hipStream_t st) {
  if (M < 1 || (d % 8) || (ldx % 8) || (ldxn % 8) || ldx < d || ldxn < d) return -1;
  hipLaunchKernelGGL(rownorm_kernel, dim3(M), dim3(ACT_THREADS), 0, st, reinterpret_cast<const __bf16*>(x), ldx, d,
                     eps, reinterpret_cast<__bf16*>(xn), ldxn);
  return int(hipGetLastError());
}

// act[m, :ffn] = f(s_m * gate) * (s_m * up) from the interleaved gate/up GEMM output gu[m, :2 ffn];
// s_m = rsqrt(mean(x[m]^2) + eps) when norm, else 1.  kind: 0 SiLU (SwiGLU), 1 tanh-GeLU (GeGLU).
CAIN_API int cain_rownorm_act(const void* x, int ldx, int d, float eps, int norm, const void* gu, int ldgu, void* act,
                              int ldact, int M, int ffn, int kind, hipStream_t st) {
  if (M < 1 || (ffn % 8) || (d % 8) || (ldx % 8) || (ldgu % 8) || (ldact % 8) || ldgu < 2 * ffn) return -1;
  const int per_row = cdiv(ffn / 8, ACT_THREADS);
  const dim3 grid(M, per_row < 4 ? per_row : 4);
  auto x_ = reinterpret_cast<const __bf16*>(x);
  auto g_ = reinterpret_cast<const __bf16*>(gu);
  auto a_ = reinterpret_cast<__bf16*>(act);
  if (kind == 1)
    hipLaunchKernelGGL(rownorm_act_kernel<1>, grid, dim3(ACT_THREADS), 0, st, x_, ldx, d, eps, norm, g_, ldgu, a_,
                       ldact, ffn);
  else
    hipLaunchKernelGGL(rownorm_act_kernel<0>, grid, dim3(ACT_THREADS), 0, st, x_, ldx, d, eps, norm, g_, ldgu, a_,
                       ldact, ffn);
  return int(hipGetLastError());
}
