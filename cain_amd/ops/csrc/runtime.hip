// Native decode runtime: the per-step kernel schedule of one model and its
// hipGraph capture/replay.
//
// The Python engine owns every buffer (torch allocations on the GPU) and hands
// the raw pointers over once in a PlanDesc.  `cain_plan_forward` enqueues one
// forward over M rows (decode: one row per live sequence; prefill: one row per
// prompt token, each with its own cache slot and position):
//
//   embed -> L x [QKV GEMM(+RMSNorm, +bias, RoPE, KV append)
//                 -> attention(+split combine) -> O GEMM(+residual)
//                 -> gate/up GEMM(+RMSNorm, act*mul) -> down GEMM(+residual)]
//                 -> LM-head GEMM(+RMSNorm) -> sample
//
// = 5 launches per layer (the unfused schedule had 9).  `cain_plan_capture` records `steps` consecutive
// decode steps into ONE hipGraph; since the sampler advances tok/pos/n_gen on
// the device, a whole generation is a handful of graph launches with no host
// round trip per token (graph-replay floor instead of ~290 host launches per
// token: MI355X_MICROARCH.md rows 'boundary', 'graph-replay-floor').
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "common.h"

constexpr int CAIN_MAX_ROWS = 256;  // rows per forward (decode batch / prefill chunk)

CAIN_API int cain_gemm(const void* Wp, const void* X, int ldx, int K, int N, int M, void* Y, int ldy,
                       const float* bias, int norm, float eps, const int* slot, const int* pos,
                       const float* cos_t, const float* sin_t, void* kc, void* vtc, int H, int Hkv, int hd, int T_max,
                       void* ws, long long ws_bytes, int epi, int waves, hipStream_t st);
CAIN_API int cain_gemm_w8(const void* Wp, const float* wscale, const void* X, int ldx, int K, int N, int M, void* Y,
                          int ldy, const float* bias, int norm, float eps, const int* slot, const int* pos,
                          const float* cos_t, const float* sin_t, void* kc, void* vtc, int H, int Hkv, int hd,
                          int T_max, int epi, hipStream_t st);
CAIN_API int cain_gemm_w4_ex(const void* Wp, const void* wsc, const void* X, int ldx, int K, int N, int M, void* Y,
                             int ldy, const float* bias, int norm, float eps, const int* slot, const int* pos,
                             const float* cos_t, const float* sin_t, void* kc, void* vtc, int H, int Hkv, int hd,
                             int T_max, void* ws, long long ws_bytes, int epi_flags, hipStream_t st);
CAIN_API int cain_gemm_q4(int fmt, const void* Wq, const void* sc, const void* dd, const float* gain, const void* X,
                          int ldx, int K, int N, int M, void* Y, int ldy, const float* bias, int norm, float eps,
                          const int* slot, const int* pos, const float* cos_t, const float* sin_t, void* kc,
                          void* vtc, int H, int Hkv, int hd, int T_max, int epi_flags, hipStream_t st);
CAIN_API int cain_gemm_w8a8(const void* Wp8, const float* wscale, const void* X8, int ld8, const float* xs, int K,
                            int N, int M, void* Y, int ldy, const float* bias, const int* slot, const int* pos,
                            const float* cos_t, const float* sin_t, void* kc, void* vtc, int H, int Hkv, int hd,
                            int T_max, void* ws, long long ws_bytes, int epi_flags, hipStream_t st);
CAIN_API int cain_gemm_w4a8(const void* Wq, const void* wsc, const void* X8, int ld8, const float* xs, int K, int N,
                            int M, void* Y, int ldy, const float* bias, const int* slot, const int* pos,
                            const float* cos_t, const float* sin_t, void* kc, void* vtc, int H, int Hkv, int hd,
                            int T_max, void* ws, long long ws_bytes, int epi_flags, hipStream_t st);
CAIN_API int cain_quant_rows(const void* x, int ldx, int K, int M, void* x8, int ld8, float* xs, int norm, float eps,
                             hipStream_t st);
CAIN_API int cain_w8a8_eligible(int N, int K, int M);
CAIN_API int cain_embed(const int* tok, const void* E, void* out, int ldo, int M, int d, float scale, hipStream_t st);
CAIN_API int cain_attention_ex(const void* q, const void* kc, const void* vtc, const int* slot, const int* pos,
                               float* part_o, float* part_ml, unsigned* counters, void* out, int ldo, int M, int H,
                               int Hkv, int hd, int T_max, int nsplit, float scale, int kv8, float kscale,
                               float vscale, hipStream_t st);
CAIN_API int cain_attention(const void* q, const void* kc, const void* vtc, const int* slot, const int* pos,
                            float* part_o, float* part_ml, unsigned* counters, void* out, int ldo, int M, int H,
                            int Hkv, int hd, int T_max, int nsplit, float scale, hipStream_t st);
CAIN_API int cain_sample(float* logits, int ldl, int V, int* tok, int* pos, int* gen, int ldg, int* n_gen,
                         const int* max_new, int* done, int* hist, const int* slot, int T_max, int M,
                         const void* params, hipStream_t st);
CAIN_API long long cain_sample_ws_bytes(int M);
CAIN_API int cain_sample_split_max();
CAIN_API int cain_sample_cm_enabled();
CAIN_API int cain_sample_cm(float* logits, int ldl, int V, const float* cmax, int* tok, int* pos, int* gen, int ldg,
                            int* n_gen, const int* max_new, int* done, int* hist, const int* slot, int T_max, int M,
                            const void* params, hipStream_t st);
CAIN_API int cain_sample_lean(float* logits, int ldl, int V, const float* cmax, int* tok, int* pos, int* gen, int ldg,
                              int* n_gen, const int* max_new, int* done, int* hist, const int* slot, int T_max, int M,
                              const void* params, hipStream_t st);
CAIN_API void cain_gemm_set_cmax(float* cmax);
CAIN_API int cain_gemm_cmax_take();
CAIN_API int cain_sample_ex(float* logits, int ldl, int V, int* tok, int* pos, int* gen, int ldg, int* n_gen,
                            const int* max_new, int* done, int* hist, const int* slot, int T_max, int M,
                            const void* params, void* ws, long long ws_bytes, hipStream_t st);

extern "C" {

// weight storage of a plan (CainPlanDesc::wfmt)
enum { WFMT_BF16 = 0, WFMT_FP8 = 1, WFMT_FP4 = 2, WFMT_Q4_0 = 3, WFMT_Q4_K = 4 };

// RMSNorm gains are folded into the weight columns of the GEMM each norm feeds (attn_norm -> wqkv,
// mlp_norm -> wgu, final_norm -> lm_head; models/weights.py fold_gain), so a norm is just a flag here.
struct CainLayer {
  const void* wqkv;
  const float* bqkv;
  const void* wo;
  const void* wgu;
  const void* wdown;
  // scales of each packed matrix (null for bf16): fp8 -- fp32 per output row; fp4 -- e8m0 bytes per 32-k block in
  // the kernel's lane order (models/weights.py pack_mxfp4)
  const void* sqkv;
  const void* so;
  const void* sgu;
  const void* sdown;
  // fp8 weights in the W8A8 wide kernel's packing (wgemm8.hip; null: W8A16 only), same scales as above
  const void* wqkv8;
  const void* wo8;
  const void* wgu8;
  const void* wdown8;
};

struct CainPlanDesc {
  int n_layers, d, H, Hkv, hd, ffn, V, act_kind, T_max, Mpad, nsplit, waves;
  float eps, embed_scale, attn_scale;
  const void* embed;
  const void* lm_head;
  const CainLayer* layers;
  void* kcache;  // [L][S][Hkv][T_max][hd] fragment-major, bf16 (kv8: e4m3)
  void* vtcache; // [L][S][Hkv][hd][T_max]
  long long kv_layer_elems;
  const float* cos_t;
  const float* sin_t;
  void* x;
  void* q;
  void* attn;
  void* act;
  float* logits;
  float* part_o;
  float* part_ml;
  unsigned* counters;
  void* gemm_ws;  // batched-GEMM workspace (counters zeroed once + split-K partials), see gemm.hip
  long long gemm_ws_bytes;
  // WFMT_FP8: e4m3 weights with per-row scales, W8A16 kernels (gemm_w8.hip) up to 64 rows (W8A8 above 16 rows
  // when the <name>8 packings are present); WFMT_FP4: MXFP4 weights, W4A16 kernels (gemm_w4.hip) up to 64 rows,
  // W4A8 (wgemm8.hip FP4, the same packed bytes) above 16 rows (cain_w4a8_set_min_rows) when x8 / xs are present
  int wfmt;
  const void* lm_head_scale;  // fp8 / fp4: scales of the packed LM head
  // 1: the KV caches hold fp8 e4m3 elements (same fragment-major offsets, one byte each, unscaled and
  // saturated at +-448): the QKV epilogue writes them (gemm_epi.h EPI_KV_FP8), attention widens them
  int kv8;
  // W8A8 (fp8 with the <name>8 packings) / W4A8 (fp4): wide forwards quantise each GEMM input per row into
  // x8 [Mpad][x8_ld] e4m3 + xs [Mpad] (wgemm8.hip quant_rows_kernel) and run the scaled-MFMA wide kernel
  const void* lm_head8;
  void* x8;
  float* xs;
  int x8_ld;
  // WFMT_Q4_*: 1 when each norm-fed weight's scale buffer ends with its fp32 RMSNorm gain (weights not gain-folded)
  int q4_gain;
};

struct CainRows {
  int* tok;
  int* pos;
  int* slot;
  // sampling state (decode rows only; may be null for prefill)
  int* n_gen;
  const int* max_new;
  int* done;
  int* hist;
  int* gen;
  int ldg;
  const void* sample_params;
};

}  // extern "C"

namespace {

struct Plan {
  CainPlanDesc d;
  std::vector<CainLayer> layers;
  // two-stage sampler workspace (sample.hip cain_sample_ex) for decode forwards of <= 64 rows, zeroed once
  void* sample_ws = nullptr;
  long long sample_ws_bytes = 0;
  // LM-head chunk maxima ([Mpad][V / 16] floats; sample.hip sample_cm_kernel)
  float* cmax = nullptr;
  ~Plan() {
    if (sample_ws) (void)hipFree(sample_ws);
    if (cmax) (void)hipFree(cmax);
  }
};

// first failing call of the last failed forward (source text + line), for the Python error message
thread_local char g_fail[160] = {0};

#define CK(x)                                                                    \
  do {                                                                           \
    int _e = (x);                                                                \
    if (_e != 0) {                                                               \
      if (!g_fail[0]) snprintf(g_fail, sizeof(g_fail), "runtime.hip:%d %s", __LINE__, #x); \
      return _e;                                                                 \
    }                                                                            \
  } while (0)

// Rows above which an fp4 plan with x8 runs W4A8 (the W4A16 kernels take up to 64): 16, the W4A8 minimum -- at 24 /
// 48 / 64 rows W4A8 decodes 7.7k / 13.6k / 16.6k tok/s against W4A16's 5.1k / 5.0k / 6.4k
// (profiles/r4/ab/w4a8_crossover.txt)
static int g_w4a8_min_rows = 16;

// rows a forward of this plan may have: 64 for the few-row-only weight formats
int max_rows(const CainPlanDesc& d) {
  if ((d.wfmt == WFMT_FP4 || d.wfmt == WFMT_FP8) && !d.x8) return d.Mpad < 64 ? d.Mpad : 64;
  if (d.wfmt == WFMT_Q4_0 || d.wfmt == WFMT_Q4_K) return d.Mpad < 64 ? d.Mpad : 64;  // 16-row launches (gemm_q4.hip)
  return d.Mpad < CAIN_MAX_ROWS ? d.Mpad : CAIN_MAX_ROWS;
}

// 5 launches per layer: QKV(+RMSNorm, bias, RoPE, KV append) -> attention(+combine) ->
// O(+residual) -> gate/up(+RMSNorm, act*mul) -> down(+residual).
int forward(const Plan& p, int M, const CainRows& r, int want_logits, int want_sample, hipStream_t st) {
  const CainPlanDesc& d = p.d;
  const int qkv_dim = (d.H + 2 * d.Hkv) * d.hd;
  const int q_dim = d.H * d.hd;
  const int epi_act = d.act_kind == 1 ? 4 : 3;
  // one GEMM of the schedule: the bf16 kernels (gemm.hip / wgemm.hip), fp8 weights (gemm_w8.hip / wgemm8.hip) or
  // MXFP4 weights (gemm_w4.hip)
  auto gemm = [&](const void* W, const void* W8, const void* ws, const void* X, int ldx, int K, int N, void* Y,
                  int ldy, const float* bias, int norm, const void* kc, const void* vc, int epi) -> int {
    void* kcm = const_cast<void*>(kc);
    void* vcm = const_cast<void*>(vc);
    if (d.wfmt == WFMT_FP4 && d.x8 && (M > g_w4a8_min_rows || M > 64) && cain_w8a8_eligible(N, K, M)) {  // W4A8
      CK(cain_quant_rows(X, ldx, K, M, d.x8, d.x8_ld, d.xs, norm, d.eps, st));
      return cain_gemm_w4a8(W, ws, d.x8, d.x8_ld, d.xs, K, N, M, Y, ldy, bias, r.slot, r.pos, d.cos_t, d.sin_t, kcm,
                            vcm, d.H, d.Hkv, d.hd, d.T_max, d.gemm_ws, d.gemm_ws_bytes, epi, st);
    }
    if (d.wfmt == WFMT_Q4_0 || d.wfmt == WFMT_Q4_K) {
      // GGUF Q4_0 / Q4_K (gemm_q4.hip): ws = [block scales: N K / 16 bytes][Q4_K: (d, dmin): N K / 64 bytes]
      // [the fp32 norm gain over K, when the plan keeps gains unfolded (a GGUF file's exact values)]
      const char* sc = static_cast<const char*>(ws);
      const char* dd = sc + (size_t)N * K / 16;
      const float* gain = d.q4_gain && norm ? reinterpret_cast<const float*>(dd + (d.wfmt == WFMT_Q4_K ? (size_t)N * K / 64 : 0))
                                            : nullptr;
      return cain_gemm_q4(d.wfmt == WFMT_Q4_K, W, sc, dd, gain, X, ldx, K, N, M, Y, ldy, bias, norm, d.eps, r.slot,
                          r.pos, d.cos_t, d.sin_t, kcm, vcm, d.H, d.Hkv, d.hd, d.T_max, epi, st);
    }
    if (d.wfmt == WFMT_FP4)
      return cain_gemm_w4_ex(W, ws, X, ldx, K, N, M, Y, ldy, bias, norm, d.eps, r.slot, r.pos, d.cos_t, d.sin_t, kcm,
                             vcm, d.H, d.Hkv, d.hd, d.T_max, d.gemm_ws, d.gemm_ws_bytes, epi, st);
    const float* wsf = static_cast<const float*>(ws);
    if (d.wfmt == WFMT_FP8 && W8 && d.x8 && cain_w8a8_eligible(N, K, M)) {  // W8A8: per-row fp8 activations
      CK(cain_quant_rows(X, ldx, K, M, d.x8, d.x8_ld, d.xs, norm, d.eps, st));
      return cain_gemm_w8a8(W8, wsf, d.x8, d.x8_ld, d.xs, K, N, M, Y, ldy, bias, r.slot, r.pos, d.cos_t, d.sin_t, kcm,
                            vcm, d.H, d.Hkv, d.hd, d.T_max, d.gemm_ws, d.gemm_ws_bytes, epi, st);
    }
    if (d.wfmt == WFMT_FP8)
      return cain_gemm_w8(W, wsf, X, ldx, K, N, M, Y, ldy, bias, norm, d.eps, r.slot, r.pos, d.cos_t, d.sin_t, kcm, vcm,
                          d.H, d.Hkv, d.hd, d.T_max, epi, st);
    return cain_gemm(W, X, ldx, K, N, M, Y, ldy, bias, norm, d.eps, r.slot, r.pos, d.cos_t, d.sin_t, kcm, vcm, d.H,
                     d.Hkv, d.hd, d.T_max, d.gemm_ws, d.gemm_ws_bytes, epi, d.waves, st);
  };
  CK(cain_embed(r.tok, d.embed, d.x, d.d, M, d.d, d.embed_scale, st));
  for (int l = 0; l < d.n_layers; ++l) {
    const CainLayer& L = p.layers[l];
    const size_t kv_off = (size_t)l * d.kv_layer_elems * (d.kv8 ? 1 : 2);  // bytes
    char* kc = static_cast<char*>(d.kcache) + kv_off;
    char* vc = static_cast<char*>(d.vtcache) + kv_off;
    CK(gemm(L.wqkv, L.wqkv8, L.sqkv, d.x, d.d, d.d, qkv_dim, d.q, q_dim, L.bqkv, 1, kc, vc,
            /*EPI_QKV_ROPE*/ 5 | (d.kv8 ? /*EPI_KV_FP8*/ 0x100 : 0)));
    CK(cain_attention_ex(d.q, kc, vc, r.slot, r.pos, d.part_o, d.part_ml, d.counters, d.attn, q_dim, M, d.H, d.Hkv,
                         d.hd, d.T_max, d.nsplit, d.attn_scale, d.kv8, 1.f, 1.f, st));
    CK(gemm(L.wo, L.wo8, L.so, d.attn, q_dim, q_dim, d.d, d.x, d.d, nullptr, 0, nullptr, nullptr, /*EPI_RESID*/ 1));
    CK(gemm(L.wgu, L.wgu8, L.sgu, d.x, d.d, d.d, 2 * d.ffn, d.act, d.ffn, nullptr, 1, nullptr, nullptr, epi_act));
    CK(gemm(L.wdown, L.wdown8, L.sdown, d.act, d.ffn, d.ffn, d.d, d.x, d.d, nullptr, 0, nullptr, nullptr,
            /*EPI_RESID*/ 1));
  }
  if (want_logits) {
    // the LM head also writes the chunk maxima the chunk-max samplers start from (the bf16 skinny / wide kernels and
    // the few-row fp8 / MXFP4 / Q4 kernels; a kernel that does not leaves cain_gemm_cmax_take() at 0)
    const int cm_mode = cain_sample_cm_enabled();
    if (p.cmax && (cm_mode == 1 || cm_mode == 3 || (cm_mode == 2 && M > 64))) cain_gemm_set_cmax(p.cmax);
    CK(gemm(d.lm_head, d.lm_head8, d.lm_head_scale, d.x, d.d, d.d, d.V, d.logits, d.V, nullptr, 1, nullptr, nullptr,
            /*EPI_F32*/ 2));
  }
  const bool cm = want_logits && cain_gemm_cmax_take();
  if (want_sample) {
    // the chunk-max sampler refuses (< 0) vocabularies beyond its chunk capacity: the two-stage / one-workgroup
    // kernels take those
    const int cm_mode = cain_sample_cm_enabled();
    const int e = !cm ? -1
                  : cm_mode == 3 ? cain_sample_lean(d.logits, d.V, d.V, p.cmax, r.tok, r.pos, r.gen, r.ldg, r.n_gen,
                                                    r.max_new, r.done, r.hist, r.slot, d.T_max, M, r.sample_params, st)
                                 : cain_sample_cm(d.logits, d.V, d.V, p.cmax, r.tok, r.pos, r.gen, r.ldg, r.n_gen,
                                                  r.max_new, r.done, r.hist, r.slot, d.T_max, M, r.sample_params, st);
    if (e > 0) CK(e);
    if (e < 0)
      CK(cain_sample_ex(d.logits, d.V, d.V, r.tok, r.pos, r.gen, r.ldg, r.n_gen, r.max_new, r.done, r.hist, r.slot,
                        d.T_max, M, r.sample_params, p.sample_ws, p.sample_ws_bytes, st));
  }
  return 0;
}

}  // namespace

extern "C" {

CAIN_API void* cain_plan_create(const CainPlanDesc* desc) {
  auto* p = new Plan();
  p->d = *desc;
  p->layers.assign(desc->layers, desc->layers + desc->n_layers);
  p->d.layers = p->layers.data();
  const int ms = desc->Mpad < cain_sample_split_max() ? desc->Mpad : cain_sample_split_max();
  if (ms > 0) {
    const long long nb = cain_sample_ws_bytes(ms);
    if (hipMalloc(&p->sample_ws, nb) == hipSuccess && hipMemset(p->sample_ws, 0, nb) == hipSuccess) {
      p->sample_ws_bytes = nb;
    } else {
      if (p->sample_ws) (void)hipFree(p->sample_ws);
      p->sample_ws = nullptr;  // the one-workgroup sampler needs no workspace
    }
  }
  // LM-head chunk maxima ([Mpad][V / 16])
  if (desc->V % 64 == 0 && desc->Mpad > 0) {
    if (hipMalloc(&p->cmax, (size_t)desc->Mpad * (desc->V / 16) * sizeof(float)) != hipSuccess) p->cmax = nullptr;
  }
  return p;
}

CAIN_API void cain_plan_destroy(void* plan) { delete static_cast<Plan*>(plan); }

CAIN_API void cain_w4a8_set_min_rows(int m) { g_w4a8_min_rows = m > 16 ? m : 16; }

CAIN_API const char* cain_plan_last_failure() { return g_fail; }

CAIN_API int cain_plan_forward(void* plan, int M, const CainRows* rows, int want_logits, int want_sample,
                               hipStream_t st) {
  auto* p = static_cast<Plan*>(plan);
  g_fail[0] = 0;
  if (M < 1 || M > max_rows(p->d)) return -1;
  return forward(*p, M, *rows, want_logits, want_sample, st);
}

// Record `steps` decode steps over M rows into a graph; returns the executable graph (or null).
CAIN_API void* cain_plan_capture(void* plan, int M, const CainRows* rows, int steps, hipStream_t st, int* err) {
  auto* p = static_cast<Plan*>(plan);
  *err = 0;
  if (M < 1 || M > max_rows(p->d) || steps < 1) {
    *err = -1;
    return nullptr;
  }
  hipGraph_t g = nullptr;
  hipError_t e = hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal);
  if (e != hipSuccess) {
    *err = int(e);
    return nullptr;
  }
  int fe = 0;
  for (int s = 0; s < steps && fe == 0; ++s) fe = forward(*p, M, *rows, 1, 1, st);
  e = hipStreamEndCapture(st, &g);
  if (fe != 0 || e != hipSuccess) {
    *err = fe ? fe : int(e);
    if (g) (void)hipGraphDestroy(g);
    return nullptr;
  }
  hipGraphExec_t ex = nullptr;
  e = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  if (e != hipSuccess) {
    *err = int(e);
    return nullptr;
  }
  return ex;
}

CAIN_API int cain_graph_launch(void* exec, hipStream_t st) {
  return int(hipGraphLaunch(static_cast<hipGraphExec_t>(exec), st));
}

CAIN_API void cain_graph_destroy(void* exec) {
  if (exec) (void)hipGraphExecDestroy(static_cast<hipGraphExec_t>(exec));
}

// ---- CU-limited streams: the batch-1 energy lever (tools/cu_sweep.py).  A stream whose hardware queue may use only
// n of the device's CUs (hipExtStreamCreateWithCUMask), chosen as whole groups of 8 consecutive mask bits spaced
// evenly over the mask: balanced over the 8 XCDs whether the mask's CU numbering interleaves the XCDs or runs
// through them one after the other (n a multiple of 64 balances exactly under both).  Kernels captured or launched
// for such a stream size their grids by cain_cu_budget().
static int g_cu_budget = 0;

static int device_cus() {
  static const int n = [] {
    int dev = 0, c = 0;
    (void)hipGetDevice(&dev);
    return hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && c > 0 ? c : 256;
  }();
  return n;
}

extern "C" int cain_cu_budget() {
  const int n = device_cus();
  return g_cu_budget > 0 && g_cu_budget < n ? g_cu_budget : n;
}

CAIN_API void cain_set_cu_budget(int n) { g_cu_budget = n > 0 ? n : 0; }
CAIN_API int cain_get_cu_budget() { return cain_cu_budget(); }

// The mask itself (host-side; tests): n_cu of total bits set, or -1.
CAIN_API int cain_cu_mask(int n_cu, int total, uint32_t* mask, int words) {
  if (total <= 0 || total % 8 || n_cu <= 0 || n_cu > total || n_cu % 8 || words * 32 < total) return -1;
  for (int i = 0; i < words; ++i) mask[i] = 0;
  const int groups = total / 8, take = n_cu / 8;
  for (int j = 0; j < take; ++j) {
    const int g = (int)((long long)j * groups / take);
    for (int b = 0; b < 8; ++b) mask[(g * 8 + b) / 32] |= 1u << ((g * 8 + b) % 32);
  }
  return 0;
}

CAIN_API void* cain_stream_create_cu_limited(int n_cu) {
  const int total = device_cus();
  std::vector<uint32_t> mask((total + 31) / 32);
  if (cain_cu_mask(n_cu, total, mask.data(), (int)mask.size()) != 0) return nullptr;
  hipStream_t st = nullptr;
  if (hipExtStreamCreateWithCUMask(&st, (uint32_t)mask.size(), mask.data()) != hipSuccess) return nullptr;
  return st;
}

CAIN_API int cain_stream_destroy(void* st) { return hipStreamDestroy(static_cast<hipStream_t>(st)) == hipSuccess ? 0 : -1; }

CAIN_API int cain_rows_size() { return int(sizeof(CainRows)); }
CAIN_API int cain_plan_desc_size() { return int(sizeof(CainPlanDesc)); }
CAIN_API int cain_layer_size() { return int(sizeof(CainLayer)); }

}  // extern "C"
