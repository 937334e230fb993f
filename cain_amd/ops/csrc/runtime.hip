// Native decode runtime: the per-step kernel schedule of one model and its
// hipGraph capture/replay.
//
// The Python engine owns every buffer (torch allocations on the GPU) and hands
// the raw pointers over once in a PlanDesc.  `cain_plan_forward` enqueues one
// forward over M rows (decode: one row per live sequence; prefill: one row per
// prompt token, each with its own cache slot and position):
//
//   embed -> L x [QKV GEMM(+RMSNorm, +bias, RoPE, KV append)
//                 -> attention(+split combine) -> O GEMM(+residual)      (CAIN_FRONT=1, <= 4 bf16 rows: ONE launch)
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
CAIN_API int cain_gemm_w8a8(const void* Wp8, const float* wscale, const void* X8, int ld8, const float* xs, int K,
                            int N, int M, void* Y, int ldy, const float* bias, const int* slot, const int* pos,
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
CAIN_API void cain_gemm_set_cmax(float* cmax);
CAIN_API int cain_gemm_cmax_take();
CAIN_API int cain_front_eligible(int M, int d, int q_dim, int hd, int H, int Hkv, int nsplit, int kv8);
CAIN_API int cain_front(const void* wqkv, const float* bqkv, const void* wo, void* x, void* q, void* attn,
                        void* kc, void* vtc, const int* slot, const int* pos, const float* cos_t, const float* sin_t,
                        int M, int d, int H, int Hkv, int hd, int T_max, float eps, int norm, float* part_o,
                        float* part_ml, unsigned* att_ctr, int nsplit, float scale, unsigned* flags,
                        unsigned long long* trace, hipStream_t st);
CAIN_API int cain_sample_ex(float* logits, int ldl, int V, int* tok, int* pos, int* gen, int ldg, int* n_gen,
                            const int* max_new, int* done, int* hist, const int* slot, int T_max, int M,
                            const void* params, void* ws, long long ws_bytes, hipStream_t st);

// hipBLASLt A/B path (opt-in library libcain_blas.so, csrc_blas/blas.hip): not linked into this library; its
// entry points are registered at run time by cain_amd.ops.enable_lt().  Unregistered (the default), every
// forward runs the hand-written kernels.
struct CainLtApi {
  int (*gemm)(const void*, const void*, int, int, int, int, void*, int, int, void*, long long, hipStream_t);
  int (*prepare)(int, int, int, int, int, int, long long);
  int (*gemm_f32)(const void*, const void*, int, int, int, int, float*, int, void*, long long, hipStream_t);
  int (*prepare_f32)(int, int, int, int, int, long long);
  int (*rownorm)(const void*, int, int, float, void*, int, int, hipStream_t);
  int (*rownorm_act)(const void*, int, int, float, int, const void*, int, void*, int, int, int, int, hipStream_t);
};
static CainLtApi g_lt{};
CAIN_API void cain_set_lt_api(const CainLtApi* a) { g_lt = a ? *a : CainLtApi{}; }

extern "C" {

// RMSNorm gains are folded into the weight columns of the GEMM each norm feeds (attn_norm -> wqkv,
// mlp_norm -> wgu, final_norm -> lm_head; models/weights.py fold_gain), so a norm is just a flag here.
struct CainLayer {
  const void* wqkv;
  const float* bqkv;
  const void* wo;
  const void* wgu;
  const void* wdown;
  // fp8 weights (CainPlanDesc::w8): per-output-row scales of each packed matrix (null for bf16)
  const float* sqkv;
  const float* so;
  const float* sgu;
  const float* sdown;
  // plain row-major bf16 copies for the hipBLASLt path (blas.hip; null: fused kernels only): Wo [d, q_dim] and
  // the 8-row-interleaved gate/up [2 ffn, d]
  const void* wo_lt;
  const void* wgu_lt;
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
  int w8;                      // 1: fp8 (e4m3) weights with per-row scales, W8A16 kernels (gemm_w8.hip), M <= 64
  const float* lm_head_scale;  // w8: scales of the packed LM head
  // forwards with >= lt_min_rows rows (0: never) run the O and gate/up projections through hipBLASLt
  // (blas.hip); gu: [Mpad, 2 ffn] bf16 gate/up output, lt_ws: the library's workspace
  int lt_min_rows;
  void* gu;
  void* lt_ws;
  long long lt_ws_bytes;
  // wide forwards with lm_head_lt set run the final RMSNorm (rownorm into xn [Mpad, d] bf16) and the LM head
  // (plain row-major [V, d] bf16, gain folded, fp32 logits) through hipBLASLt; the hand GEMM is the fallback
  const void* lm_head_lt;
  void* xn;
  // 1: the KV caches hold fp8 e4m3 elements (same fragment-major offsets, one byte each, unscaled and
  // saturated at +-448): the QKV epilogue writes them (gemm_epi.h EPI_KV_FP8), attention widens them
  int kv8;
  // W8A8 (w8 with the <name>8 packings): forwards of more than 16 rows quantise each GEMM input per row into
  // x8 [Mpad][x8_ld] e4m3 + xs [Mpad] (wgemm8.hip quant_rows_kernel) and run the fp8-MFMA wide kernel
  const void* lm_head8;
  void* x8;
  float* xs;
  int x8_ld;
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
  // layer-front launch (front.hip) hand-off counters for forwards of <= 4 rows, zeroed once (null: never used)
  unsigned* front_flags = nullptr;
  // LM-head chunk maxima ([Mpad][V / 16] floats; sample.hip sample_cm_kernel)
  float* cmax = nullptr;
  ~Plan() {
    if (sample_ws) (void)hipFree(sample_ws);
    if (front_flags) (void)hipFree(front_flags);
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

// CAIN_FRONT=1: the fused layer front (front.hip) instead of the three launches QKV / attention / O.  Off by
// default: in the graph-replayed batch-1 decode it measured 16.9 vs 14.9 us per layer (qwen2:1.5b) and 28.7 vs
// 25.8 (llama3.1:8b) -- its in-launch hand-offs cost more than the two kernel boundaries they remove
// (profiles/r3/front_trace_*.log, profiles/r3/README.md).
bool front_enabled() {
  static const bool on = [] {
    const char* e = getenv("CAIN_FRONT");
    return e && e[0] == '1';
  }();
  return on;
}

bool lt_rows(const CainPlanDesc& d, int M) { return g_lt.gemm && d.lt_min_rows > 0 && M >= d.lt_min_rows && !d.w8 && d.gu; }

// hipBLASLt heuristics allocate and synchronise: resolve them before a stream capture
int lt_prepare(const Plan& p, int M) {
  const CainPlanDesc& d = p.d;
  if (!lt_rows(d, M) || p.layers.empty()) return 0;
  const int q_dim = d.H * d.hd;
  if (p.layers[0].wo_lt) CK(g_lt.prepare(d.d, q_dim, M, q_dim, d.d, 1, d.lt_ws_bytes));
  if (p.layers[0].wgu_lt) CK(g_lt.prepare(2 * d.ffn, d.d, M, d.d, 2 * d.ffn, 0, d.lt_ws_bytes));
  // no library algorithm for the fp32-output LM head is not an error: forward() falls back to the hand GEMM
  if (d.lm_head_lt && d.xn) (void)g_lt.prepare_f32(d.V, d.d, M, d.d, d.V, d.lt_ws_bytes);
  return 0;
}

// 5 launches per layer: QKV(+RMSNorm, bias, RoPE, KV append) -> attention(+combine) ->
// O(+residual) -> gate/up(+RMSNorm, act*mul) -> down(+residual).
int forward(const Plan& p, int M, const CainRows& r, int want_logits, int want_sample, hipStream_t st) {
  const CainPlanDesc& d = p.d;
  const int qkv_dim = (d.H + 2 * d.Hkv) * d.hd;
  const int q_dim = d.H * d.hd;
  const int epi_act = d.act_kind == 1 ? 4 : 3;
  // one GEMM of the schedule: the bf16 kernels (gemm.hip) or the fp8-weight ones (gemm_w8.hip)
  auto gemm = [&](const void* W, const void* W8, const float* ws, const void* X, int ldx, int K, int N, void* Y,
                  int ldy, const float* bias, int norm, const void* kc, const void* vc, int epi) -> int {
    if (d.w8 && W8 && d.x8 && cain_w8a8_eligible(N, K, M)) {  // W8A8: per-row fp8 activations, fp8 MFMA
      CK(cain_quant_rows(X, ldx, K, M, d.x8, d.x8_ld, d.xs, norm, d.eps, st));
      return cain_gemm_w8a8(W8, ws, d.x8, d.x8_ld, d.xs, K, N, M, Y, ldy, bias, r.slot, r.pos, d.cos_t, d.sin_t,
                            const_cast<void*>(kc), const_cast<void*>(vc), d.H, d.Hkv, d.hd, d.T_max, d.gemm_ws,
                            d.gemm_ws_bytes, epi, st);
    }
    if (d.w8)
      return cain_gemm_w8(W, ws, X, ldx, K, N, M, Y, ldy, bias, norm, d.eps, r.slot, r.pos, d.cos_t, d.sin_t,
                          const_cast<void*>(kc), const_cast<void*>(vc), d.H, d.Hkv, d.hd, d.T_max, epi, st);
    return cain_gemm(W, X, ldx, K, N, M, Y, ldy, bias, norm, d.eps, r.slot, r.pos, d.cos_t, d.sin_t,
                     const_cast<void*>(kc), const_cast<void*>(vc), d.H, d.Hkv, d.hd, d.T_max, d.gemm_ws,
                     d.gemm_ws_bytes, epi, d.waves, st);
  };
  const bool lt = lt_rows(d, M);
  // few-row bf16 forwards: QKV -> attention -> O of a layer as ONE launch (front.hip)
  const bool front = p.front_flags && !d.w8 && !lt && front_enabled() &&
                     cain_front_eligible(M, d.d, q_dim, d.hd, d.H, d.Hkv, d.nsplit, d.kv8);
  CK(cain_embed(r.tok, d.embed, d.x, d.d, M, d.d, d.embed_scale, st));
  for (int l = 0; l < d.n_layers; ++l) {
    const CainLayer& L = p.layers[l];
    const size_t kv_off = (size_t)l * d.kv_layer_elems * (d.kv8 ? 1 : 2);  // bytes
    char* kc = static_cast<char*>(d.kcache) + kv_off;
    char* vc = static_cast<char*>(d.vtcache) + kv_off;
    if (front) {
      CK(cain_front(L.wqkv, L.bqkv, L.wo, d.x, d.q, d.attn, kc, vc, r.slot, r.pos, d.cos_t, d.sin_t, M, d.d, d.H,
                    d.Hkv, d.hd, d.T_max, d.eps, 1, d.part_o, d.part_ml, d.counters, d.nsplit, d.attn_scale,
                    p.front_flags, nullptr, st));
    } else {
      CK(gemm(L.wqkv, L.wqkv8, L.sqkv, d.x, d.d, d.d, qkv_dim, d.q, q_dim, L.bqkv, 1, kc, vc,
              /*EPI_QKV_ROPE*/ 5 | (d.kv8 ? /*EPI_KV_FP8*/ 0x100 : 0)));
      CK(cain_attention_ex(d.q, kc, vc, r.slot, r.pos, d.part_o, d.part_ml, d.counters, d.attn, q_dim, M, d.H,
                           d.Hkv, d.hd, d.T_max, d.nsplit, d.attn_scale, d.kv8, 1.f, 1.f, st));
    }
    if (!front) {  // (the front launch ran the O projection too)
      if (lt && L.wo_lt)
        CK(g_lt.gemm(L.wo_lt, d.attn, q_dim, q_dim, d.d, M, d.x, d.d, 1, d.lt_ws, d.lt_ws_bytes, st));
      else
        CK(gemm(L.wo, L.wo8, L.so, d.attn, q_dim, q_dim, d.d, d.x, d.d, nullptr, 0, nullptr, nullptr,
                /*EPI_RESID*/ 1));
    }
    if (lt && L.wgu_lt) {
      CK(g_lt.gemm(L.wgu_lt, d.x, d.d, d.d, 2 * d.ffn, M, d.gu, 2 * d.ffn, 0, d.lt_ws, d.lt_ws_bytes, st));
      CK(g_lt.rownorm_act(d.x, d.d, d.d, d.eps, 1, d.gu, 2 * d.ffn, d.act, d.ffn, M, d.ffn, d.act_kind, st));
    } else {
      CK(gemm(L.wgu, L.wgu8, L.sgu, d.x, d.d, d.d, 2 * d.ffn, d.act, d.ffn, nullptr, 1, nullptr, nullptr, epi_act));
    }
    CK(gemm(L.wdown, L.wdown8, L.sdown, d.act, d.ffn, d.ffn, d.d, d.x, d.d, nullptr, 0, nullptr, nullptr,
            /*EPI_RESID*/ 1));
  }
  if (want_logits) {
    int e = -2;
    if (lt && d.lm_head_lt && d.xn) {
      CK(g_lt.rownorm(d.x, d.d, d.d, d.eps, d.xn, d.d, M, st));
      e = g_lt.gemm_f32(d.lm_head_lt, d.xn, d.d, d.d, d.V, M, d.logits, d.V, d.lt_ws, d.lt_ws_bytes, st);
      if (e > 0) CK(e);  // a library failure; no plan / unsupported shape (< 0) falls back
    }
    // the LM head also writes the chunk maxima the chunk-max sampler starts from (skinny or wide kernel)
    const int cm_mode = cain_sample_cm_enabled();
    if (e != 0 && p.cmax && (cm_mode == 1 || (cm_mode == 2 && M > 64))) cain_gemm_set_cmax(p.cmax);
    if (e != 0) CK(gemm(d.lm_head, d.lm_head8, d.lm_head_scale, d.x, d.d, d.d, d.V, d.logits, d.V, nullptr, 1, nullptr,
                        nullptr, /*EPI_F32*/ 2));
  }
  const bool cm = want_logits && cain_gemm_cmax_take();
  if (want_sample) {
    if (cm)
      CK(cain_sample_cm(d.logits, d.V, d.V, p.cmax, r.tok, r.pos, r.gen, r.ldg, r.n_gen, r.max_new, r.done, r.hist,
                        r.slot, d.T_max, M, r.sample_params, st));
    else
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
  if (!desc->w8 && desc->V % 64 == 0 && desc->Mpad > 0) {  // LM-head chunk maxima ([Mpad][V / 16])
    const int rows = desc->Mpad;
    if (hipMalloc(&p->cmax, (size_t)rows * (desc->V / 16) * sizeof(float)) != hipSuccess) p->cmax = nullptr;
  }
  if (!desc->w8 && hipMalloc(&p->front_flags, 4096 * 4) == hipSuccess) {  // front.hip: 4096 flag words
    if (hipMemset(p->front_flags, 0, 4096 * 4) != hipSuccess) {
      (void)hipFree(p->front_flags);
      p->front_flags = nullptr;
    }
  } else {
    p->front_flags = nullptr;
  }
  return p;
}

CAIN_API void cain_plan_destroy(void* plan) { delete static_cast<Plan*>(plan); }

CAIN_API const char* cain_plan_last_failure() { return g_fail; }

CAIN_API int cain_plan_forward(void* plan, int M, const CainRows* rows, int want_logits, int want_sample,
                               hipStream_t st) {
  auto* p = static_cast<Plan*>(plan);
  g_fail[0] = 0;
  // W8A16 alone (no W8A8 buffers) takes at most 64 rows
  if (M < 1 || M > CAIN_MAX_ROWS || M > p->d.Mpad || (p->d.w8 && !p->d.x8 && M > 64)) return -1;
  return forward(*p, M, *rows, want_logits, want_sample, st);
}

// Record `steps` decode steps over M rows into a graph; returns the executable graph (or null).
CAIN_API void* cain_plan_capture(void* plan, int M, const CainRows* rows, int steps, hipStream_t st, int* err) {
  auto* p = static_cast<Plan*>(plan);
  *err = 0;
  if (M < 1 || M > CAIN_MAX_ROWS || M > p->d.Mpad || (p->d.w8 && !p->d.x8 && M > 64) || steps < 1) {
    *err = -1;
    return nullptr;
  }
  if ((*err = lt_prepare(*p, M)) != 0) return nullptr;
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

CAIN_API int cain_rows_size() { return int(sizeof(CainRows)); }
CAIN_API int cain_plan_desc_size() { return int(sizeof(CainPlanDesc)); }
CAIN_API int cain_layer_size() { return int(sizeof(CainLayer)); }

}  // extern "C"
