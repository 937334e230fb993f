// Token sampling on device (SURVEY §2.4 row "Sampling").
//
// One 1024-thread workgroup per row.  Ollama's default pipeline
// (repeat_penalty over the last `repeat_last_n` tokens -> temperature ->
// top-k -> top-p -> multinomial) or greedy argmax when temperature == 0.
// top-k is exact and needs two passes over the row: pass 1 takes per-thread
// maxima; the K-th largest of those 1024 maxima (wave bitonic sorts + binary
// searches) is a threshold that provably keeps all top-K elements; pass 2
// gathers the (few) elements above it, which are rank-sorted in LDS.  No histogram atomics (an earlier radix-select
// version serialised on a handful of exponent bins: 233 us/step at batch 16).
//
// The kernel also advances the decode state so a whole generation can be
// replayed from a hipGraph with no host round trip per token:
//   tok[m]  <- sampled id        (input of the next step's embedding)
//   pos[m]  += 1                 (position of that token)
//   gen[m][n_gen[m]++] <- id     (output buffer, read back once at the end)
//   hist ring of the last 64 ids (repeat penalty), done[m] on EOS / budget.
#include "common.h"

struct SampleParams {
  float temperature;
  float top_p;
  float repeat_penalty;
  int top_k;
  int repeat_last_n;
  int eos_id;
  uint64_t seed;
};

__device__ __forceinline__ uint32_t ord_u32(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

constexpr int SAMPLE_THREADS = 1024;
constexpr int HIST = 64;
constexpr int MAXC = 1024;  // candidate cap after top-k (ties included)

// Temperature / top-p / multinomial draw over the n candidates sv[0..n) (sorted: value desc, index asc).  The
// random stream is keyed by the request's seed and its token index only, not by the batch row: a request that
// continuous batching moves to another row (ContinuousBatch.retire) keeps its stream, so an Ollama `seed`
// reproduces the same tokens however the batch is packed (rows without a seed get a unique one on the host,
// engine._row_options).
__device__ int draw_topk(const float* sv, const int* si, int n, const SampleParams& P, int ng) {
  const float invT = 1.0f / P.temperature;
  const float mx = sv[0] * invT;
  float z = 0.f;
  for (int i = 0; i < n; ++i) z += __expf(sv[i] * invT - mx);
  // top-p: smallest prefix with cumulative probability >= top_p
  int cut = n;
  if (P.top_p > 0.f && P.top_p < 1.f) {
    float c = 0.f;
    for (int i = 0; i < n; ++i) {
      c += __expf(sv[i] * invT - mx) / z;
      if (c >= P.top_p) { cut = i + 1; break; }
    }
  }
  float zc = 0.f;
  for (int i = 0; i < cut; ++i) zc += __expf(sv[i] * invT - mx);
  const uint64_t r = mix64(P.seed ^ mix64(uint64_t(ng) * 0x632BE59BD9B4E019ull + 0x9E3779B97F4A7C15ull));
  const float u = float(r >> 40) * (1.0f / 16777216.0f) * zc;
  float c = 0.f;
  int pick = si[cut - 1];
  for (int i = 0; i < cut; ++i) {
    c += __expf(sv[i] * invT - mx);
    if (u < c) { pick = si[i]; break; }
  }
  return pick;
}

// Decode-state update of row m after sampling `choice` (one thread).
__device__ void advance_row(int m, int choice, int ng, const SampleParams& P, int* tok, int* pos, int* gen, int ldg,
                            int* n_gen, const int* max_new, int* done, int* hist, int T_max) {
  gen[(size_t)m * ldg + ng] = choice;
  hist[(size_t)m * HIST + (ng & (HIST - 1))] = choice;
  const int n1 = ng + 1;
  n_gen[m] = n1;
  tok[m] = choice;
  const int p1 = pos[m] + 1;
  if ((P.eos_id >= 0 && choice == P.eos_id) || n1 >= max_new[m] || p1 >= T_max) {
    done[m] = 1;
  } else {
    pos[m] = p1;
  }
}

__global__ __launch_bounds__(SAMPLE_THREADS) void sample_kernel(
    float* __restrict__ logits, int ldl, int V, int* __restrict__ tok, int* __restrict__ pos,
    int* __restrict__ gen, int ldg, int* __restrict__ n_gen, const int* __restrict__ max_new,
    int* __restrict__ done, int* __restrict__ hist, const int* __restrict__ slot, int T_max,
    const SampleParams* __restrict__ params) {
  const int m = blockIdx.x;
  if (slot[m] < 0 || done[m]) return;
  const SampleParams P = params[m];
  float* lg = logits + (size_t)m * ldl;
  const int tid = threadIdx.x;
  __shared__ int s_hist[HIST];
  __shared__ float ws_v[SAMPLE_THREADS / 64][64];
  __shared__ int ws_i[SAMPLE_THREADS / 64][64];
  __shared__ float s_tau;
  __shared__ float sv[256];
  __shared__ int si[256];
  __shared__ float cval[MAXC];
  __shared__ int cidx[MAXC];
  __shared__ int s_nc;
  __shared__ float red_v[SAMPLE_THREADS / 64];
  __shared__ int red_i[SAMPLE_THREADS / 64];
  __shared__ int s_choice;

  // ---- repeat penalty (llama.cpp semantics: once per distinct recent id), one lane per history slot
  const int* hr = hist + (size_t)m * HIST;
  const int ng = n_gen[m];
  const int nrep = (P.repeat_penalty != 1.0f && P.repeat_last_n > 0) ? min(min(P.repeat_last_n, HIST), ng) : 0;
  if (nrep > 0) {
    if (tid < HIST) s_hist[tid] = (tid < nrep) ? hr[(ng - 1 - tid) & (HIST - 1)] : -1;
    __syncthreads();
    if (tid < nrep) {
      const int id = s_hist[tid];
      bool first = id >= 0 && id < V;
      for (int j = 0; j < tid; ++j) first &= (s_hist[j] != id);
      if (first) {
        const float v = lg[id];
        lg[id] = v > 0.f ? v / P.repeat_penalty : v * P.repeat_penalty;
      }
    }
    __syncthreads();
  }

  // ---- pass 1: per-thread max (value, index); 16-byte loads, 4 in flight per thread
  const f32x4* lg4 = reinterpret_cast<const f32x4*>(lg);
  const int V4 = V >> 2;
  float bv = -INFINITY;
  int bi = 0x7fffffff;
  for (int base = tid; base < V4; base += 4 * SAMPLE_THREADS) {
    f32x4 c[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) c[u] = lg4[min(base + u * SAMPLE_THREADS, V4 - 1)];  // unconditional (clamped)
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const bool in = base + u * SAMPLE_THREADS < V4;
#pragma unroll
      for (int j = 0; j < 4; ++j) c[u][j] = in ? c[u][j] : -INFINITY;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (c[u][j] > bv) { bv = c[u][j]; bi = (base + u * SAMPLE_THREADS) * 4 + j; }
  }
  for (int i = (V4 << 2) + tid; i < V; i += SAMPLE_THREADS) {  // tail (V % 4)
    const float v = lg[i];
    if (v > bv) { bv = v; bi = i; }
  }

  int choice;
  if (P.temperature <= 0.f) {
    // ---- greedy argmax (lowest index on ties)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(bv, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
    }
    if ((tid & 63) == 0) { red_v[tid >> 6] = bv; red_i[tid >> 6] = bi; }
    __syncthreads();
    if (tid == 0) {
      float v = red_v[0];
      int ix = red_i[0];
      for (int w = 1; w < SAMPLE_THREADS / 64; ++w)
        if (red_v[w] > v || (red_v[w] == v && red_i[w] < ix)) { v = red_v[w]; ix = red_i[w]; }
      s_choice = ix;
    }
    __syncthreads();
    choice = s_choice;
  } else {
    int K = P.top_k;
    if (K <= 0 || K > 256) K = 256;
    if (K > V) K = V;
    // ---- threshold tau = K-th largest of the 1024 thread maxima.  The K largest
    // thread maxima are K distinct elements >= tau, so the K-th largest element of
    // the row is >= tau: filtering x >= tau keeps every top-K candidate.
    // Each wave bitonic-sorts its 64 maxima (value desc, thread asc) in registers;
    // only a wave's first min(K, 64) can be globally top-K, and their global rank is
    // the sum over waves of a 6-step binary search in that wave's sorted list.
    const int lane = tid & 63, wv = tid >> 6;
    float kv = bv;
    int ki = tid;
    for (int k = 2; k <= 64; k <<= 1) {
      for (int j = k >> 1; j > 0; j >>= 1) {
        const float ov = __shfl_xor(kv, j, 64);
        const int oi = __shfl_xor(ki, j, 64);
        const bool o_before = (ov > kv) || (ov == kv && oi < ki);
        const bool keep_before = ((lane & j) == 0) == ((lane & k) == 0);
        if (keep_before ? o_before : !o_before) { kv = ov; ki = oi; }
      }
    }
    ws_v[wv][lane] = kv;
    ws_i[wv][lane] = ki;
    __syncthreads();
    if (lane < K) {
      int r = lane;
      for (int w2 = 0; w2 < SAMPLE_THREADS / 64; ++w2) {
        if (w2 == wv) continue;
        int lo = 0, hi = 64;  // first index of w2's list that is NOT before (kv, ki)
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          const float mv = ws_v[w2][mid];
          const bool before = (mv > kv) || (mv == kv && ws_i[w2][mid] < ki);
          if (before) lo = mid + 1; else hi = mid;
        }
        r += lo;
      }
      if (r == K - 1) s_tau = kv;
    }
    if (tid == 0) s_nc = 0;
    __syncthreads();
    const float tau = s_tau;
    // ---- pass 2: gather candidates >= tau (few; LDS atomics only for them)
    for (int base = tid; base < V4; base += 4 * SAMPLE_THREADS) {
      f32x4 c[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) c[u] = lg4[min(base + u * SAMPLE_THREADS, V4 - 1)];  // unconditional (clamped)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const bool in = base + u * SAMPLE_THREADS < V4;
#pragma unroll
        for (int j = 0; j < 4; ++j) c[u][j] = in ? c[u][j] : -INFINITY;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (c[u][j] >= tau) {
            const int k = atomicAdd(&s_nc, 1);
            if (k < MAXC) { cval[k] = c[u][j]; cidx[k] = (base + u * SAMPLE_THREADS) * 4 + j; }
          }
    }
    for (int i = (V4 << 2) + tid; i < V; i += SAMPLE_THREADS) {
      const float v = lg[i];
      if (v >= tau) {
        const int k = atomicAdd(&s_nc, 1);
        if (k < MAXC) { cval[k] = v; cidx[k] = i; }
      }
    }
    __syncthreads();
    // ---- rank the candidates (value desc, index asc); keep the top K in sorted order
    const int nc = min(s_nc, MAXC);
    for (int a = tid; a < nc; a += SAMPLE_THREADS) {
      const float va = cval[a];
      const int ia = cidx[a];
      int r = 0;
      for (int b = 0; b < nc; ++b) {
        const float vb = cval[b];
        r += (vb > va) || (vb == va && cidx[b] < ia);
      }
      if (r < K) { sv[r] = va; si[r] = ia; }
    }
    __syncthreads();
    if (tid == 0) s_choice = draw_topk(sv, si, min(nc, K), P, ng);
    __syncthreads();
    choice = s_choice;
  }

  if (tid == 0) advance_row(m, choice, ng, P, tok, pos, gen, ldg, n_gen, max_new, done, hist, T_max);
}

// =====================================================================================================
// Two-stage sampler for few rows (single-stream decode, continuous batches of a few requests).
//
// The one-workgroup-per-row kernel above streams a row's logits through ONE CU twice: 39-48 us per token at
// batch 1 for 128-256 k vocabularies (profiles/r2/prof_b1_r2_kernel_stats.csv) -- as long as three decode
// layers of qwen2:1.5b.  Here SS_P workgroups share a row: each scans 1/SS_P of the vocabulary (repeat penalty
// for the ids it owns, then its exact local top-K by the same thread-maxima threshold + gather + rank as above,
// or its argmax when greedy) and publishes the sorted list with write-through stores; the LAST arriving
// workgroup of the row (ticket) merges the SS_P sorted lists -- each candidate's global rank is its position in
// its own list plus a binary search in every other list -- and runs the same temperature / top-p / draw and
// decode-state update as the one-workgroup kernel.  The union of local top-K lists holds the global top-K and
// (value desc, index asc) is a strict order, so both kernels draw the same token from the same logits and seed.
// =====================================================================================================
constexpr int SS_THREADS = 256;
constexpr int SS_P = 16;      // vocabulary slices (workgroups) per row
constexpr int SS_KMAX = 256;  // top-k clamp, as the one-workgroup kernel
constexpr int SS_NJ = 16;     // 16-byte chunks per thread: a slice holds <= SS_NJ * 4 * SS_THREADS elements
constexpr int SS_G = 4;       // sub-maxima per thread (threshold granularity)

struct SampleWs {  // per row: SS_P sorted candidate lists + their lengths; one ticket counter per row
  float* cv;       // [M][SS_P][SS_KMAX]
  int* ci;         // [M][SS_P][SS_KMAX]
  int* cn;         // [M][SS_P]
  unsigned* ctr;   // [M], zero between launches (the merger resets it)
};

__global__ __launch_bounds__(SS_THREADS) void sample_split_kernel(
    float* __restrict__ logits, int ldl, int V, int* __restrict__ tok, int* __restrict__ pos,
    int* __restrict__ gen, int ldg, int* __restrict__ n_gen, const int* __restrict__ max_new,
    int* __restrict__ done, int* __restrict__ hist, const int* __restrict__ slot, int T_max,
    const SampleParams* __restrict__ params, const SampleWs ws) {
  const int m = blockIdx.x, part = blockIdx.y;
  if (slot[m] < 0 || done[m]) return;  // the same for every workgroup of the row: no ticket is taken
  const SampleParams P = params[m];
  float* lg = logits + (size_t)m * ldl;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  constexpr int NW = SS_THREADS / 64;
  // this workgroup's slice [v0, v1) of the vocabulary (16-byte aligned starts)
  const int chunk = (((V + SS_P - 1) / SS_P) + 3) & ~3;
  const int v0 = min(V, part * chunk), v1 = min(V, v0 + chunk);
  const bool greedy = P.temperature <= 0.f;
  int K = P.top_k;
  if (K <= 0 || K > SS_KMAX) K = SS_KMAX;
  if (K > V) K = V;
  const int KL = greedy ? 1 : K;  // list length published per slice (at most)

  __shared__ int s_hist[HIST];
  __shared__ float ws_v[NW][64];
  __shared__ int ws_i[NW][64];
  __shared__ float sub_v[NW * SS_G][64];
  __shared__ int sub_i[NW * SS_G][64];
  __shared__ float s_tau;
  __shared__ int s_nc;
  __shared__ unsigned s_ticket;
  __shared__ float cval[MAXC];
  __shared__ int cidx[MAXC];
  __shared__ float mv[SS_P * SS_KMAX];  // merger: all lists (the stage-1 ranks reuse it as scratch)
  __shared__ int mi[SS_P * SS_KMAX];
  __shared__ int mn[SS_P];
  __shared__ float sv[SS_KMAX];
  __shared__ int si[SS_KMAX];
  __shared__ int s_choice;

  // ---- repeat penalty of the history ids this slice owns (llama.cpp semantics: once per distinct id)
  const int* hr = hist + (size_t)m * HIST;
  const int ng = n_gen[m];
  const int nrep = (P.repeat_penalty != 1.0f && P.repeat_last_n > 0) ? min(min(P.repeat_last_n, HIST), ng) : 0;
  if (nrep > 0) {
    if (tid < HIST) s_hist[tid] = (tid < nrep) ? hr[(ng - 1 - tid) & (HIST - 1)] : -1;
    __syncthreads();
    if (tid < nrep) {
      const int id = s_hist[tid];
      bool first = id >= v0 && id < v1;
      for (int j = 0; j < tid; ++j) first &= (s_hist[j] != id);
      if (first) {
        const float v = lg[id];
        lg[id] = v > 0.f ? v / P.repeat_penalty : v * P.repeat_penalty;
      }
    }
    __syncthreads();
  }

  // ---- the slice in registers: thread t holds 16-byte chunks t, t + 256, ... (SS_NJ of them, all loads in
  // flight at once -- one memory round trip), every later pass reads registers, not memory
  const int n4 = (v1 - v0) >> 2;  // whole chunks; the < 4-element tail (V % 4, last slice only) runs scalar
  const f32x4* lg4 = reinterpret_cast<const f32x4*>(lg + v0);
  // every load unconditional from a clamped chunk, masked after it returns: a select between a load and a
  // constant makes hipcc branch around each load and wait for it alone (16 dependent round trips; measured
  // 104 us per token this way at one row) -- cdna_hip_programming.md §5 item 4(c)
  f32x4 c[SS_NJ];
  if (n4 > 0) {
#pragma unroll
    for (int j = 0; j < SS_NJ; ++j) c[j] = lg4[min(tid + j * SS_THREADS, n4 - 1)];
  }
#pragma unroll
  for (int j = 0; j < SS_NJ; ++j) {
    const bool in = tid + j * SS_THREADS < n4;
#pragma unroll
    for (int e = 0; e < 4; ++e) c[j][e] = in ? c[j][e] : -INFINITY;
  }
  float tail = -INFINITY;
  const int ti = v0 + (n4 << 2) + tid;
  if (ti < v1) tail = lg[ti];
  auto elem_index = [&](int j, int e) { return v0 + (tid + j * SS_THREADS) * 4 + e; };

  float* my_v = ws.cv + ((size_t)m * SS_P + part) * SS_KMAX;
  int* my_i = ws.ci + ((size_t)m * SS_P + part) * SS_KMAX;
  if (greedy) {
    float bv = tail;
    int bi = ti < v1 ? ti : 0x7fffffff;
#pragma unroll
    for (int j = 0; j < SS_NJ; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (c[j][e] > bv) { bv = c[j][e]; bi = elem_index(j, e); }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(bv, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
    }
    if (lane == 0) { ws_v[wv][0] = bv; ws_i[wv][0] = bi; }
    __syncthreads();
    if (tid == 0) {
      float v = ws_v[0][0];
      int ix = ws_i[0][0];
      for (int w = 1; w < NW; ++w)
        if (ws_v[w][0] > v || (ws_v[w][0] == v && ws_i[w][0] < ix)) { v = ws_v[w][0]; ix = ws_i[w][0]; }
      __hip_atomic_store(my_v, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(my_i, ix, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ws.cn + (size_t)m * SS_P + part, v1 > v0 ? 1 : 0, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
  } else {
    // threshold tau = K-th largest of the SS_G * 256 sub-maxima (each thread's chunks in SS_G groups; ties
    // broken by sub-maximum id, a strict order): K distinct elements are >= tau, so every top-K element of the
    // slice is.  With SS_G = 4 sub-maxima per thread, the elements >= tau stay few even at top_k = 256.
    // Each wave bitonic-sorts each of its SS_G lists of 64 (value desc, id asc); a value's rank is its own
    // position plus a binary search in every other list.
    constexpr int JG = SS_NJ / SS_G;
#pragma unroll
    for (int g = 0; g < SS_G; ++g) {
      float kv = -INFINITY;
#pragma unroll
      for (int j = g * JG; j < (g + 1) * JG; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) kv = fmaxf(kv, c[j][e]);
      if (g == SS_G - 1) kv = fmaxf(kv, tail);
      int ki = tid * SS_G + g;
      for (int k = 2; k <= 64; k <<= 1) {
        for (int jj = k >> 1; jj > 0; jj >>= 1) {
          const float ov = __shfl_xor(kv, jj, 64);
          const int oi = __shfl_xor(ki, jj, 64);
          const bool o_before = (ov > kv) || (ov == kv && oi < ki);
          const bool keep_before = ((lane & jj) == 0) == ((lane & k) == 0);
          if (keep_before ? o_before : !o_before) { kv = ov; ki = oi; }
        }
      }
      sub_v[wv * SS_G + g][lane] = kv;
      sub_i[wv * SS_G + g][lane] = ki;
    }
    if (tid == 0) { s_nc = 0; s_tau = -INFINITY; }
    __syncthreads();
    constexpr int NL = NW * SS_G;  // sorted lists of 64
#pragma unroll
    for (int g = 0; g < SS_G; ++g) {
      const int l = wv * SS_G + g;
      if (lane < K) {
        const float kv = sub_v[l][lane];
        const int ki = sub_i[l][lane];
        int r = lane;
        for (int l2 = 0; l2 < NL; ++l2) {
          if (l2 == l) continue;
          int lo = 0, hi = 64;
          while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            const float xv = sub_v[l2][mid];
            const bool before = (xv > kv) || (xv == kv && sub_i[l2][mid] < ki);
            if (before) lo = mid + 1; else hi = mid;
          }
          r += lo;
          if (r >= K) break;
        }
        if (r == K - 1) s_tau = kv;
      }
    }
    __syncthreads();
    const float tau = s_tau;
    // gather the slice's elements >= tau from registers
#pragma unroll
    for (int j = 0; j < SS_NJ; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (c[j][e] >= tau) {
          const int k = atomicAdd(&s_nc, 1);
          if (k < MAXC) { cval[k] = c[j][e]; cidx[k] = elem_index(j, e); }
        }
    if (ti < v1 && tail >= tau) {
      const int k = atomicAdd(&s_nc, 1);
      if (k < MAXC) { cval[k] = tail; cidx[k] = ti; }
    }
    __syncthreads();
    const int nc = min(s_nc, MAXC);
    const int nl = min(nc, K);
    for (int a = tid; a < nc; a += SS_THREADS) {
      const float va = cval[a];
      const int ia = cidx[a];
      int r = 0;
      for (int b = 0; b < nc; ++b) {
        const float vb = cval[b];
        r += (vb > va) || (vb == va && cidx[b] < ia);
      }
      if (r < nl) {  // publish in rank order (write-through: the merger may sit on another XCD)
        __hip_atomic_store(my_v + r, va, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(my_i + r, ia, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    if (tid == 0) __hip_atomic_store(ws.cn + (size_t)m * SS_P + part, nl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }

  // ---- every storing wave drains, one lane takes the row's ticket; the last slice merges
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) s_ticket = __hip_atomic_fetch_add(ws.ctr + m, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  if (s_ticket != unsigned(SS_P - 1)) return;

  if (tid < SS_P) mn[tid] = __hip_atomic_load(ws.cn + (size_t)m * SS_P + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const float* rv = ws.cv + (size_t)m * SS_P * SS_KMAX;
  const int* ri = ws.ci + (size_t)m * SS_P * SS_KMAX;
  for (int e = tid; e < SS_P * KL; e += SS_THREADS) {
    const int q = e / KL, j = e - q * KL;
    if (j < mn[q]) {
      mv[q * SS_KMAX + j] = __hip_atomic_load(rv + q * SS_KMAX + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      mi[q * SS_KMAX + j] = __hip_atomic_load(ri + q * SS_KMAX + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (tid == 0) ws.ctr[m] = 0u;  // ready for the next launch (launch-ordered)
  __syncthreads();

  int choice;
  if (greedy) {
    if (tid == 0) {
      float v = -INFINITY;
      int ix = 0x7fffffff;
      for (int q = 0; q < SS_P; ++q)
        if (mn[q] > 0 && (mv[q * SS_KMAX] > v || (mv[q * SS_KMAX] == v && mi[q * SS_KMAX] < ix))) {
          v = mv[q * SS_KMAX];
          ix = mi[q * SS_KMAX];
        }
      s_choice = ix;
    }
    __syncthreads();
    choice = s_choice;
  } else {
    // global rank of each listed candidate: its own position + binary search in every other list
    int total = 0;
    for (int q = 0; q < SS_P; ++q) total += mn[q];
    const int n = min(total, K);
    for (int e = tid; e < SS_P * KL; e += SS_THREADS) {
      const int q = e / KL, j = e - q * KL;
      if (j >= mn[q]) continue;
      const float va = mv[q * SS_KMAX + j];
      const int ia = mi[q * SS_KMAX + j];
      int r = j;
      for (int q2 = 0; q2 < SS_P; ++q2) {
        if (q2 == q) continue;
        int lo = 0, hi = mn[q2];
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          const float xv = mv[q2 * SS_KMAX + mid];
          const bool before = (xv > va) || (xv == va && mi[q2 * SS_KMAX + mid] < ia);
          if (before) lo = mid + 1; else hi = mid;
        }
        r += lo;
      }
      if (r < n) { sv[r] = va; si[r] = ia; }
    }
    __syncthreads();
    if (tid == 0) s_choice = draw_topk(sv, si, n, P, ng);
    __syncthreads();
    choice = s_choice;
  }
  if (tid == 0) advance_row(m, choice, ng, P, tok, pos, gen, ldg, n_gen, max_new, done, hist, T_max);
}

// params: device array of M SampleParams (per-row options, so one captured graph
// serves trials with different seeds / temperatures).
CAIN_API int cain_sample(float* logits, int ldl, int V, int* tok, int* pos, int* gen, int ldg, int* n_gen,
                         const int* max_new, int* done, int* hist, const int* slot, int T_max, int M,
                         const void* params, hipStream_t st) {
  hipLaunchKernelGGL(sample_kernel, dim3(M), dim3(SAMPLE_THREADS), 0, st, logits, ldl, V, tok, pos, gen, ldg, n_gen,
                     max_new, done, hist, slot, T_max, reinterpret_cast<const SampleParams*>(params));
  return int(hipGetLastError());
}

// Workspace of the two-stage sampler for M rows (cain_sample_ex); zero-initialised once (the tickets self-reset).
CAIN_API long long cain_sample_ws_bytes(int M) {
  return (long long)M * SS_P * SS_KMAX * 8 + (long long)M * SS_P * 4 + (long long)M * 4 + 256;
}

// Sampler with a workspace: the two-stage kernel (SS_P workgroups per row) for rows <= 64, else the
// one-workgroup kernel.  ws must hold cain_sample_ws_bytes(M) zeroed bytes (null: one-workgroup kernel).
CAIN_API int cain_sample_ex(float* logits, int ldl, int V, int* tok, int* pos, int* gen, int ldg, int* n_gen,
                            const int* max_new, int* done, int* hist, const int* slot, int T_max, int M,
                            const void* params, void* ws, long long ws_bytes, hipStream_t st) {
  if (!ws || M > 64 || ws_bytes < cain_sample_ws_bytes(M) || V < 4 * SS_P ||
      (V + SS_P - 1) / SS_P + 3 > SS_NJ * 4 * SS_THREADS)
    return cain_sample(logits, ldl, V, tok, pos, gen, ldg, n_gen, max_new, done, hist, slot, T_max, M, params, st);
  SampleWs w{};
  char* p = static_cast<char*>(ws);
  w.ctr = reinterpret_cast<unsigned*>(p);  // first: the tickets
  p += ((size_t)M * 4 + 255) / 256 * 256;
  w.cv = reinterpret_cast<float*>(p);
  p += (size_t)M * SS_P * SS_KMAX * 4;
  w.ci = reinterpret_cast<int*>(p);
  p += (size_t)M * SS_P * SS_KMAX * 4;
  w.cn = reinterpret_cast<int*>(p);
  hipLaunchKernelGGL(sample_split_kernel, dim3(M, SS_P), dim3(SS_THREADS), 0, st, logits, ldl, V, tok, pos, gen, ldg,
                     n_gen, max_new, done, hist, slot, T_max, reinterpret_cast<const SampleParams*>(params), w);
  return int(hipGetLastError());
}

CAIN_API int cain_sample_params_size() { return int(sizeof(SampleParams)); }
