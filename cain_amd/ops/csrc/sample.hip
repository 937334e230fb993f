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
    for (int u = 0; u < 4; ++u) {
      const int i4 = base + u * SAMPLE_THREADS;
      c[u] = i4 < V4 ? lg4[i4] : f32x4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
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
      for (int u = 0; u < 4; ++u) {
        const int i4 = base + u * SAMPLE_THREADS;
        c[u] = i4 < V4 ? lg4[i4] : f32x4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
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
    if (tid == 0) {
      const int n = min(nc, K);
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
      // the random stream is keyed by the request's seed and its token index only, not by the batch row: a
      // request that continuous batching moves to another row (ContinuousBatch.retire) keeps its stream, so an
      // Ollama `seed` reproduces the same tokens however the batch is packed (rows without a seed get a unique
      // one on the host, engine._row_options)
      const uint64_t r = mix64(P.seed ^ mix64(uint64_t(ng) * 0x632BE59BD9B4E019ull + 0x9E3779B97F4A7C15ull));
      const float u = float(r >> 40) * (1.0f / 16777216.0f) * zc;
      float c = 0.f;
      int pick = si[cut - 1];
      for (int i = 0; i < cut; ++i) {
        c += __expf(sv[i] * invT - mx);
        if (u < c) { pick = si[i]; break; }
      }
      s_choice = pick;
    }
    __syncthreads();
    choice = s_choice;
  }

  if (tid == 0) {
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

CAIN_API int cain_sample_params_size() { return int(sizeof(SampleParams)); }
