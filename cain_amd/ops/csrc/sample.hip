// Token sampling on device (SURVEY §2.4 row "Sampling").
//
// One 1024-thread workgroup per row.  Ollama's default pipeline
// (repeat_penalty over the last `repeat_last_n` tokens -> temperature ->
// top-k -> top-p -> multinomial) or greedy argmax when temperature == 0.
// top-k uses an exact 4-pass radix select (8 bits/pass) on the order-preserving
// uint32 image of the logits, so the vocabulary (32k..256k) is never sorted.
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
  __shared__ uint32_t hcount[256];
  __shared__ uint32_t s_prefix, s_need, s_mask;
  __shared__ float cval[MAXC];
  __shared__ int cidx[MAXC];
  __shared__ int s_nc;
  __shared__ float red_v[SAMPLE_THREADS / 64];
  __shared__ int red_i[SAMPLE_THREADS / 64];
  __shared__ int s_choice;

  // ---- repeat penalty (llama.cpp semantics: once per distinct recent id)
  const int* hr = hist + (size_t)m * HIST;
  const int ng = n_gen[m];
  if (P.repeat_penalty != 1.0f && P.repeat_last_n > 0 && tid == 0) {
    const int n = min(min(P.repeat_last_n, HIST), ng);
    for (int i = 0; i < n; ++i) {
      int id = hr[(ng - 1 - i) & (HIST - 1)];
      bool seen = false;
      for (int j = 0; j < i; ++j) seen |= (hr[(ng - 1 - j) & (HIST - 1)] == id);
      if (seen || id < 0 || id >= V) continue;
      float v = lg[id];
      lg[id] = v > 0.f ? v / P.repeat_penalty : v * P.repeat_penalty;
    }
  }
  __syncthreads();

  int choice;
  if (P.temperature <= 0.f) {
    // ---- greedy argmax (lowest index on ties)
    float bv = -INFINITY;
    int bi = 0x7fffffff;
    for (int i = tid; i < V; i += SAMPLE_THREADS) {
      float v = lg[i];
      if (v > bv || (v == bv && i < bi)) { bv = v; bi = i; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      float ov = __shfl_xor(bv, o, 64);
      int oi = __shfl_xor(bi, o, 64);
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
    if (K <= 0 || K > MAXC) K = MAXC;
    if (K > V) K = V;
    // ---- radix select: threshold = K-th largest ordered key
    if (tid == 0) { s_prefix = 0; s_mask = 0; s_need = K; }
    __syncthreads();
    for (int pass = 0; pass < 4; ++pass) {
      const int shift = 24 - 8 * pass;
      for (int i = tid; i < 256; i += SAMPLE_THREADS) hcount[i] = 0;
      __syncthreads();
      const uint32_t pre = s_prefix, msk = s_mask;
      for (int i = tid; i < V; i += SAMPLE_THREADS) {
        uint32_t u = ord_u32(lg[i]);
        if ((u & msk) == pre) atomicAdd(&hcount[(u >> shift) & 255], 1u);
      }
      __syncthreads();
      if (tid == 0) {
        uint32_t need = s_need, acc = 0;
        int b = 255;
        for (; b > 0; --b) {
          if (acc + hcount[b] >= need) break;
          acc += hcount[b];
        }
        s_need = need - acc;
        s_prefix = pre | (uint32_t(b) << shift);
        s_mask = msk | (255u << shift);
      }
      __syncthreads();
    }
    const uint32_t thr = s_prefix;  // exact key of the K-th largest
    if (tid == 0) s_nc = 0;
    __syncthreads();
    const float invT = 1.0f / P.temperature;
    for (int i = tid; i < V; i += SAMPLE_THREADS) {
      float v = lg[i];
      if (ord_u32(v) >= thr) {
        int c = atomicAdd(&s_nc, 1);
        if (c < MAXC) { cval[c] = v * invT; cidx[c] = i; }
      }
    }
    __syncthreads();
    // rank-sort the candidates descending (value, then index); all threads
    __shared__ float sv[MAXC];
    __shared__ int si[MAXC];
    const int nc = min(s_nc, MAXC);
    for (int a = tid; a < nc; a += SAMPLE_THREADS) {
      const float va = cval[a];
      const int ia = cidx[a];
      int r = 0;
      for (int b = 0; b < nc; ++b) {
        const float vb = cval[b];
        r += (vb > va) || (vb == va && cidx[b] < ia);
      }
      sv[r] = va;
      si[r] = ia;
    }
    __syncthreads();
    if (tid == 0) {
      const int n = min(nc, K);
      const float mx = sv[0];
      float z = 0.f;
      for (int i = 0; i < n; ++i) z += __expf(sv[i] - mx);
      // top-p: smallest prefix with cumulative probability >= top_p
      int cut = n;
      if (P.top_p > 0.f && P.top_p < 1.f) {
        float c = 0.f;
        for (int i = 0; i < n; ++i) {
          c += __expf(sv[i] - mx) / z;
          if (c >= P.top_p) { cut = i + 1; break; }
        }
      }
      float zc = 0.f;
      for (int i = 0; i < cut; ++i) zc += __expf(sv[i] - mx);
      const uint64_t r = mix64(P.seed ^ mix64(uint64_t(m) * 0x632BE59BD9B4E019ull + uint64_t(ng)));
      const float u = float(r >> 40) * (1.0f / 16777216.0f) * zc;
      float c = 0.f;
      int pick = si[cut - 1];
      for (int i = 0; i < cut; ++i) {
        c += __expf(sv[i] - mx);
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
