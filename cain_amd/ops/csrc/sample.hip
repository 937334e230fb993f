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
#include <cstdlib>

#include "common.h"

struct SampleParams {
  float temperature;
  float top_p;
  float repeat_penalty;
  int top_k;
  int repeat_last_n;
  int eos_id;
  int stop[3];  // further stop ids (a chat model's turn ends: <|eot_id|>, <|end|>, <end_of_turn>, ...); -1 unused
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

// Temperature / top-p / multinomial draw over the n candidates sv[0..n) (sorted: value desc, index asc), by ONE
// wave (every lane of the calling wave calls it; all get the pick): candidate i sits in lane i % 64 of chunk i / 64,
// sums are wave reductions and the top-p cut / the pick are the first lanes whose inclusive prefix sum crosses the
// bound (shuffle scans, ballots) -- no chain of dependent LDS reads.  Both sampler kernels use it, so they draw
// the same token from the same candidates.  The random stream is keyed by the request's seed and its token index
// only, not by the batch row: a request that continuous batching moves to another row (ContinuousBatch.retire)
// keeps its stream, so an Ollama `seed` reproduces the same tokens however the batch is packed (rows without a
// seed get a unique one on the host, engine._row_options).
// Inclusive wave64 prefix sum on DPP row operations (row_shr 1 / 2 / 4 / 8 inside each 16-lane row, then
// row_bcast 15 / 31 carry the row totals): six VALU operations instead of six LDS round trips of __shfl_up.
template <int CTRL, int ROWS>
__device__ __forceinline__ float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, ROWS, 0xf, false));
}
__device__ __forceinline__ float wave_incl_scan(float v) {
  v += dpp_f<0x111, 0xf>(v);
  v += dpp_f<0x112, 0xf>(v);
  v += dpp_f<0x114, 0xf>(v);
  v += dpp_f<0x118, 0xf>(v);
  v += dpp_f<0x142, 0xa>(v);  // row_bcast:15 -> rows 1, 3
  v += dpp_f<0x143, 0xc>(v);  // row_bcast:31 -> rows 2, 3
  return v;
}
__device__ __forceinline__ float lane63(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
}
__device__ __forceinline__ float wave_total(float v) { return lane63(wave_incl_scan(v)); }

__device__ int draw_topk_wave(const float* sv, const int* si, int n, const SampleParams& P, int ng) {
  const int lane = threadIdx.x & 63;
  const float invT = 1.0f / P.temperature;
  const float mx = sv[0] * invT;
  float z = 0.f;
  for (int i = lane; i < n; i += 64) z += __expf(sv[i] * invT - mx);
  z = wave_total(z);
  // top-p: smallest prefix with cumulative probability >= top_p
  int cut = n;
  if (P.top_p > 0.f && P.top_p < 1.f) {
    float carry = 0.f;
    for (int c0 = 0; c0 < n; c0 += 64) {
      const int i = c0 + lane;
      const float pi = i < n ? __expf(sv[i < n ? i : 0] * invT - mx) / z : 0.f;
      const float c = carry + wave_incl_scan(pi);
      const unsigned long long hit = __ballot(i < n && c >= P.top_p);
      if (hit) { cut = c0 + __ffsll((long long)hit); break; }
      carry = lane63(c);
    }
  }
  float zc = 0.f;
  for (int i = lane; i < cut; i += 64) zc += __expf(sv[i] * invT - mx);
  zc = wave_total(zc);
  const uint64_t r = mix64(P.seed ^ mix64(uint64_t(ng) * 0x632BE59BD9B4E019ull + 0x9E3779B97F4A7C15ull));
  const float u = float(r >> 40) * (1.0f / 16777216.0f) * zc;
  int pick = si[cut - 1];
  float carry = 0.f;
  for (int c0 = 0; c0 < cut; c0 += 64) {
    const int i = c0 + lane;
    const float ei = i < cut ? __expf(sv[i < cut ? i : 0] * invT - mx) : 0.f;
    const float c = carry + wave_incl_scan(ei);
    const unsigned long long hit = __ballot(i < cut && u < c);
    if (hit) { pick = si[c0 + __ffsll((long long)hit) - 1]; break; }
    carry = lane63(c);
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
  const bool stop = (P.eos_id >= 0 && choice == P.eos_id) || (P.stop[0] >= 0 && choice == P.stop[0]) ||
                    (P.stop[1] >= 0 && choice == P.stop[1]) || (P.stop[2] >= 0 && choice == P.stop[2]);
  if (stop || n1 >= max_new[m] || p1 >= T_max) {
    done[m] = 1;
  } else {
    pos[m] = p1;
  }
}

// Overflow of the candidate buffer (more than MAXC elements >= tau, possible for top_k >= ~128): the K-th largest
// of the MAXC stored candidates (all >= tau) is a tighter threshold that still keeps every top-K element (the
// row's K-th largest is >= the K-th largest of any subset); the caller re-gathers with it.  Returns the new tau
// through *s_tau (every thread of the workgroup calls it; ends with a barrier).
__device__ void tighten_tau(const float* cval, const int* cidx, int K, int nthreads, float* s_tau) {
  for (int a = threadIdx.x; a < MAXC; a += nthreads) {
    const float va = cval[a];
    const int ia = cidx[a];
    int r = 0;
    for (int b = 0; b < MAXC; ++b) r += (cval[b] > va) || (cval[b] == va && cidx[b] < ia);
    if (r == K - 1) *s_tau = va;
  }
  __syncthreads();
}

typedef int i32x4 __attribute__((ext_vector_type(4)));

// Rank the n candidates cval/cidx[0..n) (value desc, index asc) and write the first K in order to sv / si (every
// thread of the workgroup calls it; ends with a barrier).  The buffers hold n rounded up to 4 (+ 4 spare entries,
// padded here with entries that rank last); each thread compares its candidate against 4 at a time with 16-byte
// LDS reads, unrolled, so the reads pipeline instead of forming a chain.  Returns min(n, K).
__device__ int rank_candidates(float* cval, int* cidx, int n, int K, float* sv, int* si, int nthreads) {
  const int n4 = (n + 3) >> 2;
  if (threadIdx.x < n4 * 4 - n) {
    cval[n + threadIdx.x] = -INFINITY;
    cidx[n + threadIdx.x] = 0x7fffffff;
  }
  __syncthreads();
  const f32x4* cv4 = reinterpret_cast<const f32x4*>(cval);
  const i32x4* ci4 = reinterpret_cast<const i32x4*>(cidx);
  for (int a = threadIdx.x; a < n; a += nthreads) {
    const float va = cval[a];
    const int ia = cidx[a];
    int r = 0;
#pragma unroll 4
    for (int b = 0; b < n4; ++b) {
      const f32x4 v = cv4[b];
      const i32x4 ix = ci4[b];
#pragma unroll
      for (int j = 0; j < 4; ++j) r += (v[j] > va) || (v[j] == va && ix[j] < ia);
    }
    if (r < K) { sv[r] = va; si[r] = ia; }
  }
  __syncthreads();
  return min(n, K);
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
  __shared__ __attribute__((aligned(16))) float cval[MAXC + 4];
  __shared__ __attribute__((aligned(16))) int cidx[MAXC + 4];
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
    for (int u = 0; u < 4; ++u) {  // unconditional loads; chunks past the row re-read chunk tid % V4
      const int i4 = base + u * SAMPLE_THREADS;
      c[u] = lg4[i4 < V4 ? i4 : tid % V4];
    }
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
    __syncthreads();
    // ---- pass 2: gather candidates >= tau (few; LDS atomics only for them); on an overflow of the candidate
    // buffer the threshold is tightened and the row gathered again (tighten_tau)
  #pragma unroll 1
  for (int attempt = 0; attempt < 4; ++attempt) {
    if (tid == 0) s_nc = 0;
    __syncthreads();
    const float tau = s_tau;
    for (int base = tid; base < V4; base += 4 * SAMPLE_THREADS) {
      f32x4 c[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {  // unconditional loads; chunks past the row re-read chunk tid % V4
        const int i4 = base + u * SAMPLE_THREADS;
        c[u] = lg4[i4 < V4 ? i4 : tid % V4];
      }
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
    if (s_nc <= MAXC) break;
    tighten_tau(cval, cidx, K, SAMPLE_THREADS, &s_tau);
    }
    // ---- rank the candidates (value desc, index asc); keep the top K in sorted order
    const int nk = rank_candidates(cval, cidx, min(s_nc, MAXC), K, sv, si, SAMPLE_THREADS);
    if (tid < 64) {
      const int pick = draw_topk_wave(sv, si, nk, P, ng);
      if (tid == 0) s_choice = pick;
    }
    __syncthreads();
    choice = s_choice;
  }

  if (tid == 0) advance_row(m, choice, ng, P, tok, pos, gen, ldg, n_gen, max_new, done, hist, T_max);
}

// =====================================================================================================
// Two-stage sampler for few rows (single-stream decode, continuous batches of a few requests).
//
// The one-workgroup-per-row kernel above streams a row's logits through ONE CU twice: 39-67 us per token at batch
// 1 for 128-256 k vocabularies -- as long as several decode layers of qwen2:1.5b.  Here SS_P workgroups share a
// row.  Each holds 1/SS_P of the vocabulary in registers (one memory round trip), applies the repeat penalty to the
// ids it owns (in registers: the logits stay unmodified) and finds its exact local top-K with the same threshold argument as the one-workgroup kernel, at
// workgroup scale: tau = the K-th largest of its 256 thread maxima (wave bitonic sorts + binary searches) keeps
// every local top-K element, the few elements >= tau (typically K..3K) go to LDS and are ranked there.  The slice
// publishes its sorted list write-through; the LAST arriving workgroup of the row (ticket) gathers the SS_P lists
// above tau_m = the largest K-th entry of any full list (again a lower bound of the row's K-th largest), ranks
// them and runs the same temperature / top-p / draw and decode-state update as the one-workgroup kernel.  The union
// of the local top-K lists holds the global top-K and (value desc, index asc) is a strict order, so both kernels
// draw the same token from the same logits and seed.  (An earlier version found each top-K by K rounds of a
// wave argmax: 105-341 us per token, profiles/r3/.)
// =====================================================================================================
constexpr int SS_THREADS = 256;
constexpr int SS_NW = SS_THREADS / 64;
constexpr int SS_P = 16;      // vocabulary slices (workgroups) per row
constexpr int SS_KMAX = 256;  // top-k clamp, as the one-workgroup kernel
constexpr int SS_NJ = 16;     // 16-byte chunks per thread: a slice holds <= SS_NJ * 4 * SS_THREADS elements

struct SampleWs {  // per row: SS_P sorted candidate lists + their lengths; one ticket counter per row
  float* cv;       // [M][SS_P][SS_KMAX]
  int* ci;         // [M][SS_P][SS_KMAX]
  int* cn;         // [M][SS_P]
  unsigned* ctr;   // [M], zero between launches (the merger resets it)
  // optional [M * SS_P][8] per-workgroup timestamps (s_memrealtime, 10 ns): start, slice loaded, tau, gathered,
  // ranked, ticket, (merger) merged + ranked, end; entry 6 of non-mergers = stage-1 candidate count
  unsigned long long* trace;
};

__device__ __forceinline__ void ss_stamp(const SampleWs& ws, int i) {
  if (ws.trace && threadIdx.x == 0)
    ws.trace[((size_t)blockIdx.x * SS_P + blockIdx.y) * 8 + i] = __builtin_amdgcn_s_memrealtime();
}

__device__ __forceinline__ bool ss_before(float av, int ai, float bv, int bi) {
  return av > bv || (av == bv && ai < bi);
}

// The K-th largest (value desc, index asc) of the workgroup's SS_THREADS keys (bv, bi), all distinct in that order;
// every thread calls it, the value lands in *s_tau (ends with a barrier).  Each wave bitonic-sorts its 64 keys in
// registers; a key's rank is its lane plus, per other wave, a 6-step binary search in that wave's sorted list.
__device__ void ss_kth(float bv, int bi, int K, float (*ws_v)[64], int (*ws_i)[64], float* s_tau) {
  static_assert(sizeof(float) * 64 % 16 == 0, "16-byte rows");
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float kv = bv;
  int ki = bi;
  for (int k = 2; k <= 64; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      const float ov = __shfl_xor(kv, j, 64);
      const int oi = __shfl_xor(ki, j, 64);
      const bool o_before = ss_before(ov, oi, kv, ki);
      const bool keep_before = ((lane & j) == 0) == ((lane & k) == 0);
      if (keep_before ? o_before : !o_before) { kv = ov; ki = oi; }
    }
  }
  ws_v[wv][lane] = kv;
  ws_i[wv][lane] = ki;
  __syncthreads();
  // a key's rank in another wave's sorted list by counting (16-byte LDS reads, all independent) rather than a
  // binary search (a chain of dependent reads)
  if (wv * 64 < SS_THREADS && K > 0) {
    int r = lane;
    const f32x4* v4 = reinterpret_cast<const f32x4*>(&ws_v[0][0]);
    const i32x4* i4 = reinterpret_cast<const i32x4*>(&ws_i[0][0]);
    for (int w2 = 0; w2 < SS_NW; ++w2) {
      if (w2 == wv) continue;
#pragma unroll
      for (int b = 0; b < 16; ++b) {
        const f32x4 v = v4[w2 * 16 + b];
        const i32x4 ix = i4[w2 * 16 + b];
#pragma unroll
        for (int j = 0; j < 4; ++j) r += ss_before(v[j], ix[j], kv, ki) ? 1 : 0;
      }
    }
    if (r == K - 1) *s_tau = kv;
  }
  __syncthreads();
}


// Append the elements e[k] (ids eid(k)) with keep(k) to cval / cidx: per wave one LDS atomic for the wave's base,
// lanes' offsets from a wave prefix sum of their counts (no per-element atomics), and no per-element branch: an
// element that is not kept (or past MAXC) is written to the lane's own trash slot cval / cidx[MAXC + 4 + lane]
// (unrolled per-element branches cost an exec-mask save each and spilled the kernel's SGPRs).  Every thread calls
// it; ends with a barrier; *s_nc = the total (may exceed MAXC: the caller tightens and gathers again).
template <int NE, class Keep, class Id>
__device__ void gather_candidates(const float (&e)[NE], Keep keep, Id eid, float* cval, int* cidx, int* s_nc) {
  const int lane = threadIdx.x & 63;
  // the keep flags as a per-lane bit mask in VGPRs (boolean lane masks would live in SGPR pairs between the two
  // loops: 65 of them spilled)
  constexpr int NW32 = (NE + 31) / 32;
  uint32_t km[NW32];
#pragma unroll
  for (int w = 0; w < NW32; ++w) km[w] = 0u;
#pragma unroll
  for (int k = 0; k < NE; ++k) km[k >> 5] |= (keep(k) ? 1u : 0u) << (k & 31);
  int cnt = 0;
#pragma unroll
  for (int w = 0; w < NW32; ++w) cnt += __builtin_popcount(km[w]);
  // inclusive wave scan of cnt
  int inc = cnt;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(inc, o, 64);
    if (lane >= o) inc += t;
  }
  const int tot = __shfl(inc, 63, 64);
  int base = 0;
  if (lane == 63 && tot > 0) base = atomicAdd(s_nc, tot);
  base = __shfl(base, 63, 64) + inc - cnt;
  const int trash = MAXC + 4 + lane;
#pragma unroll
  for (int k = 0; k < NE; ++k) {
    const int kk = (km[k >> 5] >> (k & 31)) & 1;
    const int dst = (kk && base < MAXC) ? base : trash;
    cval[dst] = e[k];
    cidx[dst] = eid(k);
    base += kk;
  }
  __syncthreads();
}

// Bitonic sort of one key per lane across the calling wave, (value desc, index asc): lane l ends with the l-th.
__device__ __forceinline__ void wave_sort_desc(float& kv, int& ki) {
  const int lane = threadIdx.x & 63;
  for (int k = 2; k <= 64; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      const float ov = __shfl_xor(kv, j, 64);
      const int oi = __shfl_xor(ki, j, 64);
      const bool o_before = ss_before(ov, oi, kv, ki);
      const bool keep_before = ((lane & j) == 0) == ((lane & k) == 0);
      if (keep_before ? o_before : !o_before) { kv = ov; ki = oi; }
    }
  }
}

__global__ __launch_bounds__(SS_THREADS) void sample_split_kernel(
    const float* __restrict__ logits, int ldl, int V, int* __restrict__ tok, int* __restrict__ pos,
    int* __restrict__ gen, int ldg, int* __restrict__ n_gen, const int* __restrict__ max_new,
    int* __restrict__ done, int* __restrict__ hist, const int* __restrict__ slot, int T_max,
    const SampleParams* __restrict__ params, const SampleWs ws) {
  const int m = blockIdx.x, part = blockIdx.y;
  if (slot[m] < 0 || done[m]) return;  // the same for every workgroup of the row: no ticket is taken
  const SampleParams P = params[m];
  const float* lg = logits + (size_t)m * ldl;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  ss_stamp(ws, 0);
  // this workgroup's slice [v0, v1) of the vocabulary (16-byte aligned starts)
  const int chunk = (((V + SS_P - 1) / SS_P) + 3) & ~3;
  const int v0 = min(V, part * chunk), v1 = min(V, v0 + chunk);
  const bool greedy = P.temperature <= 0.f;
  int K = P.top_k;
  if (K <= 0 || K > SS_KMAX) K = SS_KMAX;
  if (K > V) K = V;
  const int KL = greedy ? 1 : K;  // list length a slice publishes (at most)

  __shared__ __attribute__((aligned(16))) float ws_v[SS_NW][64];
  __shared__ __attribute__((aligned(16))) int ws_i[SS_NW][64];
  __shared__ __attribute__((aligned(16))) int s_hist[HIST];
  __shared__ __attribute__((aligned(16))) float cval[MAXC + 4 + 64];  // + 4: rank padding, + 64: trash slots
  __shared__ __attribute__((aligned(16))) int cidx[MAXC + 4 + 64];
  __shared__ float sv[SS_KMAX];
  __shared__ int si[SS_KMAX];
  __shared__ float s_tau;
  __shared__ int s_nc;
  __shared__ unsigned s_ticket;
  __shared__ int mn[SS_P];

  // ---- the slice in registers, requested first: thread t holds 16-byte chunks t, t + 256, ... (one memory round
  // trip).  Every load is unconditional, masked after it returns (a select between a load and a constant makes
  // hipcc branch around each load and wait for it alone, cdna_hip_programming.md §5 item 4(c)); chunks past the
  // slice re-read chunk tid % n4, spread over the slice.  Element (j, q) of thread t is id v0 + 4 (t + 256 j) + q;
  // slot SS_NJ * 4 is the < 4-element tail (last slice only).
  const int n4 = (v1 - v0) >> 2;
  const f32x4* lg4 = reinterpret_cast<const f32x4*>(lg + v0);
  float e[SS_NJ * 4 + 1];
  {
    const int spare = n4 > 0 ? tid % n4 : 0;
#pragma unroll
    for (int j = 0; j < SS_NJ; ++j) {
      const int i4 = tid + j * SS_THREADS;
      const f32x4 c = lg4[i4 < n4 ? i4 : spare];  // n4 == 0: a slice of < 4 elements, chunk 0 is in the row
#pragma unroll
      for (int q = 0; q < 4; ++q) e[4 * j + q] = i4 < n4 ? c[q] : -INFINITY;
    }
  }
  const int ti = v0 + (n4 << 2) + tid;
  e[SS_NJ * 4] = ti < v1 ? lg[ti < V ? ti : tid] : -INFINITY;
  auto eid = [&](int k) { return k < SS_NJ * 4 ? v0 + 4 * (tid + (k >> 2) * SS_THREADS) + (k & 3) : ti; };

  // ---- repeat penalty (llama.cpp semantics: each distinct recent id once), applied to the CANDIDATES: it only
  // lowers values, so with R = #history ids, at least K of the top K + R raw elements keep their value and the
  // (K + R)-th largest raw thread maximum is a lower bound of the penalised K-th largest; gathering raw >= that
  // bound keeps every penalised top-K element.  The history ids go to LDS while the slice is in flight.
  const int ng = n_gen[m];
  const int nrep = (P.repeat_penalty != 1.0f && P.repeat_last_n > 0) ? min(min(P.repeat_last_n, HIST), ng) : 0;
  int rs = 0;  // history ids in this slice (with repeats: an upper bound of the distinct ones)
  if (tid < HIST) {
    const int id = tid < nrep ? hist[(size_t)m * HIST + ((ng - 1 - tid) & (HIST - 1))] : -1;
    s_hist[tid] = id;
    rs = __popcll(__ballot(id >= v0 && id < v1));
  }
  if (tid < 64 && tid == 0) s_nc = rs;  // handed to every wave through LDS (s_nc is reset before its own use)

  // ---- thread max (lowest id on ties: ids grow with k); an empty thread gets a unique sentinel id
  float bv = -INFINITY;
  int bk = -1;
#pragma unroll
  for (int k = 0; k < SS_NJ * 4 + 1; ++k)
    if (e[k] > bv) { bv = e[k]; bk = k; }
  const int bi = bk >= 0 ? eid(bk) : 0x7fffff00 + tid;
  ss_stamp(ws, 1);

  // ---- tau: K-th largest thread max; gather the elements >= tau, rank them; on an overflow of the candidate
  // buffer tighten tau (tighten_tau) and gather again from the registers
  if (tid == 0) s_tau = -INFINITY;
  __syncthreads();
  const int KB = KL + s_nc;  // > SS_THREADS: no bound from the thread maxima (tau = -inf, tightened on overflow)
  ss_kth(bv, bi, KB <= SS_THREADS ? KB : 0, ws_v, ws_i, &s_tau);
  ss_stamp(ws, 2);
#pragma unroll 1
  for (int attempt = 0; attempt < 4; ++attempt) {
    if (tid == 0) s_nc = 0;
    __syncthreads();
    const float tau = s_tau;
    gather_candidates(e, [&](int k) { return e[k] >= tau && e[k] > -INFINITY; }, eid, cval, cidx, &s_nc);
    if (s_nc <= MAXC) break;
    tighten_tau(cval, cidx, min(KB, MAXC), SS_THREADS, &s_tau);  // raw values: the (K + R)-th is the bound
  }
  ss_stamp(ws, 3);
  if (ws.trace && tid == 0) ws.trace[((size_t)m * SS_P + part) * 8 + 6] = (unsigned long long)s_nc;
  const int nc1 = min(s_nc, MAXC);
  if (nrep > 0) {  // penalise the candidates whose id is in the history (16-byte LDS reads of the id list)
    const i32x4* h4 = reinterpret_cast<const i32x4*>(s_hist);
    for (int a = tid; a < nc1; a += SS_THREADS) {
      const int id = cidx[a];
      bool hit = false;
#pragma unroll
      for (int h = 0; h < HIST / 4; ++h) {
        const i32x4 hv = h4[h];
        hit |= (hv[0] == id) | (hv[1] == id) | (hv[2] == id) | (hv[3] == id);
      }
      if (hit) {
        const float v = cval[a];
        cval[a] = v > 0.f ? v / P.repeat_penalty : v * P.repeat_penalty;
      }
    }
    __syncthreads();
  }
  const int nl = rank_candidates(cval, cidx, nc1, KL, sv, si, SS_THREADS);
  ss_stamp(ws, 4);

  // ---- publish the sorted list (write-through: the merger may sit on another XCD), drain, take the row's ticket
  float* my_v = ws.cv + ((size_t)m * SS_P + part) * SS_KMAX;
  int* my_i = ws.ci + ((size_t)m * SS_P + part) * SS_KMAX;
  if (tid < nl) {
    __hip_atomic_store(my_v + tid, sv[tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(my_i + tid, si[tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (tid == 0) __hip_atomic_store(ws.cn + (size_t)m * SS_P + part, nl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) s_ticket = __hip_atomic_fetch_add(ws.ctr + m, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  ss_stamp(ws, 5);
  if (s_ticket != unsigned(SS_P - 1)) return;

  // ---- merger.  tau_m, a lower bound of the row's K-th largest: for K <= 64 the K-th largest of the SS_P lists'
  // first 64 / SS_P entries (64 actual elements: wave 0 sorts them), else the largest K-th entry of a full list.
  // Everything from the lists is read with sc1 loads (published write-through by other workgroups).
  const float* rv = ws.cv + (size_t)m * SS_P * SS_KMAX;
  const int* ri = ws.ci + (size_t)m * SS_P * SS_KMAX;
  if (wv == 0) {
    constexpr int HEADS = 64 / SS_P;
    const int q = lane / HEADS, r = lane - q * HEADS;
    const int n = __hip_atomic_load(ws.cn + (size_t)m * SS_P + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int rr = KL <= 64 ? r : KL - 1;  // K > 64: each list's K-th entry
    float hv = __hip_atomic_load(rv + q * SS_KMAX + rr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int hi = __hip_atomic_load(ri + q * SS_KMAX + rr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (r == 0) mn[q] = n;
    if (KL <= 64) {
      if (rr >= n) { hv = -INFINITY; hi = 0x7fffff00 + lane; }
      wave_sort_desc(hv, hi);
      const float t = __shfl(hv, KL - 1, 64);  // -inf when fewer than K heads exist: gather everything
      if (lane == 0) s_tau = t;
    } else {
      float t = (r == 0 && n >= KL) ? hv : -INFINITY;
      t = wave_max(t);
      if (lane == 0) s_tau = t;
    }
  }
  if (tid == 0) ws.ctr[m] = 0u;  // ready for the next launch (launch-ordered)
  __syncthreads();
  // list q = tid / 16 (SS_THREADS / SS_P threads per list), ranks r = tid % 16 + 16 u: no division
  static_assert(SS_THREADS / SS_P == 16 && SS_KMAX / 16 == 16, "merger slot mapping");
  constexpr int MS = SS_KMAX / 16;
  const int mq = tid >> 4, mr0 = tid & 15;
  const int nq = min(mn[mq], KL);
  const int nu = (KL + 15) >> 4;  // uniform
  float x[MS];
  int xi[MS];
#pragma unroll
  for (int u = 0; u < MS; ++u) {  // unconditional loads from clamped offsets; masked afterwards
    x[u] = -INFINITY, xi[u] = 0x7fffffff;
    if (u < nu) {
      const int r = mr0 + 16 * u;
      const int off = mq * SS_KMAX + min(r, max(nq - 1, 0));
      const float v = __hip_atomic_load(rv + off, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      xi[u] = __hip_atomic_load(ri + off, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      x[u] = r < nq ? v : -INFINITY;
    }
  }
#pragma unroll 1
  for (int attempt = 0; attempt < 4; ++attempt) {
    if (tid == 0) s_nc = 0;
    __syncthreads();
    const float tau = s_tau;
    gather_candidates(x, [&](int u) { return x[u] >= tau && x[u] > -INFINITY; }, [&](int u) { return xi[u]; }, cval,
                      cidx, &s_nc);
    if (s_nc <= MAXC) break;
    tighten_tau(cval, cidx, KL, SS_THREADS, &s_tau);
  }
  const int n = rank_candidates(cval, cidx, min(s_nc, MAXC), KL, sv, si, SS_THREADS);
  ss_stamp(ws, 6);
  if (tid < 64) {
    const int choice = greedy ? si[0] : draw_topk_wave(sv, si, n, P, ng);
    if (tid == 0) advance_row(m, choice, ng, P, tok, pos, gen, ldg, n_gen, max_new, done, hist, T_max);
  }
  ss_stamp(ws, 7);
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

static unsigned long long* g_sample_trace = nullptr;
// Timestamps of the next two-stage sampler launches ([M * 16][8] int64, SampleWs::trace; null: off).  Tools only.
CAIN_API void cain_sample_set_trace(void* p) { g_sample_trace = static_cast<unsigned long long*>(p); }

// Workspace of the two-stage sampler for M rows (cain_sample_ex); zero-initialised once (the tickets self-reset).
CAIN_API long long cain_sample_ws_bytes(int M) {
  return (long long)M * SS_P * SS_KMAX * 8 + (long long)M * SS_P * 4 + (long long)M * 4 + 256;
}

// Rows up to which the two-stage kernel runs (64; the decode plan sizes its workspace for min(rows, this)).  At
// 256 rows it measured slower than the one-workgroup-per-row kernel (profiles/r3/README.md).
static int g_split_max = 64;
CAIN_API int cain_sample_split_max() { return g_split_max; }
CAIN_API void cain_sample_set_split_max(int rows) { g_split_max = rows; }

// Sampler with a workspace: the two-stage kernel (SS_P workgroups per row) for rows <= cain_sample_split_max(),
// else the one-workgroup kernel.  ws must hold cain_sample_ws_bytes(M) zeroed bytes (null: one-workgroup kernel).
CAIN_API int cain_sample_ex(float* logits, int ldl, int V, int* tok, int* pos, int* gen, int ldg, int* n_gen,
                            const int* max_new, int* done, int* hist, const int* slot, int T_max, int M,
                            const void* params, void* ws, long long ws_bytes, hipStream_t st) {
  if (!ws || M > cain_sample_split_max() || ws_bytes < cain_sample_ws_bytes(M) || V < 4 * SS_P ||
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
  w.trace = g_sample_trace;
  hipLaunchKernelGGL(sample_split_kernel, dim3(M, SS_P), dim3(SS_THREADS), 0, st, logits, ldl, V, tok, pos, gen, ldg,
                     n_gen, max_new, done, hist, slot, T_max, reinterpret_cast<const SampleParams*>(params), w);
  return int(hipGetLastError());
}

// =====================================================================================================
// Chunk-maximum sampler for few rows (the single-stream decode): the LM head's skinny kernel also writes every
// row's maximum over each 16-column chunk of the vocabulary (gemm.hip, GemmArgs::cmax), so the sampler's first
// stage reads V / 16 chunk maxima instead of V logits.  One 256-thread workgroup per row:
//   1. repeat penalty in place on the logits (as sample_kernel: once per distinct recent id);
//   2. tau_c = the (K + R)-th largest of the 256 thread maxima of the chunk maxima (R = the penalised ids): at
//      least K + R distinct logits are >= tau_c, at least K of them unpenalised, so the penalised row's K-th largest
//      is >= tau_c, and every top-K logit lies in a chunk whose (unpenalised) maximum is >= tau_c -- for a penalty
//      >= 1, which only lowers logits; the penalised ids whose chunks were not gathered are added as candidates
//      themselves, which covers a penalty < 1;
//   3. the logits of the gathered chunks (typically ~K + R chunks of 16) are the candidate set, reduced with the
//      same threshold argument to the elements >= the K-th largest thread maximum, ranked (value desc, index asc)
//      and drawn by draw_topk_wave -- the same candidates in the same order as the other two kernels, so the same
//      token for the same seed.  Greedy (temperature 0): K = 1, the lowest index on ties, as sample_kernel.
// Overflows of the candidate buffers (more than MAXC chunks or elements above a threshold) tighten it
// (tighten_tau), as in the other kernels.
// =====================================================================================================
constexpr int CM_NJ = 64;  // chunk maxima (then candidate logits) per thread: V / 16 <= 64 * 256 chunks
constexpr int CM_MAPW = CM_NJ * SS_THREADS / 32;  // words of the gathered-chunk bitmap

__global__ __launch_bounds__(SS_THREADS) void sample_cm_kernel(
    float* __restrict__ logits, int ldl, int V, const float* __restrict__ cmax, int* __restrict__ tok,
    int* __restrict__ pos, int* __restrict__ gen, int ldg, int* __restrict__ n_gen, const int* __restrict__ max_new,
    int* __restrict__ done, int* __restrict__ hist, const int* __restrict__ slot, int T_max,
    const SampleParams* __restrict__ params) {
  const int m = blockIdx.x;
  if (slot[m] < 0 || done[m]) return;
  const SampleParams P = params[m];
  float* lg = logits + (size_t)m * ldl;
  const int C = V >> 4;
  const float* cm = cmax + (size_t)m * C;
  const int tid = threadIdx.x;
  __shared__ int s_hist[HIST];
  __shared__ float ws_v[SS_NW][64];
  __shared__ int ws_i[SS_NW][64];
  __shared__ float s_tau;
  __shared__ float sv[SS_KMAX];
  __shared__ int si[SS_KMAX];
  __shared__ __attribute__((aligned(16))) float cval[MAXC + 68];
  __shared__ __attribute__((aligned(16))) int cidx[MAXC + 68];
  __shared__ int s_ch[MAXC];
  __shared__ unsigned s_map[CM_MAPW];
  __shared__ int s_nc;
  __shared__ int s_choice;

  // ---- 1. repeat penalty, in place
  const int* hr = hist + (size_t)m * HIST;
  const int ng = n_gen[m];
  const int nrep = (P.repeat_penalty != 1.0f && P.repeat_last_n > 0) ? min(min(P.repeat_last_n, HIST), ng) : 0;
  if (tid < HIST) s_hist[tid] = (tid < nrep) ? hr[(ng - 1 - tid) & (HIST - 1)] : -1;
  __syncthreads();
  bool first = false;  // this thread's history id is the first occurrence of a valid id
  if (tid < nrep) {
    const int id = s_hist[tid];
    first = id >= 0 && id < V;
    for (int j = 0; j < tid; ++j) first &= (s_hist[j] != id);
    if (first) {
      const float v = lg[id];
      lg[id] = v > 0.f ? v / P.repeat_penalty : v * P.repeat_penalty;
    }
  }
  __syncthreads();

  int K = P.top_k;
  if (K <= 0 || K > SS_KMAX) K = SS_KMAX;
  if (K > V) K = V;
  if (P.temperature <= 0.f) K = 1;
  const int R = nrep;

  // ---- 2. chunk maxima: thread tid holds chunks 4 (tid + 256 j) .. + 3 (16-byte loads); threshold tau_c, then the
  // chunks >= tau_c
  float cv[CM_NJ];
  float bv = -INFINITY;
  int bi = 0x7fffffff - tid;  // distinct keys for threads without chunks
  auto cid = [&](int k) { return 4 * (tid + (k >> 2) * SS_THREADS) + (k & 3); };
  const f32x4* cm4 = reinterpret_cast<const f32x4*>(cm);
#pragma unroll
  for (int j = 0; j < CM_NJ / 4; ++j) {
    const int c4 = tid + j * SS_THREADS;
    const f32x4 v = 4 * c4 < C ? cm4[c4] : f32x4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      cv[4 * j + i] = v[i];
      if (v[i] > bv) bv = v[i], bi = 4 * c4 + i;
    }
  }
  const int Kc = K + R;
  if (Kc <= SS_THREADS) {
    ss_kth(bv, bi, Kc, ws_v, ws_i, &s_tau);
  } else {
    if (tid == 0) s_tau = -INFINITY;
    __syncthreads();
  }
  int n_ch = 0;
#pragma unroll 1
  for (int attempt = 0; attempt < 4; ++attempt) {
    if (tid == 0) s_nc = 0;
    __syncthreads();
    const float tau = s_tau;
    gather_candidates(
        cv, [&](int k) { return cid(k) < C && cv[k] >= tau; }, cid, cval, cidx, &s_nc);
    n_ch = min(s_nc, MAXC);
    if (s_nc <= MAXC) break;
    tighten_tau(cval, cidx, Kc, SS_THREADS, &s_tau);
  }
  // the gathered chunk ids, and a bitmap of them (the penalised ids' membership test)
  for (int w = tid; w < CM_MAPW; w += SS_THREADS) s_map[w] = 0u;
  __syncthreads();
  for (int k = tid; k < n_ch; k += SS_THREADS) {
    const int ch = cidx[k];
    s_ch[k] = ch;
    atomicOr(&s_map[ch >> 5], 1u << (ch & 31));
  }
  __syncthreads();

  // ---- 3. candidate logits: the gathered chunks' 16 each (chunk slot tid + 256 j: four 16-byte loads), plus the
  // penalised ids outside them
  float ev[CM_NJ + 1];
  int eidv[CM_NJ + 1];  // vocabulary ids (distinct placeholders past the candidates)
#pragma unroll
  for (int j = 0; j < CM_NJ / 16; ++j) {
    const int k = tid + j * SS_THREADS;
    const int ch = k < n_ch ? s_ch[k] : 0;
    const f32x4* src = reinterpret_cast<const f32x4*>(lg + (size_t)ch * 16);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4 v = src[q];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int e = 16 * j + 4 * q + i;
        ev[e] = k < n_ch ? v[i] : -INFINITY;
        eidv[e] = k < n_ch ? ch * 16 + 4 * q + i : 0x7ffff000 - (k * 16 + 4 * q + i);
      }
    }
  }
  int xid = -1;
  if (first) {
    const int id = s_hist[tid], ch = id >> 4;
    if (!((s_map[ch >> 5] >> (ch & 31)) & 1u)) xid = id;
  }
  ev[CM_NJ] = xid >= 0 ? lg[xid] : -INFINITY;
  eidv[CM_NJ] = xid >= 0 ? xid : 0x7fffffff - tid;
  float bv2 = -INFINITY;
  int bi2 = 0x7fffffff - tid;
#pragma unroll
  for (int k = 0; k <= CM_NJ; ++k) {
    if (ev[k] > bv2 || (ev[k] == bv2 && eidv[k] < bi2)) bv2 = ev[k], bi2 = eidv[k];
  }
  ss_kth(bv2, bi2, K, ws_v, ws_i, &s_tau);
  int nc = 0;
#pragma unroll 1
  for (int attempt = 0; attempt < 4; ++attempt) {
    if (tid == 0) s_nc = 0;
    __syncthreads();
    const float tau = s_tau;
    gather_candidates(
        ev, [&](int k) { return ev[k] >= tau && ev[k] > -INFINITY; }, [&](int k) { return eidv[k]; }, cval, cidx,
        &s_nc);
    nc = min(s_nc, MAXC);
    if (s_nc <= MAXC) break;
    tighten_tau(cval, cidx, K, SS_THREADS, &s_tau);
  }
  const int nk = rank_candidates(cval, cidx, nc, K, sv, si, SS_THREADS);
  if (tid < 64) {
    const int pick = (P.temperature <= 0.f) ? si[0] : draw_topk_wave(sv, si, nk, P, ng);
    if (tid == 0) s_choice = pick;
  }
  __syncthreads();
  if (tid == 0) advance_row(m, s_choice, ng, P, tok, pos, gen, ldg, n_gen, max_new, done, hist, T_max);
}

// The chunk-maximum sampler (V % 64 == 0, V / 16 <= 64 * 256); cmax as the LM head wrote it (cain_gemm_set_cmax).
// cain_sample_set_cm: 0 off, 1 this kernel on every forward whose LM head wrote the maxima, 2 this kernel only on
// forwards of more than 64 rows, 3 the lean kernel below on every forward whose LM head wrote them (the default).
// They draw the same tokens; at one row this kernel's one-workgroup chain of phases (37.4 us on qwen2:1.5b,
// profiles/r3/README.md) is longer than the two-stage kernel's 16-way split (29 us); at 256 rows it takes 42 us
// against the one-workgroup-per-row kernel's 62 us (+0.2-0.3 % in-graph on the headline).
static int g_sample_cm = 3;  // the lean kernel wherever the LM head wrote the maxima (cain_sample_lean, below)
CAIN_API int cain_sample_cm_enabled() { return g_sample_cm; }
// A/B switch for tests and tools (takes effect at the next forward / graph capture).
CAIN_API void cain_sample_set_cm(int on) { g_sample_cm = on; }
CAIN_API int cain_sample_cm(float* logits, int ldl, int V, const float* cmax, int* tok, int* pos, int* gen, int ldg,
                            int* n_gen, const int* max_new, int* done, int* hist, const int* slot, int T_max, int M,
                            const void* params, hipStream_t st) {
  if (!cmax || V % 64 || V / 16 > CM_NJ * SS_THREADS) return -1;  // whole 16-byte chunk-max loads
  hipLaunchKernelGGL(sample_cm_kernel, dim3(M), dim3(SS_THREADS), 0, st, logits, ldl, V, cmax, tok, pos, gen, ldg,
                     n_gen, max_new, done, hist, slot, T_max, reinterpret_cast<const SampleParams*>(params));
  return int(hipGetLastError());
}

CAIN_API int cain_sample_params_size() { return int(sizeof(SampleParams)); }


// =====================================================================================================
// Lean chunk-maximum sampler (the few-row sampler at <= 12 us).  Same inputs as sample_cm_kernel
// -- the logits and the LM head's chunk maxima (gemm_epi.h epi_cmax, written by every few-row LM-head kernel: bf16,
// fp8, MXFP4 and GGUF Q4) -- and the same candidates in the same order, so the same token for the same seed.
//
// The two-stage kernel's 29 us (profiles/r3/sampler_trace_final.log) and a first 256-thread version of this one
// (31 us; profiles/r6/sampler/) were chains of workgroup-wide phases whose cost is what each wave issues on the
// critical path: a wave64 VALU instruction takes 4 cycles, a shuffle is an LDS round trip (ds_bpermute), a rank
// pass over 128 values by one wave ~3 us.  Here 1,024 threads each hold at most 16 chunk maxima, reductions and
// scans are DPP row operations, and every rank count is split over up to 16 threads of a DPP row:
//   1. every independent load first (chunk maxima, the 64 history slots, row state, options).  The repeat penalty
//      (llama.cpp semantics: each distinct recent id once) marks the recent ids in an LDS bitmap of ids and one of
//      chunks (one atomicOr each: the first setter of an id is its distinct occurrence);
//   2. tau_c = a LOWER BOUND of the K-th largest post-penalty logit: the chunks holding no recent id have exact
//      maxima, so with the other chunks masked to -inf, G = 64 / 128 / 256 groups (G >= 2K up to K = 128) of
//      consecutive threads take their maximum (DPP row_shr), and the K-th largest group maximum (ln_bound: each
//      group's rank counted by 16 / R threads) has K distinct unpenalised logits >= it;
//   3. every chunk whose (pre-penalty) maximum is >= tau_c -- the penalty only lowers an unpenalised logit's chunk
//      mates, never the logit, so every unpenalised top-K logit lies in one -- gathered by one LDS atomic per thread
//      that has any (ln_gather), and their 16 logits loaded, 16-byte quads, two per thread;
//   4. the unpenalised logits >= tau_c of those chunks plus the distinct recent ids' penalised logits >= tau_c
//      (loaded by the history lanes in step 1, off the critical path) gathered, ranked (value desc, index asc; ln_rank)
//      and drawn (draw_topk_wave), the decode state advanced.
// A threshold that lets more than LN_CAP chunks or MAXC elements through is tightened to the exact K-th (value,
// index) pair of the gathered set (ln_tighten) and the gather repeated: exact in every case, ties included.  The
// logits are not modified (the penalty lives in registers).
// =====================================================================================================
constexpr int LN_THREADS = 1024;
constexpr int LN_NJ = 16;                     // chunk maxima per thread
constexpr int LN_C_MAX = LN_NJ * LN_THREADS;  // chunks per row: V <= 262,144
// chunks whose logits are loaded (4 quads each: two quads per thread): K <= 256 chunks without recent ids plus the
// <= 64 chunks with some
constexpr int LN_CAP = 512;
constexpr int LN_QT = LN_CAP * 4 / LN_THREADS;  // quads per thread
static_assert(LN_CAP >= SS_KMAX + HIST && LN_CAP <= MAXC, "staging capacity");

// Running max / sum over groups of GS consecutive lanes of each 16-lane DPP row (row_shr, lanes past the row start
// read the identity): the lane with (lane % GS) == GS - 1 ends with its group's total.
template <int CTRL>
__device__ __forceinline__ int dpp_i(int old, int v) {
  return __builtin_amdgcn_update_dpp(old, v, CTRL, 0xf, 0xf, false);
}
template <int GS>
__device__ __forceinline__ float group_max(float x) {
  const int ninf = __builtin_bit_cast(int, -INFINITY);
  if constexpr (GS >= 2) x = fmaxf(x, __builtin_bit_cast(float, dpp_i<0x111>(ninf, __builtin_bit_cast(int, x))));
  if constexpr (GS >= 4) x = fmaxf(x, __builtin_bit_cast(float, dpp_i<0x112>(ninf, __builtin_bit_cast(int, x))));
  if constexpr (GS >= 8) x = fmaxf(x, __builtin_bit_cast(float, dpp_i<0x114>(ninf, __builtin_bit_cast(int, x))));
  if constexpr (GS >= 16) x = fmaxf(x, __builtin_bit_cast(float, dpp_i<0x118>(ninf, __builtin_bit_cast(int, x))));
  return x;
}
template <int GS>
__device__ __forceinline__ int group_sum(int x) {
  if constexpr (GS >= 2) x += dpp_i<0x111>(0, x);
  if constexpr (GS >= 4) x += dpp_i<0x112>(0, x);
  if constexpr (GS >= 8) x += dpp_i<0x114>(0, x);
  if constexpr (GS >= 16) x += dpp_i<0x118>(0, x);
  return x;
}

// Lower bound of the K-th largest (1 <= K <= 64 R) row element behind the per-thread values tv (each an element of the
// row, or -inf): 64 R groups of GS = 16 / R consecutive threads take their maximum; group a's rank among the group
// maxima (value desc, group asc) is counted by the GS threads of group a over R^2 16-byte reads each and summed in
// the row; the group of rank K - 1 writes its maximum.  K distinct row elements are >= it.  Every thread calls it
// (R uniform); ends with a barrier.
template <int R>
__device__ float ln_bound_r(float tv, int K, float* s_g, float* s_tau) {
  constexpr int GS = 16 / R;
  const int tid = threadIdx.x, lane = tid & 63;
  tv = group_max<GS>(tv);
  const int a = tid / GS, p = tid % GS;
  if (p == GS - 1) s_g[a] = tv;
  __syncthreads();
  const float ga = s_g[a];  // (only lane GS - 1 of the group held the whole maximum)
  const f32x4* g4 = reinterpret_cast<const f32x4*>(s_g);
  int r = 0;
#pragma unroll
  for (int i = 0; i < R * R; ++i) {
    const int q = p + GS * i;
    const f32x4 v = g4[q];
#pragma unroll
    for (int j = 0; j < 4; ++j) r += (v[j] > ga) || (v[j] == ga && 4 * q + j < a);
  }
  r = group_sum<GS>(r);  // complete in lane GS - 1
  if (p == GS - 1 && r == K - 1) *s_tau = ga;  // ranks are a permutation of [0, G): one writer
  (void)lane;
  __syncthreads();
  return *s_tau;
}

// R for a bound of the K-th largest: G = 64 R >= 2 K up to K = 128 (uniform across the workgroup)
__device__ __forceinline__ float ln_bound(float tv, int K, float* s_g, float* s_tau) {
  if (K <= 32) return ln_bound_r<1>(tv, K, s_g, s_tau);
  if (K <= 64) return ln_bound_r<2>(tv, K, s_g, s_tau);
  return ln_bound_r<4>(tv, K, s_g, s_tau);
}

// Append this thread's kept items (bit k of keep) as (val(k), id(k)): one LDS atomic per thread that has any, then
// a loop over its set bits.  The list is in arrival order (ln_rank orders it); entries past MAXC are dropped, *s_nc
// counts them all.  The caller zeroes *s_nc before a barrier; ends with a barrier.
template <class Val, class Id>
__device__ void ln_gather(uint32_t keep, Val val, Id id, float* cval, int* cidx, int* s_nc) {
  const int cnt = __popc(keep);
  int base = cnt ? atomicAdd(s_nc, cnt) : 0;
  while (keep) {
    const int k = __builtin_ctz(keep);
    keep &= keep - 1;
    if (base < MAXC) {
      cval[base] = val(k);
      cidx[base] = id(k);
    }
    ++base;
  }
  __syncthreads();
}

// ln_gather for items held in a register array: the loop over the set bits is unrolled over the array (a dynamic
// register index would go through scratch memory).
template <int NE, class Id>
__device__ void ln_gather_regs(uint32_t keep, const float (&v)[NE], Id id, float* cval, int* cidx, int* s_nc) {
  const int cnt = __popc(keep);
  int base = cnt ? atomicAdd(s_nc, cnt) : 0;
#pragma unroll
  for (int k = 0; k < NE; ++k) {
    if ((keep >> k) & 1u) {
      if (base < MAXC) {
        cval[base] = v[k];
        cidx[base] = id(k);
      }
      ++base;
    }
  }
  __syncthreads();
}

// The exact K-th (value desc, id asc) of the n <= MAXC stored entries -> (*s_tv, *s_ti): a threshold pair every
// top-K item passes (the stored entries are a subset of the items above the previous threshold).  Ends with a barrier.
__device__ void ln_tighten(const float* cval, const int* cidx, int n, int K, float* s_tv, int* s_ti) {
  for (int a = threadIdx.x; a < n; a += LN_THREADS) {
    const float va = cval[a];
    const int ia = cidx[a];
    int r = 0;
    for (int b = 0; b < n; ++b) r += (cval[b] > va) || (cval[b] == va && cidx[b] < ia);
    if (r == K - 1) *s_tv = va, *s_ti = ia;
  }
  __syncthreads();
}

// Rank the n <= MAXC candidates (value desc, index asc) and write the first K in order to sv / si, TPC threads of a
// DPP row per candidate (each counts every TPC-th 16-byte group, the row sums).  Returns min(n, K); ends with a barrier.
template <int TPC>
__device__ void ln_rank_t(const float* cval, const int* cidx, int n, int K, float* sv, int* si) {
  const int tid = threadIdx.x, n4 = (n + 3) >> 2;
  const f32x4* cv4 = reinterpret_cast<const f32x4*>(cval);
  const i32x4* ci4 = reinterpret_cast<const i32x4*>(cidx);
  for (int a0 = 0; a0 < n; a0 += LN_THREADS / TPC) {
    const int a = a0 + tid / TPC, p = tid % TPC;
    const int ac = min(a, n - 1);
    const float va = cval[ac];
    const int ia = cidx[ac];
    int r = 0;
    for (int q = p; q < n4; q += TPC) {
      const f32x4 v = cv4[q];
      const i32x4 ix = ci4[q];
#pragma unroll
      for (int j = 0; j < 4; ++j) r += (v[j] > va) || (v[j] == va && ix[j] < ia);
    }
    r = group_sum<TPC>(r);
    if (a < n && p == TPC - 1 && r < K) {
      sv[r] = va;
      si[r] = ia;
    }
  }
  __syncthreads();
}

__device__ int ln_rank(float* cval, int* cidx, int n, int K, float* sv, int* si) {
  const int n4 = (n + 3) >> 2;
  if ((int)threadIdx.x < n4 * 4 - n) {  // pad to whole 16-byte groups with entries that rank last
    cval[n + threadIdx.x] = -INFINITY;
    cidx[n + threadIdx.x] = 0x7fffffff;
  }
  __syncthreads();
  if (n <= 64) ln_rank_t<16>(cval, cidx, n, K, sv, si);
  else if (n <= 128) ln_rank_t<8>(cval, cidx, n, K, sv, si);
  else if (n <= 256) ln_rank_t<4>(cval, cidx, n, K, sv, si);
  else if (n <= 512) ln_rank_t<2>(cval, cidx, n, K, sv, si);
  else ln_rank_t<1>(cval, cidx, n, K, sv, si);
  return min(n, K);
}

typedef uint32_t ln_u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(LN_THREADS) void sample_lean_kernel(
    const float* __restrict__ logits, int ldl, int V, const float* __restrict__ cmax, int* __restrict__ tok,
    int* __restrict__ pos, int* __restrict__ gen, int ldg, int* __restrict__ n_gen, const int* __restrict__ max_new,
    int* __restrict__ done, int* __restrict__ hist, const int* __restrict__ slot, int T_max,
    const SampleParams* __restrict__ params, unsigned long long* __restrict__ trace) {
  const int m = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  auto stamp = [&](int i) {
    if (trace && tid == 0) trace[(size_t)m * 8 + i] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  // ---- 1. every load that depends on no other first: the chunk maxima (thread t: chunks 4 (t + 1024 j) .. + 3;
  // unconditional clamped loads, masked after), the 64 history slots (wave 0), the row's state and options
  const int C = V >> 4, C4 = C >> 2;
  const f32x4* cm4 = reinterpret_cast<const f32x4*>(cmax + (size_t)m * C);
  f32x4 cq[LN_NJ / 4];
#pragma unroll
  for (int j = 0; j < LN_NJ / 4; ++j) cq[j] = cm4[min(tid + j * LN_THREADS, C4 - 1)];
  const int hslot = tid < HIST ? hist[(size_t)m * HIST + tid] : -1;
  const int sl = slot[m], dn = done[m], ng = n_gen[m];
  const SampleParams P = params[m];
  if (sl < 0 || dn) return;
  const float* lg = logits + (size_t)m * ldl;
  extern __shared__ __attribute__((aligned(16))) float ln_smem[];
  float* s_cm = ln_smem;                                           // [C] chunk maxima (the tightening's values)
  uint32_t* s_bm = reinterpret_cast<uint32_t*>(ln_smem + C4 * 4);  // [V / 32] recent ids, then [C / 32] their chunks
  const int bm_words = (((V + 127) >> 7) << 2);
  uint32_t* s_cbm = s_bm + bm_words;
  __shared__ float s_g[256];
  __shared__ float sv[SS_KMAX];
  __shared__ int si[SS_KMAX];
  __shared__ __attribute__((aligned(16))) float cval[MAXC + 4];
  __shared__ __attribute__((aligned(16))) int cidx[MAXC + 4];
  __shared__ float s_tau, s_tv;
  __shared__ int s_ti, s_nc, s_choice;

  const int nrep = (P.repeat_penalty != 1.0f && P.repeat_last_n > 0) ? min(min(P.repeat_last_n, HIST), ng) : 0;
  f32x4* s_cm4 = reinterpret_cast<f32x4*>(s_cm);
#pragma unroll
  for (int j = 0; j < LN_NJ / 4; ++j)
    if (tid + j * LN_THREADS < C4) s_cm4[tid + j * LN_THREADS] = cq[j];
  // history slot s holds a recent id iff it is one of the last nrep written: (ng - 1 - s) mod 64 < nrep
  int hid = (tid < HIST && ((ng - 1 - tid) & (HIST - 1)) < nrep) ? hslot : -1;
  if (hid >= V) hid = -1;
  float hv = 0.f;  // the recent id's logit (history lanes; needed in step 4 only)
  bool hfirst = false;
  float cv[LN_NJ];  // this thread's chunk maxima; the bound sees the penalised chunks' as -inf
  float bv = -INFINITY;
  if (nrep > 0) {  // (uniform)
    if (tid < HIST) hv = lg[hid >= 0 ? hid : 0];
    ln_u32x4* bm4 = reinterpret_cast<ln_u32x4*>(s_bm);
    const int nz4 = (bm_words + ((C + 127) >> 7 << 2)) >> 2;
    for (int w = tid; w < nz4; w += LN_THREADS) bm4[w] = ln_u32x4{0u, 0u, 0u, 0u};
    __syncthreads();
    if (hid >= 0) {
      const uint32_t bit = 1u << (hid & 31);
      hfirst = !(atomicOr(&s_bm[hid >> 5], bit) & bit);
      const int ch = hid >> 4;
      atomicOr(&s_cbm[ch >> 5], 1u << (ch & 31));
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < LN_NJ / 4; ++j) {
      const int c0 = 4 * (tid + j * LN_THREADS);  // 4 consecutive chunks: 4 bits of one word
      const uint32_t pb = c0 < C ? (s_cbm[c0 >> 5] >> (c0 & 31)) & 0xfu : 0u;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        cv[4 * j + i] = tid + j * LN_THREADS < C4 ? cq[j][i] : -INFINITY;
        bv = fmaxf(bv, (pb >> i) & 1u ? -INFINITY : cv[4 * j + i]);
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < LN_NJ / 4; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        cv[4 * j + i] = tid + j * LN_THREADS < C4 ? cq[j][i] : -INFINITY;
        bv = fmaxf(bv, cv[4 * j + i]);
      }
  }
  stamp(1);

  int K = P.top_k;
  if (K <= 0 || K > SS_KMAX) K = SS_KMAX;
  if (K > V) K = V;
  if (P.temperature <= 0.f) K = 1;

  // ---- 2. tau_c
  float tv = ln_bound(bv, K, s_g, &s_tau);
  int ti = 0x7fffffff;
  stamp(2);

  // ---- 3. the chunks whose maximum is >= tau_c
  auto cid = [&](int k) { return 4 * (tid + (k >> 2) * LN_THREADS) + (k & 3); };
  // (a tightening ranks the gathered chunks without recent ids: their maxima are post-penalty logits)
  auto cval_of = [&](int k) {
    const int c = cid(k);
    return nrep > 0 && ((s_cbm[c >> 5] >> (c & 31)) & 1u) ? -INFINITY : s_cm[c];
  };
  int n_ch = 0;
#pragma unroll 1
  for (int attempt = 0; attempt < 4; ++attempt) {
    if (tid == 0) s_nc = 0, s_tv = tv, s_ti = ti;  // (kept if a tightening finds no K-th)
    __syncthreads();
    uint32_t keep = 0;
#pragma unroll
    for (int k = 0; k < LN_NJ; ++k) {
      const bool in = cv[k] > tv || (cv[k] == tv && cid(k) <= ti);
      keep |= uint32_t(in && cv[k] > -INFINITY) << k;
    }
    ln_gather(keep, cval_of, cid, cval, cidx, &s_nc);
    n_ch = s_nc;
    if (n_ch <= LN_CAP) break;
    ln_tighten(cval, cidx, min(n_ch, MAXC), K, &s_tv, &s_ti);
    tv = s_tv, ti = s_ti;
  }
  n_ch = min(n_ch, LN_CAP);
  stamp(3);
  // their logits: quad tid of chunk entry tid >> 2 (chunk ids read from cidx before the next gather's first
  // barrier; without any chunk, chunk 0 is loaded and masked); the recent ids among them are masked out (their
  // penalised values come from the history lanes)
  const int nq = n_ch * 4;
  constexpr int NE = 4 * LN_QT + 1;
  float ev[NE];
  int eb[LN_QT];
  f32x4 lq[LN_QT];
#pragma unroll
  for (int u = 0; u < LN_QT; ++u) {  // quad tid + 1024 u of chunk entry (tid + 1024 u) >> 2
    const int q = tid + u * LN_THREADS;
    const int ch = nq > 0 ? cidx[min(q, nq - 1) >> 2] : 0;
    lq[u] = reinterpret_cast<const f32x4*>(lg + (size_t)ch * 16)[q & 3];
    eb[u] = ch * 16 + (q & 3) * 4;
  }
#pragma unroll
  for (int u = 0; u < LN_QT; ++u) {
    const bool qin = tid + u * LN_THREADS < nq;
    const uint32_t pen4 = nrep > 0 ? (s_bm[eb[u] >> 5] >> (eb[u] & 31)) & 0xfu : 0u;
#pragma unroll
    for (int i = 0; i < 4; ++i) ev[4 * u + i] = qin && !((pen4 >> i) & 1u) ? lq[u][i] : -INFINITY;
  }
  // the last item: the distinct recent id's penalised logit (history lanes)
  ev[NE - 1] = hfirst ? (hv > 0.f ? hv / P.repeat_penalty : hv * P.repeat_penalty) : -INFINITY;
  auto eid = [&](int k) { return k < NE - 1 ? eb[k >> 2] + (k & 3) : hid; };  // (k constant after unrolling)
  stamp(4);

  // ---- 4. the elements >= tau_c (with a tightened chunk pair (tau_c, c_K): value tau_c up to c_K's last id)
  ti = ti == 0x7fffffff ? ti : ti * 16 + 15;
  int nc = 0;
#pragma unroll 1
  for (int attempt = 0; attempt < 4; ++attempt) {
    if (tid == 0) s_nc = 0, s_tv = tv, s_ti = ti;
    __syncthreads();
    uint32_t keep = 0;
#pragma unroll
    for (int i = 0; i < NE; ++i) {
      const bool in = ev[i] > tv || (ev[i] == tv && eid(i) <= ti);
      keep |= uint32_t(in && ev[i] > -INFINITY) << i;
    }
    ln_gather_regs(keep, ev, eid, cval, cidx, &s_nc);
    nc = s_nc;
    if (nc <= MAXC) break;
    ln_tighten(cval, cidx, MAXC, K, &s_tv, &s_ti);
    tv = s_tv, ti = s_ti;
  }
  nc = min(nc, MAXC);
  stamp(5);
  const int nk = ln_rank(cval, cidx, nc, K, sv, si);
  stamp(6);
  if (tid < 64) {
    const int pick = nk == 0 ? 0 : (P.temperature <= 0.f ? si[0] : draw_topk_wave(sv, si, nk, P, ng));
    if (lane == 0) s_choice = pick;
  }
  __syncthreads();
  if (tid == 0) advance_row(m, s_choice, ng, P, tok, pos, gen, ldg, n_gen, max_new, done, hist, T_max);
  stamp(7);
}

static size_t ln_lds_bytes(int V) {
  const size_t C = (size_t)V >> 4;
  return C * sizeof(float) + (size_t)((V + 127) >> 7) * 16 + (size_t)((C + 127) >> 7) * 16;
}

// The lean chunk-maximum sampler (V % 64 == 0, V / 16 <= LN_C_MAX); cmax as the LM head wrote it.  < 0: refused.
// The trace (cain_sample_set_trace) takes [M][8] timestamps: start, penalty marked, tau_c, chunks gathered, logits
// loaded, elements gathered, ranked, end.
CAIN_API int cain_sample_lean(float* logits, int ldl, int V, const float* cmax, int* tok, int* pos, int* gen, int ldg,
                              int* n_gen, const int* max_new, int* done, int* hist, const int* slot, int T_max, int M,
                              const void* params, hipStream_t st) {
  if (!cmax || V % 64 || V / 16 > LN_C_MAX) return -1;
  static const bool attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&sample_lean_kernel),
                                               hipFuncAttributeMaxDynamicSharedMemorySize,
                                               int(ln_lds_bytes(LN_C_MAX * 16))) == hipSuccess;
  if (!attr) return -1;
  hipLaunchKernelGGL(sample_lean_kernel, dim3(M), dim3(LN_THREADS), ln_lds_bytes(V), st, logits, ldl, V, cmax, tok,
                     pos, gen, ldg, n_gen, max_new, done, hist, slot, T_max,
                     reinterpret_cast<const SampleParams*>(params), g_sample_trace);
  return int(hipGetLastError());
}
