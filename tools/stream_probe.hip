// Floor of a weight-streaming decode kernel on MI355X, graph-replayed: per-launch cost of an empty kernel, and a
// pure streaming read (no math: each workgroup reads its contiguous slice, 1 KiB per wave instruction, U loads in
// flight per wave, non-temporal) over byte sizes / grid shapes -- what the few-row GEMMs (gemm_w4.hip, gemm.hip)
// can at best reach.  Buffers rotate over 1 GiB so every launch streams from HBM.
// build: hipcc --offload-arch=gfx950 -O3 -o tools/stream_probe tools/stream_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ void empty_kernel(int* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && out[0] == 12345) out[1] = 1;
}

// grid G workgroups of W waves; workgroup b streams chunks c = b, b + G, ... of `chunk` KiB; wave w of it reads the
// KiBs w, w + W, ... of each chunk with U loads in flight
template <int U>
__global__ void stream_kernel(const u32x4* __restrict__ src, long long n_kib, int chunk_kib, unsigned* out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, W = blockDim.x >> 6;
  const long long nchunk = n_kib / chunk_kib;
  uint32_t acc = 0;
  const int per = (chunk_kib + W - 1) / W;
  for (long long c = blockIdx.x; c < nchunk; c += gridDim.x) {
    const u32x4* base = src + (size_t)c * chunk_kib * 64 + lane;
    for (int i0 = 0; i0 < per; i0 += U) {
      u32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = min(wave + (i0 + u) * W, chunk_kib - 1);
        v[u] = __builtin_nontemporal_load(base + (size_t)k * 64);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) acc ^= v[u][0] + v[u][3];
    }
  }
  if (acc == 0x9e3779b9u) out[0] = acc;  // keeps the loads
}

static float graph_us(void (*launch)(void*, int, hipStream_t), void* ctx, int reps, hipStream_t st) {
  hipGraph_t g;
  hipGraphExec_t ex;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < reps; ++i) launch(ctx, i, st);
  CK(hipStreamEndCapture(st, &g));
  CK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(ex, st));
  CK(hipStreamSynchronize(st));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int iters = 5;
  CK(hipEventRecord(a, st));
  for (int i = 0; i < iters; ++i) CK(hipGraphLaunch(ex, st));
  CK(hipEventRecord(b, st));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipGraphExecDestroy(ex));
  CK(hipGraphDestroy(g));
  return ms * 1000.f / (iters * reps);
}

struct Ctx {
  char* buf;
  long long buf_bytes;
  long long bytes;
  int grid, waves, u, chunk_kib;
  unsigned* out;
};

static void launch_empty(void* c, int, hipStream_t st) {
  auto* x = static_cast<Ctx*>(c);
  hipLaunchKernelGGL(empty_kernel, dim3(x->grid), dim3(64 * x->waves), 0, st, (int*)x->out);
}

static void launch_stream(void* c, int i, hipStream_t st) {
  auto* x = static_cast<Ctx*>(c);
  const long long nrot = x->buf_bytes / x->bytes;
  const u32x4* src = reinterpret_cast<const u32x4*>(x->buf + (i % nrot) * x->bytes);
  const long long kib = x->bytes >> 10;
  const dim3 g(x->grid), b(64 * x->waves);
  if (x->u == 2) hipLaunchKernelGGL(stream_kernel<2>, g, b, 0, st, src, kib, x->chunk_kib, x->out);
  else if (x->u == 4) hipLaunchKernelGGL(stream_kernel<4>, g, b, 0, st, src, kib, x->chunk_kib, x->out);
  else hipLaunchKernelGGL(stream_kernel<8>, g, b, 0, st, src, kib, x->chunk_kib, x->out);
}

int main() {
  hipStream_t st;
  CK(hipStreamCreate(&st));
  Ctx c{};
  c.buf_bytes = 1ll << 30;
  CK(hipMalloc(&c.buf, c.buf_bytes));
  CK(hipMemset(c.buf, 1, c.buf_bytes));
  CK(hipMalloc(&c.out, 64));
  CK(hipMemset(c.out, 0, 64));
  for (int grid : {64, 256, 1024}) {
    c.grid = grid, c.waves = 4;
    printf("{\"probe\": \"empty\", \"grid\": %d, \"us\": %.2f}\n", grid, graph_us(launch_empty, &c, 50, st));
  }
  // (MB, chunk KiB): fp4 llama QKV 12.6 MB / O 8.4 / gate-up 58.7 / down 29.4 / LM head 262 with 32-KiB tiles
  for (long long mb : {8, 12, 29, 58, 262}) {
    for (int chunk : {32, 112}) {
      if (chunk == 112 && mb != 29) continue;
      for (int waves : {4, 8}) {
        for (int u : {2, 4, 8}) {
          for (int per_cu : {1, 2, 4}) {
            c.bytes = mb << 20, c.chunk_kib = chunk, c.waves = waves, c.u = u;
            const long long nchunk = (c.bytes >> 10) / chunk;
            c.grid = (int)std::min<long long>(nchunk, 256ll * per_cu);
            const float us = graph_us(launch_stream, &c, 20, st);
            printf("{\"probe\": \"stream\", \"MB\": %lld, \"chunk_kib\": %d, \"waves\": %d, \"u\": %d, \"grid\": %d, "
                   "\"us\": %.2f, \"TBps\": %.2f}\n",
                   mb, chunk, waves, u, c.grid, us, c.bytes / us / 1e6);
            fflush(stdout);
          }
        }
      }
    }
  }
  return 0;
}
