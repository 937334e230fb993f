// Kernel-boundary cost probe: a hipGraph of back-to-back dependent kernels that each read and write B bytes,
// with the stores either plain (write-back L2) or write-through (sc1), and an empty kernel for the floor.
// Prints us per kernel for each variant.  Build: hipcc --offload-arch=gfx950 -O3 tools/boundary_probe.hip -o
// /tmp/boundary_probe ; run: /tmp/boundary_probe [MiB per kernel] [kernels per graph]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int MODE>  // 0 plain stores, 1 write-through (sc1) stores, 2 no memory traffic
__global__ __launch_bounds__(256) void step_kernel(const f32x4* __restrict__ in, f32x4* __restrict__ out, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if constexpr (MODE == 2) return;
  if (i >= n) return;
  f32x4 v = in[i];
  v = v * 1.0001f + 1.f;
  if constexpr (MODE == 0) {
    out[i] = v;
  } else {
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(out, 0, 0x7fffffff, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, i * 16, 0, 16 /* sc1 */);
  }
}

template <int MODE>
static float run(f32x4* a, f32x4* b, int n, int kernels, hipStream_t st) {
  hipGraph_t g;
  hipGraphExec_t ge;
  CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
  for (int k = 0; k < kernels; ++k) {
    f32x4* src = (k & 1) ? b : a;
    f32x4* dst = (k & 1) ? a : b;
    hipLaunchKernelGGL(step_kernel<MODE>, dim3((n + 255) / 256), dim3(256), 0, st, src, dst, n);
  }
  CHECK(hipStreamEndCapture(st, &g));
  CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int w = 0; w < 3; ++w) CHECK(hipGraphLaunch(ge, st));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  CHECK(hipEventRecord(e0, st));
  const int reps = 10;
  for (int r = 0; r < reps; ++r) CHECK(hipGraphLaunch(ge, st));
  CHECK(hipEventRecord(e1, st));
  CHECK(hipEventSynchronize(e1));
  float ms = 0.f;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  CHECK(hipGraphExecDestroy(ge));
  CHECK(hipGraphDestroy(g));
  return ms * 1000.f / (reps * kernels);
}

int main(int argc, char** argv) {
  const double mib = argc > 1 ? atof(argv[1]) : 2.0;
  const int kernels = argc > 2 ? atoi(argv[2]) : 200;
  const int n = int(mib * 1024 * 1024 / 16);
  f32x4 *a, *b;
  CHECK(hipMalloc(&a, (size_t)n * 16));
  CHECK(hipMalloc(&b, (size_t)n * 16));
  CHECK(hipMemset(a, 0, (size_t)n * 16));
  CHECK(hipMemset(b, 0, (size_t)n * 16));
  hipStream_t st;
  CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  const float t_empty = run<2>(a, b, n, kernels, st);
  const float t_plain = run<0>(a, b, n, kernels, st);
  const float t_wt = run<1>(a, b, n, kernels, st);
  printf("{\"MiB\": %.3f, \"kernels\": %d, \"empty_us\": %.2f, \"plain_us\": %.2f, \"write_through_us\": %.2f}\n", mib,
         kernels, t_empty, t_plain, t_wt);
  return 0;
}
