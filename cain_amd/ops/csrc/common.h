// Shared device helpers for the cain_amd gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));
typedef uint16_t u16x4 __attribute__((ext_vector_type(4)));

#define CAIN_API extern "C" __attribute__((visibility("default")))

// CUs the launch sizing of the persistent / CU-proportional grids assumes: the device's, or the smaller budget of
// cain_set_cu_budget (runtime.hip) while the work runs on a CU-masked stream (cain_stream_create_cu_limited).
extern "C" int cain_cu_budget();

__device__ __forceinline__ float bf2f(__bf16 v) { return static_cast<float>(v); }
__device__ __forceinline__ __bf16 f2bf(float v) { return static_cast<__bf16>(v); }  // v_cvt_pk_bf16_f32 (RNE, NaN-safe)

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Epilogue math on the hardware reciprocal / reciprocal square root (v_rcp_f32 / v_rsq_f32, ~1 ulp): hipcc's IEEE
// division and denormal-safe rsqrtf expand to ~10 dependent VALU instructions each, which made the 256-row gate/up
// epilogue (4 SiLU divisions + 1 RMSNorm division per 16 x 16 tile) ~5 us of a ~70 us kernel
// (tools/wgemm_trace.py, profiles/r3/).  Both stay far below bf16 output rounding.
__device__ __forceinline__ float fast_rcp(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ float silu_f(float g) { return g * fast_rcp(1.0f + __expf(-g)); }
__device__ __forceinline__ float gelu_tanh_f(float g) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  float u = k0 * (g + k1 * g * g * g);
  // tanh(u) = 1 - 2/(exp(2u)+1)
  float t = 1.0f - 2.0f * fast_rcp(__expf(2.0f * u) + 1.0f);
  return 0.5f * g * (1.0f + t);
}
// RMSNorm scale of a row from its sum of squares over K elements (ss / K + eps >= eps > 0: never a denormal)
__device__ __forceinline__ float rms_inv(float ss, int K, float eps) {
  return __builtin_amdgcn_rsqf(ss * fast_rcp(float(K)) + eps);
}

static inline int cdiv(int a, int b) { return (a + b - 1) / b; }

// Fragment-major KV cache (attention.hip header): element offset of (position t, head dim d) inside the
// [T_max * hd] block of one (slot, kv head).
__device__ __forceinline__ size_t kfrag_off(int t, int d, int hd) {
  return ((size_t)(t >> 4) * (hd >> 5) + (d >> 5)) * 512 + (size_t)((t & 15) + 16 * ((d & 31) >> 3)) * 8 + (d & 7);
}
__device__ __forceinline__ size_t vfrag_off(int t, int d, int hd) {
  return ((size_t)(t >> 5) * (hd >> 4) + (d >> 4)) * 512 + (size_t)((d & 15) + 16 * ((t & 15) >> 2)) * 8 +
         4 * ((t >> 4) & 1) + (t & 3);
}

// Split-K partial slabs: 16-byte write-through (sc1) buffer stores, read back by the last arriver with
// 16-byte sc1 buffer loads (L2-served, never a stale L1 line): the hand-off needs no release/acquire fence
// (cdna_hip_programming.md Guideline 16 R1; MI355X_MICROARCH.md 'Valid forms', first row).  Dword atomics did
// the same job with four instructions per 16 B.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t slab_rsrc(const float* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), 0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ void st_wt(__amdgpu_buffer_rsrc_t r, int byte_off, const f32x4& v) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, byte_off, 0, 16 /* sc1 */);
}
__device__ __forceinline__ f32x4 ld_wt(__amdgpu_buffer_rsrc_t r, int byte_off) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 16 /* sc1 */));
}

__device__ __forceinline__ void st_wt_f32(__amdgpu_buffer_rsrc_t r, int byte_off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, byte_off, 0, 16 /* sc1 */);
}
__device__ __forceinline__ float ld_wt_f32(__amdgpu_buffer_rsrc_t r, int byte_off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, byte_off, 0, 16 /* sc1 */));
}
