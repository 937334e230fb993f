// RoPE + KV-cache append (SURVEY §2.4 rows "RoPE", "KV-cache append").
//
// Input: the fused QKV projection row qkv[m] = [q (H*hd) | k (Hkv*hd) | v (Hkv*hd)]
// (bias already added by the GEMM epilogue).  Each row m belongs to cache slot
// slot[m] at position pos[m] (decode: one row per live sequence; prefill: one
// row per prompt token), so the same kernel serves both phases.
//
// Rotation: NeoX / HF "rotate_half" convention with a precomputed per-model
// cos/sin table [T_max][hd/2] (Llama-3 frequency scaling baked in on the host,
// cdna_hip_programming.md Appendix B: trig tables on host, not on device).
//
// Cache layouts (per layer):
//   K  [S][Hkv][T_max][hd]   — rows contiguous: the attention kernel's A operand
//                              (K rows, 16 B per lane) reads them directly;
//   Vt [S][Hkv][hd][T_max]   — transposed, so the P·V MFMA's A operand
//                              (V^T rows over t) is contiguous too.
#include "common.h"

__global__ __launch_bounds__(256) void rope_kv_kernel(const __bf16* __restrict__ qkv, int ldqkv,
                                                      const int* __restrict__ slot, const int* __restrict__ pos,
                                                      const float* __restrict__ cos_t, const float* __restrict__ sin_t,
                                                      __bf16* __restrict__ q_out, __bf16* __restrict__ kc,
                                                      __bf16* __restrict__ vtc, int H, int Hkv, int hd, int T_max) {
  const int m = blockIdx.x;
  const int s = slot[m];
  const int p = pos[m];
  if (s < 0) return;  // padded row
  const int half = hd >> 1;
  const __bf16* row = qkv + (size_t)m * ldqkv;
  const float* cr = cos_t + (size_t)p * half;
  const float* sr = sin_t + (size_t)p * half;
  // q and k rotations: (H + Hkv) * half pairs
  const int npairs = (H + Hkv) * half;
  for (int i = threadIdx.x; i < npairs; i += 256) {
    const int h = i / half, j = i - h * half;
    const __bf16* src = row + h * hd;  // k heads follow q heads contiguously
    float x1 = bf2f(src[j]), x2 = bf2f(src[j + half]);
    float c = cr[j], sn = sr[j];
    float y1 = x1 * c - x2 * sn, y2 = x2 * c + x1 * sn;
    if (h < H) {
      __bf16* dst = q_out + (size_t)m * H * hd + h * hd;
      dst[j] = f2bf(y1);
      dst[j + half] = f2bf(y2);
    } else {
      const int kh = h - H;
      __bf16* dst = kc + (((size_t)s * Hkv + kh) * T_max + p) * hd;
      dst[j] = f2bf(y1);
      dst[j + half] = f2bf(y2);
    }
  }
  // v: transposed append
  const __bf16* v = row + (H + Hkv) * hd;
  for (int i = threadIdx.x; i < Hkv * hd; i += 256) {
    const int kh = i / hd, d = i - kh * hd;
    vtc[(((size_t)s * Hkv + kh) * hd + d) * T_max + p] = v[i];
  }
}

CAIN_API int cain_rope_kv(const void* qkv, int ldqkv, const int* slot, const int* pos, const float* cos_t,
                          const float* sin_t, void* q_out, void* kc, void* vtc, int M, int H, int Hkv, int hd,
                          int T_max, hipStream_t st) {
  if (hd % 2) return -1;
  hipLaunchKernelGGL(rope_kv_kernel, dim3(M), dim3(256), 0, st, (const __bf16*)qkv, ldqkv, slot, pos, cos_t, sin_t,
                     (__bf16*)q_out, (__bf16*)kc, (__bf16*)vtc, H, Hkv, hd, T_max);
  return int(hipGetLastError());
}
