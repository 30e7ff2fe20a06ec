// Chip-wide f32 MFMA throughput (wall time, hipEvent): 256 x k workgroups of 64*w threads,
// every wave issuing `iters` x 4 independent v_mfma_f32_16x16x4_f32 (or 4x4x1_16b).
// Build: hipcc --offload-arch=gfx950 -O3 tools/mfma_rate.hip -o tools/mfma_rate.bin
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f4v __attribute__((ext_vector_type(4)));

template <int KIND>
__global__ void rate_kernel(float* out, int iters) {
  float a = threadIdx.x * 1e-3f, b = 1.0001f;
  f4v c0 = {}, c1 = {}, c2 = {}, c3 = {};
  float v0 = a, v1 = a + 1.f, v2 = a + 2.f, v3 = a + 3.f, v4 = a + 4.f, v5 = a + 5.f, v6 = a + 6.f, v7 = a + 7.f;
  for (int i = 0; i < iters; ++i) {
    if constexpr (KIND >= 2) {  // 16 independent VALU FMAs per 4 MFMAs (KIND 2: with MFMA, 3: VALU only)
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        v0 = fmaf(v0, b, a); v1 = fmaf(v1, b, a); v2 = fmaf(v2, b, a); v3 = fmaf(v3, b, a);
        v4 = fmaf(v4, b, a); v5 = fmaf(v5, b, a); v6 = fmaf(v6, b, a); v7 = fmaf(v7, b, a);
      }
      asm volatile("" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7));
    }
    if constexpr (KIND == 3) continue;
    if constexpr (KIND == 0 || KIND == 2) {
      c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c3, 0, 0, 0);
    } else {
      c0 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c3, 0, 0, 0);
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3] + v0 + v1 + v2 + v3 + v4 + v5 + v6 + v7;
}

int main() {
  float* d;
  hipMalloc(&d, 256 * 4 * 1024 * sizeof(float));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 4096;
  for (int kind = 0; kind < 4; ++kind)
    for (int w : {4, 8, 16}) {
      for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(e0);
        if (kind == 0)
          rate_kernel<0><<<256, 64 * w>>>(d, iters);
        else if (kind == 1)
          rate_kernel<1><<<256, 64 * w>>>(d, iters);
        else if (kind == 2)
          rate_kernel<2><<<256, 64 * w>>>(d, iters);
        else
          rate_kernel<3><<<256, 64 * w>>>(d, iters);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
      }
      float ms = 0.f;
      hipEventElapsedTime(&ms, e0, e1);
      const double mfmas = 256.0 * w * iters * 4.0;
      const double flop_per = kind == 0 ? 2048.0 : 512.0;
      const char* nm[4] = {"16x16x4_f32        ", "4x4x1_16b_f32      ", "16x16x4 + 16 v_fma ", "16 v_fma only      "};
      printf("%s waves/CU %2d (%d/SIMD): %.3f ms, %.1f TFLOP/s (MFMA part), %.2f ns per 4-MFMA group per SIMD\n",
             nm[kind], w, w / 4, ms, kind == 3 ? 0.0 : mfmas * flop_per / (ms * 1e-3) / 1e12,
             4.0 * ms * 1e6 / (mfmas / 1024.0));
    }
  return 0;
}
