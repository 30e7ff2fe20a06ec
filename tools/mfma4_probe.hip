// Layout + timing probe for v_mfma_f32_4x4x1_16b_f32 on gfx950 (no documentation of the
// multi-block forms in the guides): prints which lane / register each A, B and D element
// of the 16 blocks lives in, and the issue cost of back-to-back 4x4x1 vs 16x16x4 f32 MFMAs.
// Build: hipcc --offload-arch=gfx950 -O3 tools/mfma4_probe.hip -o /tmp/mfma4_probe
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f4v __attribute__((ext_vector_type(4)));

// A = lane-coded values: a(l) = 1 + l (so D = sum over k of a*b identifies contributors)
__global__ void layout_kernel(float* out, int mode) {
  const int l = threadIdx.x;
  f4v c = {0.f, 0.f, 0.f, 0.f};
  // mode 0: A = 1 at lane mode? -> use one-hot probes: A nonzero only at lane pa, B at lane pb
  const int pa = mode & 63, pb = (mode >> 6) & 63;
  const float a = (l == pa) ? 1.f : 0.f;
  const float b = (l == pb) ? 1.f : 0.f;
  c = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) out[l * 4 + r] = c[r];
}

__global__ void time4_kernel(float* out, int iters, long long* cyc) {
  f4v c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0, c2 = c0, c3 = c0;
  float a = threadIdx.x * 1e-3f, b = 1.0001f;
  long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c3, 0, 0, 0);
  }
  long long t1 = clock64();
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
  out[threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3];
}

__global__ void time4dep_kernel(float* out, int iters, long long* cyc) {
  f4v c0 = {0.f, 0.f, 0.f, 0.f};
  float a = threadIdx.x * 1e-3f, b = 1.0001f;
  long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c0, 0, 0, 0);
    c0 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c0, 0, 0, 0);
    c0 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c0, 0, 0, 0);
    c0 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c0, 0, 0, 0);
  }
  long long t1 = clock64();
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
  out[threadIdx.x] = c0[0];
}

__global__ void time16_kernel(float* out, int iters, long long* cyc) {
  f4v c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0, c2 = c0, c3 = c0;
  float a = threadIdx.x * 1e-3f, b = 1.0001f;
  long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c3, 0, 0, 0);
  }
  long long t1 = clock64();
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
  out[threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3];
}

int main() {
  float *d, h[256];
  long long *dc, hc;
  hipMalloc(&d, 256 * sizeof(float));
  hipMalloc(&dc, sizeof(long long));
  // A one-hot at lane pa with B all-ones-probe: find, for each A lane, which (lane, reg) of D
  // it reaches when B is one-hot at lane pb of the same block.
  printf("layout: A one-hot lane pa, B one-hot lane pb -> nonzero D (lane, reg)\n");
  const int probes[][2] = {{0, 0}, {1, 0}, {0, 1}, {2, 3}, {4, 4}, {5, 6}, {17, 18}, {63, 60}, {0, 4}, {3, 2}};
  for (auto& p : probes) {
    layout_kernel<<<1, 64>>>(d, p[0] | (p[1] << 6));
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("  A lane %2d, B lane %2d ->", p[0], p[1]);
    for (int i = 0; i < 256; ++i)
      if (h[i] != 0.f) printf(" (lane %d reg %d = %g)", i / 4, i % 4, h[i]);
    printf("\n");
  }
  const int it = 4096;
  time4_kernel<<<1, 64>>>(d, it, dc);
  hipDeviceSynchronize();
  time4_kernel<<<1, 64>>>(d, it, dc);
  hipMemcpy(&hc, dc, sizeof(hc), hipMemcpyDeviceToHost);
  printf("4x4x1_16b independent x4: %.2f clock64 ticks per MFMA\n", (double)hc / (4.0 * it));
  time4dep_kernel<<<1, 64>>>(d, it, dc);
  hipMemcpy(&hc, dc, sizeof(hc), hipMemcpyDeviceToHost);
  printf("4x4x1_16b dependent chain: %.2f ticks per MFMA\n", (double)hc / (4.0 * it));
  time16_kernel<<<1, 64>>>(d, it, dc);
  hipMemcpy(&hc, dc, sizeof(hc), hipMemcpyDeviceToHost);
  printf("16x16x4 independent x4: %.2f ticks per MFMA\n", (double)hc / (4.0 * it));
  return 0;
}
