// Layout + issue-cost probe of the f32-input multi-block MFMA forms on gfx950:
// v_mfma_f32_4x4x1_16b_f32 and v_mfma_f32_16x16x1_4b_f32 (not described in the guides).
// For every A lane (B = 1 everywhere) prints the D (lane, reg) slots it reaches, and for
// every B lane (A = 1) likewise; then the back-to-back issue cost with 1 and 2 waves per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 tools/mfma_probe2.hip -o tools/mfma_probe2.bin
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f4v __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));

__global__ void lay4(float* out, int pa, int pb) {
  const int l = threadIdx.x;
  const float a = (pa < 0 || l == pa) ? 1.f : 0.f;
  const float b = (pb < 0 || l == pb) ? 1.f : 0.f;
  f4v c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) out[l * 16 + r] = c[r];
}
__global__ void lay16(float* out, int pa, int pb) {
  const int l = threadIdx.x;
  const float a = (pa < 0 || l == pa) ? 1.f : 0.f;
  const float b = (pb < 0 || l == pb) ? 1.f : 0.f;
  f16v c = {};
  c = __builtin_amdgcn_mfma_f32_16x16x1f32(a, b, c, 0, 0, 0);
  for (int r = 0; r < 16; ++r) out[l * 16 + r] = c[r];
}

template <int KIND>
__global__ void timek(float* out, int iters, long long* cyc) {
  float a = threadIdx.x * 1e-3f, b = 1.0001f;
  long long t0 = clock64();
  float acc = 0.f;
  if constexpr (KIND == 0) {
    f4v c0 = {}, c1 = {}, c2 = {}, c3 = {};
    for (int i = 0; i < iters; ++i) {
      c0 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c3, 0, 0, 0);
    }
    acc = c0[0] + c1[1] + c2[2] + c3[3];
  } else if constexpr (KIND == 1) {
    f4v c0 = {};
    for (int i = 0; i < iters; ++i) {
      c0 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c0, 0, 0, 0);
      c0 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c0, 0, 0, 0);
      c0 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c0, 0, 0, 0);
      c0 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c0, 0, 0, 0);
    }
    acc = c0[0];
  } else if constexpr (KIND == 2) {
    f4v c0 = {}, c1 = {}, c2 = {}, c3 = {};
    for (int i = 0; i < iters; ++i) {
      c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c3, 0, 0, 0);
    }
    acc = c0[0] + c1[1] + c2[2] + c3[3];
  } else if constexpr (KIND == 3) {
    f16v c0 = {}, c1 = {};
    for (int i = 0; i < iters; ++i) {
      c0 = __builtin_amdgcn_mfma_f32_16x16x1f32(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x1f32(a, b, c1, 0, 0, 0);
      c0 = __builtin_amdgcn_mfma_f32_16x16x1f32(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x1f32(a, b, c1, 0, 0, 0);
    }
    acc = c0[0] + c1[1];
  } else if constexpr (KIND == 4) {
    // 4x4x1 with 4 independent accumulators + 4 v_exp per 4 MFMAs (softmax-like filler)
    f4v c0 = {}, c1 = {}, c2 = {}, c3 = {};
    float e = a;
    for (int i = 0; i < iters; ++i) {
      c0 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c0, 0, 0, 0);
      e = __builtin_amdgcn_exp2f(e) * 0.5f;
      c1 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c3, 0, 0, 0);
    }
    acc = c0[0] + c1[1] + c2[2] + c3[3] + e;
  }
  long long t1 = clock64();
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
  out[threadIdx.x] = acc;
}

static void dump(const char* tag, const float* h, int regs) {
  printf("%s:", tag);
  for (int l = 0; l < 64; ++l)
    for (int r = 0; r < regs; ++r)
      if (h[l * 16 + r] != 0.f) printf(" %d.%d", l, r);
  printf("\n");
}

int main() {
  float *d, h[64 * 16];
  long long *dc, hc[8];
  hipMalloc(&d, sizeof(h));
  hipMalloc(&dc, sizeof(hc));
  const int probes[] = {0, 1, 2, 3, 4, 5, 15, 16, 17, 31, 32, 48, 63};
  for (int p : probes) {
    char tag[64];
    hipMemset(d, 0, sizeof(h));
    lay4<<<1, 64>>>(d, p, -1);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    snprintf(tag, 64, "4x4x1 A lane %d -> D lane.reg", p);
    dump(tag, h, 4);
    hipMemset(d, 0, sizeof(h));
    lay4<<<1, 64>>>(d, -1, p);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    snprintf(tag, 64, "4x4x1 B lane %d -> D lane.reg", p);
    dump(tag, h, 4);
  }
  for (int p : probes) {
    char tag[64];
    hipMemset(d, 0, sizeof(h));
    lay16<<<1, 64>>>(d, p, -1);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    snprintf(tag, 64, "16x16x1 A lane %d -> D lane.reg", p);
    dump(tag, h, 16);
    hipMemset(d, 0, sizeof(h));
    lay16<<<1, 64>>>(d, -1, p);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    snprintf(tag, 64, "16x16x1 B lane %d -> D lane.reg", p);
    dump(tag, h, 16);
  }
  const int it = 4096;
  const char* names[] = {"4x4x1_16b indep x4", "4x4x1_16b dep chain", "16x16x4 indep x4", "16x16x1_4b indep x2",
                         "4x4x1_16b indep x4 + 1 exp"};
  for (int waves = 1; waves <= 4; waves *= 2) {
    for (int k = 0; k < 5; ++k) {
      auto go = [&]() {
        switch (k) {
          case 0: timek<0><<<1, 64 * waves * 4>>>(d, it, dc); break;
          case 1: timek<1><<<1, 64 * waves * 4>>>(d, it, dc); break;
          case 2: timek<2><<<1, 64 * waves * 4>>>(d, it, dc); break;
          case 3: timek<3><<<1, 64 * waves * 4>>>(d, it, dc); break;
          default: timek<4><<<1, 64 * waves * 4>>>(d, it, dc); break;
        }
      };
      go();
      hipDeviceSynchronize();
      go();
      hipMemcpy(hc, dc, sizeof(long long), hipMemcpyDeviceToHost);
      printf("%d wave(s)/SIMD  %-28s %.2f clock ticks per MFMA per wave\n", waves, names[k], (double)hc[0] / (4.0 * it));
    }
  }
  return 0;
}
