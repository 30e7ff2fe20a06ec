// Shared helpers for the hydragnn_amd gfx950 (CDNA4) kernels.
//
// Conventions used by every kernel in this directory:
//  * wave64: lane = threadIdx.x & 63; blocks are multiples of 64 threads.
//  * graphs are CSR-by-destination: edges sorted by dst, rowptr[N+1] (int32).
//    A second "by-source" view (src_rowptr, src_perm) gives atomic-free,
//    deterministic reductions onto source nodes (backward of gathers).
//  * feature rows are contiguous fp32 (row stride == F unless stated),
//    vectorised as float4 when F % 4 == 0.
#pragma once

#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>
#include <torch/library.h>

#define HY_CHECK(cond, ...) TORCH_CHECK(cond, "hydragnn_amd: ", __VA_ARGS__)
#define HY_CHECK_CUDA(t) HY_CHECK((t).is_cuda(), #t " must be a GPU tensor")
#define HY_CHECK_CONTIG(t) HY_CHECK((t).is_contiguous(), #t " must be contiguous")
#define HY_CHECK_F32(t) HY_CHECK((t).scalar_type() == at::kFloat, #t " must be float32")
#define HY_CHECK_I32(t) HY_CHECK((t).scalar_type() == at::kInt, #t " must be int32")

namespace hy {

inline hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

inline int ceil_div(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

// compute units of the current device (cached per device; persistent-grid sizing)
inline int num_cus() {
  static int cached[64] = {0};
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev < 0 || dev >= 64) dev = 0;
  if (cached[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cached[dev] = n;
  }
  return cached[dev];
}

constexpr int kWave = 64;

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

__device__ __forceinline__ float4 f4add(float4 a, float4 b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}
__device__ __forceinline__ float4 f4mul(float4 a, float4 b) {
  return make_float4(a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w);
}
__device__ __forceinline__ float4 f4scale(float4 a, float s) {
  return make_float4(a.x * s, a.y * s, a.z * s, a.w * s);
}
__device__ __forceinline__ float4 f4zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }

// Row-parallel launch geometry for [rows, F] fp32 work vectorised by float4:
// each row is served by `tpr` threads (one float4 each, looping if F/4 > tpr),
// a 256-thread block covers 256/tpr rows.
struct RowGeom {
  int tpr;        // threads per row (power of two, <= 64)
  int rows_per_block;
  int blocks;
};

inline RowGeom row_geom(int64_t rows, int F, int block = 256) {
  int f4 = (F + 3) / 4;
  int tpr = 1;
  while (tpr < f4 && tpr < 64) tpr <<= 1;
  RowGeom g;
  g.tpr = tpr;
  g.rows_per_block = block / tpr;
  g.blocks = (int)std::max<int64_t>(1, (rows + g.rows_per_block - 1) / g.rows_per_block);
  return g;
}

}  // namespace hy
