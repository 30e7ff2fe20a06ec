// Weight-gradient kernel for tall-skinny linears: dW = dY^T X, db = colsum(dY).
//
// Every GNN layer applies small dense maps (64-256 wide) to E ~ 10^4-10^6 edge rows
// or N node rows.  The weight gradient of such a map reduces over the row
// dimension: a [O x I] output with K = E.  Library GEMMs tile the OUTPUT, so a
// 64x64 gradient becomes 1-4 workgroups walking 20k+ rows (rocprof on MI355X:
// 30-105 us per call with 1-4 WGs busy on a 256-CU chip).  Here the reduction
// dimension is split instead:
//   pass 1: workgroup (tile, slab) owns a 64x64 output tile and a slab of rows.  The
//           slab streams through LDS in 32-row chunks, double buffered: all 256
//           threads issue the float4 loads of chunk c+1 before computing chunk c, so
//           one HBM/L2 latency covers 32 rows.  The products run on the fp32 matrix
//           cores (exact fp32, v_mfma_f32_16x16x4_f32), each wave a 32x32 quarter of
//           the tile, and each wave writes its partial tile (+ bias column sums);
//   pass 2: the S slab partials are summed in a fixed order, 4 waves per
//           64-output group (deterministic: no float atomics).
// Narrow problems (I <= 16) keep a VALU form (a 16-wide MFMA tile would be mostly padding).
#include "common.h"

namespace hy {

typedef float f4v __attribute__((ext_vector_type(4)));
constexpr int kWT = 64;  // output tile edge

constexpr int kWC = 32;  // rows per LDS chunk

// Stage a 32-row x 64-col chunk of one operand: thread t -> rows t/16 and t/16+16, float4 column t%16.
// Branch-free: row and column indices are clamped into range and out-of-range values
// zeroed by selects.  (The first version guarded each load with if/else; the
// compiler then drained the memory counter after every load, serialising the
// "next chunk in flight" prefetch.)  VEC: ld, col0 and ncol are multiples of 4.
template <bool VEC>
__device__ __forceinline__ void wg_load(const float* __restrict__ base, int ld, int col0, int ncol, int row0,
                                        int rend, int t, float4 (&r)[2]) {
  const int c = col0 + (t & 15) * 4;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int row_u = row0 + (t >> 4) + 16 * h;
    const bool rv = row_u < rend;
    const float* p = base + (int64_t)min(row_u, rend - 1) * ld;
    float4 v;
    if constexpr (VEC) {
      const bool cv = c < ncol;
      v = *reinterpret_cast<const float4*>(p + min(c, ncol - 4));
      if (!(rv && cv)) v = make_float4(0.f, 0.f, 0.f, 0.f);
    } else {
      const float a0 = p[min(c, ncol - 1)], a1 = p[min(c + 1, ncol - 1)];
      const float a2 = p[min(c + 2, ncol - 1)], a3 = p[min(c + 3, ncol - 1)];
      v.x = rv && c < ncol ? a0 : 0.f;
      v.y = rv && c + 1 < ncol ? a1 : 0.f;
      v.z = rv && c + 2 < ncol ? a2 : 0.f;
      v.w = rv && c + 3 < ncol ? a3 : 0.f;
    }
    r[h] = v;
  }
}

// Same chunk staging through buffer loads whose descriptor covers exactly the slab's rows:
// rows past the slab end read as zeros (hardware range check), columns past ncol read the
// next row's values (or zeros past the slab's last valid element), which only feed output
// columns that are never stored.  No select on loaded values: a select right after the load makes the
// compiler wait for it there, serialising the next-chunk prefetch with this chunk's MFMAs.
typedef __amdgpu_buffer_rsrc_t WgRsrc;
// The range ends at the LAST row's last valid column (not after a full row stride): an
// operand that is a column slice of a wider tensor (offset c0 > 0) would otherwise let the
// over-wide tile reads of its last row run up to c0 floats past the end of the storage —
// an unmapped page when the allocation ends there (observed: illegal address on MI355X).
__device__ __forceinline__ WgRsrc wg_rsrc(const float* base, int ld, int r0, int r1, int ncols) {
  const int n = r1 > r0 ? ((r1 - r0 - 1) * ld + ncols) * 4 : 0;
  return __builtin_amdgcn_make_buffer_rsrc((void*)(base + (int64_t)r0 * ld), (short)0, n, 0x00020000);
}
template <bool VEC>
__device__ __forceinline__ void wg_load_b(WgRsrc rs, int ld, int col0, int rrel, int t, float4 (&r)[2]) {
  const int c = col0 + (t & 15) * 4;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int row = rrel + (t >> 4) + 16 * h;
    const int vo = (row * ld + c) * 4;
    if constexpr (VEC) {
      r[h] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, vo, 0, 0));
    } else {
      r[h].x = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, vo, 0, 0));
      r[h].y = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, vo + 4, 0, 0));
      r[h].z = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, vo + 8, 0, 0));
      r[h].w = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, vo + 12, 0, 0));
    }
  }
}

// part layout: [S][O*I + O]   (dW partial, then db partial)
// smem: 2 buffers x (dY, X) x 32 rows x kLdsW floats (row-major chunks, 80 KB... see below)
//
// MFMA form (v_mfma_f32_16x16x4_f32, exact fp32): wave w owns the 32 x 32 output quarter
// (o half w >> 1, i half w & 1) of the workgroup's 64 x 64 tile as 2 x 2 accumulator tiles;
// per 4-row k-step a lane reads one dY value per o block and one X value per i block
// (row 4s + g of the chunk, column i) and issues 4 independent MFMAs.  The staged rows use a
// stride of 80 floats (== 16 mod 32 banks): the two row groups a ds_read_b32 lane group
// touches land on disjoint bank halves.  Each wave writes its own partial outputs straight
// from the accumulators (no cross-wave fold); the bias column sums ride along as two VALU
// adds per k-step on the waves that hold i block 0.  (The VALU 8x8-register-block form
// before this ran at ~20 % of the fp32 peak on the grouped OC20 step: 87 us.)
constexpr int kLdsW = 80;

template <bool VY, bool VX>
__device__ __forceinline__ void wgrad_partial_body(float4* smem, const float* __restrict__ dY, int ldy,
                                                   const float* __restrict__ X, int ldx, float* __restrict__ part,
                                                   int with_bias, int M, int O, int I, int rows_per_block,
                                                   int tiles_i, int tile, int s) {
  float* Ys = reinterpret_cast<float*>(smem);  // [2][kWC][kLdsW]
  float* Xs = Ys + 2 * kWC * kLdsW;            // [2][kWC][kLdsW]
  const int to0 = (tile / tiles_i) * kWT, ti0 = (tile % tiles_i) * kWT;
  const int r0 = s * rows_per_block, r1 = min(M, r0 + rows_per_block);
  const int t = threadIdx.x;
  const int lane = t & 63, w = t >> 6, i = lane & 15, g = lane >> 4;
  const int ob = (w >> 1) * 32, ib = (w & 1) * 32;  // this wave's quarter of the tile
  const bool bias_w = with_bias && ti0 == 0 && (w & 1) == 0;
  f4v acc[2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) acc[x][y] = f4v{0.f, 0.f, 0.f, 0.f};
  float bacc0 = 0.f, bacc1 = 0.f;
  const int nch = (r1 - r0 + kWC - 1) / kWC;
  float4 ry[2], rx[2];
  auto stage = [&](int b) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int row = (t >> 4) + 16 * h, c4 = (t & 15) * 4;
      *reinterpret_cast<float4*>(Ys + (b * kWC + row) * kLdsW + c4) = ry[h];
      *reinterpret_cast<float4*>(Xs + (b * kWC + row) * kLdsW + c4) = rx[h];
    }
  };
  const WgRsrc rsy = wg_rsrc(dY, ldy, r0, r1, O), rsx = wg_rsrc(X, ldx, r0, r1, I);
  if (nch > 0) {
    wg_load_b<VY>(rsy, ldy, to0, 0, t, ry);
    wg_load_b<VX>(rsx, ldx, ti0, 0, t, rx);
    stage(0);
  }
  __syncthreads();
  for (int c = 0; c < nch; ++c) {
    const int b = c & 1;
    const bool more = c + 1 < nch;
    if (more) {  // issue the next chunk's loads before computing this one
      wg_load_b<VY>(rsy, ldy, to0, (c + 1) * kWC, t, ry);
      wg_load_b<VX>(rsx, ldx, ti0, (c + 1) * kWC, t, rx);
    }
    const float* yb = Ys + b * kWC * kLdsW + ob + i;
    const float* xb = Xs + b * kWC * kLdsW + ib + i;
#pragma unroll
    for (int ks = 0; ks < kWC / 4; ++ks) {
      const int row = 4 * ks + g;
      const float a0 = yb[row * kLdsW], a1 = yb[row * kLdsW + 16];
      const float b0 = xb[row * kLdsW], b1 = xb[row * kLdsW + 16];
      acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b1, acc[1][1], 0, 0, 0);
      if (bias_w) {
        bacc0 += a0;
        bacc1 += a1;
      }
    }
    if (more) stage(b ^ 1);
    __syncthreads();
  }
  // D layout: lane (i, g) holds rows 4g + r (o) of column i (i) of each 16 x 16 tile
  float* P = part + (int64_t)s * ((int64_t)O * I + O);
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int o = to0 + ob + 16 * x + 4 * g + r, ii = ti0 + ib + 16 * y + i;
        if (o < O && ii < I) P[(int64_t)o * I + ii] = acc[x][y][r];
      }
  if (bias_w) {  // rows 4s + g of the chunk went to lane group g: fold the 4 groups
    bacc0 += __shfl_xor(bacc0, 16, 64);
    bacc0 += __shfl_xor(bacc0, 32, 64);
    bacc1 += __shfl_xor(bacc1, 16, 64);
    bacc1 += __shfl_xor(bacc1, 32, 64);
    if (g == 0) {
      const int o0 = to0 + ob + i, o1 = o0 + 16;
      if (o0 < O) P[(int64_t)O * I + o0] = bacc0;
      if (o1 < O) P[(int64_t)O * I + o1] = bacc1;
    }
  }
}

// LDS-DMA form of the same product (both operands 16-byte vectorisable): chunks are copied
// global -> LDS by buffer_load_dwordx4 ... lds (no staging registers, no ds_write pass)
// into a 3-stage ring, two chunks in flight while one is computed: the register-staged form
// above keeps only the next chunk in flight, ~0.5 us of MFMA work against ~1.5 us of load
// latency per chunk.  One wave instruction fills a 4-row x 64-column group (1 KB, lane-
// linear); groups are kGS = 264 floats apart, and k-step s of lane group g reads row
// s % 4 of group 2g + s / 4, so the two row groups of a ds_read_b32 lane group sit 528
// floats (16 banks) apart: conflict-free.  Rows past the slab read zeros (descriptor range);
// the next chunks' copies stay in flight across the barrier (counted vmcnt + raw s_barrier).
constexpr int kGS = 264, kGrp = kWC / 4, kStageF = 2 * kGrp * kGS, kNS = 3;

__device__ __forceinline__ void wgrad_glds_body(float* lds, const float* __restrict__ dY, int ldy,
                                                const float* __restrict__ X, int ldx, float* __restrict__ part,
                                                int with_bias, int M, int O, int I, int rows_per_block, int tiles_i,
                                                int tile, int s) {
  const int to0 = (tile / tiles_i) * kWT, ti0 = (tile % tiles_i) * kWT;
  const int r0 = s * rows_per_block, r1 = min(M, r0 + rows_per_block);
  const int t = threadIdx.x;
  const int lane = t & 63, w = t >> 6, i = lane & 15, g = lane >> 4;
  const int ob = (w >> 1) * 32, ib = (w & 1) * 32;
  const bool bias_w = with_bias && ti0 == 0 && (w & 1) == 0;
  const WgRsrc rsy = wg_rsrc(dY, ldy, r0, r1, O), rsx = wg_rsrc(X, ldx, r0, r1, I);
  // this lane's source element in group w * 2 + j of a chunk: row 4 grp + lane / 16, 4 columns
  const int lr = lane >> 4, lc = (lane & 15) * 4;
  auto issue = [&](int c, int st) {
    float* sb = lds + st * kStageF;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int grp = w * 2 + j, row = 4 * grp + lr;
      // the chunk offset goes into the VGPR offset, not soffset: the descriptor's range check
      // (rows past the slab read zeros) covers the VGPR + instruction offset only
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rsy, (__attribute__((address_space(3))) void*)(sb + grp * kGS), 16, ((c * kWC + row) * ldy + to0 + lc) * 4,
          0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rsx, (__attribute__((address_space(3))) void*)(sb + (kGrp + grp) * kGS), 16,
          ((c * kWC + row) * ldx + ti0 + lc) * 4, 0, 0, 0);
    }
  };
  f4v acc[2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) acc[x][y] = f4v{0.f, 0.f, 0.f, 0.f};
  float bacc0 = 0.f, bacc1 = 0.f;
  const int nch = (r1 - r0 + kWC - 1) / kWC;
  if (nch > 0) issue(0, 0);
  if (nch > 1) issue(1, 1);
  for (int c = 0; c < nch; ++c) {
    if (c + 1 < nch)
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // chunk c landed (c + 1 may be in flight)
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's copies of chunk c landed; chunk c - 1 consumed
    __builtin_amdgcn_sched_barrier(0);
    if (c + 2 < nch) issue(c + 2, (c + 2) % kNS);
    const float* yb = lds + (c % kNS) * kStageF + ob + i;
    const float* xb = lds + (c % kNS) * kStageF + kGrp * kGS + ib + i;
#pragma unroll
    for (int ks = 0; ks < kWC / 4; ++ks) {
      const int off = (2 * g + (ks >> 2)) * kGS + (ks & 3) * 64;
      const float a0 = yb[off], a1 = yb[off + 16];
      const float b0 = xb[off], b1 = xb[off + 16];
      acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b1, acc[1][1], 0, 0, 0);
      if (bias_w) {
        bacc0 += a0;
        bacc1 += a1;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  }
  float* P = part + (int64_t)s * ((int64_t)O * I + O);
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int o = to0 + ob + 16 * x + 4 * g + r, ii = ti0 + ib + 16 * y + i;
        if (o < O && ii < I) P[(int64_t)o * I + ii] = acc[x][y][r];
      }
  if (bias_w) {
    bacc0 += __shfl_xor(bacc0, 16, 64);
    bacc0 += __shfl_xor(bacc0, 32, 64);
    bacc1 += __shfl_xor(bacc1, 16, 64);
    bacc1 += __shfl_xor(bacc1, 32, 64);
    if (g == 0) {
      const int o0 = to0 + ob + i, o1 = o0 + 16;
      if (o0 < O) P[(int64_t)O * I + o0] = bacc0;
      if (o1 < O) P[(int64_t)O * I + o1] = bacc1;
    }
  }
}

template <bool VY, bool VX>
__global__ void __launch_bounds__(256) wgrad_partial_kernel(const float* __restrict__ dY, int ldy,
                                                            const float* __restrict__ X, int ldx,
                                                            float* __restrict__ part, int with_bias, int M, int O,
                                                            int I, int rows_per_block, int tiles_i) {
  __shared__ float4 smem[2 * 2 * kWC * kLdsW / 4];
  wgrad_partial_body<VY, VX>(smem, dY, ldy, X, ldx, part, with_bias, M, O, I, rows_per_block, tiles_i, blockIdx.x,
                             blockIdx.y);
}

// out[j] = sum_s part[s * ld + j]; block = 64 outputs x 16 waves splitting s; fixed order
constexpr int kSpWaves = 16;
__global__ void __launch_bounds__(64 * kSpWaves) sum_partials_kernel(const float* __restrict__ part,
                                                                     float* __restrict__ out, int S, int64_t n,
                                                                     int64_t ld) {
  __shared__ float red[kSpWaves][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t j = (int64_t)blockIdx.x * 64 + lane;
  float a[4] = {0.f, 0.f, 0.f, 0.f};
  if (j < n) {
    int s = w, k = 0;
    for (; s + 3 * kSpWaves < S; s += 4 * kSpWaves) {
#pragma unroll
      for (int q = 0; q < 4; ++q) a[q] += part[(int64_t)(s + q * kSpWaves) * ld + j];
    }
    for (; s < S; s += kSpWaves, ++k) a[k & 3] += part[(int64_t)s * ld + j];
  }
  red[w][lane] = (a[0] + a[1]) + (a[2] + a[3]);
  __syncthreads();
  if (w == 0 && j < n) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < kSpWaves; ++q) t += red[q][lane];
    out[j] = t;
  }
}

std::tuple<at::Tensor, at::Tensor> linear_wgrad(const at::Tensor& dY_, const at::Tensor& X_, bool with_bias) {
  HY_CHECK_CUDA(dY_);
  auto dY = dY_.stride(1) == 1 ? dY_ : dY_.contiguous();
  auto X = X_.stride(1) == 1 ? X_ : X_.contiguous();
  HY_CHECK_F32(dY);
  HY_CHECK_F32(X);
  HY_CHECK(dY.dim() == 2 && X.dim() == 2 && dY.size(0) == X.size(0), "wgrad expects dY [M,O], X [M,I]");
  const int64_t M = dY.size(0);
  const int O = (int)dY.size(1), I = (int)X.size(1);
  const int64_t n = (int64_t)O * I + (with_bias ? O : 0);
  auto out = at::empty({n}, dY.options());
  auto dW = out.narrow(0, 0, (int64_t)O * I).view({O, I});
  auto db = with_bias ? out.narrow(0, (int64_t)O * I, O) : at::empty({0}, dY.options());
  if (M == 0) {
    out.zero_();
    return {dW, db};
  }
  const int tiles_o = ceil_div(O, kWT), tiles_i = ceil_div(I, kWT);
  const int tiles = tiles_o * tiles_i;
  // One workgroup's 64x64 tile costs 64 FMAs per lane per row, so a slab must stay
  // short for the grid to fill 256 CUs: >= 32 rows (one LDS chunk) per slab and up to
  // ~512 workgroups (measured: 128-row slabs -> 22 WGs for a 2816-row node GEMM,
  // 16 us; the partial-sum pass is cheap next to that).
  int S = (int)std::min<int64_t>(ceil_div(M, kWC), std::max(1, 512 / tiles));
  S = std::max(S, 1);
  int rpb = (int)((M + S - 1) / S);
  rpb = ceil_div(rpb, kWC) * kWC;
  S = ceil_div(M, rpb);
  const int64_t ld = (int64_t)O * I + O;
  auto part = at::empty({S, ld}, dY.options());
  dim3 grid(tiles, S);
  // float4 path: row stride, width AND base address 16-byte aligned (a column-narrowed
  // view can have an odd storage offset)
  auto al16 = [](const at::Tensor& t) { return (reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0; };
  const bool vy = (dY.stride(0) & 3) == 0 && (O & 3) == 0 && al16(dY);
  const bool vx = (X.stride(0) & 3) == 0 && (I & 3) == 0 && al16(X);
#define HY_WGRAD(A, B)                                                                                            \
  wgrad_partial_kernel<A, B><<<grid, 256, 0, stream()>>>(dY.data_ptr<float>(), (int)dY.stride(0),               \
                                                         X.data_ptr<float>(), (int)X.stride(0), part.data_ptr<float>(), \
                                                         with_bias ? 1 : 0, (int)M, O, I, rpb, tiles_i)
  if (vy && vx)
    HY_WGRAD(true, true);
  else if (vy)
    HY_WGRAD(true, false);
  else if (vx)
    HY_WGRAD(false, true);
  else
    HY_WGRAD(false, false);
#undef HY_WGRAD
  // dW block [0, O*I) and bias block [O*I, O*I+O) are contiguous in both part and out
  sum_partials_kernel<<<ceil_div(n, 64), 64 * kSpWaves, 0, stream()>>>(part.data_ptr<float>(), out.data_ptr<float>(), S, n, ld);
  return {dW, db};
}


// ---------------------------------------------------------------------------------------
// Grouped (deferred) weight gradients: every tall linear of a backward pass records
// (dY, X, W.grad, b.grad) instead of launching its own wgrad pair; after backward ONE
// partial launch covers all of them (each workgroup looks up its problem in the kernarg
// table) and ONE reduce launch sums the slab partials in a fixed order and writes or
// accumulates into the gradient tensors.  Replaces 2 launches per linear (~33 pairs per
// GPS+PNAPlus step) with 2 per step, and the merged grid fills the chip.
constexpr int kWgMaxP = 36;  // 36 x 96 B of kernel arguments + hidden arguments < 4 KB
constexpr int kWgMaxSlabs = 64;

struct WgProb {
  const float* dy;
  const float* x;
  float* dw;
  float* db;  // nullptr: no bias
  int64_t part_off;  // float offset of this problem's [S][ld] partials in the workspace
  int ldy, ldx, M, O, I, tiles_i, S, rpb;
  int wg0;    // first partial-kernel workgroup of this problem
  int rwg0;   // first reduce-kernel workgroup
  int vec;    // bit0: dY float4 path, bit1: X float4 path
  int accumulate;
  int ldw;    // row stride of dW (a column block of a wider weight gradient: ldw > I)
  int trans;  // the problem was swapped (dY <-> X): dW is written transposed
};

struct WgArgs {
  WgProb p[kWgMaxP];
  float* ws;  // slab partials of all problems
  int n;
};

typedef __attribute__((address_space(4))) const WgArgs KWgArgs;
typedef __attribute__((address_space(4))) const WgProb KWgProb;

__device__ __forceinline__ int wg_find(KWgArgs* A, int b, bool reduce) {
  int pi = 0;
  for (int j = 1; j < A->n; ++j)
    if (b >= (reduce ? A->p[j].rwg0 : A->p[j].wg0)) pi = j;
  return pi;
}

// Narrow problems (I <= 16: radial-basis, embedding and frequency weights over E rows): a
// 64 x 64 register tile would waste >= 75% of its FMAs, so the lane owns one output row o
// (64 per workgroup) and all I columns; waves stride the slab's rows (4 in flight each),
// folded in a fixed order through LDS.  Same partial layout as wgrad_partial_body.
constexpr int kWgNarrow = 16;

__device__ __forceinline__ void wgrad_narrow_body(float4* smem, const float* __restrict__ dY, int ldy,
                                                  const float* __restrict__ X, int ldx, float* __restrict__ part,
                                                  int with_bias, int M, int O, int I, int rows_per_block, int tile,
                                                  int s) {
  constexpr int ST = kWgNarrow + 1;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int o = tile * 64 + lane, oc = min(o, O - 1);
  const int r0 = s * rows_per_block, r1 = min(M, r0 + rows_per_block);
  float* xs = reinterpret_cast<float*>(smem);  // [64 rows][ST]: the chunk's X rows, broadcast reads
  float acc[kWgNarrow], bacc = 0.f;
#pragma unroll
  for (int k = 0; k < kWgNarrow; ++k) acc[k] = 0.f;
  // buffer loads over exactly the slab's rows: rows past it read as zeros; X columns past I
  // (and dY columns past O) only feed outputs that are never stored (no selects on loads)
  const WgRsrc rsy = wg_rsrc(dY, ldy, r0, r1, O), rsx = wg_rsrc(X, ldx, r0, r1, I);
  for (int c0 = r0; c0 < r1; c0 += 64) {
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 64 * kWgNarrow / 256; ++q) {
      const int idx = threadIdx.x + 256 * q, c = idx / kWgNarrow, k = idx % kWgNarrow;
      xs[c * ST + k] = __builtin_bit_cast(
          float, __builtin_amdgcn_raw_buffer_load_b32(rsx, ((c0 - r0 + c) * ldx + min(k, I - 1)) * 4, 0, 0));
    }
    // this wave's 16 rows of the chunk: all dY loads in flight before the FMAs
    float y[16];
#pragma unroll
    for (int u = 0; u < 16; ++u)
      y[u] = __builtin_bit_cast(
          float, __builtin_amdgcn_raw_buffer_load_b32(rsy, ((c0 - r0 + w * 16 + u) * ldy + oc) * 4, 0, 0));
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const float* xr = xs + (w * 16 + u) * ST;
      bacc += y[u];
#pragma unroll
      for (int k = 0; k < kWgNarrow; ++k) acc[k] = fmaf(y[u], xr[k], acc[k]);
    }
  }
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem);  // [4][64][ST]
#pragma unroll
  for (int k = 0; k < kWgNarrow; ++k) red[(w * 64 + lane) * ST + k] = acc[k];
  red[(w * 64 + lane) * ST + kWgNarrow] = bacc;
  __syncthreads();
  float* P = part + (int64_t)s * ((int64_t)O * I + O);
  for (int idx = threadIdx.x; idx < 64 * ST; idx += 256) {
    const int ol = idx / ST, k = idx % ST, oo = tile * 64 + ol;
    if (oo >= O) continue;
    const float v = ((red[(0 * 64 + ol) * ST + k] + red[(1 * 64 + ol) * ST + k]) + red[(2 * 64 + ol) * ST + k]) +
                    red[(3 * 64 + ol) * ST + k];
    if (k < I)
      P[(int64_t)oo * I + k] = v;
    else if (k == kWgNarrow && with_bias)
      P[(int64_t)O * I + oo] = v;
  }
}

// One launch for every vectorisable problem: wide ones (I > 16) on the LDS-DMA MFMA body,
// narrow ones on the VALU body.  The LDS ring (3 workgroups per CU) bounds the occupancy
// either way, so the narrow body's registers cost nothing, and narrow workgroups fill the
// wide ones' tail.  Problems with an operand that is not 16-byte vectorisable go to a
// second launch on the register-staged MFMA body (its scalar-load variants would otherwise
// set this kernel's register count).
template <bool FALLBACK>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3)))
wgrad_grouped_partial_kernel(WgArgs) {
  __shared__ float4 smem[(FALLBACK ? 2 * 2 * kWC * kLdsW : kNS * kStageF) / 4];
  KWgArgs* A = (KWgArgs*)__builtin_amdgcn_kernarg_segment_ptr();
  const int b = blockIdx.x;
  const int pi = wg_find(A, b, false);
  KWgProb& P = A->p[pi];
  const int local = b - P.wg0;
  const int tiles = ((P.O + kWT - 1) / kWT) * P.tiles_i;
  const int tile = local % tiles, s = local / tiles;
  float* part = A->ws + P.part_off;
  const int wb = P.db != nullptr ? 1 : 0;
  if constexpr (!FALLBACK) {
    if (P.vec & 4)
      wgrad_narrow_body(smem, P.dy, P.ldy, P.x, P.ldx, part, wb, P.M, P.O, P.I, P.rpb, tile, s);
    else
      wgrad_glds_body(reinterpret_cast<float*>(smem), P.dy, P.ldy, P.x, P.ldx, part, wb, P.M, P.O, P.I, P.rpb,
                      P.tiles_i, tile, s);
  } else {
    switch (P.vec & 3) {
      case 1: wgrad_partial_body<true, false>(smem, P.dy, P.ldy, P.x, P.ldx, part, wb, P.M, P.O, P.I, P.rpb, P.tiles_i, tile, s); break;
      case 2: wgrad_partial_body<false, true>(smem, P.dy, P.ldy, P.x, P.ldx, part, wb, P.M, P.O, P.I, P.rpb, P.tiles_i, tile, s); break;
      default: wgrad_partial_body<false, false>(smem, P.dy, P.ldy, P.x, P.ldx, part, wb, P.M, P.O, P.I, P.rpb, P.tiles_i, tile, s); break;
    }
  }
}

// reduce: one output per thread, 256 consecutive outputs per workgroup (coalesced 1 KB
// per slab row); each thread walks all S slabs of its output with 8 independent
// accumulators in flight and folds them in a fixed order -> deterministic.  (The first
// form, 64 outputs per workgroup with the slabs split over 4 waves and folded through LDS,
// launched ~5,900 tiny workgroups for the OC20 step and took 33 us.)
__global__ void __launch_bounds__(256) wgrad_grouped_reduce_kernel(WgArgs) {
  KWgArgs* A = (KWgArgs*)__builtin_amdgcn_kernarg_segment_ptr();
  const int b = blockIdx.x;
  const int pi = wg_find(A, b, true);
  KWgProb& P = A->p[pi];
  const float* part = A->ws + P.part_off;
  const int64_t nw = (int64_t)P.O * P.I;
  const int64_t n = nw + (P.db != nullptr ? P.O : 0);
  const int64_t ld = nw + P.O;
  const int64_t j = (int64_t)(b - P.rwg0) * 256 + threadIdx.x;
  if (j >= n) return;
  const int S = P.S;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int s0 = 0;
  for (; s0 + 8 <= S; s0 += 8) {
#pragma unroll
    for (int u = 0; u < 8; ++u) acc[u] += part[(int64_t)(s0 + u) * ld + j];
  }
#pragma unroll
  for (int u = 0; u < 8; ++u)
    if (s0 + u < S) acc[u] += part[(int64_t)(s0 + u) * ld + j];
  const float v = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  float* dst = j < nw ? (P.trans ? P.dw + (j % P.I) * P.ldw + (j / P.I) : P.dw + (j / P.I) * P.ldw + (j % P.I))
                      : P.db + (j - nw);
  *dst = P.accumulate ? *dst + v : v;
}

void linear_wgrad_grouped(at::TensorList dYs, at::TensorList Xs, at::TensorList dWs, at::TensorList dbs,
                          at::IntArrayRef accumulate) {
  const int64_t n = (int64_t)dYs.size();
  HY_CHECK(Xs.size() == (size_t)n && dWs.size() == (size_t)n && dbs.size() == (size_t)n &&
               accumulate.size() == (size_t)n,
           "linear_wgrad_grouped: list lengths differ");
  for (int64_t c0 = 0; c0 < n; c0 += kWgMaxP) {
    const int cnt = (int)std::min<int64_t>(kWgMaxP, n - c0);
    WgArgs a{};  // every problem: the reduce launch
    a.n = cnt;
    std::vector<at::Tensor> keep;
    int64_t part_total = 0;
    int wg = 0, wg_fb = 0, rwg = 0;
    // rows per slab: the largest power of two (<= 1024) that still gives the merged grid
    // >= 768 workgroups (3 per CU: the MFMA body is latency-, not issue-bound, so a CU
    // wants a few resident workgroups), down to one 32-row LDS chunk
    int rps = 1024;
    for (; rps > kWC; rps /= 2) {
      int64_t tot = 0;
      for (int q = 0; q < cnt; ++q) {
        const auto& dY = dYs[c0 + q];
        tot += (int64_t)ceil_div(dY.size(1), kWT) * ceil_div(Xs[c0 + q].size(1), kWT) * ceil_div(dY.size(0), rps);
      }
      if (tot >= 768) break;
    }
    for (int q = 0; q < cnt; ++q) {
      const int64_t k = c0 + q;
      auto dY = dYs[k].stride(1) == 1 ? dYs[k] : dYs[k].contiguous();
      auto X = Xs[k].stride(1) == 1 ? Xs[k] : Xs[k].contiguous();
      // a wide-input, narrow-output map without bias (e.g. DimeNet's sbf projection
      // [T, 42] -> 8 over ~10^5 triplet rows): dW^T = X^T dY is a narrow problem, whose
      // VALU body has no 64 x 64 tile to waste 7/8 of and needs no 16-byte operands
      const bool swap = X.size(1) > kWgNarrow && dY.size(1) <= kWgNarrow && !(dbs[k].defined() && dbs[k].numel() > 0);
      if (swap) std::swap(dY, X);
      keep.push_back(dY);
      keep.push_back(X);
      HY_CHECK(dY.is_cuda() && X.is_cuda() && dY.scalar_type() == at::kFloat && X.scalar_type() == at::kFloat,
               "linear_wgrad_grouped: fp32 GPU operands");
      HY_CHECK(dY.dim() == 2 && X.dim() == 2 && dY.size(0) == X.size(0), "wgrad expects dY [M,O], X [M,I]");
      const int64_t M = dY.size(0);
      const int O = (int)dY.size(1), I = (int)X.size(1);
      const auto& dW = dWs[k];
      HY_CHECK(dW.scalar_type() == at::kFloat && dW.numel() == (int64_t)O * I &&
                   (dW.is_contiguous() || (dW.dim() == 2 && dW.stride(1) == 1 && dW.size(0) == (swap ? I : O))),
               "linear_wgrad_grouped: dW must be fp32 [O, I] with unit column stride");
      const bool hb = dbs[k].defined() && dbs[k].numel() > 0;
      if (hb)
        HY_CHECK(dbs[k].is_contiguous() && dbs[k].numel() == O && dbs[k].scalar_type() == at::kFloat,
                 "linear_wgrad_grouped: db must be a contiguous fp32 [O]");
      HY_CHECK(M > 0, "linear_wgrad_grouped: empty problem");
      WgProb& P = a.p[q];
      P.dy = dY.data_ptr<float>();
      P.x = X.data_ptr<float>();
      P.dw = dW.data_ptr<float>();
      P.ldw = (dW.dim() == 2 && !dW.is_contiguous()) ? (int)dW.stride(0) : (swap ? O : I);
      P.trans = swap ? 1 : 0;
      P.db = hb ? dbs[k].data_ptr<float>() : nullptr;
      P.ldy = (int)dY.stride(0);
      P.ldx = (int)X.stride(0);
      P.M = (int)M;
      P.O = O;
      P.I = I;
      const bool narrow = I <= kWgNarrow;
      auto al16 = [](const at::Tensor& t) { return (reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0; };
      const bool vy = (dY.stride(0) & 3) == 0 && (O & 3) == 0 && al16(dY);
      const bool vx = (X.stride(0) & 3) == 0 && (I & 3) == 0 && al16(X);
      P.tiles_i = narrow ? 1 : ceil_div(I, kWT);
      const int tiles = ceil_div(O, kWT) * P.tiles_i;
      // at most kWgMaxSlabs slabs per problem: the reduce pass reads S partial tiles.  Narrow
      // problems are latency-bound (one dY row per lane per load, partials of O x (I+1)
      // floats): short 128-row slabs, up to 4x as many
      const int rpb = narrow ? std::max(128, ceil_div(ceil_div(M, 4 * kWgMaxSlabs), 64) * 64)
                             : std::max(rps, ceil_div(ceil_div(M, kWgMaxSlabs), kWC) * kWC);
      const int S = ceil_div(M, rpb);
      P.S = S;
      P.rpb = rpb;
      P.part_off = part_total;
      part_total += (int64_t)S * ((int64_t)O * I + O);
      const bool fb = !narrow && (!vy || !vx);
      int& wgc = fb ? wg_fb : wg;
      P.wg0 = wgc;
      wgc += tiles * S;
      P.rwg0 = rwg;
      rwg += ceil_div((int64_t)O * I + (hb ? O : 0), 256);
      P.vec = (vy ? 1 : 0) | (vx ? 2 : 0) | (narrow ? 4 : 0);
      P.accumulate = accumulate[k] ? 1 : 0;
    }
    auto ws = at::empty({part_total}, dYs[c0].options());
    a.ws = ws.data_ptr<float>();
    // per-launch problem tables (wg_find scans p[0..n) for the owning problem)
    WgArgs am{}, af{};
    am.ws = af.ws = a.ws;
    for (int q = 0; q < cnt; ++q) {
      const WgProb& P = a.p[q];
      WgArgs& t = (!(P.vec & 4) && (P.vec & 3) != 3) ? af : am;
      t.p[t.n++] = P;
    }
    if (wg > 0) wgrad_grouped_partial_kernel<false><<<wg, 256, 0, stream()>>>(am);
    if (wg_fb > 0) wgrad_grouped_partial_kernel<true><<<wg_fb, 256, 0, stream()>>>(af);
    wgrad_grouped_reduce_kernel<<<rwg, 256, 0, stream()>>>(a);
  }
}


// ---------------------------------------------------------------------------------------
// Small-K concat-linear forward for edge-sized rows (fp32):
//   y[r, f] = b[f] + sum_j sum_k x_j[r, k] W_j[f, k]     (1-3 inputs, sum K <= 188)
// e.g. the PNAPlus edge term C = r Wr^T + edge_attr Wd^T + bc over ~23k edges, K = 65,
// F = 64.  The library path (bias broadcast copy + GEMM + addmm) cost ~32 us per layer on
// MI355X (three launches, an intermediate written and re-read); this is one pass: a
// 256-thread workgroup stages a 64-row x K tile of the inputs and the transposed
// K x 64 weight tile in LDS, each thread computes a 4 x 4 block (float4 weight reads,
// broadcast input reads) and writes 4 float4 rows (coalesced 256 B per row).
constexpr int kElK = 188;  // (KMAX + 4) floats per staged row
struct ElArgs {
  const float* x[3];
  int ldx[3];
  const float* w[3];
  int k[3];
  int nin;
  const float* b;
  float* y;
  int rows, F;
};

template <int KMAX>
__global__ void __launch_bounds__(256) edge_linear_fwd_kernel(ElArgs a) {
  // row stride: float4-aligned, and rows 4 banks apart (XS % 64 == 4) so the four rows a
  // wave reads per k-step hit disjoint banks
  constexpr int XS = (KMAX + 63) / 64 * 64 + 4;
  __shared__ __attribute__((aligned(16))) float Xs[64][XS];
  __shared__ __attribute__((aligned(16))) float Wt[KMAX][64];
  const int r0 = blockIdx.x * 64, f0 = blockIdx.y * 64;
  const int tid = threadIdx.x;
  // staging: every thread owns one row (r = tid / 4) and a strided set of 4-wide column
  // groups; the loads of a group batch are all issued before their LDS stores (a
  // load -> store loop paid one L2 latency per element)
  const int sr = tid >> 2, sq = tid & 3;
  int K = 0;
  for (int j = 0; j < a.nin; ++j) {
    const int kj = a.k[j];
    const float* xr = a.x[j] + (int64_t)min(r0 + sr, a.rows - 1) * a.ldx[j];
    const float* wr = a.w[j] + (int64_t)min(f0 + sr, a.F - 1) * kj;
    const bool vec = ((kj | a.ldx[j]) & 3) == 0 && (reinterpret_cast<uintptr_t>(a.x[j]) & 15) == 0 &&
                     (reinterpret_cast<uintptr_t>(a.w[j]) & 15) == 0;
    if (vec) {
      const int n4 = kj >> 2;
      for (int m0 = sq; m0 < n4; m0 += 16) {
        float4 xv[4], wv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int m = min(m0 + 4 * u, n4 - 1);
          xv[u] = reinterpret_cast<const float4*>(xr)[m];
          wv[u] = reinterpret_cast<const float4*>(wr)[m];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int m = m0 + 4 * u;
          if (m < n4) {
            const int c = K + 4 * m;
            *reinterpret_cast<float4*>(&Xs[sr][c]) = xv[u];
            Wt[c][sr] = wv[u].x;
            Wt[c + 1][sr] = wv[u].y;
            Wt[c + 2][sr] = wv[u].z;
            Wt[c + 3][sr] = wv[u].w;
          }
        }
      }
    } else {
      for (int c0 = sq; c0 < kj; c0 += 32) {
        float xv[8], wv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int c = min(c0 + 4 * u, kj - 1);
          xv[u] = xr[c];
          wv[u] = wr[c];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int c = c0 + 4 * u;
          if (c < kj) {
            Xs[sr][K + c] = xv[u];
            Wt[K + c][sr] = wv[u];
          }
        }
      }
    }
    K += kj;
  }
  const int K4 = (K + 3) & ~3;
  for (int idx = tid; idx < 64 * (K4 - K); idx += 256) {  // zero the k tail up to a multiple of 4
    const int r = idx / (K4 - K), c = K + idx % (K4 - K);
    Xs[r][c] = 0.f;
    Wt[c][r] = 0.f;
  }
  __syncthreads();
  const int cg = tid & 15, rg = tid >> 4;  // 4 cols (cg*4..), 4 rows (rg*4..)
  float acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[i][q] = 0.f;
  for (int k = 0; k < K4; k += 4) {
    float4 w[4], x[4];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) w[kk] = *reinterpret_cast<const float4*>(&Wt[k + kk][cg * 4]);
#pragma unroll
    for (int i = 0; i < 4; ++i) x[i] = *reinterpret_cast<const float4*>(&Xs[rg * 4 + i][k]);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float xv[4] = {x[i].x, x[i].y, x[i].z, x[i].w};
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        acc[i][0] = fmaf(xv[kk], w[kk].x, acc[i][0]);
        acc[i][1] = fmaf(xv[kk], w[kk].y, acc[i][1]);
        acc[i][2] = fmaf(xv[kk], w[kk].z, acc[i][2]);
        acc[i][3] = fmaf(xv[kk], w[kk].w, acc[i][3]);
      }
    }
  }
  const int f = f0 + cg * 4;
  float bb[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) bb[q] = (a.b != nullptr && f + q < a.F) ? a.b[f + q] : 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = r0 + rg * 4 + i;
    if (r >= a.rows) continue;
    float* yr = a.y + (int64_t)r * a.F;
    if (f + 3 < a.F && (a.F & 3) == 0) {
      *reinterpret_cast<float4*>(yr + f) =
          make_float4(acc[i][0] + bb[0], acc[i][1] + bb[1], acc[i][2] + bb[2], acc[i][3] + bb[3]);
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (f + q < a.F) yr[f + q] = acc[i][q] + bb[q];
    }
  }
}

static void edge_linear_launch(ElArgs& a, int K, int64_t rows, int64_t F) {
  const dim3 grid(ceil_div(rows, 64), ceil_div(F, 64));
  if (K <= 64)  // ~33 KB of LDS: 4 workgroups per CU
    edge_linear_fwd_kernel<64><<<grid, 256, 0, stream()>>>(a);
  else if (K <= 128)  // ~66 KB: 2 workgroups per CU (the PNAPlus+GPS edge term, K = 128)
    edge_linear_fwd_kernel<128><<<grid, 256, 0, stream()>>>(a);
  else
    edge_linear_fwd_kernel<kElK><<<grid, 256, 0, stream()>>>(a);
}

at::Tensor edge_linear_fwd(const std::vector<at::Tensor>& xs, const std::vector<at::Tensor>& ws,
                           const c10::optional<at::Tensor>& b) {
  HY_CHECK(!xs.empty() && xs.size() <= 3 && xs.size() == ws.size(), "edge_linear_fwd: 1-3 (x, W) pairs");
  ElArgs a{};
  a.nin = (int)xs.size();
  const int64_t rows = xs[0].size(0);
  const int64_t F = ws[0].size(0);
  int K = 0;
  std::vector<at::Tensor> keep;
  for (int j = 0; j < a.nin; ++j) {
    HY_CHECK_CUDA(xs[j]);
    HY_CHECK_F32(xs[j]);
    HY_CHECK(xs[j].dim() == 2 && xs[j].size(0) == rows && xs[j].stride(1) == 1, "edge_linear_fwd: x rows");
    auto w = ws[j].contiguous();
    keep.push_back(w);
    HY_CHECK(w.dim() == 2 && w.size(0) == F && w.size(1) == xs[j].size(1), "edge_linear_fwd: W shape");
    a.x[j] = xs[j].data_ptr<float>();
    a.ldx[j] = (int)xs[j].stride(0);
    a.w[j] = w.data_ptr<float>();
    a.k[j] = (int)w.size(1);
    K += a.k[j];
  }
  HY_CHECK(K >= 1 && K <= kElK, "edge_linear_fwd: total K must be in [1, 188], got ", K);
  at::Tensor bc;
  if (b.has_value() && b->defined()) {
    bc = b->contiguous();
    HY_CHECK(bc.numel() == F, "edge_linear_fwd: bias");
    a.b = bc.data_ptr<float>();
  }
  auto y = at::empty({rows, F}, xs[0].options());
  if (rows == 0 || F == 0) return y;
  a.y = y.data_ptr<float>();
  a.rows = (int)rows;
  a.F = (int)F;
  edge_linear_launch(a, K, rows, F);
  return y;
}

}  // namespace hy

TORCH_LIBRARY_FRAGMENT(hydra, m) {
  m.def("linear_wgrad(Tensor dY, Tensor X, bool with_bias) -> (Tensor, Tensor)");
  m.def("edge_linear_fwd(Tensor[] xs, Tensor[] ws, Tensor? b) -> Tensor");
  m.def("linear_wgrad_grouped(Tensor[] dYs, Tensor[] Xs, Tensor(a!)[] dWs, Tensor(b!)[] dbs, int[] accumulate) -> ()");
}

TORCH_LIBRARY_IMPL(hydra, CUDA, m) {
  m.impl("linear_wgrad", hy::linear_wgrad);
  m.impl("edge_linear_fwd", hy::edge_linear_fwd);
  m.impl("linear_wgrad_grouped", hy::linear_wgrad_grouped);
}
