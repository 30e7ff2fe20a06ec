// Weight-gradient kernel for tall-skinny linears: dW = dY^T X, db = colsum(dY).
//
// Every GNN layer applies small dense maps (64-256 wide) to E ~ 10^4-10^6 edge rows
// or N node rows.  The weight gradient of such a map reduces over the row
// dimension: a [O x I] output with K = E.  Library GEMMs tile the OUTPUT, so a
// 64x64 gradient becomes 1-4 workgroups walking 20k+ rows (rocprof on MI355X:
// 30-105 us per call with 1-4 WGs busy on a 256-CU chip).  Here the reduction
// dimension is split instead:
//   pass 1: workgroup (tile, slab) owns a 64x64 output tile and a slab of rows;
//           each of its 4 waves walks an interleaved subset of the slab's rows
//           with no LDS staging and no barriers (lane = 8x8 register block,
//           2 float4 loads of dY and of X per row feed 64 FMAs; 2-row unroll for
//           load/FMA overlap), the 4 wave accumulators are folded through a
//           padded (conflict-free) LDS image, and one fp32 partial per slab is
//           written (bias sums ride along as an extra row block);
//   pass 2: the S slab partials are summed in a fixed order, 4 waves per
//           64-output group (deterministic: no float atomics).
// fp32 in / fp32 accumulate: FMA-bound at the VALU rate, which on gfx950 equals
// the f32-MFMA rate, so the register-blocked VALU form loses nothing to MFMA.
#include "common.h"

namespace hy {

constexpr int kWT = 64;  // output tile edge

__device__ __forceinline__ void load8(const float* p, int valid, bool vec, float (&v)[8]) {
  if (vec && valid >= 8) {
    const float4 a = *reinterpret_cast<const float4*>(p);
    const float4 b = *reinterpret_cast<const float4*>(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = k < valid ? p[k] : 0.f;
  }
}

// part layout: [S][O*I + O]   (dW partial, then db partial)
__global__ void __launch_bounds__(256) wgrad_partial_kernel(const float* __restrict__ dY, int ldy,
                                                            const float* __restrict__ X, int ldx,
                                                            float* __restrict__ part, int with_bias, int M, int O,
                                                            int I, int rows_per_block, int tiles_i) {
  __shared__ float red[64 * 65];
  const int tile = blockIdx.x;
  const int to0 = (tile / tiles_i) * kWT, ti0 = (tile % tiles_i) * kWT;
  const int s = blockIdx.y;
  const int r0 = s * rows_per_block, r1 = min(M, r0 + rows_per_block);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int ob = (lane >> 3) * 8, ib = (lane & 7) * 8;
  const int ov = max(0, min(8, O - (to0 + ob))), iv = max(0, min(8, I - (ti0 + ib)));
  const bool vy = ((ldy & 3) == 0) && (((to0 + ob) & 3) == 0);
  const bool vx = ((ldx & 3) == 0) && (((ti0 + ib) & 3) == 0);
  const bool bias_lane = with_bias && ti0 == 0 && ib == 0;
  float acc[8][8];
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b) acc[a][b] = 0.f;
  float bacc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const float* yb = dY + to0 + ob;
  const float* xb = X + ti0 + ib;
  int r = r0 + w;
  for (; r + 4 < r1; r += 8) {
    float ya[8], xa[8], yc[8], xc[8];
    load8(yb + (int64_t)r * ldy, ov, vy, ya);
    load8(xb + (int64_t)r * ldx, iv, vx, xa);
    load8(yb + (int64_t)(r + 4) * ldy, ov, vy, yc);
    load8(xb + (int64_t)(r + 4) * ldx, iv, vx, xc);
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
      for (int b = 0; b < 8; ++b) acc[a][b] = fmaf(ya[a], xa[b], acc[a][b]);
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
      for (int b = 0; b < 8; ++b) acc[a][b] = fmaf(yc[a], xc[b], acc[a][b]);
    if (bias_lane) {
#pragma unroll
      for (int a = 0; a < 8; ++a) bacc[a] += ya[a] + yc[a];
    }
  }
  for (; r < r1; r += 4) {
    float ya[8], xa[8];
    load8(yb + (int64_t)r * ldy, ov, vy, ya);
    load8(xb + (int64_t)r * ldx, iv, vx, xa);
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
      for (int b = 0; b < 8; ++b) acc[a][b] = fmaf(ya[a], xa[b], acc[a][b]);
    if (bias_lane) {
#pragma unroll
      for (int a = 0; a < 8; ++a) bacc[a] += ya[a];
    }
  }
  // fold the 4 wave accumulators (fixed order) through LDS, [lane][65] padding
  for (int step = 0; step < 4; ++step) {
    if (w == step) {
#pragma unroll
      for (int a = 0; a < 8; ++a)
#pragma unroll
        for (int b = 0; b < 8; ++b) {
          const float v = acc[a][b] + (step > 0 ? red[lane * 65 + a * 8 + b] : 0.f);
          red[lane * 65 + a * 8 + b] = v;
          acc[a][b] = v;
        }
    }
    __syncthreads();
  }
  // bias: the 8 lanes with ib == 0 in every wave hold partial column sums
  float* P = part + (int64_t)s * ((int64_t)O * I + O);
  if (w == 3) {
#pragma unroll
    for (int a = 0; a < 8; ++a) {
      const int o = to0 + ob + a;
      if (o >= O) break;
#pragma unroll
      for (int b = 0; b < 8; ++b) {
        const int i = ti0 + ib + b;
        if (i < I) P[(int64_t)o * I + i] = acc[a][b];
      }
    }
  }
  if (with_bias && ti0 == 0) {
    __syncthreads();
    if (bias_lane) {
#pragma unroll
      for (int a = 0; a < 8; ++a) red[(w * 8 + (lane >> 3)) * 8 + a] = bacc[a];
    }
    __syncthreads();
    if (w == 0 && lane < 8) {
      // lane k sums the 4 waves' values for o block k (fixed order)
      float t[8];
#pragma unroll
      for (int a = 0; a < 8; ++a) t[a] = 0.f;
      for (int ww = 0; ww < 4; ++ww)
#pragma unroll
        for (int a = 0; a < 8; ++a) t[a] += red[(ww * 8 + lane) * 8 + a];
#pragma unroll
      for (int a = 0; a < 8; ++a) {
        const int o = to0 + lane * 8 + a;
        if (o < O) P[(int64_t)O * I + o] = t[a];
      }
    }
  }
}

// out[j] = sum_s part[s * ld + j]; block = 64 outputs x 4 waves splitting s; fixed order
__global__ void __launch_bounds__(256) sum_partials_kernel(const float* __restrict__ part, float* __restrict__ out,
                                                           int S, int64_t n, int64_t ld) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t j = (int64_t)blockIdx.x * 64 + lane;
  float a0 = 0.f, a1 = 0.f;
  if (j < n) {
    int s = w;
    for (; s + 4 < S; s += 8) {
      a0 += part[(int64_t)s * ld + j];
      a1 += part[(int64_t)(s + 4) * ld + j];
    }
    for (; s < S; s += 4) a0 += part[(int64_t)s * ld + j];
  }
  red[w][lane] = a0 + a1;
  __syncthreads();
  if (w == 0 && j < n) out[j] = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
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
  // ~2 x 256 workgroups; >= 64 rows per slab (16 rows per wave)
  int S = (int)std::min<int64_t>(ceil_div(M, 64), std::max(1, 512 / tiles));
  S = std::max(S, 1);
  const int rpb = (int)((M + S - 1) / S);
  S = ceil_div(M, rpb);
  const int64_t ld = (int64_t)O * I + O;
  auto part = at::empty({S, ld}, dY.options());
  dim3 grid(tiles, S);
  wgrad_partial_kernel<<<grid, 256, 0, stream()>>>(dY.data_ptr<float>(), (int)dY.stride(0), X.data_ptr<float>(),
                                                   (int)X.stride(0), part.data_ptr<float>(), with_bias ? 1 : 0,
                                                   (int)M, O, I, rpb, tiles_i);
  // dW block [0, O*I) and bias block [O*I, O*I+O) are contiguous in both part and out
  sum_partials_kernel<<<ceil_div(n, 64), 256, 0, stream()>>>(part.data_ptr<float>(), out.data_ptr<float>(), S, n, ld);
  return {dW, db};
}

}  // namespace hy

TORCH_LIBRARY_FRAGMENT(hydra, m) { m.def("linear_wgrad(Tensor dY, Tensor X, bool with_bias) -> (Tensor, Tensor)"); }

TORCH_LIBRARY_IMPL(hydra, CUDA, m) { m.impl("linear_wgrad", hy::linear_wgrad); }
