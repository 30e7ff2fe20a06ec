// Weight-gradient kernel for tall-skinny linears: dW = dY^T X, db = colsum(dY).
//
// Every GNN layer applies small dense maps (64-256 wide) to E ~ 10^4-10^6 edge rows
// or N node rows.  The weight gradient of such a map reduces over the row
// dimension: a [O x I] output with K = E.  Library GEMMs tile the OUTPUT, so a
// 64x64 gradient becomes 1-4 workgroups walking 20k+ rows (rocprof: 30-105 us per
// call on MI355X, 1-4 WGs on a 256-CU chip).  Here the reduction dimension is
// split instead: each workgroup owns a row slab and a 64x64 output tile
// (4x4 register block per thread, 32-row sub-slabs staged through LDS with
// broadcast-friendly float4 reads), writes an fp32 partial, and a second pass
// sums the partials in a fixed order (deterministic, no float atomics).  The
// bias gradient is folded into the same pass.
#include "common.h"

namespace hy {

constexpr int kWT = 64;    // output tile (O and I)
constexpr int kWR = 32;    // rows per LDS sub-slab

__global__ void __launch_bounds__(256) wgrad_partial_kernel(const float* __restrict__ dY, int ldy,
                                                            const float* __restrict__ X, int ldx,
                                                            float* __restrict__ part, float* __restrict__ dbpart,
                                                            int M, int O, int I, int rows_per_block, int tiles_i) {
  __shared__ float4 Ys[kWR][kWT / 4];
  __shared__ float4 Xs[kWR][kWT / 4];
  const int tile = blockIdx.x;
  const int to0 = (tile / tiles_i) * kWT, ti0 = (tile % tiles_i) * kWT;
  const int s = blockIdx.y;
  const int r0 = s * rows_per_block, r1 = min(M, r0 + rows_per_block);
  const int t = threadIdx.x;
  const int ty = t >> 4, tx = t & 15;  // 16 x 16 threads, 4x4 outputs each
  float acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = 0.f;
  float bacc[4] = {0.f, 0.f, 0.f, 0.f};
  const bool do_bias = dbpart != nullptr && ti0 == 0;
  const bool vy = (ldy % 4 == 0) && (to0 + kWT <= O), vx = (ldx % 4 == 0) && (ti0 + kWT <= I);
  for (int rb = r0; rb < r1; rb += kWR) {
    // stage 32 rows x 64 cols of dY and X (each thread: 2 float4 of each)
    for (int q = t; q < kWR * (kWT / 4); q += 256) {
      const int rr = q / (kWT / 4), c4 = q % (kWT / 4);
      const int row = rb + rr;
      float4 y4 = make_float4(0.f, 0.f, 0.f, 0.f), x4 = y4;
      if (row < r1) {
        const int oc = to0 + c4 * 4, ic = ti0 + c4 * 4;
        const float* yp = dY + (int64_t)row * ldy + oc;
        const float* xp = X + (int64_t)row * ldx + ic;
        if (vy) y4 = *reinterpret_cast<const float4*>(yp);
        else {
          y4.x = oc < O ? yp[0] : 0.f; y4.y = oc + 1 < O ? yp[1] : 0.f;
          y4.z = oc + 2 < O ? yp[2] : 0.f; y4.w = oc + 3 < O ? yp[3] : 0.f;
        }
        if (vx) x4 = *reinterpret_cast<const float4*>(xp);
        else {
          x4.x = ic < I ? xp[0] : 0.f; x4.y = ic + 1 < I ? xp[1] : 0.f;
          x4.z = ic + 2 < I ? xp[2] : 0.f; x4.w = ic + 3 < I ? xp[3] : 0.f;
        }
      }
      Ys[rr][c4] = y4;
      Xs[rr][c4] = x4;
    }
    __syncthreads();
#pragma unroll 8
    for (int rr = 0; rr < kWR; ++rr) {
      const float4 a = Ys[rr][ty];
      const float4 b = Xs[rr][tx];
      const float av[4] = {a.x, a.y, a.z, a.w};
      const float bv[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
      for (int u = 0; u < 4; ++u) {
#pragma unroll
        for (int v = 0; v < 4; ++v) acc[u][v] = fmaf(av[u], bv[v], acc[u][v]);
      }
      if (do_bias && tx == 0) {
#pragma unroll
        for (int u = 0; u < 4; ++u) bacc[u] += av[u];
      }
    }
    __syncthreads();
  }
  float* P = part + (int64_t)s * O * I;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int o = to0 + ty * 4 + u;
    if (o >= O) continue;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int i = ti0 + tx * 4 + v;
      if (i < I) P[(int64_t)o * I + i] = acc[u][v];
    }
  }
  if (do_bias && tx == 0) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int o = to0 + ty * 4 + u;
      if (o < O) dbpart[(int64_t)s * O + o] = bacc[u];
    }
  }
}

// out[j] = sum_s part[s, j]  (j over n elements), fixed summation order
__global__ void __launch_bounds__(256) sum_partials_kernel(const float* __restrict__ part, float* __restrict__ out,
                                                           int S, int64_t n) {
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= n) return;
  float a = 0.f;
  for (int s = 0; s < S; ++s) a += part[(int64_t)s * n + j];
  out[j] = a;
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
  auto dW = at::empty({O, I}, dY.options());
  auto db = with_bias ? at::empty({O}, dY.options()) : at::empty({0}, dY.options());
  if (M == 0) {
    dW.zero_();
    if (with_bias) db.zero_();
    return {dW, db};
  }
  const int tiles_o = ceil_div(O, kWT), tiles_i = ceil_div(I, kWT);
  const int tiles = tiles_o * tiles_i;
  // row slabs: >= 128 rows each, ~1-2k workgroups in total
  int S = (int)std::min<int64_t>(ceil_div(M, 128), std::max(1, 1536 / tiles));
  S = std::max(S, 1);
  const int rpb = (int)(((M + S - 1) / S + kWR - 1) / kWR * kWR);
  S = ceil_div(M, rpb);
  auto part = at::empty({S, O, I}, dY.options());
  auto dbp = with_bias ? at::empty({S, O}, dY.options()) : at::empty({0}, dY.options());
  dim3 grid(tiles, S);
  wgrad_partial_kernel<<<grid, 256, 0, stream()>>>(dY.data_ptr<float>(), (int)dY.stride(0), X.data_ptr<float>(),
                                                   (int)X.stride(0), part.data_ptr<float>(),
                                                   with_bias ? dbp.data_ptr<float>() : nullptr, (int)M, O, I, rpb,
                                                   tiles_i);
  const int64_t n = (int64_t)O * I;
  sum_partials_kernel<<<ceil_div(n, 256), 256, 0, stream()>>>(part.data_ptr<float>(), dW.data_ptr<float>(), S, n);
  if (with_bias)
    sum_partials_kernel<<<ceil_div(O, 256), 256, 0, stream()>>>(dbp.data_ptr<float>(), db.data_ptr<float>(), S, O);
  return {dW, db};
}

}  // namespace hy

TORCH_LIBRARY_FRAGMENT(hydra, m) { m.def("linear_wgrad(Tensor dY, Tensor X, bool with_bias) -> (Tensor, Tensor)"); }

TORCH_LIBRARY_IMPL(hydra, CUDA, m) { m.impl("linear_wgrad", hy::linear_wgrad); }
