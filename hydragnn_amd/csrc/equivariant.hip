// Channel-wise ("uvu") tensor product with per-edge weights for MACE message passing
// (gfx950).  Reference: e3nn o3.TensorProduct(irreps_node, irreps_sh, irreps_mid,
// instructions "uvu", shared_weights=False) inside MACE's
// RealAgnosticAttResidualInteractionBlock (mace_utils/modules/blocks.py:292-383);
// SURVEY K10.  The second operand is the edge's spherical harmonics (ONE channel per
// l), so for every instruction (l1 x l2 -> l3) and channel u:
//
//   out[e, u, m3] = w[e, u] * sum_{m1, m2} C[m1, m2, m3] x1[e, u, m1] Y[e, m2]
//
// (C already includes sqrt(2 l3 + 1)).  torch.einsum lowers this to batched GEMMs
// with batch = E and 1-7 wide matrices (rocprof: >50% of a MACE step in
// MT256x16x1 bmm kernels).  Here one wave owns one edge: the lanes stride over the
// channels, Y and the CG block are wave-uniform, every lane does its (u, m1, m2,
// m3) loop in registers.  Backward (one pass): dx1 and dw per lane, dY reduced over
// the channels with wave shuffles (deterministic, no atomics).
#include "common.h"

namespace hy {

// instruction table row: l1, l2, l3, m1 (channels), off1, off2, offw, offo, cgoff
constexpr int kInsCols = 9;

__global__ void __launch_bounds__(256) tp_uvu_fwd_kernel(const float* __restrict__ x1, int ld1,
                                                         const float* __restrict__ y, int ld2,
                                                         const float* __restrict__ w, int ldw,
                                                         const int* __restrict__ ins, int nins,
                                                         const float* __restrict__ cg, float* __restrict__ out,
                                                         int ldo, int64_t E) {
  const int lane = threadIdx.x & 63;
  const int64_t e = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (e >= E) return;
  for (int t = 0; t < nins; ++t) {
    const int* r = ins + t * kInsCols;
    const int d1 = 2 * r[0] + 1, d2 = 2 * r[1] + 1, d3 = 2 * r[2] + 1, m = r[3];
    const float* yb = y + e * ld2 + r[5];
    const float* C = cg + r[8];
    for (int u = lane; u < m; u += 64) {
      const float* a = x1 + e * ld1 + r[4] + u * d1;
      const float wu = w[e * ldw + r[6] + u];
      float* o = out + e * ldo + r[7] + u * d3;
      for (int k = 0; k < d3; ++k) {
        float acc = 0.f;
        for (int i = 0; i < d1; ++i) {
          const float ai = a[i];
          for (int j = 0; j < d2; ++j) acc = fmaf(C[(i * d2 + j) * d3 + k] * ai, yb[j], acc);
        }
        o[k] = wu * acc;
      }
    }
  }
}

// gx1, gy must be zero-initialised (several instructions can share an input block).
__global__ void __launch_bounds__(256) tp_uvu_bwd_kernel(const float* __restrict__ go, int ldo,
                                                         const float* __restrict__ x1, int ld1,
                                                         const float* __restrict__ y, int ld2,
                                                         const float* __restrict__ w, int ldw,
                                                         const int* __restrict__ ins, int nins,
                                                         const float* __restrict__ cg, float* __restrict__ gx1,
                                                         float* __restrict__ gy, float* __restrict__ gw, int64_t E) {
  const int lane = threadIdx.x & 63;
  const int64_t e = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (e >= E) return;
  for (int t = 0; t < nins; ++t) {
    const int* r = ins + t * kInsCols;
    const int d1 = 2 * r[0] + 1, d2 = 2 * r[1] + 1, d3 = 2 * r[2] + 1, m = r[3];
    const float* yb = y + e * ld2 + r[5];
    const float* C = cg + r[8];
    float gyl[7] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // this lane's partial dY (d2 <= 7)
    for (int u = lane; u < m; u += 64) {
      const float* a = x1 + e * ld1 + r[4] + u * d1;
      float* ga = gx1 + e * ld1 + r[4] + u * d1;
      const float* g = go + e * ldo + r[7] + u * d3;
      const float wu = w[e * ldw + r[6] + u];
      float gwu = 0.f;
      for (int i = 0; i < d1; ++i) {
        const float ai = a[i];
        float gai = 0.f;
        for (int j = 0; j < d2; ++j) {
          float s = 0.f;  // sum_k C[i, j, k] g[k]
          for (int k = 0; k < d3; ++k) s = fmaf(C[(i * d2 + j) * d3 + k], g[k], s);
          gai = fmaf(s, yb[j], gai);
          gwu = fmaf(s * ai, yb[j], gwu);
          gyl[j] = fmaf(wu * ai, s, gyl[j]);
        }
        ga[i] += wu * gai;
      }
      gw[e * ldw + r[6] + u] = gwu;
    }
    for (int j = 0; j < d2; ++j) {
      const float v = wave_sum(gyl[j]);
      if (lane == 0) gy[e * ld2 + r[5] + j] += v;
    }
  }
}

// ---------------------------------------------------------------- fused convolution
// MACE message + aggregation in one pass (reference blocks.py:354-387):
//   out[n] = sum_{e: dst_e = n} TP(x1[src_e], Y_e, w_e)
// one wave per destination node (edges are destination-sorted: the node's edges are
// one contiguous range), lanes over channels; neither the gathered [E, ld1] operand nor
// the [E, out] message tensor exists.  Backward: d x1 by a source-CSR pass (one wave
// per source node, atomic-free), dY / dw by an edge pass reading go[dst_e].
// Every (l1, l2, l3) instruction body is compiled with its degrees as template constants
// (dispatched by a wave-uniform switch): the per-lane operand and accumulator arrays then
// live in VGPRs with every loop unrolled.  (Runtime-sized loops over fixed-size arrays put
// them in scratch memory: 440-590 us per launch at MACE-multibranch size on MI355X, vs.
// the einsum/bmm composite's ~60 us per call.)
#define HY_TP_LCASES(X)                                                                                   \
  X(0, 0, 0) X(0, 1, 1) X(0, 2, 2) X(0, 3, 3) X(1, 0, 1) X(1, 1, 0) X(1, 1, 1) X(1, 1, 2) X(1, 2, 1)      \
  X(1, 2, 2) X(1, 2, 3) X(1, 3, 2) X(1, 3, 3) X(2, 0, 2) X(2, 1, 1) X(2, 1, 2) X(2, 1, 3) X(2, 2, 0)      \
  X(2, 2, 1) X(2, 2, 2) X(2, 2, 3) X(2, 3, 1) X(2, 3, 2) X(2, 3, 3) X(3, 0, 3) X(3, 1, 2) X(3, 1, 3)      \
  X(3, 2, 1) X(3, 2, 2) X(3, 2, 3) X(3, 3, 0) X(3, 3, 1) X(3, 3, 2) X(3, 3, 3)

__device__ __forceinline__ int tp_lcode(int l1, int l2, int l3) { return (l1 * 4 + l2) * 4 + l3; }

// out[n, u, :] = sum_{e in dst segment} w[e, u] * C(x1[src_e, u, :], Y_e)
// The node's edge list (edge id, gathered node) is held lane-indexed in two VGPRs (lane q:
// edge q of the chunk, loaded once per node) and broadcast with v_readlane: the index loads
// were a dependent memory latency in front of every edge's row loads, paid again for every
// instruction of the product (and, in the source-CSR backward, two of them: perm then dst).
__device__ __forceinline__ int tp_rl(int v, int q) { return __builtin_amdgcn_readlane(v, q); }

template <int L1, int L2, int L3>
__device__ __forceinline__ void conv_fwd_body(const float* __restrict__ x1, int ld1, const float* __restrict__ y,
                                              int ld2, const float* __restrict__ w, int ldw, int v_e, int v_n,
                                              int cnt, const int* r, const float* __restrict__ C, int u,
                                              float* __restrict__ o, bool first) {
  constexpr int D1 = 2 * L1 + 1, D2 = 2 * L2 + 1, D3 = 2 * L3 + 1;
  float acc[D3];
#pragma unroll
  for (int k = 0; k < D3; ++k) acc[k] = first ? 0.f : o[k];
#pragma unroll 2
  for (int q = 0; q < cnt; ++q) {
    const int e = tp_rl(v_e, q);
    const float* a = x1 + (int64_t)tp_rl(v_n, q) * ld1 + r[4] + u * D1;
    const float* yb = y + (int64_t)e * ld2 + r[5];
    const float wu = w[(int64_t)e * ldw + r[6] + u];
    float av[D1], yv[D2];
#pragma unroll
    for (int i = 0; i < D1; ++i) av[i] = a[i] * wu;
#pragma unroll
    for (int j = 0; j < D2; ++j) yv[j] = yb[j];
#pragma unroll
    for (int i = 0; i < D1; ++i)
#pragma unroll
      for (int j = 0; j < D2; ++j) {
        const float p = av[i] * yv[j];
#pragma unroll
        for (int k = 0; k < D3; ++k) acc[k] = fmaf(C[(i * D2 + j) * D3 + k], p, acc[k]);
      }
  }
#pragma unroll
  for (int k = 0; k < D3; ++k) o[k] = acc[k];
}

// gx1[n, u, :] += sum_{e in src segment} w[e, u] * C^T(go[dst_e, u, :], Y_e)
template <int L1, int L2, int L3>
__device__ __forceinline__ void conv_bwdx_body(const float* __restrict__ go, int ldo, const float* __restrict__ y,
                                               int ld2, const float* __restrict__ w, int ldw, int v_e, int v_n,
                                               int cnt, const int* r, const float* __restrict__ C, int u,
                                               float* __restrict__ o) {
  constexpr int D1 = 2 * L1 + 1, D2 = 2 * L2 + 1, D3 = 2 * L3 + 1;
  float ga[D1];
#pragma unroll
  for (int i = 0; i < D1; ++i) ga[i] = 0.f;
#pragma unroll 2
  for (int q = 0; q < cnt; ++q) {
    const int e = tp_rl(v_e, q);
    const float* g = go + (int64_t)tp_rl(v_n, q) * ldo + r[7] + u * D3;
    const float* yb = y + (int64_t)e * ld2 + r[5];
    const float wu = w[(int64_t)e * ldw + r[6] + u];
    float gv[D3], yv[D2];
#pragma unroll
    for (int k = 0; k < D3; ++k) gv[k] = g[k] * wu;
#pragma unroll
    for (int j = 0; j < D2; ++j) yv[j] = yb[j];
#pragma unroll
    for (int i = 0; i < D1; ++i)
#pragma unroll
      for (int j = 0; j < D2; ++j) {
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < D3; ++k) s = fmaf(C[(i * D2 + j) * D3 + k], gv[k], s);
        ga[i] = fmaf(s, yv[j], ga[i]);
      }
  }
#pragma unroll
  for (int i = 0; i < D1; ++i) o[i] += ga[i];
}

// per edge and channel: gw[e, u]; gY partial sums (reduced over the channels by the caller)
template <int L1, int L2, int L3>
__device__ __forceinline__ float conv_bwde_body(const float* __restrict__ a, const float* __restrict__ g,
                                                const float* __restrict__ yb, float wu,
                                                const float* __restrict__ C, float* gyl) {
  constexpr int D1 = 2 * L1 + 1, D2 = 2 * L2 + 1, D3 = 2 * L3 + 1;
  float av[D1], gv[D3], yv[D2];
#pragma unroll
  for (int i = 0; i < D1; ++i) av[i] = a[i];
#pragma unroll
  for (int k = 0; k < D3; ++k) gv[k] = g[k];
#pragma unroll
  for (int j = 0; j < D2; ++j) yv[j] = yb[j];
  float gwu = 0.f;
#pragma unroll
  for (int i = 0; i < D1; ++i)
#pragma unroll
    for (int j = 0; j < D2; ++j) {
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < D3; ++k) s = fmaf(C[(i * D2 + j) * D3 + k], gv[k], s);
      gwu = fmaf(s * av[i], yv[j], gwu);
      gyl[j] = fmaf(wu * av[i], s, gyl[j]);
    }
  return gwu;
}

__global__ void __launch_bounds__(256) tp_conv_fwd_kernel(const float* __restrict__ x1, int ld1,
                                                          const float* __restrict__ y, int ld2,
                                                          const float* __restrict__ w, int ldw,
                                                          const int* __restrict__ ins, int nins,
                                                          const float* __restrict__ cg, const int* __restrict__ src,
                                                          const int* __restrict__ drp, float* __restrict__ out,
                                                          int ldo, int N) {
  const int lane = threadIdx.x & 63;
  const int n = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (n >= N) return;
  const int e0 = drp[n], e1 = drp[n + 1];
  // one wave per (node, instruction): every instruction writes its own output block, and a
  // wave per node walking all of them left the chip at ~4 waves per CU for MACE batches
  const int t = blockIdx.y;
  for (int c0 = e0; c0 < e1 || c0 == e0; c0 += 64) {  // chunks of 64 edges (one, typically)
    const int cnt = min(64, e1 - c0);
    const int q = c0 + (lane < cnt ? lane : 0);
    const int v_e = q, v_n = cnt > 0 ? src[q < e1 ? q : e0] : 0;
    {
      const int* r = ins + t * kInsCols;
      const int m = r[3], code = tp_lcode(r[0], r[1], r[2]);
      const float* C = cg + r[8];
      for (int u = lane; u < m; u += 64) {
        float* o = out + (int64_t)n * ldo + r[7] + u * (2 * r[2] + 1);
        switch (code) {
#define HY_X(a, b, c)                                                                           \
  case (a * 4 + b) * 4 + c:                                                                     \
    conv_fwd_body<a, b, c>(x1, ld1, y, ld2, w, ldw, v_e, v_n, cnt, r, C, u, o, c0 == e0); \
    break;
          HY_TP_LCASES(HY_X)
#undef HY_X
          default:
            break;
        }
      }
    }
    if (cnt <= 0) break;
  }
}

// gx1[j] = sum_{e: src_e = j} w_e * C^T(go[dst_e], Y_e)   (gx1 zero-initialised)
__global__ void __launch_bounds__(256) tp_conv_bwd_x_kernel(const float* __restrict__ go, int ldo,
                                                            const float* __restrict__ y, int ld2,
                                                            const float* __restrict__ w, int ldw,
                                                            const int* __restrict__ ins, int nins,
                                                            const float* __restrict__ cg,
                                                            const int* __restrict__ dst, const int* __restrict__ srp,
                                                            const int* __restrict__ sperm, float* __restrict__ gx1,
                                                            int ld1, int N) {
  const int lane = threadIdx.x & 63;
  const int n = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (n >= N) return;
  // one wave per (node, x1 block): the wave of the block's first instruction accumulates
  // every instruction reading that block (disjoint gx1 slices across waves: no atomics, a
  // fixed summation order); the other instructions' waves exit
  const int tb = blockIdx.y, blk = ins[tb * kInsCols + 4];
  for (int t = 0; t < tb; ++t)
    if (ins[t * kInsCols + 4] == blk) return;
  const int b = srp[n], eN = srp[n + 1];
  for (int c0 = b; c0 < eN; c0 += 64) {  // chunks of 64 source edges (one, typically)
    const int cnt = min(64, eN - c0);
    const int q = c0 + (lane < cnt ? lane : 0);
    const int v_e = sperm ? sperm[q] : q;
    const int v_n = dst[v_e];
    for (int t = tb; t < nins; ++t) {
      const int* r = ins + t * kInsCols;
      if (r[4] != blk) continue;
      const int m = r[3], code = tp_lcode(r[0], r[1], r[2]);
      const float* C = cg + r[8];
      for (int u = lane; u < m; u += 64) {
        float* o = gx1 + (int64_t)n * ld1 + r[4] + u * (2 * r[0] + 1);
        switch (code) {
#define HY_X(a, b_, c)                                                                    \
  case (a * 4 + b_) * 4 + c:                                                              \
    conv_bwdx_body<a, b_, c>(go, ldo, y, ld2, w, ldw, v_e, v_n, cnt, r, C, u, o); \
    break;
          HY_TP_LCASES(HY_X)
#undef HY_X
          default:
            break;
        }
      }
    }
  }
}

// per edge: gw[e] and gy[e] (gy zero-initialised) from x1[src_e] and go[dst_e]; GY = false
// (edge attributes without a gradient: energy training) drops the gY partial sums and their
// per-instruction wave reductions
template <bool GY>
__global__ void __launch_bounds__(256) tp_conv_bwd_e_kernel(const float* __restrict__ go, int ldo,
                                                            const float* __restrict__ x1, int ld1,
                                                            const float* __restrict__ y, int ld2,
                                                            const float* __restrict__ w, int ldw,
                                                            const int* __restrict__ ins, int nins,
                                                            const float* __restrict__ cg, const int* __restrict__ src,
                                                            const int* __restrict__ dst, float* __restrict__ gy,
                                                            float* __restrict__ gw, int64_t E) {
  const int lane = threadIdx.x & 63;
  const int64_t e = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (e >= E) return;
  const int sn = src[e], dn = dst[e];
  for (int t = 0; t < nins; ++t) {
    const int* r = ins + t * kInsCols;
    const int d1 = 2 * r[0] + 1, d2 = 2 * r[1] + 1, d3 = 2 * r[2] + 1, m = r[3];
    const int code = tp_lcode(r[0], r[1], r[2]);
    const float* yb = y + e * ld2 + r[5];
    const float* C = cg + r[8];
    float gyl[7] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int u = lane; u < m; u += 64) {
      const float* a = x1 + (int64_t)sn * ld1 + r[4] + u * d1;
      const float* g = go + (int64_t)dn * ldo + r[7] + u * d3;
      const float wu = w[e * ldw + r[6] + u];
      float gwu = 0.f;
      switch (code) {
#define HY_X(a_, b_, c_)                                              \
  case (a_ * 4 + b_) * 4 + c_:                                        \
    gwu = conv_bwde_body<a_, b_, c_>(a, g, yb, wu, C, gyl);           \
    break;
        HY_TP_LCASES(HY_X)
#undef HY_X
        default:
          break;
      }
      gw[e * ldw + r[6] + u] = gwu;
    }
    // gyl is indexed with compile-time constants inside each case body; the reduction
    // below walks the (uniform) runtime width
    if constexpr (GY) {
#pragma unroll
      for (int j = 0; j < 7; ++j) {
        if (j < d2) {
          const float v = wave_sum(gyl[j]);
          if (lane == 0) gy[e * ld2 + r[5] + j] += v;
        }
      }
    }
  }
}

static void check_ins(const at::Tensor& ins, const at::Tensor& cg) {
  HY_CHECK(ins.device().is_cuda() && ins.scalar_type() == at::kInt && ins.dim() == 2 && ins.size(1) == kInsCols,
           "tp_uvu: instruction table must be int32 [n, 9] on the GPU");
  HY_CHECK(cg.device().is_cuda() && cg.scalar_type() == at::kFloat, "tp_uvu: cg must be fp32 on the GPU");
}

at::Tensor tp_uvu_fwd(const at::Tensor& x1_, const at::Tensor& y_, const at::Tensor& w_, const at::Tensor& ins,
                      const at::Tensor& cg, int64_t out_dim) {
  HY_CHECK_CUDA(x1_);
  auto x1 = x1_.contiguous(), y = y_.contiguous(), w = w_.contiguous();
  HY_CHECK_F32(x1);
  HY_CHECK_F32(y);
  HY_CHECK_F32(w);
  check_ins(ins, cg);
  const int64_t E = x1.size(0);
  HY_CHECK(y.size(0) == E && w.size(0) == E, "tp_uvu: operands must have one row per edge");
  auto out = at::empty({E, out_dim}, x1.options());
  if (E == 0) return out;
  tp_uvu_fwd_kernel<<<ceil_div(E, 4), 256, 0, stream()>>>(
      x1.data_ptr<float>(), (int)x1.size(1), y.data_ptr<float>(), (int)y.size(1), w.data_ptr<float>(),
      (int)w.size(1), ins.data_ptr<int>(), (int)ins.size(0), cg.data_ptr<float>(), out.data_ptr<float>(),
      (int)out_dim, E);
  return out;
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> tp_uvu_bwd(const at::Tensor& go_, const at::Tensor& x1_,
                                                          const at::Tensor& y_, const at::Tensor& w_,
                                                          const at::Tensor& ins, const at::Tensor& cg) {
  auto go = go_.contiguous(), x1 = x1_.contiguous(), y = y_.contiguous(), w = w_.contiguous();
  check_ins(ins, cg);
  const int64_t E = x1.size(0);
  auto gx1 = at::zeros_like(x1), gy = at::zeros_like(y), gw = at::empty_like(w);
  if (E == 0) return {gx1, gy, gw};
  tp_uvu_bwd_kernel<<<ceil_div(E, 4), 256, 0, stream()>>>(
      go.data_ptr<float>(), (int)go.size(1), x1.data_ptr<float>(), (int)x1.size(1), y.data_ptr<float>(),
      (int)y.size(1), w.data_ptr<float>(), (int)w.size(1), ins.data_ptr<int>(), (int)ins.size(0),
      cg.data_ptr<float>(), gx1.data_ptr<float>(), gy.data_ptr<float>(), gw.data_ptr<float>(), E);
  return {gx1, gy, gw};
}

at::Tensor tp_conv_fwd(const at::Tensor& x1, const at::Tensor& y, const at::Tensor& w, const at::Tensor& ins,
                       const at::Tensor& cg, const at::Tensor& src, const at::Tensor& drp, int64_t out_dim) {
  HY_CHECK(x1.is_cuda() && x1.is_contiguous() && y.is_contiguous() && w.is_contiguous(), "tp_conv: contiguous");
  HY_CHECK_F32(x1);
  HY_CHECK_F32(y);
  HY_CHECK_F32(w);
  HY_CHECK_I32(src);
  HY_CHECK_I32(drp);
  check_ins(ins, cg);
  const int64_t N = drp.numel() - 1, E = y.size(0);
  HY_CHECK(x1.size(0) == N && w.size(0) == E && src.numel() == E, "tp_conv: shapes");
  auto out = at::empty({N, out_dim}, x1.options());
  if (N == 0) return out;
  tp_conv_fwd_kernel<<<dim3((unsigned)ceil_div(N, 4), (unsigned)ins.size(0)), 256, 0, stream()>>>(
      x1.data_ptr<float>(), (int)x1.size(1), y.data_ptr<float>(), (int)y.size(1), w.data_ptr<float>(),
      (int)w.size(1), ins.data_ptr<int>(), (int)ins.size(0), cg.data_ptr<float>(), src.data_ptr<int>(),
      drp.data_ptr<int>(), out.data_ptr<float>(), (int)out_dim, (int)N);
  return out;
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> tp_conv_bwd(const at::Tensor& go_, const at::Tensor& x1,
                                                           const at::Tensor& y, const at::Tensor& w,
                                                           const at::Tensor& ins, const at::Tensor& cg,
                                                           const at::Tensor& src, const at::Tensor& dst,
                                                           const at::Tensor& srp,
                                                           const c10::optional<at::Tensor>& sperm, bool need_gy) {
  auto go = go_.contiguous();
  check_ins(ins, cg);
  const int64_t N = x1.size(0), E = y.size(0);
  HY_CHECK(srp.numel() == N + 1 && dst.numel() == E && go.size(0) == N, "tp_conv_bwd: shapes");
  auto gx1 = at::zeros_like(x1), gw = at::empty_like(w);
  auto gy = need_gy ? at::zeros_like(y) : at::empty({0}, y.options());
  if (N)
    tp_conv_bwd_x_kernel<<<dim3((unsigned)ceil_div(N, 4), (unsigned)ins.size(0)), 256, 0, stream()>>>(
        go.data_ptr<float>(), (int)go.size(1), y.data_ptr<float>(), (int)y.size(1), w.data_ptr<float>(),
        (int)w.size(1), ins.data_ptr<int>(), (int)ins.size(0), cg.data_ptr<float>(), dst.data_ptr<int>(),
        srp.data_ptr<int>(), sperm.has_value() ? sperm->data_ptr<int>() : nullptr, gx1.data_ptr<float>(),
        (int)x1.size(1), (int)N);
  if (E) {
    auto* kern = need_gy ? tp_conv_bwd_e_kernel<true> : tp_conv_bwd_e_kernel<false>;
    kern<<<ceil_div(E, 4), 256, 0, stream()>>>(
        go.data_ptr<float>(), (int)go.size(1), x1.data_ptr<float>(), (int)x1.size(1), y.data_ptr<float>(),
        (int)y.size(1), w.data_ptr<float>(), (int)w.size(1), ins.data_ptr<int>(), (int)ins.size(0),
        cg.data_ptr<float>(), src.data_ptr<int>(), dst.data_ptr<int>(), need_gy ? gy.data_ptr<float>() : nullptr,
        gw.data_ptr<float>(), E);
  }
  return {gx1, gy, gw};
}

}  // namespace hy

TORCH_LIBRARY_FRAGMENT(hydra, m) {
  m.def("tp_conv_fwd(Tensor x1, Tensor y, Tensor w, Tensor ins, Tensor cg, Tensor src, Tensor drp, int out_dim) -> Tensor");
  m.def(
      "tp_conv_bwd(Tensor go, Tensor x1, Tensor y, Tensor w, Tensor ins, Tensor cg, Tensor src, Tensor dst, Tensor srp, "
      "Tensor? sperm, bool need_gy=True) -> (Tensor, Tensor, Tensor)");
  m.def("tp_uvu_fwd(Tensor x1, Tensor y, Tensor w, Tensor ins, Tensor cg, int out_dim) -> Tensor");
  m.def("tp_uvu_bwd(Tensor go, Tensor x1, Tensor y, Tensor w, Tensor ins, Tensor cg) -> (Tensor, Tensor, Tensor)");
}

TORCH_LIBRARY_IMPL(hydra, CUDA, m) {
  m.impl("tp_uvu_fwd", hy::tp_uvu_fwd);
  m.impl("tp_conv_fwd", hy::tp_conv_fwd);
  m.impl("tp_conv_bwd", hy::tp_conv_bwd);
  m.impl("tp_uvu_bwd", hy::tp_uvu_bwd);
}
