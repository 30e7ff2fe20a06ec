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

}  // namespace hy

TORCH_LIBRARY_FRAGMENT(hydra, m) {
  m.def("tp_uvu_fwd(Tensor x1, Tensor y, Tensor w, Tensor ins, Tensor cg, int out_dim) -> Tensor");
  m.def("tp_uvu_bwd(Tensor go, Tensor x1, Tensor y, Tensor w, Tensor ins, Tensor cg) -> (Tensor, Tensor, Tensor)");
}

TORCH_LIBRARY_IMPL(hydra, CUDA, m) {
  m.impl("tp_uvu_fwd", hy::tp_uvu_fwd);
  m.impl("tp_uvu_bwd", hy::tp_uvu_bwd);
}
