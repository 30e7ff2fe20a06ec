// MACE symmetric contraction (product basis) on gfx950 — reference
// hydragnn/utils/mace_utils/modules/symmetric_contraction.py:92-235:
//
//   out[n, h, L, M] = sum_{nu <= correlation} sum_k W_{L,nu}[elem_n, k, h]
//                     sum_{i_1..i_nu} U_{L,nu}[M, i_1..i_nu, k] x[n, h, i_1] ... x[n, h, i_nu]
//
// The generalised Clebsch-Gordan tensors U are tiny and mostly zero; the host compiles
// their non-zeros (symmetrised, one entry per (L, M, nu, i_1..i_nu, k)) into an entry
// table grouped by output column.  One thread owns one (node, channel): its x row
// (d = (lmax+1)^2 <= 16 values) sits in LDS, the entry stream is wave-uniform (scalar
// loads), and every output column is a register accumulation — no [N, H, M, d^nu]
// intermediates (the torch path materialises them per Horner step).
//
// Backward (one pass per (node, channel)): dx via the product rule (x partials in LDS)
// and per-node weight-gradient rows dWn[n, k, h]; the per-element reduction over nodes is
// the CSR segment sum of ops/segment (deterministic).
#include "common.h"

namespace hy {
namespace sc {

constexpr int MAXD = 16, MAXK = 96;

// entry: i[3] (unused = -1), nu, k (global weight row), value
struct Ent {
  int i0, i1, i2, k;
  float v;
};
// group: output column base (column = base + h * dimL + m), dimL, first / end entry
struct Grp {
  int base, dimL, m, e0, e1;
};

__device__ __forceinline__ float prod_of(const float* xs, const Ent& e) {
  float p = xs[e.i0];
  if (e.i1 >= 0) p *= xs[e.i1];
  if (e.i2 >= 0) p *= xs[e.i2];
  return p;
}

// x [N, H, d]; W [num_elem, Ktot, H]; out [N, out_cols]
__global__ __launch_bounds__(256) void sc_fwd_kernel(const float* __restrict__ x, const int* __restrict__ elem,
                                                     const float* __restrict__ W, const Ent* __restrict__ ents,
                                                     const Grp* __restrict__ grps, int ngrp, int N, int H, int d,
                                                     int Ktot, float* __restrict__ out, int ldo) {
  __shared__ float xs_all[256 * MAXD];
  const int t = blockIdx.x * 256 + threadIdx.x;
  const int n = t / H, h = t % H;
  if (n >= N) return;
  float* xs = xs_all + threadIdx.x * MAXD;
  for (int i = 0; i < d; ++i) xs[i] = x[((int64_t)n * H + h) * d + i];
  const float* Wn = W + (int64_t)elem[n] * Ktot * H + h;
  for (int g = 0; g < ngrp; ++g) {
    const Grp G = grps[g];
    float acc = 0.f;
    for (int q = G.e0; q < G.e1; ++q) {
      const Ent e = ents[q];
      acc = fmaf(e.v * Wn[(int64_t)e.k * H], prod_of(xs, e), acc);
    }
    out[(int64_t)n * ldo + G.base + h * G.dimL + G.m] = acc;
  }
}

__global__ __launch_bounds__(256) void sc_bwd_kernel(const float* __restrict__ gout, int ldo,
                                                     const float* __restrict__ x, const int* __restrict__ elem,
                                                     const float* __restrict__ W, const Ent* __restrict__ ents,
                                                     const Grp* __restrict__ grps, int ngrp, int N, int H, int d,
                                                     int Ktot, float* __restrict__ dx, float* __restrict__ dWn) {
  __shared__ float xs_all[256 * MAXD];
  __shared__ float gx_all[256 * MAXD];
  const int t = blockIdx.x * 256 + threadIdx.x;
  const int n = t / H, h = t % H;
  if (n >= N) return;
  float* xs = xs_all + threadIdx.x * MAXD;
  float* gx = gx_all + threadIdx.x * MAXD;
  for (int i = 0; i < d; ++i) {
    xs[i] = x[((int64_t)n * H + h) * d + i];
    gx[i] = 0.f;
  }
  const float* Wn = W + (int64_t)elem[n] * Ktot * H + h;
  float* dW = dWn + (int64_t)n * Ktot * H + h;
  for (int k = 0; k < Ktot; ++k) dW[(int64_t)k * H] = 0.f;
  for (int g = 0; g < ngrp; ++g) {
    const Grp G = grps[g];
    const float go = gout[(int64_t)n * ldo + G.base + h * G.dimL + G.m];
    if (go == 0.f) continue;
    for (int q = G.e0; q < G.e1; ++q) {
      const Ent e = ents[q];
      const float a = xs[e.i0];
      const float b = e.i1 >= 0 ? xs[e.i1] : 1.f;
      const float c = e.i2 >= 0 ? xs[e.i2] : 1.f;
      dW[(int64_t)e.k * H] += e.v * go * a * b * c;
      const float s = e.v * go * Wn[(int64_t)e.k * H];
      gx[e.i0] += s * b * c;
      if (e.i1 >= 0) gx[e.i1] += s * a * c;
      if (e.i2 >= 0) gx[e.i2] += s * a * b;
    }
  }
  for (int i = 0; i < d; ++i) dx[((int64_t)n * H + h) * d + i] = gx[i];
}

}  // namespace sc

using namespace sc;

static void sc_check(const at::Tensor& x, const at::Tensor& elem, const at::Tensor& W, const at::Tensor& ents,
                     const at::Tensor& grps) {
  HY_CHECK(x.is_cuda() && x.scalar_type() == at::kFloat && x.is_contiguous() && x.dim() == 3 && x.size(2) <= MAXD,
           "symcon: x [N, H, d <= 16] fp32 contiguous");
  HY_CHECK_I32(elem);
  HY_CHECK(elem.numel() == x.size(0), "symcon: elem [N]");
  HY_CHECK(W.scalar_type() == at::kFloat && W.is_contiguous() && W.dim() == 3 && W.size(2) == x.size(1),
           "symcon: W [num_elem, Ktot, H] fp32");
  HY_CHECK(ents.scalar_type() == at::kInt && ents.dim() == 2 && ents.size(1) == 5 && ents.is_contiguous(),
           "symcon: entry table int32 [n, 5] (i0, i1, i2, k, value bits)");
  HY_CHECK(grps.scalar_type() == at::kInt && grps.dim() == 2 && grps.size(1) == 5 && grps.is_contiguous(),
           "symcon: group table int32 [g, 5]");
}

at::Tensor symcon_fwd(const at::Tensor& x, const at::Tensor& elem, const at::Tensor& W, const at::Tensor& ents,
                      const at::Tensor& grps, int64_t out_cols) {
  sc_check(x, elem, W, ents, grps);
  const int64_t N = x.size(0), H = x.size(1), d = x.size(2);
  auto out = at::empty({N, out_cols}, x.options());
  if (N == 0) return out;
  sc_fwd_kernel<<<ceil_div(N * H, 256), 256, 0, stream()>>>(
      x.data_ptr<float>(), elem.data_ptr<int>(), W.data_ptr<float>(), reinterpret_cast<const Ent*>(ents.data_ptr()),
      reinterpret_cast<const Grp*>(grps.data_ptr()), (int)grps.size(0), (int)N, (int)H, (int)d, (int)W.size(1),
      out.data_ptr<float>(), (int)out_cols);
  return out;
}

std::tuple<at::Tensor, at::Tensor> symcon_bwd(const at::Tensor& gout_, const at::Tensor& x, const at::Tensor& elem,
                                              const at::Tensor& W, const at::Tensor& ents, const at::Tensor& grps) {
  sc_check(x, elem, W, ents, grps);
  auto gout = gout_.contiguous();
  const int64_t N = x.size(0), H = x.size(1), d = x.size(2);
  auto dx = at::empty_like(x);
  auto dWn = at::empty({N, W.size(1), H}, x.options());
  if (N == 0) return {dx, dWn};
  sc_bwd_kernel<<<ceil_div(N * H, 256), 256, 0, stream()>>>(
      gout.data_ptr<float>(), (int)gout.size(1), x.data_ptr<float>(), elem.data_ptr<int>(), W.data_ptr<float>(),
      reinterpret_cast<const Ent*>(ents.data_ptr()), reinterpret_cast<const Grp*>(grps.data_ptr()), (int)grps.size(0),
      (int)N, (int)H, (int)d, (int)W.size(1), dx.data_ptr<float>(), dWn.data_ptr<float>());
  return {dx, dWn};
}

}  // namespace hy

TORCH_LIBRARY_FRAGMENT(hydra, m) {
  m.def("symcon_fwd(Tensor x, Tensor elem, Tensor W, Tensor ents, Tensor grps, int out_cols) -> Tensor");
  m.def("symcon_bwd(Tensor gout, Tensor x, Tensor elem, Tensor W, Tensor ents, Tensor grps) -> (Tensor, Tensor)");
}

TORCH_LIBRARY_IMPL(hydra, CUDA, m) {
  m.impl("symcon_fwd", hy::symcon_fwd);
  m.impl("symcon_bwd", hy::symcon_bwd);
}
