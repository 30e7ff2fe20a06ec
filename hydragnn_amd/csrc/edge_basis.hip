// Radial edge bases (gfx950), SURVEY K7: the distance featurisations of the SchNet / PAINN
// stacks as one launch each way instead of 3-5 elementwise launches.
//   kind 0  Gaussian smearing  out[e,k] = exp(coeff (d_e - off_k)^2)          (SCFStack / PyG GaussianSmearing)
//   kind 1  sinc expansion     out[e,k] = sin((k+1) pi d_e / c) / d_e          (PAINNStack sinc_expansion)
//   kind 2  cosine cutoff      out[e]   = 0.5 (cos(pi d_e / c) + 1) [* (d_e < c) if masked]
// Backward: dd[e] = sum_k g[e,k] d out[e,k] / d d_e (one launch, analytic).  Higher-order
// derivatives (force training) use the composite torch path (ops/geometry.py under
// composite_mode).
#include "common.h"

namespace hy {

constexpr float kPi = 3.14159265358979323846f;

__device__ __forceinline__ float basis_val(int kind, float d, int k, float a, float b, const float* __restrict__ off,
                                           float& deriv) {
  if (kind == 0) {  // a = coeff
    const float t = d - off[k];
    const float v = expf(a * t * t);
    deriv = v * 2.f * a * t;
    return v;
  }
  // kind 1: a = pi / c
  const float w = (float)(k + 1) * a;
  float s, co;
  sincosf(w * d, &s, &co);
  const float inv = 1.f / d;
  deriv = (w * co - s * inv) * inv;
  return s * inv;
}

template <bool BWD>
__global__ void __launch_bounds__(256) edge_basis_kernel(const float* __restrict__ d, const float* __restrict__ off,
                                                         const float* __restrict__ g, float* __restrict__ out,
                                                         int64_t E, int K, int kind, float a, float b, int masked) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (kind == 2) {  // cosine cutoff, one value per edge
    if (t >= E) return;
    const float x = d[t];
    float s, c;
    sincosf(a * x, &s, &c);
    const bool in = !masked || x < b;
    if (BWD)
      out[t] = in ? g[t] * (-0.5f * a * s) : 0.f;
    else
      out[t] = in ? 0.5f * (c + 1.f) : 0.f;
    return;
  }
  if (!BWD) {
    if (t >= E * K) return;
    const int64_t e = t / K;
    const int k = (int)(t % K);
    float dv;
    out[t] = basis_val(kind, d[e], k, a, b, off, dv);
    return;
  }
  if (t >= E) return;  // one thread per edge: dd = sum_k g * dout/dd (fixed order)
  const float x = d[t];
  float acc = 0.f;
  for (int k = 0; k < K; ++k) {
    float dv;
    basis_val(kind, x, k, a, b, off, dv);
    acc = fmaf(g[t * K + k], dv, acc);
  }
  out[t] = acc;
}

// kind 0: (d, offsets, coeff); kind 1: (d, K, pi/c); kind 2: (d, pi/c, cutoff, masked)
at::Tensor edge_basis_fwd(const at::Tensor& d_, const c10::optional<at::Tensor>& off_, int64_t K, int64_t kind,
                          double a, double b, bool masked) {
  HY_CHECK_CUDA(d_);
  auto d = d_.contiguous().view({-1});
  HY_CHECK_F32(d);
  HY_CHECK(kind >= 0 && kind <= 2, "edge_basis: kind 0-2");
  const int64_t E = d.numel();
  at::Tensor off;
  const float* op = nullptr;
  if (kind == 0) {
    HY_CHECK(off_.has_value() && off_->numel() == K, "edge_basis: gaussian offsets");
    off = off_->contiguous();
    HY_CHECK_F32(off);
    op = off.data_ptr<float>();
  }
  auto out = kind == 2 ? at::empty({E}, d.options()) : at::empty({E, K}, d.options());
  const int64_t n = kind == 2 ? E : E * K;
  if (n == 0) return out;
  edge_basis_kernel<false><<<ceil_div(n, 256), 256, 0, stream()>>>(d.data_ptr<float>(), op, nullptr,
                                                                  out.data_ptr<float>(), E, (int)K, (int)kind,
                                                                  (float)a, (float)b, masked ? 1 : 0);
  return out;
}

at::Tensor edge_basis_bwd(const at::Tensor& g_, const at::Tensor& d_, const c10::optional<at::Tensor>& off_, int64_t K,
                          int64_t kind, double a, double b, bool masked) {
  HY_CHECK_CUDA(d_);
  auto d = d_.contiguous().view({-1});
  auto g = g_.contiguous();
  const int64_t E = d.numel();
  HY_CHECK(g.numel() == (kind == 2 ? E : E * K), "edge_basis_bwd: grad shape");
  at::Tensor off;
  const float* op = nullptr;
  if (kind == 0) {
    off = off_->contiguous();
    op = off.data_ptr<float>();
  }
  auto dd = at::empty({E}, d.options());
  if (E == 0) return dd;
  edge_basis_kernel<true><<<ceil_div(E, 256), 256, 0, stream()>>>(d.data_ptr<float>(), op, g.data_ptr<float>(),
                                                                 dd.data_ptr<float>(), E, (int)K, (int)kind, (float)a,
                                                                 (float)b, masked ? 1 : 0);
  return dd;
}

}  // namespace hy

TORCH_LIBRARY_FRAGMENT(hydra, m) {
  m.def("edge_basis_fwd(Tensor d, Tensor? off, int K, int kind, float a, float b, bool masked) -> Tensor");
  m.def("edge_basis_bwd(Tensor g, Tensor d, Tensor? off, int K, int kind, float a, float b, bool masked) -> Tensor");
}

TORCH_LIBRARY_IMPL(hydra, CUDA, m) {
  m.impl("edge_basis_fwd", hy::edge_basis_fwd);
  m.impl("edge_basis_bwd", hy::edge_basis_bwd);
}
